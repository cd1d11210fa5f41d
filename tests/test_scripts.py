"""Node bootstrap scripts under stub binaries (systemctl, kubeadm, apt-get, kubectl, ...)
with every written file redirected under ROOT."""
import os
import sys
import subprocess

import pytest

from fake_node import make_node

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(REPO, "deploy", "scripts")
STUBS = ["systemctl", "kubeadm", "apt-get", "apt-mark", "modprobe", "sysctl", "ss", "curl",
         "kubectl", "crio", "crictl", "swapoff", "udevadm", "tar", "crun", "conmon", "chown",
         "git"]


@pytest.fixture()
def env(tmp_path):
    stub = tmp_path / "stubs"
    stub.mkdir()
    log = tmp_path / "calls.log"
    for s in STUBS:
        body = f'#!/bin/bash\necho "{s} $*" >> "{log}"\n'
        if s == "curl":   # honour -o so the files the scripts download exist under ROOT
            body += ('prev=""; for a in "$@"; do [[ "$prev" == "-o" ]] && '
                     'echo "-----BEGIN PGP PUBLIC KEY BLOCK-----" > "$a"; prev="$a"; done\n')
        if s == "kubeadm":
            body += ('if [[ "$1" == init ]]; then echo "kubeadm join 10.0.0.1:6443 --token abc.def '
                     '--discovery-token-ca-cert-hash sha256:00"; fi\n')
        (stub / s).write_text(body)
        (stub / s).chmod(0o755)
    root = tmp_path / "root"
    (root / "etc").mkdir(parents=True)
    (root / "etc" / "fstab").write_text("UUID=1 / ext4 defaults 0 1\n/swap.img none swap sw 0 0\n")
    e = dict(os.environ, PATH=f"{stub}:{os.environ['PATH']}", ROOT=str(root), SUDO_USER="")
    return e, root, log


def sh(script, *args, env, check=True):
    r = subprocess.run(["bash", os.path.join(SCRIPTS, script), *args], env=env,
                       capture_output=True, text=True)
    if check:
        assert r.returncode == 0, r.stdout + r.stderr
    return r


def calls(log):
    return log.read_text().splitlines() if log.exists() else []


def test_control_plane(env):
    e, root, log = env
    sh("k8s_setup.sh", "--role", "control_plane", "--kube-version=v1.32.1", "--yes", "--untaint",
       "--label-gpu", env=e)
    c = calls(log)
    init = [x for x in c if x.startswith("kubeadm init")][0]
    assert "--cri-socket unix:///var/run/crio/crio.sock" in init
    assert "--kubernetes-version v1.32.1" in init and "--pod-network-cidr 192.168.0.0/16" in init
    assert "stable:/v1.32/deb" in (root / "etc/apt/sources.list.d/kubernetes.list").read_text()
    assert "br_netfilter" in (root / "etc/modules-load.d/k8s.conf").read_text()
    assert "ip_forward" in (root / "etc/sysctl.d/99-kubernetes-cri.conf").read_text()
    assert "#/swap.img" in (root / "etc/fstab").read_text()
    assert any("calico.yaml" in x for x in c)
    assert any("taint nodes --all node-role.kubernetes.io/control-plane-" in x for x in c)
    assert any("label node" in x and "gpu=true" in x for x in c)
    assert any(x == "apt-get install -y kubelet kubeadm kubectl" for x in c)
    assert list((root / "var/log").glob("kubeadm-init-*.log"))


def test_fix_coredns(env):
    e, root, log = env
    sh("k8s_setup.sh", "--yes", "--role=cp", "--fix-coredns", env=e)
    c = calls(log)
    patch = [x for x in c if "patch deployment coredns" in x]
    assert patch and '"appArmorProfile":{"type":"Unconfined"}' in patch[0]
    assert any("rollout restart deployment coredns" in x for x in c)


def test_ha_control_plane_endpoint(env):
    e, root, log = env
    sh("k8s_setup.sh", "--yes", "--role=cp", "--control-plane-endpoint=10.0.0.100:6443", env=e)
    init = [x for x in calls(log) if x.startswith("kubeadm init")][0]
    assert "--control-plane-endpoint 10.0.0.100:6443 --upload-certs" in init


def test_worker_join_reference_form(env):
    e, root, log = env
    join = "kubeadm join 10.0.0.1:6443 --token abc --discovery-token-ca-cert-hash sha256:00"
    sh("k8s_setup.sh", "--yes", "--role=node", f"--join={join}", env=e)
    j = [x for x in calls(log) if x.startswith("kubeadm join")]
    assert j and j[0].endswith("--cri-socket unix:///var/run/crio/crio.sock")


def test_worker_join_honours_cri_socket_and_yes_anywhere(env):
    e, root, log = env
    sh("k8s_setup.sh", "--role", "worker", "--join", "kubeadm join 1.2.3.4:6443 --token t",
       "--cri-socket", "unix:///run/containerd/containerd.sock", "--yes", env=e)
    j = [x for x in calls(log) if x.startswith("kubeadm join")][0]
    assert j.endswith("--cri-socket unix:///run/containerd/containerd.sock")


def test_args_validated_before_destructive_steps(env):
    e, root, log = env
    r = sh("k8s_setup.sh", "--yes", env=e, check=False)
    assert r.returncode != 0 and "--role" in r.stderr
    r = sh("k8s_setup.sh", "--role=node", "--yes", env=e, check=False)
    assert r.returncode != 0
    r = sh("k8s_setup.sh", "--role=cp", "--kube-version=latest", "--yes", env=e, check=False)
    assert r.returncode != 0
    assert calls(log) == []          # nothing was reset or installed


def test_dry_run_prints(env):
    e, root, log = env
    r = sh("k8s_setup.sh", "--role=cp", "--yes", "--dry-run", env=e)
    assert "DRY: kubeadm init" in r.stdout and not any(x.startswith("kubeadm init") for x in calls(log))


def test_crio_setup(env):
    e, root, log = env
    (root / "usr/local/bin").mkdir(parents=True)
    sh("crio_setup.sh", "--crio-version", "v1.33", "--proxy=http://127.0.0.1:8118", env=e)
    assert "isv:/cri-o:/stable:/v1.33" in (root / "etc/apt/sources.list.d/cri-o.list").read_text()
    assert "HTTPS_PROXY=http://127.0.0.1:8118" in (root / "etc/systemd/system/crio.service.d/proxy.conf").read_text()
    assert any(x == "apt-get install -y cri-o" for x in calls(log))


def test_gpu_crio_setup(env):
    e, root, log = env
    subprocess.run(["bash", os.path.join(REPO, "native", "build.sh")], check=True)
    make_node(str(root), n_gpus=8)
    sh("gpu-crio-setup.sh", "--with-hook", "--skip-apt", env=e)
    import tomli
    for f in (root / "etc/crio/crio.conf.d").iterdir():     # every drop-in must parse
        tomli.loads(f.read_text())
    conf = (root / "etc/crio/crio.conf.d/99-amd.conf").read_text()
    assert "[crio.runtime.runtimes.amd]" in conf and "default_runtime" not in conf
    assert 'default_runtime = "crun"' in (root / "etc/crio/crio.conf.d/98-crun-default.conf").read_text()
    cdi = (root / "etc/cdi/amd.yaml").read_text()
    assert cdi.count("renderD") >= 16
    assert (root / "usr/share/containers/oci/hooks.d/oci-amd-hook.json").exists()
    assert "hooks_dir" in (root / "etc/crio/crio.conf.d/99-amd-hooks.conf").read_text()
    assert (root / "usr/local/bin/amd-container-runtime").exists()
    assert "render" in (root / "etc/udev/rules.d/70-amdgpu-kfd.rules").read_text()
    c = calls(log)
    assert "systemctl restart crio" in c
    assert any("runtimeclasses.yaml" in x for x in c) and any("amd-gpu-device-plugin.yaml" in x for x in c)
    # --set-default makes the amd handler the default runtime
    sh("gpu-crio-setup.sh", "--set-default", "--skip-apt", "--no-kubectl", env=e)
    assert 'default_runtime = "amd"' in (root / "etc/crio/crio.conf.d/99-amd.conf").read_text()
    assert not (root / "etc/crio/crio.conf.d/98-crun-default.conf").exists()


def test_ha_setup_systemd(env):
    e, root, log = env
    sh("ha_setup.sh", "--vip=10.0.0.100", "--interface", "eth0", "--state=master",
       "--peer=cp1=10.0.0.11", "--peer", "cp2=10.0.0.12", "--peer=cp3=10.0.0.13", "--yes", env=e)
    ka = (root / "etc/keepalived/keepalived.conf").read_text()
    assert "state MASTER" in ka and "priority 101" in ka and "interface eth0" in ka
    assert "10.0.0.100" in ka and "fall 10" in ka and "rise 2" in ka and "interval 3" in ka
    chk = root / "etc/keepalived/check_apiserver.sh"
    assert os.access(chk, os.X_OK) and "127.0.0.1:8443/healthz" in chk.read_text()
    hp = (root / "etc/haproxy/haproxy.cfg").read_text()
    assert "bind *:8443" in hp and "uri /healthz" in hp
    for i in (1, 2, 3):
        assert f"server cp{i} 10.0.0.1{i}:6443 check" in hp
    c = calls(log)
    assert "apt-get install -y keepalived haproxy" in c
    assert "systemctl enable --now keepalived" in c and "systemctl enable --now haproxy" in c
    r = subprocess.run(["bash", "-n", str(chk)], capture_output=True)
    assert r.returncode == 0


def test_ha_setup_static_pods_and_validation(env):
    e, root, log = env
    sh("ha_setup.sh", "--vip=10.0.0.100", "--interface=ens5", "--peer=a=10.0.0.2",
       "--mode=static-pods", "--yes", env=e)
    assert "state BACKUP" in (root / "etc/keepalived/keepalived.conf").read_text()
    man = (root / "etc/kubernetes/manifests/haproxy.yaml").read_text()
    assert "path: /etc/haproxy/haproxy.cfg" in man and "mountPath: /usr/local/etc/haproxy/haproxy.cfg" in man
    assert (root / "etc/kubernetes/manifests/keepalived.yaml").exists()
    assert not any(x.startswith("systemctl") for x in calls(log))
    for bad in (["--interface=eth0", "--peer=a=1.2.3.4"],                     # no vip
                ["--vip=10.0.0.1", "--peer=a=1.2.3.4"],                       # no interface
                ["--vip=10.0.0.1", "--interface=eth0"],                       # no peers
                ["--vip=10.0.0.1", "--interface=eth0", "--peer=a=1.2.3.4", "--lb-port=6443"]):
        r = sh("ha_setup.sh", *bad, env=e, check=False)
        assert r.returncode != 0


def test_proxy_setup(env):
    e, root, log = env
    sh("proxy_setup.sh", "--socks=127.0.0.1:1080", "--ssh-tunnel", "me@bastion", env=e)
    conf = (root / "etc/privoxy/config").read_text()
    assert "listen-address  127.0.0.1:8118" in conf and "forward-socks5  /  127.0.0.1:1080" in conf
    unit = (root / "etc/systemd/system/kgc-socks-tunnel.service").read_text()
    assert "ssh -N -D 127.0.0.1:1080" in unit and "Restart=always" in unit and "me@bastion" in unit
    c = calls(log)
    assert "systemctl restart privoxy" in c and "apt-get install -y privoxy" in c
    assert sh("proxy_setup.sh", env=e, check=False).returncode != 0


def _signed_by(list_file):
    import re
    m = re.search(r"signed-by=([^\]\s]+)", list_file.read_text())
    assert m, list_file.read_text()
    return m.group(1)


def test_apt_signed_by_keys_exist(env):
    """apt rejects a repo whose signed-by file is missing: every list must point at the
    exact file the script downloaded the key to."""
    e, root, log = env
    sh("k8s_setup.sh", "--yes", "--role=cp", env=e)
    sh("crio_setup.sh", env=e)
    for lst in ("kubernetes.list", "cri-o.list"):
        key = _signed_by(root / "etc/apt/sources.list.d" / lst)
        assert (root / key.lstrip("/")).is_file(), f"{lst}: signed-by {key} not written"
        assert key.endswith(".asc")   # armoured key: apt needs the .asc suffix to read it


def _fake_crun(dir_, version):
    dir_.mkdir(parents=True, exist_ok=True)
    c = dir_ / "crun"
    c.write_text(f'#!/bin/bash\n[[ "$1" == --version ]] && echo "crun version {version}"\n')
    c.chmod(0o755)
    return c


def test_gpu_crio_crun_version_gate(env, tmp_path):
    """crun >= 1.21 is used where it is found (its path goes into the crun handler and the
    shim's defaults); an older crun triggers the source build of 1.21 (reference
    gpu-crio-setup.sh:43-56) with the caller's cwd untouched."""
    e, root, log = env
    new = _fake_crun(tmp_path / "newbin", "1.22")
    e2 = dict(e, PATH=f"{new.parent}:{e['PATH']}")
    sh("gpu-crio-setup.sh", "--skip-apt", "--no-kubectl", env=e2)
    conf = (root / "etc/crio/crio.conf.d/98-crun-default.conf").read_text()
    import tomli
    assert tomli.loads(conf)["crio"]["runtime"]["runtimes"]["crun"]["runtime_path"] == str(new)
    assert f"AMD_CONTAINER_RUNTIME_LOWLEVEL={new}" in \
        (root / "etc/default/amd-container-runtime").read_text()
    assert not any(x.startswith("git clone") for x in calls(log))
    old = _fake_crun(tmp_path / "oldbin", "1.14.1")
    e3 = dict(e, PATH=f"{old.parent}:{e['PATH']}", CRUN_SRC_DIR=str(tmp_path / "crun-src"))
    r = sh("gpu-crio-setup.sh", "--skip-apt", "--no-kubectl", env=e3)
    clone = [x for x in calls(log) if x.startswith("git clone")]
    assert clone and "--branch 1.21" in clone[0] and "containers/crun" in clone[0]
    assert "no crun >= 1.21" in r.stderr                 # stub build produced nothing


def test_bringup_dry_run_full_ordered_log(env):
    """bringup.sh --dry-run: every step of the single-node bring-up, in order."""
    e, root, log = env
    r = sh("bringup.sh", "--single-node", "--dry-run",
           "--values=" + os.path.join(REPO, "deploy/values/values-llama3-8b-tp1.yaml"), env=e)
    out = r.stdout
    order = ["step 1: CRI-O", "apt-get install -y cri-o",
             "step 2: Kubernetes", "kubeadm init", "taint nodes --all",
             "step 3: native", "native/build.sh",
             "step 4: GPU enablement", "amd-ctk runtime configure",
             "step 4b: engine image kgc/engine:", "podman build -f", "deploy/docker/Dockerfile",
             "crictl inspecti kgc/engine:",
             "step 5:", "wait for amd.com/gpu on the node",
             "step 6:", "k8s.render -f", "--engine-image kgc/engine --engine-tag",
             "| kubectl apply -f -",
             "step 7:", "wait for serving-engine Deployments", "wait for vllm-router-service",
             "step 8:", "port-forward svc/vllm-router-service 30080:80",
             "curl -sf http://127.0.0.1:30080/v1/models", "bring-up complete"]
    pos = 0
    for needle in order:
        i = out.find(needle, pos)
        assert i >= 0, f"{needle!r} missing or out of order in:\n{out}"
        pos = i
    assert calls(log) == [] or not any(c.startswith("kubeadm init") for c in calls(log))


def test_bringup_waits_and_smokes(env, tmp_path):
    """Deploy + wait + smoke against stub kubectl/curl (node already bootstrapped)."""
    e, root, log = env
    stub = tmp_path / "stubs2"
    stub.mkdir()
    (stub / "kubectl").write_text(f'''#!/bin/bash
echo "kubectl $*" >> "{log}"
case "$*" in
  *"get nodes"*) echo 8 ;;
  *"get endpoints"*) echo 10.0.0.5 ;;
  "apply -f -") cat > "{tmp_path}/applied.yaml" ;;
  *port-forward*) sleep 30 ;;
esac
''')
    (stub / "curl").write_text(f'''#!/bin/bash
echo "curl $*" >> "{log}"
prev=""; for a in "$@"; do [[ "$prev" == "-o" ]] && echo '{{"data": [{{"id": "llama-3-8b"}}]}}' > "$a"; prev="$a"; done
exit 0
''')
    for f in stub.iterdir():
        f.chmod(0o755)
    e2 = dict(e, PATH=f"{stub}:{e['PATH']}", WAIT_INTERVAL="0", PYTHON=sys.executable)
    r = sh("bringup.sh", "--skip-node-setup", "--port=31999", env=e2)
    assert "serving model: llama-3-8b" in r.stdout
    applied = (tmp_path / "applied.yaml").read_text()
    assert "vllm-router-service" in applied and "amd.com/gpu" in applied
    c = calls(log)
    assert any("rollout status deployment" in x for x in c)
    assert any("/v1/completions" in x for x in c)


def _stub(d, name, body):
    d.mkdir(exist_ok=True)
    (d / name).write_text("#!/bin/bash\n" + body)
    (d / name).chmod(0o755)


def test_bringup_missing_image_fails_before_apply(env, tmp_path):
    """No engine image on the node, no podman / buildah, no --image-tar: bring-up stops
    at step 4b with a clear message and applies nothing (instead of 30 min of
    ImagePullBackOff at step 7)."""
    e, root, log = env
    d = tmp_path / "nobuild"
    _stub(d, "crictl", f'echo "crictl $*" >> "{log}"; exit 1\n')
    # hide the default podman / buildah stubs (and any real ones) behind failing lookups
    _stub(d, "podman", "exit 127\n")
    path = f"{d}:{e['PATH']}"
    e2 = dict(e, PATH=path, PYTHON=sys.executable, WAIT_INTERVAL="0")
    r = sh("bringup.sh", "--skip-node-setup", "--no-build", env=e2, check=False)
    assert r.returncode != 0
    assert "not on this node and --no-build" in r.stderr
    assert not any(c.startswith("kubectl apply") for c in calls(log))
    # with building allowed but the build (podman) failing: also stops before apply
    r = sh("bringup.sh", "--skip-node-setup", env=e2, check=False)
    assert r.returncode != 0 and "podman build of kgc/engine" in r.stderr
    assert not any(c.startswith("kubectl apply") for c in calls(log))


def test_bringup_side_loads_image_tar(env, tmp_path):
    """--image-tar: podman load into CRI-O's store, then crictl inspecti, then render with
    exactly that image."""
    e, root, log = env
    tar = tmp_path / "engine.tar"
    tar.write_text("x")
    r = sh("bringup.sh", "--single-node", "--dry-run", f"--image-tar={tar}",
           "--image=registry.local/kgc/engine:test1", env=dict(e, PYTHON=sys.executable))
    out = r.stdout
    i = out.find(f"podman load -i {tar}")
    j = out.find("crictl inspecti registry.local/kgc/engine:test1")
    k = out.find("--engine-image registry.local/kgc/engine --engine-tag test1")
    assert 0 <= i < j < k, out
    assert "podman build" not in out
