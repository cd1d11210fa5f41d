"""libamdgpu-topo, amd-container-runtime (OCI shim), amd-container-hook and amd-ctk
against fake MI355X sysfs / bundle fixtures."""
import json
import os
import subprocess

import pytest
import yaml

from fake_node import make_bundle, make_node

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "native")


@pytest.fixture(scope="session", autouse=True)
def built():
    subprocess.run(["bash", os.path.join(ROOT, "native", "build.sh")], check=True)


def run(tool, *args, env=None, input=None, check=True):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([os.path.join(BIN, tool), *args], capture_output=True, text=True,
                       env=e, input=input)
    if check and r.returncode != 0:
        raise AssertionError(f"{tool} rc={r.returncode}: {r.stderr}")
    return r


def topo(root):
    return json.loads(run("amdgpu-topo", "--root", root).stdout)


def test_topology_8x_mi355x(tmp_path):
    root = make_node(str(tmp_path))
    t = topo(root)
    assert t["kfd_present"]
    g = t["gpus"]
    assert len(g) == 8
    assert all(x["gfx"] == "gfx950" for x in g)
    assert [x["render_minor"] for x in g] == list(range(128, 136))
    assert [x["card"] for x in g] == list(range(8))
    assert all(len(x["xgmi_peers"]) == 7 for x in g)          # full mesh
    assert g[0]["pci_bdf"] == "0000:05:00.0" and g[5]["numa_node"] == 1
    assert g[0]["vram_bytes"] == 288 * 10**9 and g[0]["cu_count"] == 256
    assert all(x["healthy"] for x in g)
    assert "gfx950" in run("amdgpu-topo", "--root", root, "--table").stdout


def test_topology_cpx_and_faults(tmp_path):
    root = make_node(str(tmp_path), n_gpus=2, partitions=4, missing_render=(1,), ras_ue={6: 2})
    g = topo(root)["gpus"]
    assert len(g) == 8 and all(x["partitions"] == 4 for x in g)
    assert [x["partition"] for x in g[:4]] == [0, 1, 2, 3]
    assert not g[1]["healthy"] and "render" in g[1]["health_reason"]
    assert not g[6]["healthy"] and "ue=2" in g[6]["health_reason"]
    assert len(g[0]["xgmi_peers"]) == 4                      # peers on the other GPU only


def test_topo_ctypes_binding(tmp_path):
    from kubernetes_gpu_cluster_amd.k8s.topo import enumerate_gpus
    root = make_node(str(tmp_path), n_gpus=3)
    gpus = enumerate_gpus(root)
    assert [x["index"] for x in gpus] == [0, 1, 2]


def _shim(bundle, root, *extra, env=None):
    return run("amd-container-runtime", "--kgc-dry-run", f"--kgc-root={root}", "create",
               "--bundle", bundle, "ctr1", *extra,
               env=dict(AMD_CONTAINER_RUNTIME_LOG="", **(env or {})))


def test_runtime_shim_injects_devices(tmp_path):
    root = make_node(str(tmp_path / "node"))
    b = make_bundle(str(tmp_path / "b"), env=["AMD_VISIBLE_DEVICES=0,3"])
    cfg = json.loads(_shim(b, root).stdout)
    paths = [d["path"] for d in cfg["linux"]["devices"]]
    assert paths == ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/card0", "/dev/dri/renderD131",
                     "/dev/dri/card3"]
    rules = [r for r in cfg["linux"]["resources"]["devices"] if r.get("allow")]
    assert {(r["major"], r["minor"]) for r in rules} == {(235, 0), (226, 128), (226, 0),
                                                        (226, 131), (226, 3)}
    assert sorted(cfg["process"]["user"]["additionalGids"]) == [44, 109]
    assert "AMD_VISIBLE_DEVICES=0,3" in cfg["process"]["env"]


def test_runtime_shim_annotation_all_and_noop(tmp_path):
    root = make_node(str(tmp_path / "node"), n_gpus=4)
    b = make_bundle(str(tmp_path / "b"), annotations={"amd.com/gpu.devices": "all"})
    cfg = json.loads(_shim(b, root).stdout)
    assert len(cfg["linux"]["devices"]) == 1 + 2 * 4
    b2 = make_bundle(str(tmp_path / "b2"))
    cfg2 = json.loads(_shim(b2, root).stdout)
    assert "devices" not in cfg2["linux"]
    b3 = make_bundle(str(tmp_path / "b3"), env=["AMD_VISIBLE_DEVICES=9"])
    r = run("amd-container-runtime", "--kgc-dry-run", f"--kgc-root={root}", "create",
            "--bundle", b3, "x", env={"AMD_CONTAINER_RUNTIME_LOG": ""}, check=False)
    assert r.returncode == 1 and "out of range" in r.stderr


def test_runtime_shim_execs_lowlevel(tmp_path):
    root = make_node(str(tmp_path / "node"), n_gpus=2)
    b = make_bundle(str(tmp_path / "b"), env=["AMD_VISIBLE_DEVICES=1"])
    log = tmp_path / "argv.txt"
    fake = tmp_path / "fake-crun"
    fake.write_text(f"#!/bin/sh\necho \"$@\" > {log}\n")
    fake.chmod(0o755)
    run("amd-container-runtime", f"--kgc-root={root}", "--root", "/run/x", "create", "--bundle", b,
        "ctr9", env={"AMD_CONTAINER_RUNTIME_LOWLEVEL": str(fake),
                     "AMD_CONTAINER_RUNTIME_LOG": str(tmp_path / "shim.log")})
    assert log.read_text().split() == ["--root", "/run/x", "create", "--bundle", b, "ctr9"]
    cfg = json.load(open(os.path.join(b, "config.json")))
    assert "/dev/dri/renderD129" in [d["path"] for d in cfg["linux"]["devices"]]
    assert "1 GPU(s)" in (tmp_path / "shim.log").read_text()
    # non-create verbs pass straight through
    run("amd-container-runtime", "state", "ctr9", env={"AMD_CONTAINER_RUNTIME_LOWLEVEL": str(fake),
                                                       "AMD_CONTAINER_RUNTIME_LOG": ""})
    assert log.read_text().split() == ["state", "ctr9"]


def test_hook_dry_run(tmp_path):
    root = make_node(str(tmp_path / "node"), n_gpus=2)
    b = make_bundle(str(tmp_path / "b"), env=["AMD_VISIBLE_DEVICES=all"])
    r = run("amd-container-hook", "prestart", "--root", root, "--dry-run",
            input=json.dumps({"ociVersion": "1.0.2", "id": "c", "pid": 1, "bundle": b}))
    lines = r.stdout.strip().splitlines()
    # the container /dev tmpfs only exists in the container's mount namespace: the hook
    # enters it (state.pid) before creating any node
    assert lines[0] == "setns /proc/1/ns/mnt"
    assert lines[1].endswith("/rootfs/dev/kfd c 235 0")
    assert len(lines) == 6
    r = run("amd-container-hook", "createContainer", "--root", root, "--dry-run",
            input=json.dumps({"pid": 7, "bundle": b}))
    assert not r.stdout.startswith("setns")      # already in the container namespace
    r = run("amd-container-hook", "prestart", "--root", root, "--dry-run",
            input=json.dumps({"bundle": make_bundle(str(tmp_path / "b2"))}))
    assert r.stdout == ""
    # a GPU container without a pid cannot be served: fail instead of a silent no-op
    r = subprocess.run([os.path.join(BIN, "amd-container-hook"), "prestart", "--root", root],
                       input=json.dumps({"bundle": b}), capture_output=True, text=True)
    assert r.returncode != 0 and "pid" in r.stderr


def test_ctk(tmp_path):
    root = make_node(str(tmp_path / "node"), n_gpus=2)
    out = tmp_path / "cdi" / "amd.yaml"
    run("amd-ctk", "cdi", "generate", "--root", root, "--output", str(out))
    spec = yaml.safe_load(out.read_text())
    assert spec["kind"] == "amd.com/gpu" and spec["cdiVersion"] == "0.6.0"
    names = [d["name"] for d in spec["devices"]]
    assert names[:2] == ["0", "0x0000000000abc000"] and names[-1] == "all"
    assert spec["containerEdits"]["deviceNodes"][0]["path"] == "/dev/kfd"
    conf = tmp_path / "99-amd.conf"
    run("amd-ctk", "runtime", "configure", "--runtime=crio", f"--config={conf}", "--set-as-default")
    t = conf.read_text()
    assert 'default_runtime = "amd"' in t and "[crio.runtime.runtimes.amd]" in t
    assert 'runtime_path = "/usr/local/bin/amd-container-runtime"' in t
    import tomli
    run("amd-ctk", "runtime", "configure", "--runtime=crio", f"--config={conf}",
        "--set-as-default", "--cdi.enabled=true")
    doc = tomli.loads(conf.read_text())                    # a duplicate table would raise
    rt = doc["crio"]["runtime"]
    assert rt["enable_cdi"] is True and rt["default_runtime"] == "amd"
    assert rt["runtimes"]["amd"]["runtime_type"] == "oci"
    hooks = tmp_path / "99-amd-hooks.conf"
    run("amd-ctk", "crio", "hooks-dir", f"--config={hooks}")
    assert tomli.loads(hooks.read_text())["crio"]["runtime"]["hooks_dir"]
    run("amd-ctk", "hook", "install", "--hooks-dir", str(tmp_path / "hooks.d"))
    h = json.load(open(tmp_path / "hooks.d" / "oci-amd-hook.json"))
    assert h["stages"] == ["prestart"] and h["hook"]["args"] == ["amd-container-hook", "prestart"]
    info = json.loads(run("amd-ctk", "info", "--root", root).stdout)
    assert len(info["gpus"]) == 2


def test_sanitizer_build_clean(tmp_path):
    """ASan/UBSan build of the shim + topo over the fixtures (host-code sanitizers)."""
    subprocess.run(["bash", os.path.join(ROOT, "native", "build.sh")], check=True,
                   env=dict(os.environ, SANITIZE="1"))
    root = make_node(str(tmp_path / "node"), n_gpus=8, partitions=2)
    b = make_bundle(str(tmp_path / "b"), env=["AMD_VISIBLE_DEVICES=0-3,0x0000000000abc005"])
    asan = os.path.join(ROOT, "build", "native-asan")
    for cmd in ([f"{asan}/amdgpu-topo", "--root", root],
                [f"{asan}/amd-container-runtime", "--kgc-dry-run", f"--kgc-root={root}", "create",
                 "--bundle", b, "c"],
                [f"{asan}/amd-ctk", "cdi", "generate", "--root", root]):
        r = subprocess.run(cmd, capture_output=True, text=True,
                           env=dict(os.environ, AMD_CONTAINER_RUNTIME_LOG="",
                                    ASAN_OPTIONS="detect_leaks=1"))
        assert r.returncode == 0, r.stderr
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
