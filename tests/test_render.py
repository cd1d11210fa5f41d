"""values-*.yaml -> manifests renderer (SURVEY.md §2.7 schema) and Helm chart parity."""
import glob
import os
import re

import pytest
import yaml
from hypothesis import given, settings, strategies as st

from kubernetes_gpu_cluster_amd.k8s.render import ValuesError, render, to_yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = sorted(glob.glob(os.path.join(ROOT, "deploy/values/*.yaml")))
REF = sorted(glob.glob("/root/reference/values-01-minimal-example*.yaml"))


def _load(p):
    with open(p) as f:
        return yaml.safe_load(f)


def _by_kind(objs, kind):
    return [o for o in objs if o["kind"] == kind]


def _check_invariants(objs, values):
    deps = [d for d in _by_kind(objs, "Deployment") if d["metadata"]["name"].endswith("-deployment-vllm")]
    assert len(deps) == len(values["servingEngineSpec"]["modelSpec"])
    for d, ms in zip(deps, values["servingEngineSpec"]["modelSpec"]):
        tpl = d["spec"]["template"]
        lab = tpl["metadata"]["labels"]
        assert lab["app.kubernetes.io/name"] == "vllm-stack"
        assert lab["app.kubernetes.io/component"] == "serving-engine"
        c = tpl["spec"]["containers"][0]
        res = c["resources"]
        assert "nvidia.com/gpu" not in str(res)
        if int(ms.get("requestGPU", 1)):
            assert int(res["limits"]["amd.com/gpu"]) >= int(ms.get("requestGPU", 1))
        else:
            assert "amd.com/gpu" not in res["limits"]
            assert "--device" in c["args"]
        shm = [m for m in c["volumeMounts"] if m["mountPath"] == "/dev/shm"]
        assert len(shm) <= 1
        names = [v["name"] for v in tpl["spec"]["volumes"]]
        for m in c["volumeMounts"]:
            assert m["name"] in names
        assert d["spec"]["replicas"] == ms.get("replicaCount", 1)
        assert c["args"][:2] == ["--model", str(ms["modelURL"])]
    svc = [s for s in _by_kind(objs, "Service") if s["metadata"]["name"] == "vllm-router-service"]
    assert svc and svc[0]["spec"]["ports"][0]["port"] == 80


@pytest.mark.parametrize("path", OURS + REF, ids=[os.path.basename(os.path.dirname(p)) + "/" + os.path.basename(p) for p in OURS + REF])
def test_render_all_values(path):
    v = _load(path)
    objs = render(v, release="vllm")
    _check_invariants(objs, v)
    yaml.safe_load_all(to_yaml(objs))     # round-trips


def test_values8_mapping():
    v = _load(os.path.join(ROOT, "deploy/values/values-01-minimal-example8.yaml"))
    dep = render(v)[0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    a = c["args"]
    assert a[a.index("--tensor-parallel-size") + 1] == "2"
    assert a[a.index("--dtype") + 1] == "float16"
    assert "--disable-custom-all-reduce" in a and "--enforce-eager" in a
    assert c["resources"]["limits"]["amd.com/gpu"] == "2"
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["PYTORCH_HIP_ALLOC_CONF"] == "expandable_segments:True"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    shm = [m for m in c["volumeMounts"] if m["mountPath"] == "/dev/shm"]
    assert len(shm) == 1
    assert dep["spec"]["template"]["spec"]["runtimeClassName"] == "crun"
    assert dep["metadata"]["name"] == "vllm-qwen3-deployment-vllm"


def test_pp_and_cpu():
    v4 = _load(os.path.join(ROOT, "deploy/values/values-01-minimal-example4.yaml"))
    c = render(v4)[0]["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == "2"      # PP=2 folded into the pod
    vc = _load(os.path.join(ROOT, "deploy/values/values-opt125m-cpu.yaml"))
    c = render(vc)[0]["spec"]["template"]["spec"]["containers"][0]
    assert "amd.com/gpu" not in c["resources"]["requests"]
    assert c["args"][c["args"].index("--device") + 1] == "cpu"


def test_errors():
    with pytest.raises(ValuesError):
        render({})
    with pytest.raises(ValuesError):
        render({"servingEngineSpec": {"modelSpec": [{"name": "a"}]}})
    with pytest.raises(ValuesError):
        render({"servingEngineSpec": {"modelSpec": [{"name": "a", "modelURL": "x", "bogus": 1}]}})
    with pytest.raises(ValuesError):
        render({"servingEngineSpec": {"modelSpec": [{"name": "a", "modelURL": "x"},
                                                    {"name": "A", "modelURL": "y"}]}})


def test_golden_example2():
    v = _load(os.path.join(ROOT, "deploy/values/values-01-minimal-example2.yaml"))
    got = to_yaml(render(v, release="vllm"))
    golden = os.path.join(ROOT, "tests/fixtures/golden_values2.yaml")
    if not os.path.exists(golden):
        with open(golden, "w") as f:
            f.write(got)
    assert got == open(golden).read()


_name = st.text(alphabet="abcdefghijklmnopqrstuvwxyz0123456789-", min_size=1, max_size=20)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.fixed_dictionaries(
    {"name": _name, "modelURL": st.sampled_from(["meta-llama/Meta-Llama-3-8B", "/models/x"])},
    optional={"replicaCount": st.integers(1, 8), "requestGPU": st.integers(0, 8),
              "requestCPU": st.integers(1, 64), "shmSize": st.sampled_from(["1Gi", "10Gi"]),
              "vllmConfig": st.fixed_dictionaries({}, optional={
                  "tensorParallelSize": st.sampled_from([1, 2, 4, 8]),
                  "pipelineParallelSize": st.sampled_from([1, 2]),
                  "maxModelLen": st.integers(128, 131072),
                  "extraArgs": st.lists(st.sampled_from(["--enforce-eager", "--trust-remote-code"]))})}),
    min_size=1, max_size=3, unique_by=lambda d: d["name"].strip("-") or "x"))
def test_render_fuzz(specs):
    v = {"servingEngineSpec": {"runtimeClassName": "", "modelSpec": specs}}
    try:
        objs = render(v)
    except ValuesError:
        return    # e.g. names colliding after DNS-1123 normalisation
    _check_invariants(objs, v)
    for d, ms in zip([o for o in objs if o["kind"] == "Deployment"], specs):
        vc = ms.get("vllmConfig") or {}
        deg = vc.get("tensorParallelSize", 1) * vc.get("pipelineParallelSize", 1)
        if ms.get("requestGPU", 1):
            lim = int(d["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"])
            assert lim == max(ms.get("requestGPU", 1), deg)


def test_chart_parity():
    """No helm binary offline: the chart must expose the same contract as the renderer."""
    tpl = open(os.path.join(ROOT, "deploy/chart/kgc-stack/templates/engine.yaml")).read()
    rt = open(os.path.join(ROOT, "deploy/chart/kgc-stack/templates/router.yaml")).read()
    for key in ("servingEngineSpec.modelSpec", "replicaCount", "requestCPU", "requestMemory",
                "amd.com/gpu", "tensorParallelSize", "pipelineParallelSize",
                "gpuMemoryUtilization", "maxModelLen", "extraArgs", "shmSize", "nodeSelector",
                "affinity", "topologySpreadConstraints", "tolerations", "runtimeClassName",
                "extraVolumes", "extraVolumeMounts", "-deployment-vllm", "serving-engine",
                "PYTORCH_HIP_ALLOC_CONF", "/health", "vllmApiKey", "VLLM_API_KEY"):
        assert key in tpl, key
    assert "vllm-router-service" in rt and "port: 80" in rt and "pods" in rt
    assert "vllmApiKey" in rt and "VLLM_API_KEY" in rt
    for t in (tpl, rt):
        opens = len(re.findall(r"{{-?\s*(if|range|with|define)\b", t))
        assert opens == len(re.findall(r"{{-?\s*end\s*-?}}", t))
    mn = open(os.path.join(ROOT, "deploy/chart/kgc-stack/templates/engine-multinode.yaml")).read()
    for key in ("StatefulSet", "worker_node", "--nnodes", "--master-addr", "--node-rank-offset",
                "apps.kubernetes.io/pod-index", "clusterIP: None", "engine-worker"):
        assert key in mn, key
    # template actions balance (no helm binary: a cheap structural check)
    for t in (tpl, mn):
        opens = len(re.findall(r"{{-?\s*(if|range|with|define)\b", t))
        assert opens == len(re.findall(r"{{-?\s*end\s*-?}}", t))
    yaml.safe_load(open(os.path.join(ROOT, "deploy/chart/kgc-stack/Chart.yaml")))


def test_multinode_leader_worker_statefulsets():
    v = _load(os.path.join(ROOT, "deploy/values/multinode/values-llama3-70b-2nodes-pp2.yaml"))
    objs = render(v, release="vllm", namespace="ml")
    sts = {o["metadata"]["name"]: o for o in _by_kind(objs, "StatefulSet")}
    assert set(sts) == {"vllm-llama3-70b-2n-leader", "vllm-llama3-70b-2n-worker"}
    assert not [d for d in _by_kind(objs, "Deployment") if "-deployment-vllm" in d["metadata"]["name"]]
    lead, wk = sts["vllm-llama3-70b-2n-leader"], sts["vllm-llama3-70b-2n-worker"]
    assert lead["spec"]["replicas"] == 1 and wk["spec"]["replicas"] == 1
    lc = lead["spec"]["template"]["spec"]["containers"][0]
    wc = wk["spec"]["template"]["spec"]["containers"][0]
    master = "vllm-llama3-70b-2n-leader-0.vllm-llama3-70b-2n-leader.ml.svc.cluster.local"
    for c in (lc, wc):
        a = c["args"]
        assert a[a.index("--nnodes") + 1] == "2" and a[a.index("--master-addr") + 1] == master
        assert c["resources"]["limits"]["amd.com/gpu"] == "4"
    assert lc["command"][-1].endswith("api_server") and "--node-rank" in lc["args"]
    assert wc["command"][-1].endswith("worker_node")
    assert "--host" not in wc["args"] and "--port" not in wc["args"]
    assert any(e["name"] == "POD_INDEX" for e in wc["env"])
    # the router discovers only the leader; the engine Service targets only the leader
    assert lead["spec"]["template"]["metadata"]["labels"]["app.kubernetes.io/component"] == "serving-engine"
    assert wk["spec"]["template"]["metadata"]["labels"]["app.kubernetes.io/component"] == "engine-worker"
    heads = [s for s in _by_kind(objs, "Service") if s["spec"].get("clusterIP") == "None"]
    assert {s["metadata"]["name"] for s in heads} == set(sts)
    # the rendered argv parse with each entrypoint's own parser
    from kubernetes_gpu_cluster_amd.entrypoints.api_server import make_parser as api_parser
    from kubernetes_gpu_cluster_amd.entrypoints.worker_node import make_parser as wk_parser
    ns = wk_parser().parse_args(wc["args"])
    assert ns.nnodes == 2 and ns.node_rank_offset == 1 and ns.pipeline_parallel_size == 2
    ns = api_parser().parse_args(lc["args"])
    assert ns.nnodes == 2 and ns.node_rank == 0 and ns.tensor_parallel_size == 4
    bad = dict(v)
    bad["servingEngineSpec"]["modelSpec"][0]["vllmConfig"]["nnodes"] = 3
    with pytest.raises(ValuesError):
        render(bad)


def test_vllm_api_key_reaches_engines_and_router():
    """servingEngineSpec.vllmApiKey (vllm-stack chart key): VLLM_API_KEY on every engine
    container and on the router (its /v1/models polls), literal or from a Secret."""
    v = _load(os.path.join(ROOT, "deploy/values/values-llama3-8b-tp1.yaml"))
    for key, want in (("k1", {"name": "VLLM_API_KEY", "value": "k1"}),
                      ({"secretName": "s", "secretKey": "api"},
                       {"name": "VLLM_API_KEY", "valueFrom": {"secretKeyRef": {"name": "s", "key": "api"}}})):
        v2 = dict(v, servingEngineSpec=dict(v["servingEngineSpec"], vllmApiKey=key))
        objs = render(v2)
        deps = _by_kind(objs, "Deployment")
        assert deps and all(want in d["spec"]["template"]["spec"]["containers"][0]["env"]
                            for d in deps), deps
    objs = render(v)
    assert all(not any(e.get("name") == "VLLM_API_KEY"
                       for e in d["spec"]["template"]["spec"]["containers"][0].get("env", []))
               for d in _by_kind(objs, "Deployment"))
