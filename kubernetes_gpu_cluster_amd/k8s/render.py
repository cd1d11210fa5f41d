"""Helm-values -> Kubernetes manifests renderer (the source of truth behind the
``deploy/chart`` Helm chart).

Input is the reference's ``servingEngineSpec`` values schema (SURVEY.md §2.7;
``values-01-minimal-example*.yaml``).  Output: per ``modelSpec`` entry an engine
Deployment + Service, plus the router Deployment, ``vllm-router-service`` (port 80,
``old_README.md:1175``) and the router's pod-discovery RBAC.

MI355X-specific mapping:
* ``requestGPU`` -> ``amd.com/gpu`` (reference chart: ``nvidia.com/gpu``); the pod
  requests max(requestGPU, tensorParallelSize * pipelineParallelSize) GPUs, since
  TP/PP run as in-pod workers over xGMI (a ``raySpec`` head is accepted and folded
  into the same pod).  ``requestGPU: 0`` renders a CPU pod (``--device cpu``).
* ``vllm/vllm-openai`` images map to the kgc engine image (``--engine-image``).
* ``shmSize`` -> one ``/dev/shm`` Memory emptyDir; an ``extraVolumeMounts`` entry
  for /dev/shm is de-duplicated (values-8/9 declare both forms).
* Engine pods carry ``app.kubernetes.io/name: vllm-stack`` and
  ``app.kubernetes.io/component: serving-engine`` so the reference's anti-affinity /
  spread selectors (``values-01-minimal-example2.yaml:23-49``) bind.
* ``PYTORCH_CUDA_ALLOC_CONF`` is mirrored to ``PYTORCH_HIP_ALLOC_CONF``.
* ``lmcacheConfig`` is accepted and ignored.
* ``vllmConfig.nnodes: N`` (extension) spreads one engine replica over N pods, the
  in-house replacement for the reference's KubeRay multi-pod pipeline
  (``values-01-minimal-example4.yaml:42-46``): a leader StatefulSet (API server +
  driver, node 0; ``component: serving-engine``, so the router discovers only it) and
  a worker StatefulSet of N-1 pods (``entrypoints.worker_node``, node rank = pod index
  + 1), rendezvousing at the leader's stable headless-service DNS name.  Each pod gets
  ``requestGPU`` GPUs, or ``tp*pp/N`` when that is larger.

    python -m kubernetes_gpu_cluster_amd.k8s.render -f values.yaml --release vllm | kubectl apply -f -
"""
from __future__ import annotations

import argparse
import copy
import re
import sys
from typing import Any, Optional

import yaml

DEFAULT_ENGINE_IMAGE = "kgc/engine"
DEFAULT_ENGINE_TAG = "0.1.0-rocm7.2-gfx950"
ROUTER_SERVICE = "vllm-router-service"
ENGINE_PORT = 8000
ROUTER_PORT = 8080
LABEL_NAME = "vllm-stack"

_KNOWN_MODEL_KEYS = {
    "name", "repository", "tag", "imagePullPolicy", "modelURL", "replicaCount", "requestCPU",
    "requestMemory", "requestGPU", "env", "shmSize", "vllmConfig", "lmcacheConfig",
    "nodeSelector", "extraVolumes", "extraVolumeMounts", "raySpec", "affinity",
    "topologySpreadConstraints", "tolerations", "hf_token", "pvcStorage", "labels",
    "annotations", "priorityClassName", "serviceAccountName",
}


class ValuesError(ValueError):
    pass


def _dns1123(s: str) -> str:
    s = re.sub(r"[^a-z0-9-]+", "-", s.lower()).strip("-")
    return s[:63] or "model"


def _flag_present(args: list[str], flag: str) -> bool:
    return any(a == flag or a.startswith(flag + "=") for a in args)


def engine_args(ms: dict) -> list[str]:
    """vllmConfig + extraArgs -> engine argv (``api_server``)."""
    vc = ms.get("vllmConfig") or {}
    extra = [str(a) for a in (vc.get("extraArgs") or [])]
    args = ["--model", str(ms["modelURL"]), "--host", "0.0.0.0", "--port", str(ENGINE_PORT),
            "--served-model-name", str(ms["modelURL"])]
    mapping = [("tensorParallelSize", "--tensor-parallel-size"),
               ("pipelineParallelSize", "--pipeline-parallel-size"),
               ("gpuMemoryUtilization", "--gpu-memory-utilization"),
               ("maxModelLen", "--max-model-len"), ("dtype", "--dtype"),
               ("maxNumSeqs", "--max-num-seqs"), ("blockSize", "--block-size"),
               ("maxNumBatchedTokens", "--max-num-batched-tokens"),
               ("apiServerCount", "--api-server-count")]
    for key, flag in mapping:
        if key in vc and vc[key] is not None and not _flag_present(extra, flag):
            args += [flag, str(vc[key])]
    for key, flag in [("enableChunkedPrefill", "--enable-chunked-prefill"),
                      ("enforceEager", "--enforce-eager"),
                      ("disableCustomAllReduce", "--disable-custom-all-reduce"),
                      ("trustRemoteCode", "--trust-remote-code")]:
        if vc.get(key) and not _flag_present(extra, flag):
            args.append(flag)
    if int(ms.get("requestGPU", 1) or 0) == 0 and not _flag_present(extra, "--device"):
        args += ["--device", "cpu"]
    return args + extra


def _parallel_degree(args: list[str]) -> int:
    def get(flag, default=1):
        for i, a in enumerate(args):
            if a == flag and i + 1 < len(args):
                return int(args[i + 1])
            if a.startswith(flag + "="):
                return int(a.split("=", 1)[1])
        return default
    tp = get("--tensor-parallel-size", get("-tp"))
    pp = get("--pipeline-parallel-size", get("-pp"))
    return tp * pp


def _image(ms: dict, engine_image: str, engine_tag: str) -> str:
    repo = ms.get("repository") or engine_image
    if repo.startswith("vllm/") or "vllm-openai" in repo:
        return f"{engine_image}:{engine_tag}"
    return f"{repo}:{ms.get('tag', engine_tag)}"


def _quantity(v: Any) -> str:
    return str(v)


def render_engine(ms: dict, release: str, namespace: str, engine_image: str, engine_tag: str,
                  runtime_class: str) -> list[dict]:
    unknown = set(ms) - _KNOWN_MODEL_KEYS
    if unknown:
        raise ValuesError(f"modelSpec {ms.get('name')}: unknown keys {sorted(unknown)}")
    for req in ("name", "modelURL"):
        if req not in ms:
            raise ValuesError(f"modelSpec entry missing required key {req!r}")
    name = _dns1123(ms["name"])
    args = engine_args(ms)
    gpus = int(ms.get("requestGPU", 1) or 0)
    degree = _parallel_degree(args)
    if gpus:
        gpus = max(gpus, degree)
    labels = {"app.kubernetes.io/name": LABEL_NAME, "app.kubernetes.io/component": "serving-engine",
              "app.kubernetes.io/instance": release, "model": name}
    labels.update(ms.get("labels") or {})
    resources = {"requests": {}, "limits": {}}
    if "requestCPU" in ms:
        resources["requests"]["cpu"] = _quantity(ms["requestCPU"])
    if "requestMemory" in ms:
        resources["requests"]["memory"] = _quantity(ms["requestMemory"])
        resources["limits"]["memory"] = _quantity(ms["requestMemory"])
    if gpus:
        resources["requests"]["amd.com/gpu"] = str(gpus)
        resources["limits"]["amd.com/gpu"] = str(gpus)
    env = [dict(e) for e in (ms.get("env") or [])]
    names = {e["name"] for e in env}
    for e in list(env):
        if e["name"] == "PYTORCH_CUDA_ALLOC_CONF" and "PYTORCH_HIP_ALLOC_CONF" not in names:
            env.append({"name": "PYTORCH_HIP_ALLOC_CONF", "value": e.get("value", "")})
    if gpus and "HSA_ENABLE_IPC_MODE_LEGACY" not in names:
        env.append({"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"})
    volumes = [copy.deepcopy(v) for v in (ms.get("extraVolumes") or [])]
    mounts = [copy.deepcopy(m) for m in (ms.get("extraVolumeMounts") or [])]
    shm_mount = next((m for m in mounts if m.get("mountPath") == "/dev/shm"), None)
    if ms.get("shmSize"):
        if shm_mount is None:
            volumes.append({"name": "dshm", "emptyDir": {"medium": "Memory",
                                                         "sizeLimit": str(ms["shmSize"])}})
            mounts.append({"name": "dshm", "mountPath": "/dev/shm"})
        else:   # one /dev/shm: the declared volume wins, sized by shmSize
            for v in volumes:
                if v.get("name") == shm_mount["name"] and "emptyDir" in v:
                    v["emptyDir"].setdefault("medium", "Memory")
                    v["emptyDir"]["sizeLimit"] = str(ms["shmSize"])
    seen = set()
    dedup = []
    for m in mounts:
        if m.get("mountPath") in seen:
            continue
        seen.add(m.get("mountPath"))
        dedup.append(m)
    mounts = dedup
    probe = {"httpGet": {"path": "/health", "port": ENGINE_PORT}, "periodSeconds": 10,
             "failureThreshold": 3, "timeoutSeconds": 5}
    container = {
        "name": "engine", "image": _image(ms, engine_image, engine_tag),
        "imagePullPolicy": ms.get("imagePullPolicy", "IfNotPresent"),
        "command": ["python3", "-m", "kubernetes_gpu_cluster_amd.entrypoints.api_server"],
        "args": args, "ports": [{"name": "http", "containerPort": ENGINE_PORT}],
        "env": env, "resources": resources, "volumeMounts": mounts,
        "startupProbe": dict(probe, failureThreshold=180),
        "readinessProbe": probe, "livenessProbe": dict(probe, failureThreshold=6),
    }
    spec: dict = {"containers": [container], "volumes": volumes}
    rc = ms.get("runtimeClassName", runtime_class)
    if rc:
        spec["runtimeClassName"] = rc
    for k in ("nodeSelector", "affinity", "topologySpreadConstraints", "tolerations",
              "priorityClassName", "serviceAccountName"):
        if ms.get(k):
            spec[k] = copy.deepcopy(ms[k])
    dep_name = f"{release}-{name}-deployment-vllm"
    sel = {"app.kubernetes.io/instance": release, "model": name,
           "app.kubernetes.io/component": "serving-engine"}
    nnodes = int((ms.get("vllmConfig") or {}).get("nnodes", 1) or 1)
    if nnodes > 1:
        return _render_multinode(ms, name, release, namespace, nnodes, degree, labels, sel,
                                 spec, container)
    dep = {"apiVersion": "apps/v1", "kind": "Deployment",
           "metadata": {"name": dep_name, "namespace": namespace, "labels": labels,
                        "annotations": dict(ms.get("annotations") or {})},
           "spec": {"replicas": int(ms.get("replicaCount", 1)),
                    "selector": {"matchLabels": sel},
                    "strategy": {"type": "Recreate"} if gpus else {"type": "RollingUpdate"},
                    "template": {"metadata": {"labels": labels}, "spec": spec}}}
    svc = {"apiVersion": "v1", "kind": "Service",
           "metadata": {"name": f"{release}-{name}-engine-service", "namespace": namespace,
                        "labels": labels},
           "spec": {"selector": sel, "ports": [{"name": "http", "port": ENGINE_PORT,
                                                "targetPort": ENGINE_PORT}]}}
    return [dep, svc]


MULTINODE_PORT = 29500


def _render_multinode(ms, name, release, namespace, nnodes, degree, labels, sel, spec,
                      container) -> list[dict]:
    """Leader + worker StatefulSets for one engine spread over ``nnodes`` pods."""
    if degree % nnodes:
        raise ValuesError(f"modelSpec {name}: tp*pp={degree} does not split over nnodes={nnodes}")
    per_pod = max(int(ms.get("requestGPU", 1) or 0), degree // nnodes)
    if int(ms.get("requestGPU", 1) or 0) == 0:
        raise ValuesError(f"modelSpec {name}: nnodes > 1 needs GPU pods")
    for obj in (container["resources"]["requests"], container["resources"]["limits"]):
        obj["amd.com/gpu"] = str(per_pod)
    out = []
    reps = int(ms.get("replicaCount", 1))
    for r in range(reps):
        sfx = f"-r{r}" if reps > 1 else ""
        leader, worker = f"{release}-{name}{sfx}-leader", f"{release}-{name}{sfx}-worker"
        group = {"kgc.amd.com/engine-group": f"{name}{sfx}"}
        master = f"{leader}-0.{leader}.{namespace}.svc.cluster.local"
        dist = ["--nnodes", str(nnodes), "--master-addr", master,
                "--master-port", str(MULTINODE_PORT)]
        lead_c = copy.deepcopy(container)
        lead_c["args"] = list(container["args"]) + ["--node-rank", "0"] + dist
        lead_c["ports"] = lead_c["ports"] + [{"name": "dist", "containerPort": MULTINODE_PORT}]
        wk_c = copy.deepcopy(container)
        wk_args, skip = [], False
        for a in container["args"]:          # api-server-only flags
            if skip:
                skip = False
                continue
            if a in ("--host", "--port"):
                skip = True
                continue
            wk_args.append(a)
        wk_c["command"] = ["python3", "-m", "kubernetes_gpu_cluster_amd.entrypoints.worker_node"]
        wk_c["args"] = wk_args + dist + ["--node-rank-offset", "1", "--health-port", str(ENGINE_PORT)]
        wk_c["env"] = wk_c["env"] + [{"name": "POD_INDEX", "valueFrom": {"fieldRef": {
            "fieldPath": "metadata.labels['apps.kubernetes.io/pod-index']"}}}]
        wk_c["ports"] = [{"name": "health", "containerPort": ENGINE_PORT}]
        lead_labels = dict(labels, **group)
        wk_labels = dict(labels, **group)
        wk_labels["app.kubernetes.io/component"] = "engine-worker"
        lead_sel = dict(sel, **group)
        wk_sel = dict(sel, **group)
        wk_sel["app.kubernetes.io/component"] = "engine-worker"

        def sts(nm, lbl, sl, c, replicas):
            pod_spec = copy.deepcopy(spec)
            pod_spec["containers"] = [c]
            return {"apiVersion": "apps/v1", "kind": "StatefulSet",
                    "metadata": {"name": nm, "namespace": namespace, "labels": lbl,
                                 "annotations": dict(ms.get("annotations") or {})},
                    "spec": {"serviceName": nm, "replicas": replicas,
                             "podManagementPolicy": "Parallel",
                             "selector": {"matchLabels": sl},
                             "template": {"metadata": {"labels": lbl}, "spec": pod_spec}}}

        def headless(nm, lbl, sl, ports):
            return {"apiVersion": "v1", "kind": "Service",
                    "metadata": {"name": nm, "namespace": namespace, "labels": lbl},
                    "spec": {"clusterIP": "None", "publishNotReadyAddresses": True,
                             "selector": sl, "ports": ports}}
        out += [headless(leader, lead_labels, lead_sel,
                         [{"name": "dist", "port": MULTINODE_PORT},
                          {"name": "http", "port": ENGINE_PORT}]),
                headless(worker, wk_labels, wk_sel, [{"name": "health", "port": ENGINE_PORT}]),
                sts(leader, lead_labels, lead_sel, lead_c, 1),
                sts(worker, wk_labels, wk_sel, wk_c, nnodes - 1)]
    out.append({"apiVersion": "v1", "kind": "Service",
                "metadata": {"name": f"{release}-{name}-engine-service", "namespace": namespace,
                             "labels": labels},
                "spec": {"selector": sel, "ports": [{"name": "http", "port": ENGINE_PORT,
                                                     "targetPort": ENGINE_PORT}]}})
    return out


def _api_key_env(v) -> Optional[dict]:
    """servingEngineSpec.vllmApiKey (as the vllm-stack chart takes it): a literal key or
    {secretName, secretKey} -> the VLLM_API_KEY env entry of every engine and the router."""
    if not v:
        return None
    if isinstance(v, str):
        return {"name": "VLLM_API_KEY", "value": v}
    if isinstance(v, dict) and v.get("secretName") and v.get("secretKey"):
        return {"name": "VLLM_API_KEY", "valueFrom": {"secretKeyRef": {
            "name": v["secretName"], "key": v["secretKey"]}}}
    raise ValuesError("servingEngineSpec.vllmApiKey: a string or {secretName, secretKey}")


def render_router(release: str, namespace: str, engine_image: str, engine_tag: str,
                  router: dict, key_env: Optional[dict] = None) -> list[dict]:
    labels = {"app.kubernetes.io/name": LABEL_NAME, "app.kubernetes.io/component": "router",
              "app.kubernetes.io/instance": release}
    sa = f"{release}-router-sa"
    selector = f"app.kubernetes.io/component=serving-engine,app.kubernetes.io/instance={release}"
    args = ["--port", str(ROUTER_PORT), "--k8s-label-selector", selector,
            "--k8s-port", str(ENGINE_PORT), "--routing-logic",
            router.get("routingLogic", "least-outstanding")]
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount",
         "metadata": {"name": sa, "namespace": namespace, "labels": labels}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
         "metadata": {"name": f"{release}-pod-reader", "namespace": namespace, "labels": labels},
         "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list", "watch"]}]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
         "metadata": {"name": f"{release}-router-pod-reader", "namespace": namespace,
                      "labels": labels},
         "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": namespace}],
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role",
                     "name": f"{release}-pod-reader"}},
        {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"name": f"{release}-deployment-router", "namespace": namespace,
                      "labels": labels},
         "spec": {"replicas": int(router.get("replicaCount", 1)),
                  "selector": {"matchLabels": {"app.kubernetes.io/component": "router",
                                               "app.kubernetes.io/instance": release}},
                  "template": {"metadata": {"labels": labels},
                               "spec": {"serviceAccountName": sa, "containers": [{
                                   "name": "router", "image": f"{engine_image}:{engine_tag}",
                                   "command": ["python3", "-m",
                                               "kubernetes_gpu_cluster_amd.router.router"],
                                   "args": args,
                                   **({"env": [key_env]} if key_env else {}),
                                   "ports": [{"name": "http", "containerPort": ROUTER_PORT}],
                                   "resources": {"requests": {"cpu": str(router.get("requestCPU", 1)),
                                                              "memory": str(router.get("requestMemory", "1Gi"))}},
                                   "readinessProbe": {"httpGet": {"path": "/metrics",
                                                                  "port": ROUTER_PORT}},
                               }]}}}},
        {"apiVersion": "v1", "kind": "Service",
         "metadata": {"name": ROUTER_SERVICE, "namespace": namespace, "labels": labels},
         "spec": {"type": router.get("serviceType", "ClusterIP"),
                  "selector": {"app.kubernetes.io/component": "router",
                               "app.kubernetes.io/instance": release},
                  "ports": [{"name": "router-sport", "port": 80, "targetPort": ROUTER_PORT}]}},
    ]


def render(values: dict, release: str = "vllm", namespace: str = "default",
           engine_image: str = DEFAULT_ENGINE_IMAGE, engine_tag: str = DEFAULT_ENGINE_TAG) -> list[dict]:
    if not isinstance(values, dict) or "servingEngineSpec" not in values:
        raise ValuesError("values must contain servingEngineSpec")
    ses = values["servingEngineSpec"] or {}
    specs = ses.get("modelSpec") or []
    if not specs:
        raise ValuesError("servingEngineSpec.modelSpec is empty")
    names = [_dns1123(m.get("name", "")) for m in specs]
    if len(set(names)) != len(names):
        raise ValuesError(f"duplicate modelSpec names {names}")
    rc = ses.get("runtimeClassName", "") or ""
    key_env = _api_key_env(ses.get("vllmApiKey"))
    out = []
    for ms in specs:
        ms = dict(ms)
        if key_env:
            ms["env"] = list(ms.get("env") or []) + [key_env]
        ms.setdefault("runtimeClassName", rc)
        rcn = ms.pop("runtimeClassName")
        out += render_engine(ms, release, namespace, engine_image, engine_tag, rcn)
    if (values.get("routerSpec") or {}).get("enableRouter", True):
        out += render_router(release, namespace, engine_image, engine_tag,
                             values.get("routerSpec") or {}, key_env)
    return out


class _NoAliasDumper(yaml.SafeDumper):
    def ignore_aliases(self, data):  # kubectl-friendly: no &anchors / *aliases
        return True


def to_yaml(objs: list[dict]) -> str:
    return yaml.dump_all(objs, Dumper=_NoAliasDumper, sort_keys=False)


def main(argv=None):
    ap = argparse.ArgumentParser(description="render values-*.yaml to Kubernetes manifests")
    ap.add_argument("-f", "--values", required=True)
    ap.add_argument("--release", default="vllm")
    ap.add_argument("--namespace", default="default")
    ap.add_argument("--engine-image", default=DEFAULT_ENGINE_IMAGE)
    ap.add_argument("--engine-tag", default=DEFAULT_ENGINE_TAG)
    a = ap.parse_args(argv)
    with open(a.values) as f:
        values = yaml.safe_load(f)
    sys.stdout.write(to_yaml(render(values, a.release, a.namespace, a.engine_image, a.engine_tag)))


if __name__ == "__main__":
    main()
