#!/usr/bin/env bash
# One-command bring-up of a single MI355X node that serves (north star: "a single
# 8xMI355X node comes up and serves with one command").  Chains the steps of the
# reference workflow (README.md:45-110, old_README.md:1077-1176) in order and checks
# each one before moving on:
#
#   1. CRI-O + crictl                       crio_setup.sh
#   2. kubeadm control plane, untainted,    k8s_setup.sh --role=control_plane --untaint --label-gpu
#      Calico, node labelled gpu=true
#   3. native node tools                    native/build.sh (OCI shim, hook, amd-ctk, amdgpu-topo)
#   4. GPU enablement                       gpu-crio-setup.sh (runtime handler, CDI, device plugin)
#   4b. engine image in CRI-O's store       --image-tar: podman load; otherwise podman / buildah
#                                           build of deploy/docker/Dockerfile when missing;
#                                           always `crictl inspecti` before anything is applied
#   5. wait until the node advertises amd.com/gpu
#   6. values -> manifests | kubectl apply  python -m kubernetes_gpu_cluster_amd.k8s.render
#   7. wait for the engine Deployments and the vllm-router-service endpoints
#   8. smoke: port-forward svc/vllm-router-service and GET /v1/models (+ one completion)
#
#   sudo bash deploy/scripts/bringup.sh --single-node \
#        [--values=deploy/values/values-llama3-8b-tp1.yaml] [--proxy=URL] [--kube-version=v1.33.3]
#        [--image-tar=kgc-engine.tar | --no-build] [--image=kgc/engine:TAG] [--port=30080]
#        [--timeout=1800] [--skip-node-setup] [--dry-run]
#
# --dry-run prints the full ordered call log (the sub-scripts run in their own dry-run
# mode) without changing the machine.  --skip-node-setup starts at step 5 on a node that
# is already bootstrapped.  Exits non-zero at the first step that fails.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
source "$HERE/lib.sh"

VALUES="$REPO/deploy/values/values-llama3-8b-tp1.yaml"
PROXY="${PROXY:-}"
KUBE_VERSION=""
IMAGE_TAR=""
IMAGE="${IMAGE:-}"
BUILD=1
PORT=30080
TIMEOUT=1800
SKIP_NODE=0
PYTHON="${PYTHON:-python3}"

while [[ $# -gt 0 ]]; do
  arg="$1"; val=""
  case "$arg" in
    --*=*) val="${arg#*=}"; arg="${arg%%=*}" ;;
    --values|--proxy|--kube-version|--image-tar|--image|--port|--timeout)
      [[ $# -ge 2 ]] || die "$arg needs a value"; val="$2"; shift ;;
  esac
  case "$arg" in
    --single-node) ;;                       # the only topology this script brings up
    --values) VALUES="$val" ;;
    --proxy) PROXY="$val" ;;
    --kube-version) KUBE_VERSION="$val" ;;
    --image-tar) IMAGE_TAR="$val" ;;
    --image) IMAGE="$val" ;;
    --no-build) BUILD=0 ;;
    --port) PORT="$val" ;;
    --timeout) TIMEOUT="$val" ;;
    --skip-node-setup) SKIP_NODE=1 ;;
    --dry-run) DRY_RUN=1 ;;
    --yes|-y) ASSUME_YES=1 ;;
    -h|--help) sed -n 2,29p "$0"; exit 0 ;;
    *) die "unknown argument $1" ;;
  esac
  shift
done
[[ -f "$VALUES" ]] || die "values file not found: $VALUES"
if [[ -z "$IMAGE" ]]; then             # the renderer's default engine image
  IMAGE=$(cd "$REPO" && "$PYTHON" -c 'from kubernetes_gpu_cluster_amd.k8s.render import \
DEFAULT_ENGINE_IMAGE as i, DEFAULT_ENGINE_TAG as t; print(f"{i}:{t}")') \
    || die "cannot read the default engine image from the renderer"
fi
[[ "$IMAGE" == *:* ]] || die "--image must be REPOSITORY:TAG (got $IMAGE)"
export DRY_RUN ASSUME_YES ROOT

sub_flags=()
[[ "$DRY_RUN" == "1" ]] && sub_flags+=(--dry-run)
step() { log "==== step $1: $2"; }

node_setup() {
  step 1 "CRI-O"
  bash "$HERE/crio_setup.sh" ${PROXY:+--proxy="$PROXY"} "${sub_flags[@]}"
  step 2 "Kubernetes control plane (single node)"
  bash "$HERE/k8s_setup.sh" --yes --role=control_plane --untaint --label-gpu \
    ${PROXY:+--proxy="$PROXY"} ${KUBE_VERSION:+--kube-version="$KUBE_VERSION"} "${sub_flags[@]}"
  step 3 "native node tools"
  run bash "$REPO/native/build.sh"
  step 4 "GPU enablement"
  bash "$HERE/gpu-crio-setup.sh" --yes "${sub_flags[@]}"
}

image_present() { crictl inspecti "$IMAGE" >/dev/null 2>&1; }

# The engine Deployments reference $IMAGE with imagePullPolicy IfNotPresent: an offline
# node that lacks it would sit in ImagePullBackOff until step 7 times out.  Put it into
# CRI-O's store here (podman / buildah as root share containers/storage with CRI-O) and
# refuse to apply manifests for an image the node does not have.
ensure_image() {
  step 4b "engine image $IMAGE"
  if [[ -n "$IMAGE_TAR" ]]; then          # offline node: side-load the saved image
    [[ "$DRY_RUN" == "1" || -f "$IMAGE_TAR" ]] || die "--image-tar $IMAGE_TAR not found"
    run podman load -i "$IMAGE_TAR" || die "loading $IMAGE_TAR into CRI-O's store failed"
  elif [[ "$DRY_RUN" == "1" ]] || ! image_present; then
    if [[ "$BUILD" != "1" ]]; then
      [[ "$DRY_RUN" == "1" ]] || die "engine image $IMAGE is not on this node and --no-build was given"
    elif [[ "$DRY_RUN" == "1" ]] || have_cmd podman; then
      run podman build -f "$REPO/deploy/docker/Dockerfile" -t "$IMAGE" "$REPO" \
        || die "podman build of $IMAGE failed"
    elif have_cmd buildah; then
      run buildah bud -f "$REPO/deploy/docker/Dockerfile" -t "$IMAGE" "$REPO" \
        || die "buildah build of $IMAGE failed"
    else
      die "engine image $IMAGE is not in CRI-O's store and neither podman nor buildah is" \
          "installed: build deploy/docker/Dockerfile elsewhere and pass --image-tar"
    fi
  fi
  if [[ "$DRY_RUN" == "1" ]]; then
    printf "DRY: crictl inspecti %s\n" "$IMAGE"
  else
    image_present || die "engine image $IMAGE is still not in CRI-O's store (crictl inspecti);" \
                         "not applying manifests that would sit in ImagePullBackOff"
    log "engine image $IMAGE is on the node"
  fi
}

# wait_for DESC CMD...: retry CMD every 5 s until it succeeds or TIMEOUT elapses
wait_for() {
  local desc="$1"; shift
  if [[ "$DRY_RUN" == "1" ]]; then printf "DRY: wait for %s: %s\n" "$desc" "$*"; return 0; fi
  local t0=$SECONDS
  until "$@"; do
    (( SECONDS - t0 >= TIMEOUT )) && die "timed out after ${TIMEOUT}s waiting for $desc"
    sleep "${WAIT_INTERVAL:-5}"
  done
  log "$desc: ready after $((SECONDS - t0))s"
}

gpus_advertised() {
  local n
  n=$(kubectl get nodes -o 'jsonpath={.items[*].status.allocatable.amd\.com/gpu}' 2>/dev/null \
      | tr ' ' '\n' | awk '{s += $1} END {print s + 0}')
  [[ "${n:-0}" -gt 0 ]]
}

engines_ready() {
  kubectl rollout status deployment -l app.kubernetes.io/component=serving-engine \
    --timeout=10s >/dev/null 2>&1
}

router_endpoints() {
  local ips
  ips=$(kubectl get endpoints vllm-router-service -o 'jsonpath={.subsets[*].addresses[*].ip}' \
        2>/dev/null || true)
  [[ -n "$ips" ]]
}

models_ok() { curl -sf --max-time 5 "http://127.0.0.1:$PORT/v1/models" -o "$MODELS_OUT"; }

deploy_and_smoke() {
  step 5 "node advertises amd.com/gpu"
  wait_for "amd.com/gpu on the node" gpus_advertised
  step 6 "render $(basename "$VALUES") and apply"
  if [[ "$DRY_RUN" == "1" ]]; then
    (cd "$REPO" && "$PYTHON" -m kubernetes_gpu_cluster_amd.k8s.render -f "$VALUES" \
      --engine-image "${IMAGE%:*}" --engine-tag "${IMAGE##*:}" >/dev/null)
    printf "DRY: %s -m kubernetes_gpu_cluster_amd.k8s.render -f %s --engine-image %s --engine-tag %s | kubectl apply -f -\n" \
      "$PYTHON" "$VALUES" "${IMAGE%:*}" "${IMAGE##*:}"
  else
    (cd "$REPO" && "$PYTHON" -m kubernetes_gpu_cluster_amd.k8s.render -f "$VALUES" \
      --engine-image "${IMAGE%:*}" --engine-tag "${IMAGE##*:}") \
      | kubectl apply -f - || die "kubectl apply failed"
  fi
  step 7 "engine pods and router service"
  wait_for "serving-engine Deployments" engines_ready
  wait_for "vllm-router-service endpoints" router_endpoints
  step 8 "smoke through svc/vllm-router-service"
  if [[ "$DRY_RUN" == "1" ]]; then
    printf "DRY: kubectl port-forward svc/vllm-router-service %s:80\n" "$PORT"
    printf "DRY: curl -sf http://127.0.0.1:%s/v1/models\n" "$PORT"
    return 0
  fi
  MODELS_OUT=$(mktemp)
  kubectl port-forward svc/vllm-router-service "$PORT:80" >/dev/null 2>&1 &
  PF_PID=$!
  trap 'kill "$PF_PID" 2>/dev/null || true; rm -f "$MODELS_OUT"' EXIT
  wait_for "GET /v1/models through the router" models_ok
  local model
  model=$("$PYTHON" -c 'import json,sys; print(json.load(open(sys.argv[1]))["data"][0]["id"])' \
          "$MODELS_OUT") || die "/v1/models returned no model"
  log "serving model: $model"
  curl -sf --max-time 120 "http://127.0.0.1:$PORT/v1/completions" \
    -H 'content-type: application/json' \
    -d "{\"model\": \"$model\", \"prompt\": \"Hello\", \"max_tokens\": 8}" >/dev/null \
    || die "completion through the router failed"
  log "node is serving: http://127.0.0.1:$PORT/v1 (kubectl port-forward svc/vllm-router-service $PORT:80)"
}

require_root
[[ "$SKIP_NODE" == "1" ]] || node_setup
ensure_image
# kubectl as root on the control plane (k8s_setup copies admin.conf to $SUDO_USER's home)
if [[ -z "${KUBECONFIG:-}" && -f "${ROOT}/etc/kubernetes/admin.conf" ]]; then
  export KUBECONFIG="${ROOT}/etc/kubernetes/admin.conf"
fi
deploy_and_smoke
log "bring-up complete"
