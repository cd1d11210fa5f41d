#!/usr/bin/env bash
# MI355X GPU enablement for a CRI-O node (replaces the reference's NVIDIA
# gpu-crio-setup.sh:138-154).  One injection mechanism, no runtime conflicts:
#   1. conmon + crun present (crun >= 1.21, the version the reference needed)
#   2. amd node tools installed: amd-container-runtime (OCI shim), amd-container-hook,
#      amd-ctk, amdgpu-topo, libamdgpu_topo.so (built by native/build.sh)
#   3. CRI-O runtime handler "amd" -> amd-container-runtime (amd-ctk runtime configure);
#      crun stays the default runtime (the working end state of old_README.md:1335-1361)
#   4. CDI spec /etc/cdi/amd.yaml (amd-ctk cdi generate) for CDI-aware clients
#   5. optional prestart hook (--with-hook) + hooks_dir drop-in
#   6. udev rule: /dev/kfd and /dev/dri/renderD* group render, mode 0660
#   7. RuntimeClasses crun + amd and the amd.com/gpu device-plugin DaemonSet (kubectl)
#   8. verify: GPU table, runtime config
#   sudo bash gpu-crio-setup.sh [--set-default] [--with-hook] [--skip-apt] [--no-kubectl]
set -uo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
source "$HERE/lib.sh"

SET_DEFAULT=0
WITH_HOOK=0
SKIP_APT=${SKIP_APT:-0}
NO_KUBECTL=0
PREFIX=/usr/local
BIN_SRC="${BIN_SRC:-$REPO/build/native}"

for a in "$@"; do
  case "$a" in
    --set-default) SET_DEFAULT=1 ;;
    --with-hook) WITH_HOOK=1 ;;
    --skip-apt) SKIP_APT=1 ;;
    --no-kubectl) NO_KUBECTL=1 ;;
    --dry-run) DRY_RUN=1 ;;
    --yes|-y) ASSUME_YES=1 ;;
    *) die "unknown argument $a" ;;
  esac
done

apt_install() {
  [[ "$SKIP_APT" == "1" ]] && { warn "SKIP_APT=1: not installing $*"; return 1; }
  local i
  for i in 1 2 3; do
    run apt-get -o Acquire::Retries=3 update -y && break
    warn "apt-get update attempt $i failed"; sleep 2
  done
  run apt-get install -y "$@"
}

install_runtime_deps() {
  have_cmd conmon || apt_install conmon || warn "conmon missing"
  if ! have_cmd crun; then
    apt_install crun || warn "crun missing: build crun >= 1.21 from source"
  fi
}

install_node_tools() {
  if [[ ! -x "$BIN_SRC/amd-ctk" ]]; then
    log "building native node tools"
    run bash "$REPO/native/build.sh" || die "native build failed"
  fi
  mkdir -p "${ROOT}$PREFIX/bin" "${ROOT}$PREFIX/lib"
  for b in amd-container-runtime amd-container-hook amd-ctk amdgpu-topo; do
    run install -m 0755 "$BIN_SRC/$b" "${ROOT}$PREFIX/bin/$b"
  done
  run install -m 0644 "$BIN_SRC/libamdgpu_topo.so" "${ROOT}$PREFIX/lib/libamdgpu_topo.so"
}

CTK() { run "$BIN_SRC/amd-ctk" "$@"; }

configure_crio() {
  local args=(runtime configure --runtime=crio --config="${ROOT}/etc/crio/crio.conf.d/99-amd.conf"
              --runtime-path="$PREFIX/bin/amd-container-runtime")
  [[ "$SET_DEFAULT" == "1" ]] && args+=(--set-as-default)
  CTK "${args[@]}"
  write_file /etc/crio/crio.conf.d/98-crun-default.conf '[crio.runtime]
default_runtime = "crun"

[crio.runtime.runtimes.crun]
runtime_path = "/usr/bin/crun"
runtime_type = "oci"
runtime_root = "/run/crun"
'
  [[ "$SET_DEFAULT" == "1" ]] && rm -f "${ROOT}/etc/crio/crio.conf.d/98-crun-default.conf"
  CTK cdi generate --root="${ROOT:-/}" --output="${ROOT}/etc/cdi/amd.yaml"
  if [[ "$WITH_HOOK" == "1" ]]; then
    CTK hook install --hooks-dir="${ROOT}/usr/share/containers/oci/hooks.d" \
        --hook-path="$PREFIX/bin/amd-container-hook"
    CTK crio hooks-dir --config="${ROOT}/etc/crio/crio.conf.d/99-amd-hooks.conf"
  fi
}

udev_rules() {
  write_file /etc/udev/rules.d/70-amdgpu-kfd.rules 'KERNEL=="kfd", GROUP="render", MODE="0660"
SUBSYSTEM=="drm", KERNEL=="renderD*", GROUP="render", MODE="0660"
'
  run udevadm control --reload-rules || true
  run udevadm trigger || true
}

restart_crio() {
  run systemctl restart crio || warn "crio restart failed"
  run systemctl restart kubelet || true
}

apply_cluster_objects() {
  [[ "$NO_KUBECTL" == "1" ]] && return 0
  have_cmd kubectl || { warn "kubectl not found: apply deploy/manifests/*.yaml manually"; return 0; }
  run kubectl apply -f "$REPO/deploy/manifests/runtimeclasses.yaml" || warn "RuntimeClasses"
  run kubectl apply -f "$REPO/deploy/manifests/amd-gpu-device-plugin.yaml" || warn "device plugin"
}

verify() {
  log "GPUs:"
  run "$BIN_SRC/amdgpu-topo" --root "${ROOT:-/}" --table || true
  have_cmd crun && run crun --version | head -n1 || true
  have_cmd crio && run crio --version | head -n1 || true
  ls -1 "${ROOT}/etc/crio/crio.conf.d/" 2>/dev/null || true
  head -n 12 "${ROOT}/etc/cdi/amd.yaml" 2>/dev/null || true
}

main() {
  require_root
  install_runtime_deps
  install_node_tools
  configure_crio
  udev_rules
  restart_crio
  apply_cluster_objects
  verify
  log "MI355X GPU enablement complete"
}

[[ "${BASH_SOURCE[0]}" == "$0" ]] && main
