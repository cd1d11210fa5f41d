#!/usr/bin/env bash
# MI355X GPU enablement for a CRI-O node (replaces the reference's NVIDIA
# gpu-crio-setup.sh:138-154).  One injection mechanism, no runtime conflicts:
#   1. conmon + crun >= 1.21 (the version the reference needed): the newest crun found
#      (/usr/local first, then PATH), else apt, else a source build of crun 1.21;
#      the detected path goes into the crun runtime handler and the shim's environment
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

CRUN_MIN=1.21               # older distro crun broke pods ("unknown version specified",
CRUN_PATH=""                # reference old_README.md:774,1186-1199; gpu-crio-setup.sh:43-56)

# version_ge A B: A >= B in version order
version_ge() { [[ "$(printf '%s\n%s\n' "$2" "$1" | sort -V | head -n1)" == "$2" ]]; }

crun_version() {    # "crun version 1.21" -> 1.21 (empty when crun is missing / unparsable)
  local c="${1:-crun}"
  "$c" --version 2>/dev/null | awk 'NR==1 && $2=="version" {print $3}'
}

find_crun() {       # newest usable crun: the source build in /usr/local wins over the distro's
  local c
  for c in /usr/local/bin/crun "$(command -v crun 2>/dev/null)"; do
    [[ -n "$c" && -x "$c" ]] || continue
    local v; v=$(crun_version "$c")
    if [[ -n "$v" ]] && version_ge "$v" "$CRUN_MIN"; then CRUN_PATH="$c"; return 0; fi
  done
  return 1
}

build_crun() {      # source build of crun $CRUN_MIN into /usr/local (cwd untouched)
  local src="${CRUN_SRC_DIR:-/usr/local/src/crun-$CRUN_MIN}"
  log "building crun $CRUN_MIN from source in $src"
  apt_install git make gcc automake autoconf libtool pkg-config libsystemd-dev libcap-dev \
    libseccomp-dev libyajl-dev go-md2man python3 || warn "crun build deps not installed"
  run rm -rf "$src"
  run git clone --depth 1 --branch "$CRUN_MIN" https://github.com/containers/crun.git "$src" \
    || return 1
  run bash -c "cd '$src' && ./autogen.sh && ./configure --prefix=/usr/local && make -j\$(nproc) && make install"
}

install_runtime_deps() {
  have_cmd conmon || apt_install conmon || warn "conmon missing"
  find_crun && { log "crun $(crun_version "$CRUN_PATH") at $CRUN_PATH"; return 0; }
  apt_install crun || true
  find_crun && { log "crun $(crun_version "$CRUN_PATH") at $CRUN_PATH"; return 0; }
  build_crun || warn "crun $CRUN_MIN source build failed"
  if ! find_crun; then
    CRUN_PATH=$(command -v crun 2>/dev/null || echo /usr/local/bin/crun)
    warn "no crun >= $CRUN_MIN found; configuring $CRUN_PATH anyway"
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
  # the shim execs this crun (not whatever crun is first in CRI-O's PATH)
  write_file /etc/default/amd-container-runtime "AMD_CONTAINER_RUNTIME_LOWLEVEL=$CRUN_PATH
"
  [[ "$SET_DEFAULT" == "1" ]] && args+=(--set-as-default)
  CTK "${args[@]}"
  write_file /etc/crio/crio.conf.d/98-crun-default.conf '[crio.runtime]
default_runtime = "crun"

[crio.runtime.runtimes.crun]
runtime_path = "'"$CRUN_PATH"'"
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
