#!/usr/bin/env bash
# Kubernetes node bootstrap for MI355X GPU nodes (kubeadm + CRI-O).
# CLI-compatible with the reference's k8s_setup.sh (k8s_setup.sh:5-47):
#   sudo bash k8s_setup.sh --yes --role=control_plane
#   sudo bash k8s_setup.sh --yes --role=node --join="$(ssh cp 'kubeadm token create --print-join-command')"
# Differences from the reference: flags are parsed before any
# destructive step; --yes may appear anywhere; both --flag=value and --flag value
# work; --join honours --cri-socket; the apt repo follows --kube-version.
# Extra flags: --control-plane-endpoint=VIP:6443 (HA, multi-cp.md:290),
#   --pod-network-cidr, --cni=calico|none, --untaint, --label-gpu, --skip-reset,
#   --proxy=http://host:port (optional egress proxy for apt/CRI-O), --dry-run,
#   --fix-coredns (run CoreDNS AppArmor-unconfined: the fix that made CoreDNS start
#   on the reference's nodes, old_README.md:780-836).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "$HERE/lib.sh"

ROLE=""
KUBE_VERSION="v1.33.3"
CRI_SOCKET="unix:///var/run/crio/crio.sock"
JOIN_CMD=""
CP_ENDPOINT=""
POD_CIDR="192.168.0.0/16"
CNI="calico"
CALICO_VERSION="v3.28.0"
UNTAINT=0
LABEL_GPU=0
SKIP_RESET=0
FIX_COREDNS=0
PROXY="${PROXY:-}"

usage() { sed -n '2,14p' "$0"; exit "${1:-0}"; }

parse_args() {
  while [[ $# -gt 0 ]]; do
    local arg="$1" val=""
    case "$arg" in
      --*=*) val="${arg#*=}"; arg="${arg%%=*}" ;;
      --yes|-y|--untaint|--label-gpu|--skip-reset|--fix-coredns|--dry-run|-h|--help) ;;
      --*) [[ $# -ge 2 ]] || die "$arg needs a value"; val="$2"; shift ;;
    esac
    case "$arg" in
      --yes|-y) ASSUME_YES=1 ;;
      --role)
        case "${val//-/_}" in
          control_plane|control*|cp|master) ROLE="control_plane" ;;
          node|worker) ROLE="node" ;;
          *) die "unknown role '$val' (control_plane|node)" ;;
        esac ;;
      --kube-version) KUBE_VERSION="$val" ;;
      --cri-socket) CRI_SOCKET="$val" ;;
      --join) JOIN_CMD="$val" ;;
      --control-plane-endpoint) CP_ENDPOINT="$val" ;;
      --pod-network-cidr) POD_CIDR="$val" ;;
      --cni) CNI="$val" ;;
      --untaint) UNTAINT=1 ;;
      --label-gpu) LABEL_GPU=1 ;;
      --skip-reset) SKIP_RESET=1 ;;
      --fix-coredns) FIX_COREDNS=1 ;;
      --proxy) PROXY="$val" ;;
      --dry-run) DRY_RUN=1 ;;
      -h|--help) usage 0 ;;
      *) die "unknown argument $arg" ;;
    esac
    shift
  done
  [[ -n "$ROLE" ]] || die "--role=control_plane|node is required"
  [[ "$ROLE" == "node" && -z "$JOIN_CMD" ]] && die "--role=node needs --join='kubeadm join ...'"
  [[ "$KUBE_VERSION" =~ ^v?[0-9]+\.[0-9]+\.[0-9]+$ ]] || die "bad --kube-version $KUBE_VERSION"
  return 0
}

stop_disable_service() {
  local s="$1"
  if have_cmd systemctl && systemctl list-unit-files 2>/dev/null | grep -q "^$s"; then
    run systemctl stop "$s" || true
    run systemctl disable "$s" || true
  fi
}

free_port_6443() {
  local pids=""
  if have_cmd ss; then
    pids=$(ss -ltnp 2>/dev/null | awk '/:6443 /{print $NF}' | grep -o 'pid=[0-9]*' | cut -d= -f2 | sort -u || true)
  fi
  for p in $pids; do
    run kill -TERM "$p" || true
  done
  [[ -n "$pids" ]] && sleep 1
  for p in $pids; do
    kill -0 "$p" 2>/dev/null && run kill -KILL "$p" || true
  done
  return 0
}

reset_node() {
  log "resetting previous Kubernetes state"
  stop_disable_service kubelet
  if have_cmd kubeadm; then run kubeadm reset -f --cri-socket "$CRI_SOCKET" || true; fi
  free_port_6443
  local paths=(/etc/kubernetes /var/lib/kubelet /var/lib/etcd)
  if confirm "remove ${paths[*]} ?"; then
    for p in "${paths[@]}"; do run rm -rf --one-file-system "${ROOT}$p"; done
  fi
}

disable_swap() {
  log "disabling swap"
  run swapoff -a || true
  local fstab="${ROOT}/etc/fstab"
  if [[ -f "$fstab" ]] && grep -qE '^[^#].*\sswap\s' "$fstab"; then
    backup /etc/fstab
    awk '{ if ($0 !~ /^#/ && $3 == "swap") print "#" $0; else print $0 }' "$fstab" > "$fstab.new"
    mv "$fstab.new" "$fstab"
  fi
  if have_cmd systemctl; then
    for u in $(systemctl list-units --type=swap --no-legend 2>/dev/null | awk '{print $1}'); do
      run systemctl mask "$u" || true
    done
  fi
}

setup_netfilters() {
  log "kernel modules and sysctls"
  write_file /etc/modules-load.d/k8s.conf $'overlay\nbr_netfilter\n'
  run modprobe overlay || true
  run modprobe br_netfilter || true
  write_file /etc/sysctl.d/99-kubernetes-cri.conf \
$'net.bridge.bridge-nf-call-iptables  = 1\nnet.bridge.bridge-nf-call-ip6tables = 1\nnet.ipv4.ip_forward                 = 1\n'
  run sysctl --system >/dev/null || true
}

install_k8s_apt() {
  local minor; minor=$(kube_minor "$KUBE_VERSION")
  log "installing kubelet/kubeadm/kubectl from pkgs.k8s.io $minor"
  # apt reads an ASCII-armoured key directly when the file ends in .asc, so the key is
  # stored exactly where signed-by points (no gpg --dearmor step to get out of sync)
  local keyring=/etc/apt/keyrings/kubernetes-apt-keyring.asc
  write_file /etc/apt/sources.list.d/kubernetes.list \
    "deb [signed-by=${keyring}] https://pkgs.k8s.io/core:/stable:/${minor}/deb/ /
"
  mkdir -p "${ROOT}/etc/apt/keyrings"
  run curl -fsSL ${PROXY:+--proxy "$PROXY"} "https://pkgs.k8s.io/core:/stable:/${minor}/deb/Release.key" \
    -o "${ROOT}${keyring}" \
    || die "could not fetch the Kubernetes apt key from pkgs.k8s.io (network / --proxy?)"
  run apt-get update -y || die "apt-get update failed (the pkgs.k8s.io repository is unusable)"
  run apt-get install -y kubelet kubeadm kubectl || die "installing kubeadm failed"
  run apt-mark hold kubelet kubeadm kubectl || true
  run systemctl enable --now kubelet || true
}

setup_crio_proxy() {
  [[ -z "$PROXY" ]] && return 0
  write_file /etc/systemd/system/crio.service.d/proxy.conf "[Service]
Environment=\"HTTP_PROXY=$PROXY\" \"HTTPS_PROXY=$PROXY\"
Environment=\"NO_PROXY=localhost,127.0.0.1,::1,.svc,.cluster.local,10.96.0.0/12,10.244.0.0/16,$POD_CIDR\"
"
  run systemctl daemon-reload || true
  run systemctl restart crio || true
}

post_init_kubeconfig() {
  local user="${SUDO_USER:-root}" home
  home=$(getent passwd "$user" 2>/dev/null | cut -d: -f6 || true)
  home=${home:-/root}
  mkdir -p "${ROOT}${home}/.kube"
  if [[ -f "${ROOT}/etc/kubernetes/admin.conf" ]]; then
    cp "${ROOT}/etc/kubernetes/admin.conf" "${ROOT}${home}/.kube/config"
    run chown "$user" "${ROOT}${home}/.kube/config" || true
  fi
}

init_control_plane() {
  local ts logf; ts=$(date +%Y%m%d-%H%M%S); logf="${ROOT}/var/log/kubeadm-init-$ts.log"
  mkdir -p "$(dirname "$logf")"
  local args=(init --cri-socket "$CRI_SOCKET" --kubernetes-version "$KUBE_VERSION"
              --pod-network-cidr "$POD_CIDR")
  [[ -n "$CP_ENDPOINT" ]] && args+=(--control-plane-endpoint "$CP_ENDPOINT" --upload-certs)
  log "kubeadm ${args[*]}"
  if [[ "$DRY_RUN" == "1" ]]; then
    run kubeadm "${args[@]}"       # and keep going: the dry run prints the post-init calls too
  else
    kubeadm "${args[@]}" 2>&1 | tee "$logf"
    grep -qE 'kubeadm join .* --token' "$logf" || die "kubeadm init did not print a join command (see $logf)"
    post_init_kubeconfig
  fi
  local kc=(kubectl --kubeconfig "${ROOT}/etc/kubernetes/admin.conf")
  if [[ "$CNI" == "calico" ]]; then
    run "${kc[@]}" apply -f "https://raw.githubusercontent.com/projectcalico/calico/${CALICO_VERSION}/manifests/calico.yaml" \
      || warn "calico apply failed"
  fi
  if [[ "$UNTAINT" == "1" ]]; then
    run "${kc[@]}" taint nodes --all node-role.kubernetes.io/control-plane- || true
  fi
  if [[ "$LABEL_GPU" == "1" ]]; then
    run "${kc[@]}" label node "$(hostname)" gpu=true --overwrite || true
  fi
  if [[ "$FIX_COREDNS" == "1" ]]; then
    # AppArmor-confined CoreDNS crash-looped on the reference's hosts; the pod-level
    # appArmorProfile field (k8s >= 1.30) replaces the deprecated annotation
    run "${kc[@]}" -n kube-system patch deployment coredns --type=strategic -p \
      '{"spec":{"template":{"spec":{"securityContext":{"appArmorProfile":{"type":"Unconfined"}}}}}}' \
      || warn "coredns patch failed"
    run "${kc[@]}" -n kube-system rollout restart deployment coredns || true
  fi
}

join_node() {
  local cmd="$JOIN_CMD"
  [[ "$cmd" == *"--cri-socket"* ]] || cmd="$cmd --cri-socket $CRI_SOCKET"
  log "joining: $cmd"
  # shellcheck disable=SC2086
  run bash -c "$cmd"
}

main() {
  parse_args "$@"
  require_root
  log "role=$ROLE kube=$KUBE_VERSION cri=$CRI_SOCKET"
  [[ "$SKIP_RESET" == "1" ]] || reset_node
  disable_swap
  setup_netfilters
  install_k8s_apt
  setup_crio_proxy
  if [[ "$ROLE" == "control_plane" ]]; then init_control_plane; else join_node; fi
  log "done"
}

[[ "${BASH_SOURCE[0]}" == "$0" ]] && main "$@"
