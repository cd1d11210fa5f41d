#!/usr/bin/env bash
# HA control-plane front end for a multi-control-plane cluster: a keepalived-managed
# virtual IP plus an haproxy TCP load balancer over the kube-apiservers.  This is the
# scripted form of the reference's manual multi-cp.md procedure (multi-cp.md:36-188;
# VRRP check every 3 s, fall 10 / rise 2; haproxy /healthz checks over TLS).
#
#   sudo bash ha_setup.sh --vip=10.0.0.100 --interface=eth0 --state=MASTER \
#        --peer=cp1=10.0.0.11 --peer=cp2=10.0.0.12 --peer=cp3=10.0.0.13
#   # then on the first control plane:
#   sudo bash k8s_setup.sh --yes --role=control_plane --control-plane-endpoint=10.0.0.100:8443
#
# Flags (both --flag=value and --flag value):
#   --vip=IP             virtual IP (required)
#   --interface=IF       NIC that carries the VIP (required)
#   --state=MASTER|BACKUP  initial VRRP role (default BACKUP); priority 101 / 100
#   --priority=N         override the VRRP priority
#   --router-id=N        VRRP virtual_router_id, same on all LB hosts (default 51)
#   --auth-pass=S        VRRP password, same on all LB hosts (default: derived from --vip)
#   --lb-port=P          port haproxy listens on = the endpoint port (default 8443)
#   --apiserver-port=P   kube-apiserver port on every control plane (default 6443)
#   --peer=NAME=ADDR     one per control-plane node (repeatable, required)
#   --mode=systemd|static-pods  run keepalived/haproxy as host services (default) or as
#                        kubelet static pods written to /etc/kubernetes/manifests
#   --skip-install       do not apt-get install keepalived/haproxy
#   --yes, --dry-run
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "$HERE/lib.sh"

VIP="" IFACE="" STATE="BACKUP" PRIORITY="" ROUTER_ID=51 AUTH_PASS="" LB_PORT=8443
API_PORT=6443 MODE="systemd" SKIP_INSTALL=0
PEERS=()

usage() { sed -n '2,28p' "$0"; exit "${1:-0}"; }

parse_args() {
  while [[ $# -gt 0 ]]; do
    local arg="$1" val=""
    case "$arg" in
      --*=*) val="${arg#*=}"; arg="${arg%%=*}" ;;
      --yes|-y|--skip-install|--dry-run|-h|--help) ;;
      --*) [[ $# -ge 2 ]] || die "$arg needs a value"; val="$2"; shift ;;
    esac
    case "$arg" in
      --vip) VIP="$val" ;;
      --interface) IFACE="$val" ;;
      --state) STATE="${val^^}" ;;
      --priority) PRIORITY="$val" ;;
      --router-id) ROUTER_ID="$val" ;;
      --auth-pass) AUTH_PASS="$val" ;;
      --lb-port) LB_PORT="$val" ;;
      --apiserver-port) API_PORT="$val" ;;
      --peer) PEERS+=("$val") ;;
      --mode) MODE="$val" ;;
      --skip-install) SKIP_INSTALL=1 ;;
      --yes|-y) ASSUME_YES=1 ;;
      --dry-run) DRY_RUN=1 ;;
      -h|--help) usage 0 ;;
      *) die "unknown argument $arg" ;;
    esac
    shift
  done
  [[ "$VIP" =~ ^[0-9]+\.[0-9]+\.[0-9]+\.[0-9]+$ ]] || die "--vip=IPv4 is required"
  [[ -n "$IFACE" ]] || die "--interface is required"
  [[ "$STATE" == MASTER || "$STATE" == BACKUP ]] || die "--state must be MASTER or BACKUP"
  [[ ${#PEERS[@]} -ge 1 ]] || die "at least one --peer=NAME=ADDR is required"
  local p
  for p in "${PEERS[@]}"; do
    [[ "$p" =~ ^[A-Za-z0-9._-]+=[A-Za-z0-9.:-]+$ ]] || die "bad --peer '$p' (NAME=ADDR)"
  done
  [[ "$MODE" == systemd || "$MODE" == static-pods ]] || die "--mode systemd|static-pods"
  [[ "$LB_PORT" =~ ^[0-9]+$ && "$API_PORT" =~ ^[0-9]+$ ]] || die "ports must be numeric"
  # the LB usually runs on the control planes themselves: it cannot share their port
  [[ "$LB_PORT" != "$API_PORT" ]] || die "--lb-port must differ from --apiserver-port"
  if [[ -z "$PRIORITY" ]]; then
    if [[ "$STATE" == MASTER ]]; then PRIORITY=101; else PRIORITY=100; fi
  fi
  if [[ -z "$AUTH_PASS" ]]; then
    # VRRP PASS auth is at most 8 characters; derive a stable one from the VIP
    AUTH_PASS=$(printf "%s" "$VIP" | cksum | cut -c1-8)
  fi
  return 0
}

keepalived_conf() {
  cat <<EOF
# keepalived VRRP for the Kubernetes API VIP $VIP (written by ha_setup.sh)
global_defs {
    router_id kgc_apiserver_lb
    enable_script_security
    script_user root
}

vrrp_script apiserver_alive {
    script "/etc/keepalived/check_apiserver.sh"
    interval 3
    timeout 2
    weight -2
    fall 10
    rise 2
}

vrrp_instance kube_api {
    state $STATE
    interface $IFACE
    virtual_router_id $ROUTER_ID
    priority $PRIORITY
    advert_int 1
    authentication {
        auth_type PASS
        auth_pass $AUTH_PASS
    }
    virtual_ipaddress {
        $VIP
    }
    track_script {
        apiserver_alive
    }
}
EOF
}

check_script() {
  cat <<EOF
#!/bin/sh
# Healthy when the load balancer answers locally and, on the VIP holder, through the VIP.
fail() { echo "check_apiserver: \$*" >&2; exit 1; }
curl -sfk --max-time 2 -o /dev/null "https://127.0.0.1:$LB_PORT/healthz" \\
  || fail "no /healthz via 127.0.0.1:$LB_PORT"
if ip -o addr show 2>/dev/null | grep -qw "$VIP"; then
  curl -sfk --max-time 2 -o /dev/null "https://$VIP:$LB_PORT/healthz" \\
    || fail "no /healthz via VIP $VIP:$LB_PORT"
fi
exit 0
EOF
}

haproxy_cfg() {
  local p name addr
  cat <<EOF
# haproxy: TCP pass-through to the kube-apiservers (written by ha_setup.sh)
global
    log stdout format raw local0
    maxconn 4096

defaults
    log global
    mode tcp
    option tcplog
    option dontlognull
    retries 1
    timeout connect 5s
    timeout client 35s
    timeout server 35s
    timeout check 10s

frontend kube_apiserver
    bind *:$LB_PORT
    default_backend kube_apiservers

backend kube_apiservers
    balance roundrobin
    option httpchk
    http-check connect ssl
    http-check send meth GET uri /healthz
    http-check expect status 200
    default-server inter 3s fall 3 rise 2
EOF
  for p in "${PEERS[@]}"; do
    name="${p%%=*}"; addr="${p#*=}"
    printf "    server %s %s:%s check verify none\n" "$name" "$addr" "$API_PORT"
  done
}

static_pod() {  # name image host_conf container_conf -> kubelet static pod manifest
  local name="$1" image="$2" host_conf="$3" ctr_conf="$4"
  cat <<EOF
apiVersion: v1
kind: Pod
metadata:
  name: $name
  namespace: kube-system
spec:
  hostNetwork: true
  priorityClassName: system-node-critical
  containers:
  - name: $name
    image: $image
    securityContext:
      capabilities:
        add: ["NET_ADMIN", "NET_BROADCAST", "NET_RAW"]
    volumeMounts:
    - {name: conf, mountPath: $ctr_conf, readOnly: true}
  volumes:
  - name: conf
    hostPath: {path: $host_conf, type: File}
EOF
}

main() {
  parse_args "$@"
  require_root
  log "HA front end: VIP $VIP on $IFACE ($STATE, priority $PRIORITY), haproxy :$LB_PORT -> ${#PEERS[@]} apiservers :$API_PORT"
  if [[ "$MODE" == systemd && "$SKIP_INSTALL" == 0 && "${SKIP_APT:-0}" != 1 ]]; then
    run apt-get install -y keepalived haproxy
  fi
  backup /etc/keepalived/keepalived.conf
  backup /etc/haproxy/haproxy.cfg
  write_file /etc/keepalived/keepalived.conf "$(keepalived_conf)"$'\n'
  write_file /etc/keepalived/check_apiserver.sh "$(check_script)"$'\n'
  chmod 0755 "${ROOT}/etc/keepalived/check_apiserver.sh"
  write_file /etc/haproxy/haproxy.cfg "$(haproxy_cfg)"$'\n'
  if [[ "$MODE" == static-pods ]]; then
    write_file /etc/kubernetes/manifests/keepalived.yaml \
      "$(static_pod keepalived osixia/keepalived:2.0.20 /etc/keepalived/keepalived.conf \
         /usr/local/etc/keepalived/keepalived.conf)"$'\n'
    write_file /etc/kubernetes/manifests/haproxy.yaml \
      "$(static_pod haproxy haproxy:2.8 /etc/haproxy/haproxy.cfg \
         /usr/local/etc/haproxy/haproxy.cfg)"$'\n'
    log "static pods written; kubelet starts them once it runs (kubeadm init)"
  else
    run systemctl enable --now haproxy
    run systemctl enable --now keepalived
    run systemctl restart haproxy
    run systemctl restart keepalived
  fi
  log "next: k8s_setup.sh --role=control_plane --control-plane-endpoint=$VIP:$LB_PORT"
}

main "$@"
