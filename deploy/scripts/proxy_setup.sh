#!/usr/bin/env bash
# Optional egress proxy for air-gapped / filtered sites: privoxy on 127.0.0.1:8118
# forwarding to a SOCKS5 upstream that the operator provides (an SSH -D tunnel, a
# corporate SOCKS gateway, ...).  k8s_setup.sh --proxy=http://127.0.0.1:8118 then uses
# it for apt and CRI-O image pulls.  Mirrors the reference's privoxy_setup.sh /
# ssh-tunel.md behaviour (privoxy_setup.sh:1-38); unlike xray_setup.sh it never
# downloads a client configuration from anywhere.
#
#   sudo bash proxy_setup.sh --socks=127.0.0.1:1080 [--listen=127.0.0.1:8118]
#   sudo bash proxy_setup.sh --socks=127.0.0.1:1080 --ssh-tunnel=user@bastion [--ssh-key=/path]
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "$HERE/lib.sh"

SOCKS="" LISTEN="127.0.0.1:8118" TUNNEL="" SSH_KEY=""

parse_args() {
  while [[ $# -gt 0 ]]; do
    local arg="$1" val=""
    case "$arg" in
      --*=*) val="${arg#*=}"; arg="${arg%%=*}" ;;
      --yes|-y|--dry-run) ;;
      --*) [[ $# -ge 2 ]] || die "$arg needs a value"; val="$2"; shift ;;
    esac
    case "$arg" in
      --socks) SOCKS="$val" ;;
      --listen) LISTEN="$val" ;;
      --ssh-tunnel) TUNNEL="$val" ;;
      --ssh-key) SSH_KEY="$val" ;;
      --yes|-y) ASSUME_YES=1 ;;
      --dry-run) DRY_RUN=1 ;;
      *) die "unknown argument $arg" ;;
    esac
    shift
  done
  [[ "$SOCKS" =~ ^[A-Za-z0-9.-]+:[0-9]+$ ]] || die "--socks=HOST:PORT is required"
  [[ "$LISTEN" =~ ^[0-9.]+:[0-9]+$ ]] || die "bad --listen $LISTEN"
  return 0
}

main() {
  parse_args "$@"
  require_root
  [[ "${SKIP_APT:-0}" == 1 ]] || run apt-get install -y privoxy
  backup /etc/privoxy/config
  write_file /etc/privoxy/config "# privoxy: local HTTP proxy -> SOCKS5 $SOCKS (proxy_setup.sh)
listen-address  $LISTEN
forward-socks5  /  $SOCKS  .
forward         localhost/  .
forward         127.*.*.*/  .
forward         10.*.*.*/   .
forward         192.168.*.*/ .
toggle 0
enable-remote-toggle 0
enable-edit-actions 0
buffer-limit 4096
"
  if [[ -n "$TUNNEL" ]]; then
    local port="${SOCKS##*:}"
    write_file /etc/systemd/system/kgc-socks-tunnel.service "[Unit]
Description=SOCKS5 tunnel for the cluster egress proxy (ssh -D $port)
After=network-online.target
Wants=network-online.target

[Service]
ExecStart=/usr/bin/ssh -N -D 127.0.0.1:$port ${SSH_KEY:+-i $SSH_KEY }-o ServerAliveInterval=30 -o ServerAliveCountMax=3 -o ExitOnForwardFailure=yes $TUNNEL
Restart=always
RestartSec=5

[Install]
WantedBy=multi-user.target
"
    run systemctl daemon-reload
    run systemctl enable --now kgc-socks-tunnel.service
  fi
  run systemctl restart privoxy
  run systemctl enable privoxy
  log "proxy ready: export http_proxy=http://$LISTEN https_proxy=http://$LISTEN"
}

main "$@"
