#!/usr/bin/env bash
# CRI-O + crictl install (reference crio_setup.sh shape: opensuse isv:/cri-o repo,
# crictl tarball, optional proxy drop-in).
#   sudo bash crio_setup.sh [--crio-version v1.33] [--crictl-version v1.33.0] [--proxy URL]
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "$HERE/lib.sh"

CRIO_VERSION="v1.33"
CRICTL_VERSION="v1.33.0"
PROXY="${PROXY:-}"

while [[ $# -gt 0 ]]; do
  case "$1" in
    --crio-version=*) CRIO_VERSION="${1#*=}" ;;
    --crio-version) CRIO_VERSION="$2"; shift ;;
    --crictl-version=*) CRICTL_VERSION="${1#*=}" ;;
    --crictl-version) CRICTL_VERSION="$2"; shift ;;
    --proxy=*) PROXY="${1#*=}" ;;
    --proxy) PROXY="$2"; shift ;;
    --dry-run) DRY_RUN=1 ;;
    *) die "unknown argument $1" ;;
  esac
  shift
done

require_root
KEYRING=/etc/apt/keyrings/cri-o-apt-keyring.asc   # armoured key; apt accepts .asc as-is
write_file /etc/apt/sources.list.d/cri-o.list \
  "deb [signed-by=$KEYRING] https://download.opensuse.org/repositories/isv:/cri-o:/stable:/$CRIO_VERSION/deb/ /
"
mkdir -p "${ROOT}/etc/apt/keyrings"
run curl -fsSL ${PROXY:+--proxy "$PROXY"} \
  "https://download.opensuse.org/repositories/isv:/cri-o:/stable:/$CRIO_VERSION/deb/Release.key" \
  -o "${ROOT}${KEYRING}" \
  || die "could not fetch the CRI-O apt key from download.opensuse.org (network / --proxy?)"
if [[ -n "$PROXY" ]]; then
  write_file /etc/apt/apt.conf.d/95kgc-proxy "Acquire::http::Proxy \"$PROXY\";
Acquire::https::Proxy \"$PROXY\";
"
fi
run apt-get update -y || die "apt-get update failed (the CRI-O repository is unusable)"
run apt-get install -y cri-o || die "installing cri-o failed"
run systemctl enable --now crio || true

arch=$(uname -m); [[ "$arch" == "x86_64" ]] && arch=amd64
tarball="crictl-$CRICTL_VERSION-linux-$arch.tar.gz"
run curl -fsSL ${PROXY:+--proxy "$PROXY"} -o "/tmp/$tarball" \
  "https://github.com/kubernetes-sigs/cri-tools/releases/download/$CRICTL_VERSION/$tarball" \
  && run tar -C "${ROOT}/usr/local/bin" -xzf "/tmp/$tarball" || warn "crictl download failed"

if [[ -n "$PROXY" ]]; then
  write_file /etc/systemd/system/crio.service.d/proxy.conf "[Service]
Environment=\"HTTP_PROXY=$PROXY\" \"HTTPS_PROXY=$PROXY\" \"NO_PROXY=127.0.0.1,localhost,10.0.0.0/8,192.168.0.0/16\"
"
  run systemctl daemon-reload || true
  run systemctl restart crio || true
fi
have_cmd crio && run crio --version || true
log "CRI-O $CRIO_VERSION ready"
