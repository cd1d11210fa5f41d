#!/usr/bin/env bash
# Shared helpers for the node bootstrap scripts.
#   ROOT=<dir>   prefix for every file the scripts write/read (tests use a tmp dir)
#   DRY_RUN=1    print commands instead of executing them (files still go to $ROOT)
#   ASSUME_YES=1 never prompt
ROOT=${ROOT:-}
DRY_RUN=${DRY_RUN:-0}
ASSUME_YES=${ASSUME_YES:-0}

log()   { printf "\033[1;34m[INFO]\033[0m %s\n" "$*"; }
warn()  { printf "\033[1;33m[WARN]\033[0m %s\n" "$*" >&2; }
error() { printf "\033[1;31m[ERR ]\033[0m %s\n" "$*" >&2; }
die()   { error "$*"; exit 1; }
have_cmd() { command -v "$1" >/dev/null 2>&1; }

# run CMD...: execute (or print under DRY_RUN); returns the command's status
run() {
  if [[ "$DRY_RUN" == "1" ]]; then
    printf "DRY: %s\n" "$*"
    return 0
  fi
  "$@"
}

require_root() {
  [[ -n "$ROOT" || "$DRY_RUN" == "1" ]] && return 0
  [[ "$(id -u)" -eq 0 ]] || die "run as root (sudo)"
}

confirm() {
  [[ "$ASSUME_YES" == "1" ]] && return 0
  read -r -p "$1 [y/N] " ans
  [[ "$ans" == "y" || "$ans" == "Y" ]]
}

# write_file PATH CONTENT: atomic write under $ROOT, creating parent dirs
write_file() {
  local dst="${ROOT}$1"
  mkdir -p "$(dirname "$dst")"
  printf "%s" "$2" > "$dst.tmp.$$" && mv "$dst.tmp.$$" "$dst"
  log "wrote $1"
}

# backup PATH: timestamped copy next to the original
backup() {
  local f="${ROOT}$1"
  [[ -f "$f" ]] || return 0
  cp -a "$f" "$f.bak.$(date +%Y%m%d%H%M%S)"
}

# kube_minor v1.33.3 -> v1.33
kube_minor() { local v="${1#v}"; echo "v${v%.*}"; }
