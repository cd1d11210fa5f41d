#!/usr/bin/env bash
# Build the native node tools (C++17, host only) into build/native/:
#   libamdgpu_topo.so, amdgpu-topo, amd-container-runtime, amd-container-hook, amd-ctk
# SANITIZE=1 builds an AddressSanitizer/UBSan variant into build/native-asan/.
set -euo pipefail
cd "$(dirname "$0")"
CXX=${CXX:-g++}
OUT=../build/native
FLAGS=(-O2 -std=c++17 -Wall -Wextra -Wno-unused-parameter -fPIC)
if [[ "${SANITIZE:-0}" == "1" ]]; then
  OUT=../build/native-asan
  FLAGS+=(-g -fsanitize=address,undefined -fno-omit-frame-pointer)
fi
mkdir -p "$OUT"
TOPO=(topo/amdgpu_topo.cpp)
DEV=(container/devices.cpp)
# each artefact is linked under a private name and renamed into place (atomic): a
# concurrent build (parallel test workers) never exposes a half-written binary
tmp="$OUT/.tmp.$$"
mkdir -p "$tmp"
trap 'rm -rf "$tmp"' EXIT
pids=()
$CXX "${FLAGS[@]}" -shared -o "$tmp/libamdgpu_topo.so" "${TOPO[@]}" & pids+=($!)
$CXX "${FLAGS[@]}" -o "$tmp/amdgpu-topo" topo/topo_cli.cpp "${TOPO[@]}" & pids+=($!)
$CXX "${FLAGS[@]}" -o "$tmp/amd-container-runtime" container/runtime_main.cpp "${DEV[@]}" "${TOPO[@]}" & pids+=($!)
$CXX "${FLAGS[@]}" -o "$tmp/amd-container-hook" container/hook_main.cpp "${DEV[@]}" "${TOPO[@]}" & pids+=($!)
$CXX "${FLAGS[@]}" -o "$tmp/amd-ctk" container/ctk_main.cpp "${DEV[@]}" "${TOPO[@]}" & pids+=($!)
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
if [[ $rc == 0 ]]; then
  for f in libamdgpu_topo.so amdgpu-topo amd-container-runtime amd-container-hook amd-ctk; do
    mv -f "$tmp/$f" "$OUT/$f"
  done
fi
exit $rc
