#!/usr/bin/env bash
# Kernel-level profile of any engine command with rocprofv3, summarised.
#   tools/profile.sh <out_dir> -- python bench.py --steps 1 --warmup 1
#   PMC=1 tools/profile.sh <out_dir> -- python tools/attn_bench.py   (counter pass: MFMA /
#        LDS / HBM counters; collected in its own run, never combined with API tracing)
# Writes <out_dir>/run_results.db (rocpd) and <out_dir>/summary.txt (kernel families and
# the steady-state decode-step anatomy from tools/trace_summary.py).
set -euo pipefail
out="${1:?usage: tools/profile.sh OUT_DIR -- CMD...}"; shift
[[ "${1:-}" == "--" ]] && shift
[[ $# -gt 0 ]] || { echo "no command" >&2; exit 2; }
mkdir -p "$out"
export TMPDIR=/tmp
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
if [[ "${PMC:-0}" == "1" ]]; then
  # one counter group per pass keeps the run within the hardware counter slots
  rocprofv3 --kernel-trace --stats \
    --pmc SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT TCC_EA0_RDREQ_sum \
    -d "$out" -o pmc -- "$@"
  echo "counters under $out (pmc_*)"
  exit 0
fi
rocprofv3 --kernel-trace --stats -d "$out" -o run -- "$@"
db=$(find "$out" -name 'run_results.db' | head -1)
if [[ -n "$db" ]]; then
  python "$HERE/trace_summary.py" "$db" --steps ${DETAIL:+--detail} | tee "$out/summary.txt"
else
  csv=$(find "$out" -name '*kernel_trace.csv' | head -1)
  python "$HERE/trace_summary.py" "$csv" --steps ${DETAIL:+--detail} | tee "$out/summary.txt"
fi
