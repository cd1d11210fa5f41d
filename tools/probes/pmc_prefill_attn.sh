export TMPDIR=/tmp
set -e
for sh in 32x512 1x16384; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_pf_$sh -o p -- python tools/prefill_attn_bench.py --shapes $sh --chunked 0 > gpurun_out/pmc_pf_$sh.log 2>&1
  python tools/pmc_summary.py $(find gpurun_out/pmc_pf_$sh -name 'p_results.db' | head -1) --match prefill > gpurun_out/pmc_pf_$sh.txt
done
