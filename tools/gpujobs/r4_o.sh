set -o pipefail
bash tools/gpu_steps.sh \
 "t_dec|300|python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'paged_decode' -m gpu" \
 "attn_b1|300|for c in 640 2048 4096; do for w in 0 8; do KGC_DECODE_WIDE_MAX_PAIRS=\$w python tools/attn_bench.py --batch 1 --ctx \$c --ragged 0 >> gpurun_out/r4o_attn_b1.jsonl || exit 2; done; done" \
 "p_wide|300|DETAIL=1 bash tools/profile.sh /tmp/pw -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4o_wide.log 2>&1 && cp /tmp/pw/summary.txt gpurun_out/r4o_wide_summary.txt" \
 "p_nowide|300|KGC_DECODE_WIDE_MAX_PAIRS=0 DETAIL=1 bash tools/profile.sh /tmp/pz -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4o_nowide.log 2>&1 && cp /tmp/pz/summary.txt gpurun_out/r4o_nowide_summary.txt" \
 "t_eng|400|python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -m gpu"
