set -o pipefail
bash tools/gpu_steps.sh \
 "t_eng|500|python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k 'norm_free or logits_match or skinny or tune or graph' -m gpu" \
 "p_b1|200|DETAIL=1 bash tools/profile.sh /tmp/pb1 -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4r_b1.log 2>&1 && cp /tmp/pb1/summary.txt gpurun_out/r4r_b1_summary.txt" \
 "b8|200|python bench.py --mode engine --num-prompts 8 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4r_b8.json 2>/dev/null"
