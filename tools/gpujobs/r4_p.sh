set -o pipefail
bash tools/gpu_steps.sh \
 "t_sk|300|python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k 'norm_free or skinny or logits_match or tune' -m gpu" \
 "p_b1|300|DETAIL=1 bash tools/profile.sh /tmp/pw -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4p_b1.log 2>&1 && cp /tmp/pw/summary.txt gpurun_out/r4p_b1_summary.txt" \
 "b1|300|python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4p_b1.json 2>gpurun_out/r4p_b1.err" \
 "b8|300|python bench.py --mode engine --num-prompts 8 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4p_b8.json 2>/dev/null" \
 "b32|300|python bench.py --mode engine --num-prompts 32 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4p_b32.json 2>/dev/null"
