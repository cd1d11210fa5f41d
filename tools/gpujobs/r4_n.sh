set -o pipefail
bash tools/gpu_steps.sh \
 "t_sk|300|python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k 'norm_free or skinny or logits_match or pp2_stage_graphs' -m gpu" \
 "p_new|300|DETAIL=1 bash tools/profile.sh /tmp/pn -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4n_new.log 2>&1 && cp /tmp/pn/summary.txt gpurun_out/r4n_new_summary.txt" \
 "p_base|300|KGC_OPS_SO=build/ab/_kgc_ops_base.so DETAIL=1 bash tools/profile.sh /tmp/pb -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4n_base.log 2>&1 && cp /tmp/pb/summary.txt gpurun_out/r4n_base_summary.txt" \
 "b8_new|300|python bench.py --mode engine --num-prompts 8 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4n_b8_new.json 2>/dev/null" \
 "b8_base|300|KGC_OPS_SO=build/ab/_kgc_ops_base.so python bench.py --mode engine --num-prompts 8 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4n_b8_base.json 2>/dev/null"
