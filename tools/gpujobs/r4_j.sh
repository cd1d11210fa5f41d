set -o pipefail
bash tools/gpu_steps.sh \
 "t_rs|300|python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k 'norm_free or skinny or logits_match or graph_equals' -m gpu" \
 "b1_rs1|300|python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4j_b1_rs1.json 2>/dev/null" \
 "b1_rs0|300|KGC_RS_LAYER=0 python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4j_b1_rs0.json 2>/dev/null" \
 "prof_b1|300|bash tools/profile.sh /tmp/prof_b1 -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4j_prof_b1.log 2>&1 && cp /tmp/prof_b1/summary.txt gpurun_out/r4j_prof_b1_summary.txt" \
 "prof_b1_0|300|KGC_RS_LAYER=0 bash tools/profile.sh /tmp/prof_b1z -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4j_prof_b1z.log 2>&1 && cp /tmp/prof_b1z/summary.txt gpurun_out/r4j_prof_b1z_summary.txt"
