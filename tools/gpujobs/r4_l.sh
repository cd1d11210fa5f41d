set -o pipefail
bash tools/gpu_steps.sh \
 "t_rs|300|python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k 'norm_free or skinny or logits_match' -m gpu" \
 "prof_rs1|300|DETAIL=1 bash tools/profile.sh /tmp/p1 -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4l_prof_rs1.log 2>&1 && cp /tmp/p1/summary.txt gpurun_out/r4l_prof_rs1_summary.txt" \
 "prof_rs0|300|KGC_RS_LAYER=0 DETAIL=1 bash tools/profile.sh /tmp/p0 -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4l_prof_rs0.log 2>&1 && cp /tmp/p0/summary.txt gpurun_out/r4l_prof_rs0_summary.txt"
