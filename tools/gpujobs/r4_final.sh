set -o pipefail
bash tools/gpu_steps.sh \
 "t_fix|200|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k tail_fused -m gpu" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r4.log 2>&1; tail -3 gpurun_out/smoke_r4.log" \
 "bench|500|python bench.py > gpurun_out/bench_r4.json 2> gpurun_out/bench_r4.err" \
 "prof|400|bash tools/profile.sh /tmp/prof_f -- python bench.py --mode engine --steps 1 --warmup 0 > gpurun_out/r4f_prof.log 2>&1 && cp /tmp/prof_f/summary.txt gpurun_out/r4f_prof_summary.txt" \
 "prof_b1|300|bash tools/profile.sh /tmp/prof_b1 -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4f_prof_b1.log 2>&1 && cp /tmp/prof_b1/summary.txt gpurun_out/r4f_prof_b1_summary.txt"
