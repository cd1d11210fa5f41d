set -o pipefail
bash tools/gpu_steps.sh \
 "bench|600|python bench.py > gpurun_out/bench_r4f.json 2> gpurun_out/bench_r4f.err" \
 "prof|500|DETAIL=1 bash tools/profile.sh /tmp/prof_f -- python bench.py --mode engine --steps 1 --warmup 0 > gpurun_out/r4f4_prof.log 2>&1 && cp /tmp/prof_f/summary.txt gpurun_out/r4f4_prof_summary.txt"
