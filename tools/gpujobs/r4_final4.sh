set -o pipefail
bash tools/gpu_steps.sh \
 "prof|400|DETAIL=1 bash tools/profile.sh /tmp/prof_f -- python bench.py --mode engine --steps 1 --warmup 0 > gpurun_out/r4f4_prof.log 2>&1 && cp /tmp/prof_f/summary.txt gpurun_out/r4f4_prof_summary.txt" \
 "mixtral|700|python bench.py --model mixtral-8x7b --steps 1 --warmup 1 > gpurun_out/bench_mixtral_r4.json 2> gpurun_out/bench_mixtral_r4.err"
