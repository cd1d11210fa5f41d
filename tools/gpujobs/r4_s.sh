set -o pipefail
bash tools/gpu_steps.sh \
 "e256|400|python bench.py --mode engine --steps 1 --warmup 1 > gpurun_out/r4s_e256.json 2> gpurun_out/r4s_e256.err" \
 "prof|400|DETAIL=1 bash tools/profile.sh /tmp/prof_s -- python bench.py --mode engine --steps 1 --warmup 0 > gpurun_out/r4s_prof.log 2>&1 && cp /tmp/prof_s/summary.txt gpurun_out/r4s_prof_summary.txt"
