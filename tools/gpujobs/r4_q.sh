set -o pipefail
bash tools/gpu_steps.sh \
 "mixtral|1000|python bench.py --model mixtral-8x7b --steps 1 --warmup 1 > gpurun_out/bench_mixtral_r4.json 2> gpurun_out/bench_mixtral_r4.err"
