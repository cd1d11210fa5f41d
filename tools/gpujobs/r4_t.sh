set -o pipefail
bash tools/gpu_steps.sh \
 "b70|1100|python bench.py --model llama-3-70b --steps 1 --warmup 1 > gpurun_out/bench_70b_r4.json 2> gpurun_out/bench_70b_r4.err"
