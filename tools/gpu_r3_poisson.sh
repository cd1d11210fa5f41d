set -o pipefail
mkdir -p gpurun_out/r3p
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_allreduce_gpu.py -k "timeout or (matches_sum and 2)" -s > gpurun_out/r3p/ar_timeout.log 2>&1 && \
KGC_FAKE_ENGINE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 8 --device cpu --model llama-3-8b --steps 1 --warmup 1 > gpurun_out/r3p/fake_dp8.log 2>&1 && \
timeout -k 10 330 python -u bench/serve_bench.py --launch --gpus 1 --num-prompts 1024 --request-rate 40 --json-out gpurun_out/r3p/poisson_decode_first.json > gpurun_out/r3p/poisson_decode_first.log 2>&1 && \
timeout -k 10 330 python -u bench/serve_bench.py --launch --gpus 1 --num-prompts 1024 --request-rate 40 --json-out gpurun_out/r3p/poisson_pf_bounded.json -- --prefill-first > gpurun_out/r3p/poisson_pf_bounded.log 2>&1 && \
timeout -k 10 330 python -u bench/serve_bench.py --launch --gpus 1 --num-prompts 1024 --request-rate 40 --json-out gpurun_out/r3p/poisson_pf_unbounded.json -- --prefill-first --prefill-first-max-defer 1000000 > gpurun_out/r3p/poisson_pf_unbounded.log 2>&1
echo rc=$?
