set -o pipefail
export KGC_BENCH_DEVICES=0,0
bash tools/gpu_steps.sh \
 "dp2_shared|900|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --num-prompts 64 --output-len 64 --steps 1 --warmup 1 --num-gpu-blocks-override 4096 > gpurun_out/r4m_dp2.json"
