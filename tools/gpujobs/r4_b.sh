set -o pipefail
bash tools/gpu_steps.sh \
 "t_ar|500|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_allreduce_gpu.py tests/test_world_emulation_gpu.py -m gpu" \
 "t_decode|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'paged_decode or dgemm or sample' -m gpu" \
 "attn_w1|200|python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --rope 4 > gpurun_out/r4b_attn_w1.jsonl && python tools/attn_bench.py --batch 32 --ctx 2600 --ragged 0.25 >> gpurun_out/r4b_attn_w1.jsonl && python tools/attn_bench.py --batch 1 --ctx 640 --ragged 0 --rope 0 >> gpurun_out/r4b_attn_w1.jsonl" \
 "eng_w1|400|python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4b_eng_w1.json" \
 "eng_w0|400|KGC_DECODE_WAVE=0 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4b_eng_w0.json"
