set -o pipefail
bash tools/gpu_steps.sh \
 "t_kern|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'paged_decode or sample or prefill_rope' -m gpu" \
 "attn|200|python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --rope 4 > gpurun_out/r4d_attn.jsonl && python tools/attn_bench.py --batch 32 --ctx 2600 --ragged 0.25 >> gpurun_out/r4d_attn.jsonl && python tools/attn_bench.py --batch 1 --ctx 640 --ragged 0 --rope 0 >> gpurun_out/r4d_attn.jsonl && python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --nq 8 --nkv 1 --rope 4 >> gpurun_out/r4d_attn.jsonl" \
 "smp|120|python tools/sample_bench.py > gpurun_out/r4d_sample.jsonl" \
 "t_ar|400|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_allreduce_gpu.py tests/test_world_emulation_gpu.py -m gpu" \
 "t_wv|240|python -u -m pytest -x -q --timeout 120 --timeout-method thread tools/research/test_research_gpu.py -k wv" \
 "wv_bench|400|python tools/research/wv_bench.py > gpurun_out/r4d_wv.jsonl"
