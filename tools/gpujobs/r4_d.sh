set -o pipefail
bash tools/gpu_steps.sh \
 "t_kern|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'paged_decode or sample or prefill_rope' -m gpu" \
 "attn|200|python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --rope 4 > gpurun_out/r4d_attn.jsonl && python tools/attn_bench.py --batch 32 --ctx 2600 --ragged 0.25 >> gpurun_out/r4d_attn.jsonl && python tools/attn_bench.py --batch 1 --ctx 640 --ragged 0 --rope 0 >> gpurun_out/r4d_attn.jsonl && python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --nq 8 --nkv 1 --rope 4 >> gpurun_out/r4d_attn.jsonl" \
 "smp|120|python tools/sample_bench.py > gpurun_out/r4d_sample.jsonl" \
 "t_ar|400|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_allreduce_gpu.py tests/test_world_emulation_gpu.py -m gpu" \
 "t_eng|900|python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k 'tp_on_one_gpu or pp2 or two_node or graph_equals or rope_fused' -m gpu" \
 "eng|400|python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4d_eng.json 2> gpurun_out/r4d_eng.err" \
 "eng_pr0|400|KGC_PREFILL_ROPE_FUSED=0 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4d_eng_pr0.json 2> gpurun_out/r4d_eng_pr0.err" \
 "prof|400|bash tools/profile.sh /tmp/prof_d -- python bench.py --mode engine --steps 1 --warmup 0 > gpurun_out/r4d_prof.log 2>&1 && cp /tmp/prof_d/summary.txt gpurun_out/r4d_prof_summary.txt"
