set -o pipefail
bash tools/gpu_steps.sh \
 "t_smp|200|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k sample -m gpu && python tools/sample_bench.py --batches 1,256 > gpurun_out/r4d2_sample.jsonl" \
 "t_eng|900|python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k 'tp_on_one_gpu or pp2 or two_node or graph_equals or rope_fused' -m gpu" \
 "eng|400|python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4d_eng.json 2> gpurun_out/r4d_eng.err" \
 "eng_pr0|400|KGC_PREFILL_ROPE_FUSED=0 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4d_eng_pr0.json 2> gpurun_out/r4d_eng_pr0.err" \
 "eng_b1|300|python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 --log-level info > gpurun_out/r4d_eng_b1.json 2> gpurun_out/r4d_eng_b1.err"
