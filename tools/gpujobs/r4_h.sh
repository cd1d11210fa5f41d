set -o pipefail
bash tools/gpu_steps.sh \
 "t_2s|300|python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k 'two_stream or tp_on_one_gpu' -m gpu" \
 "eng_s1|400|python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4h_eng_s1.json 2> gpurun_out/r4h_eng_s1.err" \
 "eng_s0|400|KGC_PREFILL_STREAMS=0 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r4h_eng_s0.json 2> gpurun_out/r4h_eng_s0.err"
