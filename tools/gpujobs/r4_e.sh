set -o pipefail
T8="tests/test_engine_gpu.py::test_tp_on_one_gpu_matches_tp1[8-True-tiny-llama-gqa8-False-False]"
bash tools/gpu_steps.sh \
 "t_smp|200|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k sample -m gpu && python tools/sample_bench.py --batches 1,256 > gpurun_out/r4e_sample.jsonl" \
 "tp8_a|200|python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu" \
 "tp8_b|200|KGC_PREFILL_ROPE_FUSED=0 python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu" \
 "tp8_c|200|KGC_VP_SAMPLING=0 python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu" \
 "tp8_d|200|KGC_TP_AR_NORM=0 KGC_PREFILL_ROPE_FUSED=0 KGC_VP_SAMPLING=0 python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu"
