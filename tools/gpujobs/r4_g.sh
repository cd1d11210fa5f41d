set -o pipefail
T8="tests/test_engine_gpu.py::test_tp_on_one_gpu_matches_tp1[8-True-tiny-llama-gqa8-False-False]"
bash tools/gpu_steps.sh \
 "gloo|200|python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gloo_cuda_gpu.py -m gpu" \
 "tp8_c|200|KGC_VP_SAMPLING=0 python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu" \
 "t_pf|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'prefill_attention or prefill_rope or paged_decode_rope' -m gpu"
