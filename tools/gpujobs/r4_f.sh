set -o pipefail
T8="tests/test_engine_gpu.py::test_tp_on_one_gpu_matches_tp1[8-True-tiny-llama-gqa8-False-False]"
bash tools/gpu_steps.sh \
 "hf|300|python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k 'logits_match_hf and not fused' -m gpu" \
 "tp8_g|200|KGC_SKINNY_GEMM=0 KGC_DGEMM=0 python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu" \
 "tp8_h|200|KGC_DECODE_WAVE=0 KGC_SKINNY_GEMM=0 KGC_DGEMM=0 KGC_PREFILL_ROPE_FUSED=0 KGC_TP_AR_NORM=0 python -u -m pytest -q -x --timeout 150 --timeout-method thread '$T8' -m gpu"
