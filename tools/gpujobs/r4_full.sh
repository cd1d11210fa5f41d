set -o pipefail
bash tools/gpu_steps.sh \
 "full|1100|python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/gpu_tests_full_r4.log 2>&1; tail -5 gpurun_out/gpu_tests_full_r4.log"
