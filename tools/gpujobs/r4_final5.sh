set -o pipefail
bash tools/gpu_steps.sh \
 "full|600|python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/gpu_tests_full_r4.log 2>&1; tail -5 gpurun_out/gpu_tests_full_r4.log" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r4.log 2>&1; tail -3 gpurun_out/smoke_r4.log" \
 "bench|500|python bench.py > gpurun_out/bench_r4g.json 2> gpurun_out/bench_r4g.err"
