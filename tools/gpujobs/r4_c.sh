set -o pipefail
bash tools/gpu_steps.sh \
 "t_kern2|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'paged_decode or prefill_rope or acc_norm or accnorm or skinny or sample' -m gpu" \
 "attn|200|python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --rope 4 > gpurun_out/r4c_attn.jsonl && python tools/attn_bench.py --batch 32 --ctx 2600 --ragged 0.25 >> gpurun_out/r4c_attn.jsonl && python tools/attn_bench.py --batch 1 --ctx 640 --ragged 0 --rope 0 >> gpurun_out/r4c_attn.jsonl && KGC_DECODE_WAVE=0 python tools/attn_bench.py --batch 1 --ctx 640 --ragged 0 --rope 0 >> gpurun_out/r4c_attn.jsonl" \
 "rope_ab|200|python tools/prefill_rope_bench.py > gpurun_out/r4c_rope.jsonl && KGC_ROPE_KVG=0 python tools/prefill_rope_bench.py >> gpurun_out/r4c_rope.jsonl" \
 "ar_bench|300|python tools/allreduce_rms_bench.py --world 2 > gpurun_out/r4c_arbench.jsonl && python tools/allreduce_rms_bench.py --world 4 >> gpurun_out/r4c_arbench.jsonl" \
 "eng_b1|300|python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4c_eng_b1.json 2> gpurun_out/r4c_eng_b1.err" \
 "clock|260|timeout -s KILL 220 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d /tmp/pmc_pf -o p -- python tools/prefill_gemm_probe.py --tables default --reps 100 --layers 4 > gpurun_out/r4c_pf_probe.jsonl && python tools/pmc_summary.py \$(find /tmp/pmc_pf -name 'p_results.db') > gpurun_out/r4c_pf_clock.txt" \
 "smi|200|(for i in \$(seq 40); do rocm-smi --showpower --showclocks --csv; sleep 1; done > gpurun_out/r4c_smi.txt 2>&1) & python tools/prefill_gemm_probe.py --tables default --reps 400 --layers 4 > gpurun_out/r4c_pf_sustained.jsonl; wait" \
 "prof|400|bash tools/profile.sh /tmp/prof_c -- python bench.py --mode engine --steps 1 --warmup 0 > gpurun_out/r4c_prof.log 2>&1 && cp /tmp/prof_c/summary.txt gpurun_out/r4c_prof_summary.txt"
