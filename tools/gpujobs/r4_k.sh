set -o pipefail
bash tools/gpu_steps.sh \
 "attn_b1|300|for c in 640 2048; do for z in 1 2 3 4 8 16; do python tools/attn_bench.py --batch 1 --ctx \$c --ragged 0 --z \$z >> gpurun_out/r4k_attn_b1.jsonl || exit 2; done; done" \
 "prof_b1d|300|DETAIL=1 bash tools/profile.sh /tmp/prof_b1 -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4k_prof_b1.log 2>&1 && cp /tmp/prof_b1/summary.txt gpurun_out/r4k_prof_b1_summary.txt" \
 "b8_rs1|300|python bench.py --mode engine --num-prompts 8 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4k_b8_rs1.json 2>/dev/null" \
 "b8_rs0|300|KGC_RS_LAYER=0 python bench.py --mode engine --num-prompts 8 --output-len 128 --steps 1 --warmup 1 > gpurun_out/r4k_b8_rs0.json 2>/dev/null"
