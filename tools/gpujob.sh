#!/bin/bash
# One GPU job = named recipes run in order through tools/gpu_steps.sh (each under its own
# time limit; a step that times out, aborts or faults ends the call there).
#
#   gpurun --timeout 1200 -- 'TAG=r5a bash tools/gpujob.sh tests_kern bench prof'
#   TAG=r5b K="paged_decode or dgemm" bash tools/gpujob.sh tests_k attn
#   TAG=r5c ENV="KGC_DGEMM=0" bash tools/gpujob.sh eng            (env for bench / prof steps)
#
# Outputs land in gpurun_out/<TAG>_<recipe>.*  Recipes:
#   full      pytest -m gpu over tests/ (the driver's round-end tier)
#   tests_k   pytest -m gpu -k "$K" over tests/
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py (the driver's headline command)
#   eng       python bench.py --mode engine --steps 2 --warmup 1
#   b1        batch 1, 128 output tokens, engine mode
#   prof      rocprofv3 anatomy of one engine wave (DETAIL=1 per-instantiation)
#   prof_b1   the same at batch 1
#   attn      decode attention microbench (B = 256 / 32 / 1 and the 70B TP = 8 rank heads)
#   dgemm     K9m microbench at M = 256
#   b70       Llama-3-70B one-GPU service bench
#   mixtral   Mixtral 8x7B one-GPU service bench
#   phantom   Llama-3-70B TP = 8 rank-0 stand-in (one GPU), engine mode + anatomy
#   dgemm8    K9m microbench at M = 256 on the Llama-3-70B TP = 8 shard shapes
#   prof_mix  rocprofv3 anatomy of one Mixtral 8x7B engine wave (DETAIL=1)
#   phantom_mix  Mixtral 8x7B EP = 8 rank-0 stand-in (one GPU), engine mode + anatomy
#   py        python $PY (a probe / microbench; limit $PYT seconds, default 300)
set -o pipefail
TAG="${TAG:-job}"
K="${K:-}"
ENVS="${ENV:-}"
mkdir -p gpurun_out
O="gpurun_out/${TAG}"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
steps=()
for r in "$@"; do
  case "$r" in
    full)    steps+=("full|900|$PT tests -m gpu > ${O}_full.log 2>&1; tail -5 ${O}_full.log") ;;
    tests_k) steps+=("tests_k|600|$PT tests -m gpu -k '$K' > ${O}_tests_k.log 2>&1; tail -5 ${O}_tests_k.log") ;;
    smoke)   steps+=("smoke|200|python -c 'import __graft_entry__ as g; g.smoke()' > ${O}_smoke.log 2>&1; tail -3 ${O}_smoke.log") ;;
    bench)   steps+=("bench|600|env $ENVS python bench.py > ${O}_bench.json 2> ${O}_bench.err") ;;
    eng)     steps+=("eng|450|env $ENVS python bench.py --mode engine --steps 2 --warmup 1 > ${O}_eng.json 2> ${O}_eng.err") ;;
    b1)      steps+=("b1|300|env $ENVS python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > ${O}_b1.json 2> ${O}_b1.err") ;;
    prof)    steps+=("prof|450|env $ENVS DETAIL=1 bash tools/profile.sh /tmp/prof_${TAG} -- python bench.py --mode engine --steps 1 --warmup 0 > ${O}_prof.log 2>&1 && cp /tmp/prof_${TAG}/summary.txt ${O}_prof_summary.txt") ;;
    prof_b1) steps+=("prof_b1|300|env $ENVS DETAIL=1 bash tools/profile.sh /tmp/profb1_${TAG} -- python bench.py --mode engine --num-prompts 1 --output-len 128 --steps 1 --warmup 1 > ${O}_prof_b1.log 2>&1 && cp /tmp/profb1_${TAG}/summary.txt ${O}_prof_b1_summary.txt") ;;
    attn)    steps+=("attn|300|python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --rope 4 > ${O}_attn.jsonl && python tools/attn_bench.py --batch 32 --ctx 2600 --ragged 0.25 >> ${O}_attn.jsonl && python tools/attn_bench.py --batch 1 --ctx 640 --ragged 0 --rope 0 >> ${O}_attn.jsonl && python tools/attn_bench.py --batch 256 --ctx 640 --ragged 0 --nq 8 --nkv 1 --rope 4 >> ${O}_attn.jsonl") ;;
    moe)     steps+=("moe|400|python tools/moe_bench.py --tokens 1 16 64 128 256 --no-loop > ${O}_moe.jsonl 2> ${O}_moe.err") ;;
    dgemm)   steps+=("dgemm|500|python tools/dgemm_bench.py --ms 256 --splits 1,2,3,4,5,6,8,12,16 > ${O}_dgemm.jsonl 2> ${O}_dgemm.err") ;;
    phantom_mix) steps+=("phantom_mix|600|env $ENVS KGC_TP_PHANTOM=8 DETAIL=1 bash tools/profile.sh /tmp/phm_${TAG} -- python bench.py --mode engine --model mixtral-8x7b --moe-parallel ep --steps 1 --warmup 1 > ${O}_phantom_mix.log 2>&1 && cp /tmp/phm_${TAG}/summary.txt ${O}_phantom_mix_summary.txt") ;;
    dgemm8)  steps+=("dgemm8|500|python tools/dgemm_bench.py --model llama-3-70b --tp 8 --ms 256 --copies 8 --shapes qkv,o,gate_up,down --splits 1,2,3,4,6,8,12,16 > ${O}_dgemm8.jsonl 2> ${O}_dgemm8.err") ;;
    prof_mix) steps+=("prof_mix|900|env $ENVS DETAIL=1 bash tools/profile.sh /tmp/pmix_${TAG} -- python bench.py --mode engine --model mixtral-8x7b --steps 1 --warmup 1 > ${O}_prof_mix.log 2>&1 && cp /tmp/pmix_${TAG}/summary.txt ${O}_prof_mix_summary.txt") ;;
    b70)     steps+=("b70|1100|env $ENVS python bench.py --model llama-3-70b --steps 1 --warmup 1 > ${O}_b70.json 2> ${O}_b70.err") ;;
    mixtral) steps+=("mixtral|1000|env $ENVS python bench.py --model mixtral-8x7b --steps 1 --warmup 1 > ${O}_mixtral.json 2> ${O}_mixtral.err") ;;
    phantom) steps+=("phantom|600|env $ENVS KGC_TP_PHANTOM=8 DETAIL=1 bash tools/profile.sh /tmp/ph_${TAG} -- python bench.py --mode engine --model llama-3-70b --steps 1 --warmup 1 > ${O}_phantom.log 2>&1 && cp /tmp/ph_${TAG}/summary.txt ${O}_phantom_summary.txt") ;;
    py)      steps+=("py|${PYT:-300}|python $PY > ${O}_py.jsonl 2> ${O}_py.err") ;;
    *) echo "unknown recipe $r" >&2; exit 2 ;;
  esac
done
bash tools/gpu_steps.sh "${steps[@]}"
