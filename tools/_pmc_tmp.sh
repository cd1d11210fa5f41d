set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/pmc2 -o p -- python3 $R/tools/dgemm_bench.py --shapes gate_up --only 6:1:1 --no-lib --copies 8 > $R/gpurun_out/pmc2.log 2>&1
