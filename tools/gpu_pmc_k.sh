#!/bin/bash
# SQ / TCP / TCC / TA counters per kernel (launch averages, tools/pmc_sq.py) of tools/exp_bench.py on
# the bench workload, one rocprofv3 --pmc pass per counter group.  OUT: directory under gpurun_out/;
# EXP_N / EXP_SEED / EXP_PARAMS as exp_bench.py; PMC_CMD: another program to profile (default the bench
# workload through tools/exp_bench.py), PMC_NODES: the node count per-node figures divide by.
set -u
O=gpurun_out/${OUT:-pmck}
mkdir -p $O
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  EXP_STEPS=2 timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o p \
    -- ${PMC_CMD:-python tools/exp_bench.py} > $O/p$i.txt 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "STOP: pass $i exited $rc"; tail -3 $O/p$i.txt; exit $rc; fi
done
PMC_NODES=${PMC_NODES:-${EXP_N:-16777216}} python tools/pmc_sq.py $O $O/pmc_k.json > /dev/null && echo pmc ok
