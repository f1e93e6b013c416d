#!/bin/bash
# SQ / TCP / TCC counters of the dense-round kernels on the bench workload (one counter group per
# pass, each under its own time limit), summarized per launch by tools/pmc_sq.py.
# usage: gpu_pmc_sq.sh <out> ; BENCH="..." overrides the profiled command.
set -u
O=gpurun_out/${1:-pmc_sq}
mkdir -p $O
export TMPDIR=/tmp
B=${BENCH:-python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dense-only}
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o p -- $B > $O/p$i.out 2>&1 \
    || { echo "STOP: pass $i exited $?"; tail -5 $O/p$i.out; exit 1; }
done
python tools/pmc_sq.py $O $O/pmc_sq.json > /dev/null && echo "pmc ok"
