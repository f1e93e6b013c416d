#!/bin/bash
# Counters of the first dense round (EXP_AUTO=1 tools/exp_rounds.py): HBM bytes, request sizes,
# L2 hits, SQ activity; one counter group per pass.  Summary per dense kernel (last dispatch).
set -u
O=gpurun_out/pmc3
mkdir -p $O
export TMPDIR=/tmp EXP_AUTO=1
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
B="python tools/exp_rounds.py"
P=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
  P=$((P+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O -o p$P -- $B > $O/p$P.txt 2>&1; ok $?
done
for k in bin_emit bin_serve bin_apply; do echo "== $k"; python tools/pmc_dispatch.py $O $k | tail -1; done
echo done
