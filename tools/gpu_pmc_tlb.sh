set -u
export TMPDIR=/tmp
O=gpurun_out/vmm_tlb; mkdir -p $O
for v in default s8 s64; do
  L=exp/lib$v.so; [ $v = default ] && L=""
  GOSSIP_LIB=$L EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_PARAMS=place_tries=1 EXP_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/$v -o p -- python tools/exp_bench.py > $O/$v.txt 2>&1 || { echo "STOP $v"; exit 1; }
  tail -1 $O/$v.txt
done
