#!/bin/bash
# Round 5: direct-round commits read D only at S_t's nonzero nodes.  Parity of the sparse paths,
# then the bench workload at 2^24 and 2^27 under alld_frac choices (which rounds go direct).
set -u
O=gpurun_out/${1:-r05_cm}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_big_paths.py tests/test_gpu_faults.py tests/test_gpu_cfg4_full.py -k "sparse or cfg4_single or auto" -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -1 $O/pytest.txt
SWEEP_N=16777216 SWEEP_STEPS=10 timeout -k 10 300 python tools/sweep_single.py - "alld_frac=0.004" "alld_frac=0.001" - "alld_frac=0.004" "alld_frac=0.001" > $O/sweep.16777216.txt 2>&1; ok $?
cat $O/sweep.16777216.txt
SWEEP_N=134217728 SWEEP_STEPS=6 timeout -k 10 400 python tools/sweep_single.py - "alld_frac=0.004" "alld_frac=0.001" - "alld_frac=0.004" "alld_frac=0.001" > $O/sweep.134217728.txt 2>&1; ok $?
cat $O/sweep.134217728.txt
echo done
