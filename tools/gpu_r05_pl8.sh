#!/bin/bash
# Two-phase placement (the slab, then the replies' array alone): dense-path parity, three logged
# processes (exp/libplog.so) and three default ones (tools/place_probe4.py).
set -u
O=gpurun_out/${1:-r05_pl8}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4_full.py::test_cfg4_single_engine_equals_oracle tests/test_gpu_big_paths.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1 || { echo STOP tests; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for rep in 1 2 3; do
  GOSSIP_LIB=exp/libplog.so timeout -k 10 150 python tools/place_probe4.py >> $O/log.txt 2>&1 || { echo STOP; tail -5 $O/log.txt; exit 1; }
done
for rep in 1 2 3; do
  timeout -k 10 150 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo STOP; tail -5 $O/probe.txt; exit 1; }
done
grep -v amdgpu.ids $O/log.txt
cat $O/probe.txt
