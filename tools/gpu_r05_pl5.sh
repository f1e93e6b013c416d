#!/bin/bash
# Placement calibration (param place_tries): processes alternating 1 / 4 tries (tools/place_probe4.py),
# after the dense-path parity tests on the calibrated default.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_pl5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4_full.py::test_cfg4_single_engine_equals_oracle -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1 || { echo STOP tests; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for rep in 1 2 3 4; do
  for t in 1 4; do
    PROBE_TRIES=$t timeout -k 10 120 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo "STOP"; tail -5 $O/probe.txt; exit 1; }
    tail -1 $O/probe.txt
  done
done
