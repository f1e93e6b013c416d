#!/bin/bash
# Replicated dense rounds: the sharded GPU tests that run them, then the per-rank
# device-time probe and the gloo rehearsal lines at G = 2 and 4.  Every step under its own limit.
set -u
O=gpurun_out/${OUT:-rep}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: $2 exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_group.py tests/test_gpu_multiprocess.py -m gpu -v \
  --timeout 300 --timeout-method thread -x -k "${K:-replicat}" > $O/pytest_gpu.txt 2>&1
rc=$?; tail -4 $O/pytest_gpu.txt; ok $rc pytest
if [ "${REH:-1}" = 1 ]; then  # gloo rehearsals of the N > 1 bench line on one GPU: the planner's plan and model
  for G in 2 4; do
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $G --master-addr 127.0.0.1 \
      --master-port $((29515 + G)) bench.py --gpus $G --steps 2 --warmup 1 --backend gloo \
      > $O/bench_rehearsal_gloo_G$G.json 2> $O/rehearsal_G$G.err; ok $? "rehearsal G=$G"
    grep '^{' $O/bench_rehearsal_gloo_G$G.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($G, d['value'], d.get('verified'), json.dumps(d['roofline']['plan_model']))"
  done
fi
