#!/bin/bash
# Round 5 end: two- and four-rank gloo rehearsals of bench.py on one GPU (ranks share the device;
# not a measurement: the line says so) with the placement calibration in the sharded engines.
set -u
O=gpurun_out/${1:-r05_reh}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo > $O/bench_rehearsal_gloo_G2.json 2> $O/rehearsal_G2.err; ok $?
cat $O/bench_rehearsal_gloo_G2.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 2 --warmup 1 --backend gloo > $O/bench_rehearsal_gloo_G4.json 2> $O/rehearsal_G4.err; ok $?
cat $O/bench_rehearsal_gloo_G4.json
echo done
