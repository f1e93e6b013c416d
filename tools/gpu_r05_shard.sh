#!/bin/bash
# Round 5: the sharded paths after the link-aware planner and the whole-round N > 1 roofline:
# the sharded / group / multiprocess GPU tests, a two-rank gloo rehearsal of bench.py (its line
# carries round_wall_us and link_bytes_per_round), and tools/shard_probe.py at 2 x 2^26 with the
# link-aware plan and with the fixed thresholds (link_gbps=0).  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_shard}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_sharded.py tests/test_gpu_multiprocess.py -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_shard.txt 2>&1; ok $?
tail -1 $O/pytest_shard.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo > $O/bench_rehearsal_gloo_G2.json 2> $O/bench_rehearsal.err; ok $?
cat $O/bench_rehearsal_gloo_G2.json
timeout -k 10 300 python tools/shard_probe.py 2 26 > $O/probe_G2.txt 2>&1; ok $?
tail -3 $O/probe_G2.txt
timeout -k 10 300 python tools/shard_probe.py 2 26 link_gbps=0 > $O/probe_G2_fixed.txt 2>&1; ok $?
tail -3 $O/probe_G2_fixed.txt
echo done
