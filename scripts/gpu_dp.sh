#!/bin/bash
# Multi-rank rehearsal on one GPU: xgmi kernel tests (all-reduce + gather channel), the DP learner
# matrix (low-rank fc exchange vs full all-reduce, replicas bit-equal), the 2-rank bench; then
# (DP_APEX=N) an N-actor Ape-X run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dp
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { echo "dist tests failed"; tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
DQN_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 200 --warmup 20 --replay 100000 \
    > $OUT/bench2.log 2>&1 || { echo "bench2 failed"; tail -30 $OUT/bench2.log; exit 1; }
grep '^{' $OUT/bench2.log | tail -1 | cut -c1-1500
if [ -n "${DP_APEX:-}" ]; then
  timeout -k 20 240 python scripts/bench_apex.py --actors $DP_APEX --seconds 60 > $OUT/apex.log 2>&1 \
      || { echo apex failed; tail -20 $OUT/apex.log; exit 1; }
  tail -1 $OUT/apex.log
fi
