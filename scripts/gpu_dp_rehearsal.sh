#!/bin/bash
# Multi-rank rehearsal on ONE GPU: DP learner tests (2 ranks over gloo on cuda:0) and the
# torchrun bench path with 2 ranks. Each GPU step has its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread \
    > $OUT/pytest_dist_gpu.log 2>&1 || { echo "dist tests rc=$?"; tail -40 $OUT/pytest_dist_gpu.log; exit 1; }
tail -3 $OUT/pytest_dist_gpu.log
DQN_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 \
    > $OUT/bench_gloo2.log 2>&1 || { echo "bench2 rc=$?"; tail -30 $OUT/bench_gloo2.log; exit 1; }
tail -1 $OUT/bench_gloo2.log
echo DP_DONE
