#!/bin/bash
# 2 ranks on one GPU (gloo process group, xgmi transport over same-device IPC): the DP step
# with the low-rank fc exchange (default), the full all-reduce in stream order, and the full
# all-reduce on a forked graph branch (the previous schedule). Timings include both ranks'
# work on the one GPU; the comparison between schedules is what they are for.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dpvar
mkdir -p $OUT
run() {
  local name=$1; shift
  env DQN_DIST_BACKEND=gloo "$@" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr=127.0.0.1 --master-port=$((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 1000 --warmup 50 \
      --replay 100000 ${EXTRA:-} > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -20 $OUT/$name.log; exit 1; }
  echo "$name: $(grep '^{' $OUT/$name.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['allreduce'], c['lowrank_dense'], c['replicas_equal'])")"
}
run lowrank
EXTRA="--extra=--lowrank_dense=0" run full_serial
EXTRA="--extra=--lowrank_dense=0" run full_fork DQN_AR_FORK=1
