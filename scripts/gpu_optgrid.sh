#!/bin/bash
# Optimizer+pack grid sweep (DQN_OPT_GRID: blocks of the update launch; <= 256 grid-strides over
# the work items with a flat ticket, larger = one block per item up to the cap)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/optgrid
for V in dqn rainbow; do
  for G in 256 512 1024 2048; do
    DQN_OPT_GRID=$G timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --variant $V --replay 200000 \
        > gpurun_out/optgrid/${V}_$G.log 2>&1 || { echo "bench $V $G failed"; tail -5 gpurun_out/optgrid/${V}_$G.log; exit 1; }
    echo "$V grid $G: $(tail -1 gpurun_out/optgrid/${V}_$G.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
