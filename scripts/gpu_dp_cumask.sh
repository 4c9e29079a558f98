#!/bin/bash
# 2 ranks on one GPU with disjoint CU masks (HSA_CU_MASK: each rank's queues on half of the
# CUs) -- a closer stand-in for two GPUs than sharing every CU: one-step vs 8-step graphs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/cumask
mkdir -p $OUT
export DQN_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 LOCAL_RANK=0
for G in 1 8; do
  for MASK in split shared; do
    P=$((29600 + G * 10 + ${#MASK}))
    if [ $MASK = split ]; then M0="0:0-127"; M1="0:128-255"; else M0=""; M1=""; fi
    HSA_CU_MASK=$M1 RANK=1 MASTER_PORT=$P timeout -k 10 150 python3 bench.py --gpus 2 --steps 1000 --warmup 50 \
        --replay 100000 --graph_steps $G > $OUT/r1_${G}_$MASK.log 2>&1 &
    PID=$!
    HSA_CU_MASK=$M0 RANK=0 MASTER_PORT=$P timeout -k 10 150 python3 bench.py --gpus 2 --steps 1000 --warmup 50 \
        --replay 100000 --graph_steps $G > $OUT/r0_${G}_$MASK.log 2>&1
    R0=$?
    wait $PID
    R1=$?
    [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || { echo "G=$G $MASK failed: $R0 $R1"; tail -5 $OUT/r0_${G}_$MASK.log; exit 1; }
    echo "G=$G cu=$MASK: $(grep '^{' $OUT/r0_${G}_$MASK.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['replicas_equal'])")"
  done
done
