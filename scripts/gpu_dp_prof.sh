#!/bin/bash
# Kernel trace of rank 0 of a 2-rank DP bench on one GPU (rank 1 runs unprofiled beside it):
# the low-rank exchange's kernels (xgmi_allgather, wgrad_multi, multi-range xgmi_allreduce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out/dpprof
V=${DP_VARIANT:-dqn}
export DQN_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 WORLD_SIZE=2 LOCAL_RANK=0
cd /tmp && export TMPDIR=/tmp
RANK=1 timeout -k 10 200 python3 $REPO/bench.py --gpus 2 --steps 300 --warmup 30 --replay 100000 --variant $V \
    > $REPO/gpurun_out/dpprof/rank1_$V.log 2>&1 &
P1=$!
RANK=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/dpprof/$V -o run --output-format csv -- \
    python3 $REPO/bench.py --gpus 2 --steps 300 --warmup 30 --replay 100000 --variant $V \
    > $REPO/gpurun_out/dpprof/rank0_$V.log 2>&1
R0=$?
wait $P1
R1=$?
[ $R0 -eq 0 ] && [ $R1 -eq 0 ] || { echo "ranks failed: $R0 $R1"; tail -5 $REPO/gpurun_out/dpprof/rank0_$V.log; exit 1; }
grep '^{' $REPO/gpurun_out/dpprof/rank0_$V.log | cut -c1-200
python3 $REPO/scripts/kstats.py $REPO/gpurun_out/dpprof/$V/run_kernel_trace.csv 16
