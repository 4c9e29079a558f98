#!/bin/bash
# How much of the grouped weight-gradient launch is its fp32 atomics? Kernel traces of the
# flagship with the default chunking, 256-row conv chunks, and (numerically wrong, timing only)
# plain stores instead of atomics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out/wgp
cd /tmp && export TMPDIR=/tmp
for cfg in default mc256 noatomic; do
  case $cfg in
    default) E="";;
    mc256) E="DQN_WGRAD_MC=256";;
    noatomic) E="DQN_WGRAD_PROBE_NOATOMIC=1";;
  esac
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/wgp/$cfg -o run --output-format csv -- \
      python3 $REPO/bench.py --steps 100 --warmup 20 --replay 200000 > $REPO/gpurun_out/wgp/$cfg.log 2>&1 || { echo "$cfg failed"; exit 1; }
  echo "$cfg: $(python3 $REPO/scripts/kstats.py $REPO/gpurun_out/wgp/$cfg/run_kernel_trace.csv 3 | grep wgrad_group)"
done
