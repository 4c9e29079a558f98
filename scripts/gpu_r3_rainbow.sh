#!/bin/bash
# Round 3 Rainbow: bench bf16 / fp16 (optimizer store policy DQN_OPT_NT 0/1), kernel stats and
# the PMC passes (HBM bytes) of the Rainbow step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3rb}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
for cfg in "bf16:0" "bf16:1" "fp16:0"; do
  dt=${cfg%%:*}; nt=${cfg#*:}
  DQN_OPT_NT=$nt timeout -k 10 300 python bench.py --variant rainbow --dtype $dt --steps 1000 --warmup 100 > $OUT/bench_${dt}_nt$nt.log 2>&1; ok $? bench_${dt}_nt$nt
  tail -1 $OUT/bench_${dt}_nt$nt.log | cut -c1-330
done
PROF_NAME=${R3_OUT:-r3rb}/prof PROF_ARGS="--variant rainbow --steps 100 --warmup 20 --replay 200000" PROF_TOP=16 timeout -k 10 300 bash scripts/gpu_prof.sh; ok $? prof
if [ -n "${PMC:-}" ]; then
  BENCH_ARGS="--variant rainbow --steps 60 --warmup 10 --replay 200000" PMC_OUT=${R3_OUT:-r3rb}/pmc timeout -k 10 900 bash scripts/profile_counters.sh | tail -25; ok $? pmc
fi
echo ALL_DONE
