#!/bin/bash
# Deterministic conv wgrad: partial-count sweep (DQN_DET_GROUPS) and kernel traces det on / off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3det}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
for g in ${DET_GROUPS:-4 8 13 50}; do
  DQN_DET_GROUPS=$g timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench_g$g.log 2>&1; ok $? bench_g$g
  echo "groups=$g $(tail -1 $OUT/bench_g$g.log | cut -c150-260)"
done
for det in 1 0; do
  PROF_NAME=${R3_OUT:-r3det}/prof_det$det PROF_ARGS="--steps 200 --warmup 20 --replay 200000" PROF_EXTRA="--det_wgrad=$det" PROF_TOP=12 timeout -k 10 300 bash scripts/gpu_prof.sh; ok $? prof_det$det
done
echo ALL_DONE
