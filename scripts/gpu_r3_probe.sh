#!/bin/bash
# Round 3 probes: the fused-fc / deterministic-wgrad tests, then the optimizer store policy
# (DQN_OPT_NT), deterministic conv wgrad vs fp32 atomics (--det_wgrad), and the price of the
# atomics (DQN_WGRAD_PROBE_NOATOMIC: timing only, wrong gradients).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3probe}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_fused_fc_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_fc.log 2>&1; ok $? pytest_fc
tail -4 $OUT/pytest_fc.log
for nt in 0 1; do
  DQN_OPT_NT=$nt timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim_nt$nt.log 2>&1; ok $? probe_nt$nt
  tail -1 $OUT/probe_optim_nt$nt.log
done
for det in 1 0; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --extra="--det_wgrad=$det" > $OUT/bench_det$det.log 2>&1; ok $? bench_det$det
  tail -1 $OUT/bench_det$det.log | cut -c1-300
done
DQN_OPT_NT=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench_nt1.log 2>&1; ok $? bench_nt1
tail -1 $OUT/bench_nt1.log | cut -c1-300
DQN_WGRAD_PROBE_NOATOMIC=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --extra="--det_wgrad=0" > $OUT/bench_noatomic.log 2>&1; ok $? bench_noatomic
tail -1 $OUT/bench_noatomic.log | cut -c1-300
echo ALL_DONE
