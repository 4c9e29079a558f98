#!/bin/bash
# Round 3 probes: optimizer store policy (DQN_OPT_NT), the price of the conv wgrad fp32 atomics
# (DQN_WGRAD_PROBE_NOATOMIC: timing only), then the multi-rank DP rehearsals at world 2/4/8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3probe}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
for nt in 0 1; do
  DQN_OPT_NT=$nt timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim_nt$nt.log 2>&1; ok $? probe_nt$nt
  tail -1 $OUT/probe_optim_nt$nt.log
  DQN_OPT_NT=$nt timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench_nt$nt.log 2>&1; ok $? bench_nt$nt
  tail -1 $OUT/bench_nt$nt.log | cut -c1-300
done
DQN_WGRAD_PROBE_NOATOMIC=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench_noatomic.log 2>&1; ok $? bench_noatomic
tail -1 $OUT/bench_noatomic.log | cut -c1-300
timeout -k 10 600 python -u -m pytest tests/test_fused_fc_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_fc.log 2>&1; ok $? pytest_fc
tail -2 $OUT/pytest_fc.log
timeout -k 10 400 python -u -m pytest tests/test_apex_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_apex.log 2>&1; ok $? pytest_apex
tail -8 $OUT/pytest_apex.log
timeout -k 10 1000 python -u -m pytest tests/test_dist_gpu.py -v --timeout 400 --timeout-method thread > $OUT/pytest_dist.log 2>&1; ok $? pytest_dist
tail -25 $OUT/pytest_dist.log
echo ALL_DONE
