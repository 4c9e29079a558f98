#!/bin/bash
# Round 3: grouped conv wgrad with several M-chunks per block (DQN_WGRAD_MLOOP, fp32 atomics once
# per chunk group): oracle tests with the setting, then a bench sweep; plus HBM reference rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3wgrad}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 120 python scripts/probe_hbm.py > $OUT/probe_hbm.log 2>&1; ok $? probe_hbm
tail -1 $OUT/probe_hbm.log
DQN_WGRAD_MLOOP=4,2,2 timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_fused_fc_gpu.py -x -q \
    --timeout 200 --timeout-method thread > $OUT/pytest_mloop.log 2>&1; ok $? pytest_mloop
tail -2 $OUT/pytest_mloop.log
for m in ${MLOOPS:-"1,1,1" "2,1,1" "2,2,2" "4,2,2" "4,1,1" "8,3,2"}; do
  DQN_WGRAD_MLOOP=$m timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench_$m.log 2>&1; ok $? bench_$m
  echo "$m $(tail -1 $OUT/bench_$m.log | cut -c1-200)"
done
echo ALL_DONE
