#!/bin/bash
# Round 4: the multi-rank GPU evidence on one MI355X -- the DP / xgmi / async-PS / Ape-X rehearsal
# tests and the async-PS throughput bench (native server thread). Each GPU step has its own time
# limit; a failing step (beyond test failures) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R4_OUT:-r4dist}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
T=${TESTS:-"tests/test_dist_gpu.py tests/test_apex_dp.py"}
timeout -k 10 900 python -u -m pytest $T -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
grep -E "passed|failed|PASSED|FAILED|XFAIL|XPASS|Error" $OUT/pytest.log | tail -60
if [ -n "${PS_STEPS:-6000}" ]; then
  timeout -k 10 400 python scripts/bench_async_ps.py --transport xgmi --workers 2 --steps ${PS_STEPS:-6000} \
      > $OUT/async_ps.json 2> $OUT/async_ps.err; ok $? async_ps
  cat $OUT/async_ps.json
fi
echo ALL_DONE
