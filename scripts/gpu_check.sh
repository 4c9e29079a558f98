#!/bin/bash
# One GPU-box session: kernel tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok_or_stop() {  # rc 0 = pass, 1 = test failures (keep going); anything else = stop
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what (rc=$rc)"; exit "$rc"; fi
}
STEPS=${STEPS:-300}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  ok_or_stop $? pytest_gpu
  tail -5 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
ok_or_stop $? smoke
tail -2 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps $STEPS --warmup 30 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
ok_or_stop $? bench
tail -3 $OUT/bench.log
if [ "${PROFILE:-1}" == "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 100 --warmup 20 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  ok_or_stop $? rocprof
  find $OUT/prof -name "*kernel_stats.csv" | head -3
fi
echo ALL_DONE
