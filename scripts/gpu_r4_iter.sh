#!/bin/bash
# Round 4 build -> measure iteration: selected GPU tests, flagship A/B benches, kernel trace.
# Each GPU step has its own time limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R4_OUT:-r4iter}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
  grep -E "passed|failed|PASSED|FAILED|Error" $OUT/pytest.log | tail -30
fi
for v in ${BENCHES:-"dqn:--fuse_wgrad_update=1" "dqn:--fuse_wgrad_update=0"}; do
  IFS=: read var ex <<< "$v"
  tag=$(echo "$var$ex" | tr -c 'a-zA-Z0-9_=\n' '_')
  timeout -k 10 300 python bench.py --variant $var --steps ${NSTEPS:-2000} --warmup 100 --extra="$ex" > $OUT/bench_$tag.log 2>&1; ok $? bench_$tag
  tail -1 $OUT/bench_$tag.log | cut -c1-250
done
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof -o run --output-format csv -- \
      python3 $REPO/bench.py --variant ${PROF} --steps 200 --warmup 20 --replay 200000 > $REPO/$OUT/prof.log 2>&1; ok $? rocprof
  cd $REPO
  python scripts/kstats.py $OUT/prof/run_kernel_trace.csv 14 > $OUT/kstats.md; cat $OUT/kstats.md
fi
echo ALL_DONE
