#!/bin/bash
# Round 4 start state of the tree: the whole GPU test suite, the flagship + variant benches and a kernel
# trace of the flagship step. Each GPU step has its own time limit; a crash / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R4_OUT:-r4base}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
  tail -3 $OUT/pytest.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke
tail -1 $OUT/smoke.log
for v in ${BENCH_VARIANTS:-"dqn:bf16:2000" "rainbow:bf16:1000"}; do
  IFS=: read var dt n <<< "$v"
  if [ "$var" = cnn ]; then a="--network cnn"; else a="--variant $var"; fi
  timeout -k 10 300 python bench.py $a --dtype $dt --steps $n --warmup 100 > $OUT/bench_${var}_$dt.log 2>&1; ok $? bench_${var}_$dt
  tail -1 $OUT/bench_${var}_$dt.log | cut -c1-330
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof -o run --output-format csv -- \
    python3 $REPO/bench.py --steps 200 --warmup 20 --replay 200000 > $REPO/$OUT/prof.log 2>&1; ok $? rocprof
cd $REPO
python scripts/kstats.py $OUT/prof/run_kernel_trace.csv 16 > $OUT/kstats.md; cat $OUT/kstats.md
echo ALL_DONE
