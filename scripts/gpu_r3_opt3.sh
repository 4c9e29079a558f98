#!/bin/bash
# Round 3: optimizer end-of-launch bookkeeping by block 0 polling no-return arrival counters (no
# returning ticket per block). Full GPU suite, the optimizer alone with phase stamps, flagship +
# Rainbow benches and kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R3_OUT:-r3opt3}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
  tail -3 $OUT/pytest.log
fi
DQN_OPT_PROF=1 timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim.log 2>&1; ok $? probe_optim
tail -1 $OUT/probe_optim.log
for v in ${BENCH_VARIANTS:-"dqn:bf16:2000" "rainbow:bf16:1000"}; do
  IFS=: read var dt n <<< "$v"
  timeout -k 10 300 python bench.py --variant $var --dtype $dt --steps $n --warmup 100 > $OUT/bench_${var}_$dt.log 2>&1; ok $? bench_${var}_$dt
  tail -1 $OUT/bench_${var}_$dt.log | cut -c1-300
done
DQN_OPT_PROF=1 timeout -k 10 300 python bench.py --variant rainbow --steps 200 --warmup 20 > $OUT/bench_rb_prof.log 2>&1; ok $? bench_rb_prof
tail -1 $OUT/bench_rb_prof.log
cd /tmp && export TMPDIR=/tmp
for var in dqn rainbow; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof_$var -o run --output-format csv -- \
      python3 $REPO/bench.py --variant $var --steps 200 --warmup 20 --replay 200000 > $REPO/$OUT/prof_$var.log 2>&1; ok $? rocprof_$var
  python3 $REPO/scripts/kstats.py $REPO/$OUT/prof_$var/run_kernel_trace.csv 10 > $REPO/$OUT/kstats_$var.md; cat $REPO/$OUT/kstats_$var.md
done
echo ALL_DONE
