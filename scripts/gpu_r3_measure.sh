#!/bin/bash
# Round 3 phase measurements: head / trunk s_memtime phases, the optimizer launch alone, a
# flagship bench and a kernel trace of the flagship and Rainbow steps. Each GPU step has its own
# time limit; a crash / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R3_OUT:-r3measure}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 120 python scripts/probe_head.py > $OUT/probe_head.log 2>&1; ok $? probe_head
tail -2 $OUT/probe_head.log
timeout -k 10 120 python scripts/probe_head.py --distributional --noisy --dueling --double_dqn --optimizer=adam \
    --prioritized_replay > $OUT/probe_head_c51.log 2>&1; ok $? probe_head_c51
tail -2 $OUT/probe_head_c51.log
timeout -k 10 120 python scripts/probe_trunk.py > $OUT/probe_trunk.log 2>&1; ok $? probe_trunk
tail -8 $OUT/probe_trunk.log
timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim.log 2>&1; ok $? probe_optim
tail -1 $OUT/probe_optim.log
for v in ${BENCH_VARIANTS:-"dqn:bf16:2000" "rainbow:bf16:1000"}; do
  IFS=: read var dt n <<< "$v"
  timeout -k 10 300 python bench.py --variant $var --dtype $dt --steps $n --warmup 100 > $OUT/bench_${var}_$dt.log 2>&1; ok $? bench_${var}_$dt
  tail -1 $OUT/bench_${var}_$dt.log | cut -c1-300
done
if [ "${PROFILE:-1}" == "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  for var in dqn rainbow; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof_$var -o run --output-format csv -- \
        python3 $REPO/bench.py --variant $var --steps 200 --warmup 20 --replay 200000 > $REPO/$OUT/prof_$var.log 2>&1; ok $? rocprof_$var
    python3 $REPO/scripts/kstats.py $REPO/$OUT/prof_$var/run_kernel_trace.csv 12 > $REPO/$OUT/kstats_$var.md; cat $REPO/$OUT/kstats_$var.md
  done
  cd $REPO
fi
echo ALL_DONE
