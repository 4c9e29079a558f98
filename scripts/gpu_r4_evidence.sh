#!/bin/bash
# Round 4 evidence: variant benches (flagship, dd, Rainbow, the fp32 build), kernel traces of the
# flagship and of the fp32 build, and the flagship's hardware-counter passes. Each GPU step has
# its own time limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R4_OUT:-r4ev}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in "dqn::2000" "dd::2000" "rainbow::1000" "dqn:--dtype=fp32:1000"; do
  IFS=: read var ex n <<< "$v"
  tag=$(echo "$var$ex" | tr -c 'a-zA-Z0-9_=\n' '_')
  timeout -k 10 300 python bench.py --variant $var --steps $n --warmup 100 --extra="$ex" > $OUT/bench_$tag.log 2>&1; ok $? bench_$tag
  tail -1 $OUT/bench_$tag.log | cut -c1-220
done
cd /tmp && export TMPDIR=/tmp
for v in "dqn:" "dqn:--dtype=fp32"; do
  IFS=: read var ex <<< "$v"
  tag=$(echo "$var$ex" | tr -c 'a-zA-Z0-9_=\n' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof_$tag -o run --output-format csv -- \
      python3 $REPO/bench.py --variant $var --steps 200 --warmup 20 --replay 200000 --extra="$ex" > $REPO/$OUT/prof_$tag.log 2>&1; ok $? rocprof_$tag
  python3 $REPO/scripts/kstats.py $REPO/$OUT/prof_$tag/run_kernel_trace.csv 14 > $REPO/$OUT/kstats_$tag.md; cat $REPO/$OUT/kstats_$tag.md
done
cd $REPO
PMC_OUT=r4ev/pmc BENCH_ARGS="--steps 60 --warmup 10" timeout -k 10 900 bash scripts/profile_counters.sh; ok $? pmc
echo ALL_DONE
