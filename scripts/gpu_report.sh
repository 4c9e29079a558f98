#!/bin/bash
# One GPU call producing the committed evidence: variant benches, rocprofv3 kernel stats
# of the flagship and Rainbow steps, and the PMC counter passes. Every GPU step has its
# own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/report
mkdir -p $OUT
run_bench() {   # name, args
  timeout -k 10 300 python bench.py $2 > $OUT/bench_$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -5 $OUT/bench_$1.log; exit 1; }
  tail -1 $OUT/bench_$1.log >> $OUT/benches.jsonl
  echo "$1: $(python -c "import json; d=json.loads(open('$OUT/bench_$1.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['dtype'])")"
}
rm -f $OUT/benches.jsonl
run_bench default ""
run_bench dqn "--steps 1000 --warmup 100"
run_bench dqn_fp16 "--steps 1000 --warmup 100 --dtype fp16"
run_bench dqn_sep "--steps 1000 --warmup 100 --fuse_acting 0"
run_bench cnn "--network cnn --steps 1000 --warmup 100"
run_bench dd "--variant dd --steps 1000 --warmup 100"
run_bench rainbow "--variant rainbow --steps 500 --warmup 50"
run_bench rainbow_fp16 "--variant rainbow --steps 500 --warmup 50 --dtype fp16"
run_bench torch_cnn "--network cnn --backend torch --steps 200 --warmup 20"
PROF_NAME=report/prof_dqn PROF_ARGS="--steps 100 --warmup 20" PROF_TOP=16 bash scripts/gpu_prof.sh > $OUT/kstats_dqn.txt || exit 1
PROF_NAME=report/prof_rainbow PROF_ARGS="--variant rainbow --steps 100 --warmup 20" PROF_TOP=24 bash scripts/gpu_prof.sh > $OUT/kstats_rainbow.txt || exit 1
BENCH_ARGS="--steps 60 --warmup 10" bash scripts/profile_counters.sh > $OUT/pmc.txt 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.txt; exit 1; }
echo REPORT_DONE
