#!/bin/bash
# Round GPU session: full GPU tests, flagship bench, variant benches (Double+Dueling,
# Rainbow, reference cnn), Ape-X bench, kernel-stats profile. Each GPU step has its
# own time limit; a crash / abort / timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
stop_on() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; stop_on $? pytest_gpu
  tail -3 $OUT/pytest_gpu.log
fi
run_bench() {   # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$name.log 2>&1; stop_on $? "bench $name"
  tail -1 $OUT/bench_$name.log
}
run_bench nature --steps 400 --warmup 40
run_bench dd --steps 400 --warmup 40 --variant dd
run_bench rainbow --steps 300 --warmup 30 --variant rainbow
run_bench rainbow16 --steps 300 --warmup 30 --variant rainbow --dtype fp16
run_bench cnn --steps 300 --warmup 30 --network cnn
if [ "${APEX:-1}" == "1" ]; then
  timeout -k 10 200 python scripts/bench_apex.py --actors 16 --seconds 45 > $OUT/apex.log 2>&1; stop_on $? apex
  tail -1 $OUT/apex.log
fi
if [ "${PROFILE:-1}" == "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
  stop_on $? rocprof
  cd $GRAFT_REPO_ROOT
fi
if [ "${PMC:-0}" == "1" ]; then
  bash scripts/profile_counters.sh > $OUT/pmc_run.log 2>&1; stop_on $? pmc
  tail -25 $OUT/pmc_run.log
fi
echo ALL_DONE
