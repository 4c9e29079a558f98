#!/bin/bash
# Iteration run on one GPU: GPU tests, A/B benches given as "NAME:ENV:ARGS" triples in
# $BENCHES (';'-separated), optional rocprofv3 kernel stats of the flagship bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
if [ "${TESTS:-1}" == "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
IFS=';' read -ra BS <<< "${BENCHES:-}"
for b in "${BS[@]}"; do
  name=${b%%:*}; rest=${b#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 300 python bench.py $args > $OUT/bench_$name.log 2>&1 \
      || { echo "bench $name rc=$?"; tail -20 $OUT/bench_$name.log; exit 1; }
  echo "$name: $(python -c "import json,sys; d=json.loads(open('$OUT/bench_$name.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
if [ "${PROFILE:-0}" == "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 \
      || { echo "rocprof rc=$?"; exit 1; }
  cd $GRAFT_REPO_ROOT
  python scripts/kstats.py $OUT/prof/run_kernel_trace.csv 14
fi
echo ITER_DONE
