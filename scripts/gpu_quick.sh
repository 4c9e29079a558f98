#!/bin/bash
# Quick GPU iteration: executor/kernel tests, flagship bench (200k and 1M replay), rocprof
# kernel stats of the flagship and the head phase probe. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for R in 200000 1000000; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --replay $R ${BENCH_EXTRA:-} > $OUT/bench_$R.log 2>&1 \
      || { echo "bench failed"; tail -5 $OUT/bench_$R.log; exit 1; }
  echo "replay $R: $(tail -1 $OUT/bench_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['env_frames_per_sec'])")"
done
PROF_NAME=quick/prof PROF_ARGS="--steps 100 --warmup 20 --replay 200000 ${BENCH_EXTRA:-}" PROF_TOP=14 bash scripts/gpu_prof.sh || exit 1
timeout -k 10 100 python scripts/probe_head.py 2>&1 | grep cycles
