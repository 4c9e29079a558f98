#!/bin/bash
# Rainbow iteration: C51 / noisy GPU tests, C51 head probe, Rainbow bench, kernel stats and
# PMC passes (HBM bytes, LDS conflicts) of the Rainbow step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rb
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 100 python scripts/probe_head.py --dueling --double_dqn --distributional --noisy --optimizer=adam \
    > $OUT/probe_c51.log 2>&1 || { echo "probe failed"; tail -5 $OUT/probe_c51.log; exit 1; }
grep cycles $OUT/probe_c51.log
timeout -k 10 150 python bench.py --variant rainbow --steps 1000 --warmup 100 > $OUT/bench.log 2>&1 \
    || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
echo "rainbow: $(tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
PROF_NAME=rb/prof PROF_ARGS="--variant rainbow --steps 100 --warmup 20 --replay 200000" PROF_TOP=16 bash scripts/gpu_prof.sh || exit 1
if [ -n "${PMC:-}" ]; then
  BENCH_ARGS="--variant rainbow --steps 60 --warmup 10 --replay 200000" PMC_OUT=rb/pmc bash scripts/profile_counters.sh | tail -25
fi
