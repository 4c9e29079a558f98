#!/bin/bash
# One build -> measure iteration on the GPU box:
#   STEP_TESTS  pytest files (default: the executor + kernel GPU tests; none: skip), STEP_K: a -k expression
#   STEP_BENCH  space-separated bench variants (dqn dd rainbow), 2000 steps each
#   STEP_PROF   one bench variant to kernel-trace (rocprofv3 --kernel-trace --stats), empty: none
# Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/step
mkdir -p $OUT
if [ "${STEP_TESTS:-x}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest ${STEP_TESTS:-tests/test_executor_gpu.py tests/test_kernels_gpu.py} -m gpu -x -q \
      ${STEP_K:+-k "$STEP_K"} \
      --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for V in ${STEP_BENCH:-dqn rainbow}; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --variant $V ${STEP_BENCH_ARGS:-} > $OUT/bench_$V.log 2>&1 \
      || { echo "bench $V failed"; tail -5 $OUT/bench_$V.log; exit 1; }
  echo "$V: $(tail -1 $OUT/bench_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['env_frames_per_sec'])")"
done
if [ -n "${STEP_PROF:-}" ]; then
  PROF_NAME=step/prof_$STEP_PROF PROF_ARGS="--steps 100 --warmup 20 --replay 200000 --variant $STEP_PROF" PROF_TOP=12 \
      bash scripts/gpu_prof.sh || exit 1
fi
