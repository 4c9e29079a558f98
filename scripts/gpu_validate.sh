#!/bin/bash
# Full GPU validation: every gpu-marked test, smoke(), the flagship bench and the Rainbow bench,
# then (VALIDATE_PROF=1) kernel stats of Rainbow with and without PER. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/validate
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for V in dqn rainbow; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --variant $V > $OUT/bench_$V.log 2>&1 \
      || { echo "bench $V failed"; tail -5 $OUT/bench_$V.log; exit 1; }
  echo "$V: $(tail -1 $OUT/bench_$V.log | cut -c1-400)"
done
if [ "${VALIDATE_PROF:-0}" = 1 ]; then
  PROF_NAME=validate/prof_rb PROF_ARGS="--steps 100 --warmup 20 --replay 200000 --variant rainbow" PROF_TOP=12 \
      bash scripts/gpu_prof.sh || exit 1
  PROF_NAME=validate/prof_rb_noper PROF_ARGS="--steps 100 --warmup 20 --replay 200000 --variant dd" \
      PROF_EXTRA="--distributional --noisy --optimizer=adam --lr=0.0000625" PROF_TOP=12 bash scripts/gpu_prof.sh || exit 1
fi
