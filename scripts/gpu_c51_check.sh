#!/bin/bash
# C51 head change check: GPU tests touching C51 / Rainbow, Rainbow bench, rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "c51 or rainbow or RAINBOW or distributional or noisy" > gpurun_out/pytest_c51.log 2>&1 \
    || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_c51.log; exit 1; }
tail -2 gpurun_out/pytest_c51.log
timeout -k 10 200 python bench.py --variant rainbow --steps 1000 --warmup 100 > gpurun_out/bench_rb.log 2>&1 \
    || { echo "bench rc=$?"; tail -5 gpurun_out/bench_rb.log; exit 1; }
tail -1 gpurun_out/bench_rb.log | cut -c1-260
PROF_NAME=prof_rb PROF_ARGS="--variant rainbow --steps 100 --warmup 20 --replay 200000" PROF_TOP=16 bash scripts/gpu_prof.sh
