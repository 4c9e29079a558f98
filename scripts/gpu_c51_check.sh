#!/bin/bash
# C51 head change check: GPU tests touching C51 / Rainbow, phase probe, Rainbow bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "c51 or rainbow or distributional or noisy" > gpurun_out/pytest_c51.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_c51.log; exit 1; }
tail -2 gpurun_out/pytest_c51.log
PYTHONPATH=. timeout -k 10 200 python scripts/probe_c51.py > gpurun_out/probe_c51.log 2>&1 || { echo "probe rc=$?"; exit 1; }
grep -v amdgpu gpurun_out/probe_c51.log | head -2
timeout -k 10 200 python bench.py --variant rainbow --steps 500 --warmup 50 > gpurun_out/bench_rb.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_rb.log; exit 1; }
tail -1 gpurun_out/bench_rb.log | cut -c1-260
