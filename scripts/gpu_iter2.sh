#!/bin/bash
# Head iteration: executor / kernel GPU tests, head phase probes (scalar + C51), flagship and
# Rainbow benches. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/iter
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 100 python scripts/probe_head.py > $OUT/probe_scalar.log 2>&1 || { echo "probe failed"; tail -5 $OUT/probe_scalar.log; exit 1; }
grep cycles $OUT/probe_scalar.log
timeout -k 10 100 python scripts/probe_head.py --dueling --double_dqn --distributional --noisy --optimizer=adam \
    > $OUT/probe_c51.log 2>&1 || { echo "probe failed"; tail -5 $OUT/probe_c51.log; exit 1; }
grep cycles $OUT/probe_c51.log
for V in dqn rainbow; do
  timeout -k 10 150 python bench.py --variant $V --steps 1000 --warmup 100 > $OUT/bench_$V.log 2>&1 \
      || { echo "bench failed"; tail -5 $OUT/bench_$V.log; exit 1; }
  echo "$V: $(tail -1 $OUT/bench_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['env_frames_per_sec'])")"
done
