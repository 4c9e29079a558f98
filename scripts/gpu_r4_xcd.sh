#!/bin/bash
# A/B of the XCD-aware block order of the dense launches (DQN_XCD_ORDER=0 / 1), interleaved,
# then the fused-fc / executor GPU tests with it on. Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4xcd
mkdir -p $OUT
for rep in 1 2; do
  for v in dqn rainbow dd; do
    for x in 0 1; do
      DQN_XCD_ORDER=$x timeout -k 10 300 python bench.py --variant $v --steps 2000 --warmup 200 > $OUT/${v}_x${x}_$rep.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$OUT/${v}_x${x}_$rep.log').read().strip().splitlines()[-1]); print('$v xcd=$x rep=$rep', d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_fused_fc_gpu.py tests/test_executor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; echo pytest rc=$?; tail -3 $OUT/pytest.log
