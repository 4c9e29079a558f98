#!/bin/bash
# A/B: fc dgrad tiles 16 x 32 split-K 2 (0) vs 16 x 16 split-K 4 (DQN_FCDG16=1), interleaved; tests with 1.
# (DQN_FCDG16 was a temporary switch for this A/B; 16 x 16 split-K 4 is now the only fc dgrad tiling)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4fcdg
mkdir -p $OUT
for rep in 1 2; do
  for v in dqn rainbow dd; do
    for x in 0 1; do
      DQN_FCDG16=$x timeout -k 10 300 python bench.py --variant $v --steps 2000 --warmup 200 > $OUT/${v}_t${x}_$rep.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$OUT/${v}_t${x}_$rep.log').read().strip().splitlines()[-1]); print('$v fcdg16=$x rep=$rep', d['value'], d['ms_per_step'])"
    done
  done
done
DQN_FCDG16=1 timeout -k 10 600 python -u -m pytest tests/test_fused_fc_gpu.py tests/test_executor_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; echo pytest rc=$?; tail -2 $OUT/pytest.log
