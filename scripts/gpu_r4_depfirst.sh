#!/bin/bash
# A/B: the fused launch's range-dependent update jobs placed right after the weight-gradient tiles
# (DQN_DEP_FIRST=1) or at the end of the grid (0), interleaved; then the GPU tests with 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4dep
mkdir -p $OUT
for rep in 1 2; do
  for v in dqn rainbow; do
    for x in 0 1; do
      DQN_DEP_FIRST=$x timeout -k 10 300 python bench.py --variant $v --steps 2000 --warmup 200 > $OUT/${v}_d${x}_$rep.log 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$OUT/${v}_d${x}_$rep.log').read().strip().splitlines()[-1]); print('$v dep_first=$x rep=$rep', d['value'], d['ms_per_step'])"
    done
  done
done
DQN_DEP_FIRST=1 DQN_OPT_PROF=1 timeout -k 10 200 python scripts/probe_split.py --iters 50 --real-only --dueling --double_dqn --distributional --noisy --prioritized_replay --optimizer=adam --lr=0.0000625 > $OUT/rb_split.json 2> $OUT/rb_split.err || exit $?
DQN_DEP_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_fused_fc_gpu.py tests/test_executor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; echo pytest rc=$?; tail -3 $OUT/pytest.log
