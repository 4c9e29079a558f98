#!/bin/bash
# Round 3 lean validation: the GEMM / optimizer / DP GPU tests, smoke and one flagship bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3lean}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests/test_executor_gpu.py tests/test_fused_fc_gpu.py tests/test_dist_gpu.py \
    tests/test_kernels_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
tail -2 $OUT/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench.log 2>&1; ok $? bench
tail -1 $OUT/bench.log | cut -c1-300
echo ALL_DONE
