#!/bin/bash
# Round 3: Ape-X native ingest tests and the multi-rank DP / async-PS rehearsals (world 2/4/8
# ranks on one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3multi}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_apex_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_apex.log 2>&1; ok $? pytest_apex
tail -8 $OUT/pytest_apex.log
timeout -k 10 700 python -u -m pytest tests/test_dist_gpu.py -v --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1; ok $? pytest_dist
tail -30 $OUT/pytest_dist.log
echo ALL_DONE
