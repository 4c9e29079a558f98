#!/bin/bash
# Round 3: trunk tile permutation + wgrad staging swizzle -- kernel numerics tests, bench, the
# LDS-conflict PMC pass over the flagship bench, then Ape-X 256 actors within the CFS quota.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R3_OUT:-r3lds}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_fused_fc_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench.log 2>&1; ok $? bench
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace -d $REPO/$OUT/pmc_lds/pass1 -o pass1 --output-format csv -- \
    python3 $REPO/bench.py --steps 60 --warmup 10 > $REPO/$OUT/pmc_lds.log 2>&1; ok $? pmc_lds
cd $REPO
python3 scripts/pmc_summary.py $OUT/pmc_lds > $OUT/pmc_lds.md; head -8 $OUT/pmc_lds.md | cut -c1-200
timeout -k 20 200 python scripts/bench_apex.py --actors 256 --seconds 45 --extra="--apex_graph_steps=16" > $OUT/apex256.log 2>&1; ok $? apex256
tail -1 $OUT/apex256.log | cut -c1-600
echo ALL_DONE
