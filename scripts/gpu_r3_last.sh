#!/bin/bash
# Round 3: Ape-X GPU tests + 14 / 256 actors with the paced default, then the kernarg / graph-length A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3last}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_apex_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_apex.log 2>&1; ok $? pytest_apex
tail -2 $OUT/pytest_apex.log
for n in 14 256; do
  timeout -k 20 200 python scripts/bench_apex.py --actors $n --seconds 45 --extra="--apex_graph_steps=16" > $OUT/apex$n.log 2>&1; ok $? apex$n
  tail -1 $OUT/apex$n.log | cut -c1-330
done
R3_OUT=r3last/ab bash scripts/gpu_r3_ab.sh
