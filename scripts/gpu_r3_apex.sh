#!/bin/bash
# Round 3 Ape-X: native-ingest tests, then 256 actors (BASELINE config 4 shape) with the native
# ingest thread + CPU reservation at apex_graph_steps 4 and 16, and the 14-actor row.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3apex}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_apex_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_apex.log 2>&1; ok $? pytest_apex
tail -6 $OUT/pytest_apex.log
for cfg in ${APEX_CFGS:-256:16 256:4 14:16}; do
  n=${cfg%%:*}; g=${cfg#*:}
  timeout -k 20 200 python scripts/bench_apex.py --actors $n --seconds ${APEX_SECS:-45} --extra="--apex_graph_steps=$g" > $OUT/apex${n}_g$g.log 2>&1; ok $? apex${n}_g$g
  tail -1 $OUT/apex${n}_g$g.log | cut -c1-420
done
echo ALL_DONE
