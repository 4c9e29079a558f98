#!/bin/bash
# Round 3 Ape-X at 256 actors on the box's 16-CPU CFS quota: pinned actors (default) vs paced,
# unpinned actors (--apex_pace) vs no CPU reservation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3apexpace}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
i=0
for x in "--apex_pace=0.9" "--apex_pace=0.7" "--apex_reserve_cpus=0" ""; do
  i=$((i + 1))
  timeout -k 20 200 python scripts/bench_apex.py --actors 256 --seconds ${APEX_SECS:-45} --extra="--apex_graph_steps=16 $x" > $OUT/apex256_$i.log 2>&1; ok $? apex256_$i
  echo "[$x] $(tail -1 $OUT/apex256_$i.log | cut -c1-330)"
done
echo ALL_DONE
