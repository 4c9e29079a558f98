#!/bin/bash
# Round 3: re-sweep the latency-bound layer GEMM tile variants (DQN_TILES="kind:variant") on the
# round-3 step (fc wgrad in the optimizer, 256-row wgrad chunks); base runs bracket the sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3tiles}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
i=0
for t in base 4:1 4:2 6:1 6:2 7:1 8:1 8:2 base; do
  i=$((i + 1))
  if [ "$t" = base ]; then unset DQN_TILES; else export DQN_TILES=$t; fi
  timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/t$i.log 2>&1; ok $? tiles_$t
  python3 -c "import json; d=json.loads(open('$OUT/t$i.log').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'])"
done
echo ALL_DONE
