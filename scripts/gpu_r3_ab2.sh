#!/bin/bash
# Round 3: fc dgrad tiles A/B (DQN_TILES=6:2: 16 x 16 blocks, split-K 4 vs the default 16 x 32,
# split-K 2), alternating on one box, flagship and Rainbow.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3ab2}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
for rep in 1 2 3; do
  for t in base 6:2; do
    if [ "$t" = base ]; then unset DQN_TILES; else export DQN_TILES=$t; fi
    timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/dqn_${t/:/_}_$rep.log 2>&1; ok $? dqn_$t
    python3 -c "import json; d=json.loads(open('$OUT/dqn_${t/:/_}_$rep.log').read().strip().splitlines()[-1]); print('dqn $t', $rep, d['value'])"
  done
done
for t in base 6:2; do
  if [ "$t" = base ]; then unset DQN_TILES; else export DQN_TILES=$t; fi
  for v in dd rainbow; do
    timeout -k 10 300 python bench.py --variant $v --steps 1000 --warmup 100 > $OUT/${v}_${t/:/_}.log 2>&1; ok $? ${v}_$t
    python3 -c "import json; d=json.loads(open('$OUT/${v}_${t/:/_}.log').read().strip().splitlines()[-1]); print('$v $t', d['value'])"
  done
done
echo ALL_DONE
