#!/bin/bash
# Round 3: grouped conv wgrad with 256-row M-chunks (DQN_WGRAD_MC=256: half the blocks and the fp32
# atomic bytes) vs the default 128-row chunks, alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3knobs}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
for rep in 1 2 3; do
  for mc in 128 256; do
    DQN_WGRAD_MC=$mc timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/mc${mc}_$rep.log 2>&1; ok $? mc${mc}_$rep
    python3 -c "import json; d=json.loads(open('$OUT/mc${mc}_$rep.log').read().strip().splitlines()[-1]); print('mc$mc', $rep, d['value'], d['ms_per_step'])"
  done
done
for mc in 128 256; do
  DQN_WGRAD_MC=$mc timeout -k 10 300 python bench.py --variant rainbow --steps 1000 --warmup 100 > $OUT/rb_mc$mc.log 2>&1; ok $? rb_mc$mc
  python3 -c "import json; d=json.loads(open('$OUT/rb_mc$mc.log').read().strip().splitlines()[-1]); print('rainbow mc$mc', d['value'], d['ms_per_step'])"
done
echo ALL_DONE
