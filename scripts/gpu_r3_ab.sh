#!/bin/bash
# Round 3 A/B on one box (alternating runs): HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device
# memory) and 16-step graphs vs the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3ab}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
for rep in 1 2 3; do
  for cfg in base devk g16 devk_g16; do
    env=""; args=""
    case $cfg in devk) env="HIP_FORCE_DEV_KERNARG=1";; g16) args="--graph_steps 16";;
                 devk_g16) env="HIP_FORCE_DEV_KERNARG=1"; args="--graph_steps 16";; esac
    env $env timeout -k 10 300 python bench.py --steps 2000 --warmup 100 $args > $OUT/${cfg}_$rep.log 2>&1; ok $? ${cfg}_$rep
    python3 -c "import json,sys; d=json.loads(open('$OUT/${cfg}_$rep.log').read().strip().splitlines()[-1]); print('$cfg', $rep, d['value'], d['ms_per_step'], d['graph_steps'])"
  done
done
echo ALL_DONE
