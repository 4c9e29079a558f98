#!/bin/bash
# Round 3: why the 8-rank xgmi self-test fails with 8 ranks on ONE GPU -- per-call timing, exact-sum
# and timeout flags per rank (XGMI_CFGS = "hwqueues:world:selftest:wire ...").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3x8}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for cfg in ${XGMI_CFGS:-4:4:0:fp32 4:8:0:fp32 1:8:0:fp32 2:8:0:fp32}; do
  IFS=: read hq w st wire <<< "$cfg"
  name=w${w}_q${hq}_st${st}_$wire
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 150 python scripts/probe_xgmi_world.py --world $w --calls 3 --timeout 110 --selftest $st --wire $wire > $OUT/$name.json 2> $OUT/$name.err; ok $? $name
  tail -1 $OUT/$name.json | cut -c1-1500
done
echo ALL_DONE
