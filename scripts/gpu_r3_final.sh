#!/bin/bash
# Round 3 end state: the whole GPU suite, smoke, the variant benches and the flagship PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R3_OUT:-r3final}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $? pytest
  tail -4 $OUT/pytest.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke
tail -1 $OUT/smoke.log
for v in ${BENCH_VARIANTS:-"dqn:bf16:2000" "dd:bf16:1000" "rainbow:bf16:1000" "rainbow:fp16:1000" "dqn:fp32:1000"}; do
  IFS=: read var dt n <<< "$v"
  timeout -k 10 300 python bench.py --variant $var --dtype $dt --steps $n --warmup 100 > $OUT/bench_${var}_$dt.log 2>&1; ok $? bench_${var}_$dt
  tail -1 $OUT/bench_${var}_$dt.log | cut -c1-300
done
if [ "${PMC:-1}" == "1" ]; then
  PMC_OUT=r3final/pmc BENCH_ARGS="--steps 60 --warmup 20 --replay 200000 --graph_steps 1" timeout -k 10 900 bash scripts/profile_counters.sh > $OUT/pmc.log 2>&1; ok $? pmc
  tail -14 $OUT/pmc.log
fi
echo ALL_DONE
