#!/bin/bash
# Round-4 end-of-session check: benches (flagship, Rainbow, dd), smoke(), the whole GPU suite in one
# process, a flagship kernel trace. Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R4_OUT:-r4final}
mkdir -p $OUT
for v in dqn rainbow dqn rainbow dd; do
  timeout -k 10 300 python bench.py --variant $v --steps 2000 --warmup 200 > $OUT/bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$OUT/bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['graph_steps'])" | tee -a $OUT/bench_summary.txt
done
[ -n "${SKIP_SUITE:-}" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof -o run --output-format csv -- \
    python3 $REPO/bench.py --steps 400 --warmup 50 --replay 200000 > $REPO/$OUT/prof.log 2>&1 || exit $?
cd $REPO
python scripts/kstats.py $OUT/prof/run_kernel_trace.csv 10 > $OUT/kstats.md; cat $OUT/kstats.md
echo ALL_DONE
