#!/bin/bash
# Round 3: fused fc weight gradient in the optimizer launch -- new tests, the optimizer probe,
# A/B benches (fused vs --fuse_fc_wgrad=0), the CLI user paths and a kernel trace.
# Each GPU step has its own time limit; a crash / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R3_OUT:-r3fc}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest ${R3_TESTS:-tests/test_fused_fc_gpu.py tests/test_cli_paths_gpu.py} -x -v --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1; ok $? pytest_new
tail -4 $OUT/pytest_new.log
timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim.log 2>&1; ok $? probe_optim
tail -1 $OUT/probe_optim.log
for v in "fused:" "unfused:--fuse_fc_wgrad=0"; do
  name=${v%%:*}; ex=${v#*:}
  timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --extra="$ex" > $OUT/bench_$name.log 2>&1; ok $? bench_$name
  tail -1 $OUT/bench_$name.log | cut -c1-400
done
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --variant rainbow > $OUT/bench_rainbow.log 2>&1; ok $? bench_rainbow
tail -1 $OUT/bench_rainbow.log | cut -c1-400
for p in device host; do
  timeout -k 10 300 python scripts/bench_paths.py --path $p --steps ${R3_PATH_STEPS:-3000} > $OUT/paths_$p.log 2>&1; ok $? paths_$p
  tail -1 $OUT/paths_$p.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --replay 200000 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
ok $? rocprof
echo ALL_DONE
