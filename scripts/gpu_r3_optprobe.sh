#!/bin/bash
# Round 3: price the optimizer launch's parts -- the arrival ticket (DQN_OPT_PROBE_NOTICKET, timing
# only), the fc weight tiles (probe_optim's no_fc_tiles variant) -- flagship alone and Rainbow in
# a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R3_OUT:-r3optprobe}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim.log 2>&1; ok $? probe_optim
tail -1 $OUT/probe_optim.log
DQN_OPT_PROBE_NOTICKET=1 timeout -k 10 120 python scripts/probe_optim.py > $OUT/probe_optim_noticket.log 2>&1; ok $? probe_optim_noticket
tail -1 $OUT/probe_optim_noticket.log
cd /tmp && export TMPDIR=/tmp
for nt in 0 1; do
  if [ $nt = 1 ]; then export DQN_OPT_PROBE_NOTICKET=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof_rb$nt -o run --output-format csv -- \
      python3 $REPO/bench.py --variant rainbow --steps 200 --warmup 20 --replay 200000 > $REPO/$OUT/prof_rb$nt.log 2>&1; ok $? rocprof_rb$nt
  python3 $REPO/scripts/kstats.py $REPO/$OUT/prof_rb$nt/run_kernel_trace.csv 4 > $REPO/$OUT/kstats_rb$nt.md; cat $REPO/$OUT/kstats_rb$nt.md
done
echo ALL_DONE
