#!/bin/bash
# rocprofv3 kernel trace of one bench configuration: PROF_NAME, PROF_ARGS (bench.py args),
# PROF_EXTRA (one --extra config string).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
NAME=${PROF_NAME:-prof}
mkdir -p gpurun_out/$(dirname $NAME)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/$NAME -o run --output-format csv -- \
    python3 $REPO/bench.py ${PROF_ARGS:-} ${PROF_EXTRA:+--extra="$PROF_EXTRA"} > $REPO/gpurun_out/$NAME.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $REPO/gpurun_out/$NAME.log; exit 1; }
cd $REPO
tail -1 gpurun_out/$NAME.log | cut -c1-200
python scripts/kstats.py gpurun_out/$NAME/run_kernel_trace.csv ${PROF_TOP:-20}
