#!/bin/bash
# Same-box kernel-trace A/B: rocprofv3 kernel stats of bench.py for each "LABEL:BENCH FLAGS" spec.
#   OUT=gpurun_out/x BENCH_ARGS="--steps 200 --warmup 20" bash scripts/gpu_trace_ab.sh "a:" "b:--dp_path=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=${OUT:-gpurun_out/trace_ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%:*}
  flags=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/prof_$label" -o run --output-format csv -- \
      python3 "$REPO/bench.py" ${BENCH_ARGS:---steps 200 --warmup 20 --replay 200000} $flags > "$REPO/$OUT/prof_$label.log" 2>&1
  rc=$?
  echo "[trace $label] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 "$REPO/scripts/kstats.py" "$REPO/$OUT/prof_$label/run_kernel_trace.csv" 8 > "$REPO/$OUT/kstats_$label.md"
  cat "$REPO/$OUT/kstats_$label.md"
done
