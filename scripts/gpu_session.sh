#!/bin/bash
# One parameterised GPU-box evidence session (replaces the per-round gpu_r3_* / gpu_r4_* scripts).
# Every GPU step runs under its own time limit and the first failing step ends the session.
#
#   TESTS=1              pytest -m gpu (whole suite; PYTEST_ARGS to narrow it)
#   SMOKE=1              __graft_entry__.smoke()
#   BENCH="dqn:: dd:: rainbow:: rainbow:--dtype=fp16 dqn:--dtype=fp32"
#                        bench.py per "variant:extra flags:" spec (STEPS / WARMUP)
#   TRACE="dqn: rainbow:"  rocprofv3 kernel trace + kstats table per "variant:extra" spec
#   PMC=1                hardware-counter passes over the flagship (scripts/profile_counters.sh)
#   OUT=gpurun_out/<tag> where everything lands
# e.g. gpurun -- 'BENCH="dqn:: rainbow::" TRACE="dqn:" OUT=gpurun_out/r5ev bash scripts/gpu_session.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=${OUT:-gpurun_out/session}
mkdir -p "$OUT"
STEPS=${STEPS:-2000}
WARMUP=${WARMUP:-100}
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
tag_of() { echo "$1" | tr -c 'a-zA-Z0-9_=\n' '_'; }
if [ "${TESTS:-0}" == "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} \
      > "$OUT/pytest_gpu.log" 2>&1
  ok $? pytest_gpu
  tail -3 "$OUT/pytest_gpu.log"
fi
if [ "${SMOKE:-0}" == "1" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $? smoke
  tail -1 "$OUT/smoke.log"
fi
for spec in ${BENCH:-}; do
  IFS=: read -r var ex _ <<< "$spec"
  tag=$(tag_of "$var$ex")
  timeout -k 10 300 python bench.py --variant "$var" --steps "$STEPS" --warmup "$WARMUP" --extra="$ex" \
      > "$OUT/bench_$tag.log" 2>&1
  ok $? "bench $tag"
  grep '^{' "$OUT/bench_$tag.log" | tail -1 >> "$OUT/bench.jsonl"
  grep '^{' "$OUT/bench_$tag.log" | tail -1 | cut -c1-240
done
if [ -n "${TRACE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  for spec in $TRACE; do
    IFS=: read -r var ex <<< "$spec"
    tag=$(tag_of "$var$ex")
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/prof_$tag" -o run --output-format csv -- \
        python3 "$REPO/bench.py" --variant "$var" --steps 200 --warmup 20 --replay 200000 --extra="$ex" \
        > "$REPO/$OUT/prof_$tag.log" 2>&1
    ok $? "trace $tag"
    python3 "$REPO/scripts/kstats.py" "$REPO/$OUT/prof_$tag/run_kernel_trace.csv" 14 > "$REPO/$OUT/kstats_$tag.md"
    cat "$REPO/$OUT/kstats_$tag.md"
  done
  cd "$REPO"
fi
if [ "${PMC:-0}" == "1" ]; then
  PMC_OUT=${OUT#gpurun_out/}/pmc BENCH_ARGS="${PMC_ARGS:---steps 60 --warmup 10}" timeout -k 10 900 \
      bash scripts/profile_counters.sh
  ok $? pmc
fi
echo ALL_DONE
