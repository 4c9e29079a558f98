#!/bin/bash
# Bench A/B on one GPU box: for each "LABEL=ENV..." spec, `python bench.py $BENCH_ARGS` with those
# env assignments, ROUNDS times alternating; one JSON line per run into $OUT (gpurun_out/...).
#   OUT=gpurun_out/x.jsonl ROUNDS=2 BENCH_ARGS="--steps 2000 --warmup 100" scripts/gpu_ab.sh "mix0=DQN_WG_MIX=0" "mix1=DQN_WG_MIX=1"
set -o pipefail
OUT=${OUT:-gpurun_out/ab.jsonl}
ROUNDS=${ROUNDS:-2}
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    label=${spec%%=*}
    envs=${spec#*=}
    line=$(env $envs timeout -k 10 300 python bench.py $BENCH_ARGS 2>>"${OUT%.jsonl}.err" | grep '^{') || exit 1
    echo "{\"label\": \"$label\", \"round\": $r, \"env\": \"$envs\", \"bench\": $line}" >> "$OUT"
    echo "$label round $r: $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
