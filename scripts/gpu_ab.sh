#!/bin/bash
# Bench A/B on one GPU box: for each "LABEL:BENCH FLAGS" spec, `python bench.py $BENCH_ARGS <flags>`,
# ROUNDS times alternating; one JSON line per run into $OUT (gpurun_out/...). Kernel tuning constants
# are config flags (ops/tuning.py), e.g.
#   OUT=gpurun_out/x.jsonl ROUNDS=2 BENCH_ARGS="--steps 2000 --warmup 100" scripts/gpu_ab.sh \
#       "c3:" "c2:--extra=--kernel_tuning=wg_conv_chunks=2"
set -o pipefail
OUT=${OUT:-gpurun_out/ab.jsonl}
ROUNDS=${ROUNDS:-2}
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    label=${spec%%:*}
    flags=${spec#*:}
    line=$(timeout -k 10 300 python bench.py $BENCH_ARGS $flags 2>>"${OUT%.jsonl}.err" | grep '^{') || exit 1
    echo "{\"label\": \"$label\", \"round\": $r, \"flags\": \"$flags\", \"bench\": $line}" >> "$OUT"
    echo "$label round $r: $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
