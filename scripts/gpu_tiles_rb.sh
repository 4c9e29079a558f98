#!/bin/bash
# DQN_TILES sweep of the dense forward / dgrad tiles for the Rainbow and dd steps (4 instances x
# 2 hidden layers: 512 blocks at the flagship's 16-row tiles)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tiles_rb
mkdir -p $OUT
for V in rainbow dd; do
  for T in "" "4:1" "4:2" "6:1" "6:2"; do
    tag=$(echo "${T:-default}" | tr ':,' '-_')
    DQN_TILES="$T" timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --variant $V --replay 200000 \
        > $OUT/${V}_$tag.log 2>&1 || { echo "bench $V '$T' failed"; tail -5 $OUT/${V}_$tag.log; exit 1; }
    echo "$V tiles='$T': $(tail -1 $OUT/${V}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
