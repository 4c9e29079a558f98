#!/bin/bash
# Tile-variant sweep of the layer GEMMs (DQN_TILES, csrc/kernels/qnet.hip tile_variant):
# oracle check of every variant set, then the flagship bench for each. One GPU call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tiles
mkdir -p $OUT
rm -f $OUT/sweep.jsonl
for T in "${@}"; do
  tag=$(echo "$T" | tr ':,' '-_')
  [ -z "$tag" ] && tag=default
  DQN_TILES="$T" timeout -k 10 200 python -m pytest tests/test_executor_gpu.py -x -q -k "loss_and_grad_match_oracle" \
      --timeout 120 --timeout-method thread > $OUT/test_$tag.log 2>&1 || { echo "oracle FAILED for '$T': $(grep -m1 AssertionError $OUT/test_$tag.log)" | tee -a $OUT/sweep.txt; }
  DQN_TILES="$T" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > $OUT/bench_$tag.log 2>&1 || { echo "bench failed '$T'"; tail -5 $OUT/bench_$tag.log; exit 1; }
  v=$(tail -1 $OUT/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
  echo "tiles='$T' -> $v" | tee -a $OUT/sweep.txt
done
