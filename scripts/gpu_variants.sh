#!/bin/bash
# Benches of every variant (BASELINE configs, bf16 / fp16 / fp32 builds) + rocprof kernel stats
# of one variant (PROF_VARIANT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/variants
mkdir -p $OUT
rm -f $OUT/benches.jsonl
run() {   # name, args
  timeout -k 10 180 python bench.py $2 > $OUT/bench_$1.log 2>&1 || { echo "bench $1 failed"; tail -5 $OUT/bench_$1.log; exit 1; }
  tail -1 $OUT/bench_$1.log >> $OUT/benches.jsonl
  echo "$1: $(tail -1 $OUT/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['dtype'], d['env_frames_per_sec'])")"
}
run dqn "--steps 2000 --warmup 200"
run dqn_fp16 "--steps 2000 --warmup 200 --dtype fp16"
run dqn_fp32 "--steps 1000 --warmup 100 --dtype fp32"
run cnn "--network cnn --steps 2000 --warmup 200"
run cnn_fp32 "--network cnn --steps 1000 --warmup 100 --dtype fp32"
run dd "--variant dd --steps 2000 --warmup 200"
run rainbow "--variant rainbow --steps 1000 --warmup 100"
run rainbow_fp16 "--variant rainbow --steps 1000 --warmup 100 --dtype fp16"
run torch_cnn "--network cnn --backend torch --dtype fp32 --steps 200 --warmup 20"
if [ -n "${PROF_VARIANT:-}" ]; then
  PROF_NAME=variants/prof_$PROF_VARIANT PROF_ARGS="--variant $PROF_VARIANT --steps 100 --warmup 20 --replay 200000" PROF_TOP=${PROF_TOP:-20} bash scripts/gpu_prof.sh || exit 1
fi
