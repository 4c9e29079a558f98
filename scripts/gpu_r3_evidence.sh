#!/bin/bash
# Round 3 evidence runs: Ape-X at 256 / 14 actors (native ingest), the two CLI user paths (host agent
# loop vs --device_envs), the async PS over both transports, and the flagship PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/${R3_OUT:-r3evidence}
mkdir -p $OUT
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_fused_fc_gpu.py tests/test_kernels_gpu.py tests/test_executor_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $OUT/pytest_opt.log 2>&1; ok $? pytest_opt
tail -2 $OUT/pytest_opt.log
for v in "dqn:bf16:2000" "rainbow:bf16:1000"; do
  IFS=: read var dt n <<< "$v"
  timeout -k 10 300 python bench.py --variant $var --dtype $dt --steps $n --warmup 100 > $OUT/bench_${var}_$dt.log 2>&1; ok $? bench_${var}_$dt
  tail -1 $OUT/bench_${var}_$dt.log | cut -c1-300
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $OUT/bench_devkernarg.log 2>&1; ok $? bench_devkernarg
echo "devkernarg $(tail -1 $OUT/bench_devkernarg.log | cut -c1-260)"
timeout -k 10 120 python scripts/probe_wgrad.py > $OUT/probe_wgrad.log 2>&1; ok $? probe_wgrad
tail -3 $OUT/probe_wgrad.log
for cfg in ${APEX_CFGS:-256:16 14:16}; do
  n=${cfg%%:*}; g=${cfg#*:}
  timeout -k 20 200 python scripts/bench_apex.py --actors $n --seconds ${APEX_SECS:-45} --extra="--apex_graph_steps=$g" > $OUT/apex${n}_g$g.log 2>&1; ok $? apex${n}_g$g
  tail -1 $OUT/apex${n}_g$g.log | cut -c1-600
done
timeout -k 10 400 python scripts/bench_paths.py --path host --steps 2000 > $OUT/path_host.log 2>&1; ok $? path_host
tail -1 $OUT/path_host.log
timeout -k 10 400 python scripts/bench_paths.py --path device --steps 20000 > $OUT/path_device.log 2>&1; ok $? path_device
tail -1 $OUT/path_device.log
for tr in ${PS_TRANSPORTS:-xgmi}; do
  timeout -k 10 300 python scripts/bench_async_ps.py --transport $tr --workers 2 --steps 300 > $OUT/async_ps_$tr.log 2>&1; ok $? async_ps_$tr
  tail -1 $OUT/async_ps_$tr.log
done
if [ "${PMC:-1}" == "1" ]; then
  PMC_OUT=r3evidence/pmc BENCH_ARGS="--steps 60 --warmup 20 --replay 200000 --graph_steps 1" timeout -k 10 900 bash scripts/profile_counters.sh > $OUT/pmc.log 2>&1; ok $? pmc
  tail -14 $OUT/pmc.log
fi
echo ALL_DONE
