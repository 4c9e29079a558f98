set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/apex
timeout -k 10 100 python scripts/probe_head.py > gpurun_out/apex/probe_head.log 2>&1 || { echo probe failed; tail -5 gpurun_out/apex/probe_head.log; exit 1; }
cat gpurun_out/apex/probe_head.log | grep cycles
timeout -k 20 240 python scripts/bench_apex.py --actors 256 --seconds 60 > gpurun_out/apex/apex256.log 2>&1 || { echo apex failed; tail -20 gpurun_out/apex/apex256.log; exit 1; }
tail -1 gpurun_out/apex/apex256.log
