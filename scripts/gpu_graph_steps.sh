set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/gsteps
timeout -k 10 200 python -u -m pytest tests/test_executor_gpu.py -q -x -k "step_many or fused_acting_per or fused_sampling" --timeout 120 --timeout-method thread > gpurun_out/gsteps/tests.log 2>&1 || { tail -30 gpurun_out/gsteps/tests.log; exit 1; }
tail -1 gpurun_out/gsteps/tests.log
for V in dqn rainbow; do
  for G in 1 8 32; do
    timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --variant $V --graph_steps $G > gpurun_out/gsteps/${V}_$G.log 2>&1 || { echo "$V $G failed"; tail -5 gpurun_out/gsteps/${V}_$G.log; exit 1; }
    echo "$V G=$G: $(tail -1 gpurun_out/gsteps/${V}_$G.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['env_frames_per_sec'], d['config']['steps_per_graph_launch'])")"
  done
done
