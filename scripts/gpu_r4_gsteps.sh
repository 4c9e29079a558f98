set -u
mkdir -p gpurun_out/r4gs
for g in 8 16 32 8 32; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --graph_steps $g > gpurun_out/r4gs/g$g.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/r4gs/g$g.log').read().strip().splitlines()[-1]); print($g, d['value'], d['ms_per_step'], d['graph_steps'])"
done
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_models_optim.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4gs/pytest.log 2>&1; echo pytest rc=$?; tail -3 gpurun_out/r4gs/pytest.log
