#!/bin/bash
# Bounds-checked debug pass: the GPU test suite against the debug build
# (-O1 -g, device DQN_ASSERTs) with serialized, blocking launches so a failing check or
# fault is attributed to the launch that caused it. Build it first, on the CPU:
#   DQN_DEBUG=1 python setup.py build_ext --inplace     (-> dist_dqn_amd/_C_debug*.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DQN_DEBUG_EXT=1 AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 900 \
    python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not two_ranks" > gpurun_out/pytest_gpu_debug.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_debug.log
exit $rc
