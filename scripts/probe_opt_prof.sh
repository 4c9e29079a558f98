#!/bin/bash
# Optimizer+pack launch duration under probe modes / with and without the PER sampler block.
set -u
cd $GRAFT_REPO_ROOT
run() { # name probe args
  DQN_OPT_PROBE=$2 PROF_NAME=probe/$1 PROF_ARGS="$3" PROF_TOP=40 bash scripts/gpu_prof.sh > gpurun_out/probe/k_$1.txt || exit 1
  echo "== $1"; grep -E "optim_pack|c51_head|head_loss" gpurun_out/probe/k_$1.txt
}
mkdir -p gpurun_out/probe
run rb0 0 "--variant rainbow --steps 100 --warmup 20"
run rb7 7 "--variant rainbow --steps 100 --warmup 20"
run dd 0 "--variant dd --steps 100 --warmup 20"
run ddper 0 "--variant dd --extra=--prioritized_replay --steps 100 --warmup 20"
