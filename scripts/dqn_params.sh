#!/bin/bash
# DQN hyper-parameter presets (same names/values as the reference's
# scripts/dqn_params.sh: CONTROL, ATARI) plus the MI355X north-star presets.
# Single source of truth is dist_dqn_amd/config.py (PRESETS); this wrapper
# keeps the reference's shell interface: dqn_params_for_env <env_type> <env_name>.

dqn_params_for_env() {
  if [ "$#" -ne 2 ]; then
    echo "Usage: dqn_params_for_env <env_type> <env_name>. Options for env_type:" \
         "[control, atari, nature, double_dueling, apex, rainbow]." >&2
    return 1
  fi
  python -c "from dist_dqn_amd.config import dqn_params_for_env; print(dqn_params_for_env('$1', '$2'))"
}
