#!/bin/bash
# DQN on a single node with 0 or 1 GPU (reference: scripts/dqn_single_node.sh).
#   dqn_single_node.sh <env_type> <env_name> [extra flags...]
if [ "$#" -lt 2 ]; then
  echo "Usage: $0 <env_type> <env_name> [extra flags]. env_type: control, atari, nature, double_dueling, apex, rainbow."
  exit 1
fi
SCRIPTS_DIR=$( cd "$(dirname "${BASH_SOURCE}")" ; pwd -P )
cd "$SCRIPTS_DIR/.."
source "$SCRIPTS_DIR/dqn_params.sh"
dqn_params=$(dqn_params_for_env $1 $2) || exit 1
shift 2
BASE_LOG_DIR=${BASE_LOG_DIR:-/tmp}
TRAIN_LOG_DIR="$BASE_LOG_DIR/train"
GYM_LOG_DIR="$BASE_LOG_DIR/gym"
echo "Starting DQN. Train logs: $TRAIN_LOG_DIR, monitor logs: $GYM_LOG_DIR"
exec python -m dist_dqn_amd $dqn_params --logdir=$TRAIN_LOG_DIR --monitor --monitor_path=$GYM_LOG_DIR \
  --disable_video "$@"
