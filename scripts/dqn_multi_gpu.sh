#!/bin/bash
# Single-node multi-GPU DQN (reference: scripts/dqn_multi_gpu.sh).
#   dqn_multi_gpu.sh <env_type> <env_name> <num_gpus> [extra flags...]
#
# The reference starts 1 parameter server + (num_gpus - 1) workers on localhost
# gRPC ports and leaves GPU 0 to the PS. Here all num_gpus GPUs run learner
# ranks of one torch.distributed job (RCCL over xGMI, synchronous data
# parallelism: gradients all-reduced every step, no parameter server).
if [ "$#" -lt 3 ]; then
  echo "Usage: $0 <env_type> <env_name> <num_gpus> [extra flags]."
  exit 1
fi
SCRIPTS_DIR=$( cd "$(dirname "${BASH_SOURCE}")" ; pwd -P )
cd "$SCRIPTS_DIR/.."
source "$SCRIPTS_DIR/dqn_params.sh"
dqn_params=$(dqn_params_for_env $1 $2) || exit 1
NUM_GPUS=$3
shift 3
if [[ "$NUM_GPUS" -lt 1 ]]; then NUM_GPUS=1; fi
BASE_LOG_DIR=${BASE_LOG_DIR:-/tmp}
TRAIN_LOG_DIR="$BASE_LOG_DIR/train"
GYM_LOG_DIR="$BASE_LOG_DIR/gym"
PORT=${MASTER_PORT:-29511}
echo "Starting $NUM_GPUS learner ranks. Train logs: $TRAIN_LOG_DIR, per-rank monitor logs under $GYM_LOG_DIR"
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node=$NUM_GPUS --master-addr 127.0.0.1 \
  --master-port $PORT -m dist_dqn_amd $dqn_params --sync --logdir=$TRAIN_LOG_DIR --monitor \
  --monitor_path=$GYM_LOG_DIR --disable_video "$@"
