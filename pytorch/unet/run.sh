#!/bin/bash
# UNet launcher (reference: pytorch/unet/run.sh -- torchrun + interactive prompts with defaults).
# Defaults to mpirun (HOSTFILE=<file>: ranks over several nodes, NPROC_PER_NODE * NNODES in total);
# LAUNCHER=torchrun for the reference-style launch.  PROMPT=1 asks interactively.
set -e
cd "$(dirname "$0")"
validate_ip() {
  local ip=$1
  if [[ $ip =~ ^([0-9]{1,3}\.){3}[0-9]{1,3}$ ]]; then
    for o in $(echo "$ip" | tr '.' ' '); do ((o >= 0 && o <= 255)) || return 1; done; return 0
  fi
  return 1
}
ask() { local var=$1 msg=$2 def=$3; if [ "${PROMPT:-0}" = "1" ] && [ -t 0 ]; then read -p "$msg [default: $def]: " v; eval "$var=\"\${v:-$def}\""; else eval "$var=\"\${$var:-$def}\""; fi; }
DEFAULT_IP=$(hostname -I 2>/dev/null | awk '{print $1}'); DEFAULT_IP=${DEFAULT_IP:-127.0.0.1}
ask LAUNCHER "Launcher (mpirun or torchrun)" mpirun
ask NPROC_PER_NODE "Processes per node (nproc_per_node)" 1
ask NNODES "Number of nodes (nnodes)" 1
ask NODE_RANK "Node rank (node_rank)" 0
if [[ $NODE_RANK -eq 0 ]]; then MASTER_ADDR=${MASTER_ADDR:-$DEFAULT_IP}; else ask MASTER_ADDR "Master address" 127.0.0.1; fi
validate_ip "$MASTER_ADDR" || { echo "Error: Invalid IP address format for master_addr: $MASTER_ADDR"; exit 1; }
ask MASTER_PORT "Master port" 29500
ask NUM_EPOCHS "Number of epochs" 100
ask BATCH_SIZE "Batch size per process" 128
ask LEARNING_RATE "Learning rate" 0.001
ask RANDOM_SEED "Random seed" 42
ask MODEL_DIR "Model directory" saved_models
ask MODEL_FILENAME "Model filename" model.pth
ask RESUME_PROMPT "Resume from a checkpoint? (yes or no)" no
RESUME=""; [[ $RESUME_PROMPT == "yes" ]] && RESUME="--resume"
EXTRA=${EXTRA_ARGS:-}
if [[ ! "$EXTRA" =~ --synthetic ]] && [[ ! -d data ]]; then echo "The 'data' directory does not exist. Please create it before running this script."; exit 1; fi
mkdir -p "$MODEL_DIR" logs
ARGS="--num_epochs $NUM_EPOCHS --batch_size $BATCH_SIZE --learning_rate $LEARNING_RATE --random_seed $RANDOM_SEED --model_dir $MODEL_DIR --model_filename $MODEL_FILENAME $RESUME $EXTRA"
MPIRUN=$(command -v mpirun || echo /opt/conda/bin/mpirun)
if [ "$LAUNCHER" = "mpirun" ]; then
  exec "$MPIRUN" ${HOSTFILE:+-hostfile "$HOSTFILE"} -n "$((NPROC_PER_NODE * NNODES))" python train.py $ARGS
else
  exec python -m torch.distributed.run --nproc_per_node=$NPROC_PER_NODE --nnodes=$NNODES --node_rank=$NODE_RANK \
       --master_addr=$MASTER_ADDR --master_port=$MASTER_PORT train.py $ARGS
fi
