#!/bin/bash
# Launcher for hello_world.py (reference: pytorch/hello_world/run.sh, torchrun-only + prompts).
# Non-interactive by default; every value can come from the environment:
#   LAUNCHER=mpirun|torchrun  NPROC=2  NNODES=1  NODE_RANK=0  MASTER_ADDR  MASTER_PORT  BACKEND  OP
# With a TTY and PROMPT=1 it asks like the reference does.
set -e
cd "$(dirname "$0")"
ask() { local var=$1 msg=$2 def=$3; if [ "${PROMPT:-0}" = "1" ] && [ -t 0 ]; then read -p "$msg [default: $def]: " v; eval "$var=\"\${v:-$def}\""; else eval "$var=\"\${$var:-$def}\""; fi; }
ask LAUNCHER "Launcher (mpirun or torchrun)" mpirun
ask NPROC "Processes per node (nproc_per_node)" 2
ask NNODES "Number of nodes (nnodes)" 1
ask NODE_RANK "Node rank (node_rank)" 0
ask MASTER_ADDR "Master address (master_addr)" 127.0.0.1
ask MASTER_PORT "Master port (master_port)" 29500
ask BACKEND "Backend (nccl, gloo or mpi)" gloo
ask OP "Operation (send, allreduce, both)" both
MPIRUN=$(command -v mpirun || echo /opt/conda/bin/mpirun)
if [ "$LAUNCHER" = "mpirun" ]; then
  exec "$MPIRUN" ${HOSTFILE:+-hostfile "$HOSTFILE"} -n "$NPROC" python hello_world.py --backend "$BACKEND" --op "$OP"
else
  exec python -m torch.distributed.run --nproc_per_node="$NPROC" --nnodes="$NNODES" --node_rank="$NODE_RANK" \
       --master_addr="$MASTER_ADDR" --master_port="$MASTER_PORT" hello_world.py --backend "$BACKEND" --op "$OP"
fi
