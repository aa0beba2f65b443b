#!/bin/bash
# ResNet launcher (the reference ships none that works for ResNet).
# LAUNCHER=mpirun|torchrun NPROC=8 SCRIPT=main.py|resnet.py EXTRA_ARGS="--arch resnet50 --synthetic ..."
# HOSTFILE=<file> (mpirun): spread the NPROC ranks over the listed nodes
set -e
cd "$(dirname "$0")"
LAUNCHER=${LAUNCHER:-mpirun}; NPROC=${NPROC:-1}; SCRIPT=${SCRIPT:-main.py}
MPIRUN=$(command -v mpirun || echo /opt/conda/bin/mpirun)
if [ "$LAUNCHER" = "mpirun" ]; then
  exec "$MPIRUN" ${HOSTFILE:+-hostfile "$HOSTFILE"} -n "$NPROC" python "$SCRIPT" ${EXTRA_ARGS:-}
else
  exec python -m torch.distributed.run --standalone --nproc_per_node="$NPROC" "$SCRIPT" ${EXTRA_ARGS:-}
fi
