#!/bin/bash
# Real-data-path throughput of the reference's own ResNet-18 / CIFAR-10 run (pytorch/resnet/main.py):
# a CIFAR-10-sized binary dataset (50,000 random 32x32x3 records; no network for the real files) fed by
# the device-resident pipeline vs torch DataLoader workers, eager and hipGraph steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/cifar
export HSA_ENABLE_IPC_MODE_LEGACY=0
D=/tmp/dlmpi_cifar && mkdir -p $D/cifar-10-batches-bin
python - <<'PY'
import numpy as np
g = np.random.default_rng(0)
for i, name in enumerate([f"data_batch_{k}.bin" for k in range(1, 6)] + ["test_batch.bin"]):
    r = g.integers(0, 256, size=(10000, 3073), dtype=np.uint8); r[:, 0] %= 10
    r.tofile(f"/tmp/dlmpi_cifar/cifar-10-batches-bin/{name}")
PY
for mode in 1 0; do
  for graph in "" "--graph"; do
    tag=dev${mode}${graph:+_graph}
    timeout -k 10 300 python pytorch/resnet/main.py --num_epochs 2 --eval_every 1000 --data_root $D \
      --data_on_device $mode $graph --model_dir /tmp/dlmpi_models > gpurun_out/cifar/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -20 gpurun_out/cifar/$tag.log; exit 1; }
    echo "$tag: $(grep throughput gpurun_out/cifar/$tag.log | tail -1)"
  done
done
