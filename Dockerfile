# MI355X (gfx950) container for deeplearning_mpi_amd.
# Reference equivalent: /root/reference/pytorch/unet/Dockerfile (miniconda + CUDA torch + sshd for
# multi-node).  Here: a ROCm PyTorch base, MPICH for the mpirun launcher/bootstrap, openssh for
# multi-node mpirun, and the native extension compiled in-tree for gfx950.
#
#   docker build -t dlmpi-amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host \
#              --shm-size 64g --network host -it dlmpi-amd
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

ENV DEBIAN_FRONTEND=noninteractive \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950

RUN apt-get update && apt-get install -y --no-install-recommends \
        mpich libmpich-dev openssh-server openssh-client build-essential git \
    && rm -rf /var/lib/apt/lists/* \
    && mkdir -p /var/run/sshd

# multi-node mpirun: key-based ssh between the nodes of the job (mount/copy your keys; the
# reference enables root password login, which we deliberately do not)
RUN sed -i 's/#\?PermitRootLogin.*/PermitRootLogin prohibit-password/' /etc/ssh/sshd_config
EXPOSE 22 29500

WORKDIR /workspace
COPY requirements.txt /workspace/requirements.txt
RUN pip install --no-cache-dir -r /workspace/requirements.txt
COPY . /workspace
# compile every HIP kernel for gfx950 + the torch/RCCL binding + the MPI bootstrap, in-tree
RUN python -m deeplearning_mpi_amd.build \
    && mkdir -p pytorch/unet/data pytorch/unet/logs pytorch/unet/saved_models pytorch/resnet/saved_models

CMD ["/bin/bash"]
