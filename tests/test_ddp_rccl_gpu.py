"""The RCCL data plane of DDP on one GPU: a world-size-1 ``RcclComm`` with the bucketed reducer forced
on, so every piece of the multi-rank path runs -- bucket all-reduces (ncclAvg) on the comm stream
fenced after the side (weight-gradient) stream, the asynchronous per-forward BatchNorm buffer
broadcast (K5) joined before the first BN finalize, the end-of-backward join -- eagerly and inside
a captured hipGraph, with the auxiliary streams (side, branch) on.  With one rank every collective
is an identity, so the results must be bit-identical to the single-process step (VERDICT r1:
"the RCCL multi-rank path has never run").  One process, one device: RCCL refuses two ranks on
one GPU, so the N-rank run itself is the driver's 8-GPU bench."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rccl_comm():
    from deeplearning_mpi_amd._ext import native
    from deeplearning_mpi_amd.parallel.bootstrap import LaunchInfo
    from deeplearning_mpi_amd.parallel.comm import RcclCommunicator

    torch.cuda.set_device(0)
    C = native()
    nc = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0)
    return RcclCommunicator(LaunchInfo("single", 0, 1, 0, 1), torch.device(DEV, 0), nc)


def _train(model, comm, make_opt, loss_fn, batches, graph, aux):
    import deeplearning_mpi_amd as dl
    from deeplearning_mpi_amd.optim import Adam, clip_grad_norm_
    from deeplearning_mpi_amd.utils.graphs import CapturedStep

    model.engine_setup(DEV)
    if aux:
        model._be.aux_min_pixels = 0   # side + branch streams on at this small size
    ddp = dl.DistributedDataParallel(model, comm=comm, _force_reducer=comm is not None)
    assert (ddp.reducer is not None) == (comm is not None)
    opt = make_opt(model)
    x, y = batches[0][0].clone(), batches[0][1].clone()

    def step():
        opt.zero_grad()
        loss = loss_fn(ddp, x, y)
        loss.backward()
        if isinstance(opt, Adam):
            clip_grad_norm_(model.parameters(), 1.0, optimizer=opt)
        opt.step()
        return loss

    cs = CapturedStep(step, warmup=2, inputs=(x, y), enabled=graph)
    losses = []
    for bx, by in batches:
        cs.set_inputs(bx, by)
        losses.append(cs().clone())
    torch.cuda.synchronize()
    if graph:
        assert cs.graph is not None
    return (torch.stack(losses), [p.detach().clone() for p in model.parameters()],
            [b.detach().clone() for b in model.buffers()])


def _check(make, make_opt, loss_fn, batches, aux):
    comm = _rccl_comm()
    try:
        torch.manual_seed(0)
        m0 = make().to(DEV)
        ref = _train(copy.deepcopy(m0), None, make_opt, loss_fn, batches, graph=False, aux=aux)
        for graph in (False, True):
            got = _train(copy.deepcopy(m0), comm, make_opt, loss_fn, batches, graph=graph, aux=aux)
            assert torch.equal(ref[0], got[0]), (graph, ref[0], got[0])
            for a, b in zip(ref[1] + ref[2], got[1] + got[2]):
                assert torch.equal(a, b), graph
    finally:
        comm.destroy()


@pytest.mark.parametrize("dual", [False, True])
def test_resnet50_rccl_reducer_eager_and_graph_match_single_process(dual, monkeypatch):
    """dual: the dual 1x1 data gradient (models/engine.py DUAL_DGRAD) forced on every eligible conv
    (at the bench size it is on for layers 1-2), so its weight kernel, the [dy | z] GEMMs and the
    prologue weight gradients run under the reducer and inside the captured graph too."""
    from deeplearning_mpi_amd.models import engine, resnet50

    monkeypatch.setattr(engine, "DUAL_DGRAD", True)
    monkeypatch.setattr(engine, "DUAL_MIN_ROWS", 0 if dual else 1 << 40)
    from deeplearning_mpi_amd.ops import cross_entropy
    from deeplearning_mpi_amd.optim import SGD

    g = torch.Generator(device=DEV).manual_seed(5)
    batches = [(torch.randn(8, 3, 64, 64, device=DEV, generator=g),
                torch.randint(100, (8,), device=DEV, generator=g)) for _ in range(5)]
    _check(lambda: resnet50(num_classes=100),
           lambda m: SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-5),
           lambda d, x, y: cross_entropy(d(x), y), batches, aux=True)


def test_unet_rccl_reducer_eager_and_graph_match_single_process():
    from deeplearning_mpi_amd.models import UNet
    from deeplearning_mpi_amd.ops import bce_with_logits
    from deeplearning_mpi_amd.optim import Adam

    g = torch.Generator(device=DEV).manual_seed(6)
    batches = [(torch.randn(2, 3, 64, 64, device=DEV, generator=g),
                (torch.rand(2, 64, 64, device=DEV, generator=g) > 0.5).float()) for _ in range(5)]
    _check(lambda: UNet(out_classes=1),
           lambda m: Adam(m.parameters(), lr=1e-3),
           lambda d, x, y: bce_with_logits(d(x).squeeze(1), y), batches, aux=True)
