"""hipGraph capture of whole training steps: replaying the captured step must reproduce the eager
steps bit-for-bit (every kernel is deterministic), including new batches copied into the captured
inputs, SGD momentum, Adam's device-side bias corrections and the clip/skip path."""
import copy

import pytest
import torch

from deeplearning_mpi_amd.models import UNet, resnet18
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy
from deeplearning_mpi_amd.optim import SGD, Adam, clip_grad_norm_
from deeplearning_mpi_amd.utils.graphs import CapturedStep

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(model, opt_fn, loss_fn, batches, graph):
    opt = opt_fn(model)
    x = batches[0][0].clone()
    y = batches[0][1].clone()

    def step():
        opt.zero_grad()
        loss = loss_fn(model, x, y)
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
    return torch.stack(losses), [p.detach().clone() for p in model.parameters()], \
        [b.detach().clone() for b in model.buffers()]


def _check(make, opt_fn, loss_fn, batches):
    torch.manual_seed(0)
    m1 = make().to(DEV)
    m2 = copy.deepcopy(m1)
    l1, p1, b1 = _run(m1, opt_fn, loss_fn, batches, graph=False)
    l2, p2, b2 = _run(m2, opt_fn, loss_fn, batches, graph=True)
    assert torch.equal(l1, l2), (l1, l2)
    for a, b in zip(p1, p2):
        assert torch.equal(a, b)
    for a, b in zip(b1, b2):
        assert torch.equal(a, b)


def test_resnet18_sgd_step_graph_replay_matches_eager():
    g = torch.Generator(device=DEV).manual_seed(3)
    batches = [(torch.randn(32, 3, 32, 32, device=DEV, generator=g),
                torch.randint(10, (32,), device=DEV, generator=g)) for _ in range(6)]
    _check(lambda: resnet18(num_classes=10),
           lambda m: SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-5),
           lambda m, x, y: cross_entropy(m(x), y), batches)


def test_unet_adam_clip_step_graph_replay_matches_eager():
    g = torch.Generator(device=DEV).manual_seed(4)
    batches = [(torch.randn(2, 3, 64, 64, device=DEV, generator=g),
                (torch.rand(2, 64, 64, device=DEV, generator=g) > 0.5).float()) for _ in range(6)]
    _check(lambda: UNet(out_classes=1),
           lambda m: Adam(m.parameters(), lr=1e-3),
           lambda m, x, y: bce_with_logits(m(x).squeeze(1), y), batches)
