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


def _sgd(m):
    return SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-5)


def _cifar_batches(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return [(torch.randn(32, 3, 32, 32, device=DEV, generator=g),
             torch.randint(10, (32,), device=DEV, generator=g)) for _ in range(n)]


def test_eager_eval_after_replays_sees_updated_weights():
    """replays update the fp32 masters through raw pointers; an eager forward after them
    (evaluation, a ragged last batch) must recast the bf16 compute weights instead of reusing the
    copy from before the replays.  Train (graph) -> eval -> train (graph) -> eval must equal the
    all-eager run, evals included."""
    batches = _cifar_batches(8, 21)
    xe = torch.randn(16, 3, 32, 32, device=DEV, generator=torch.Generator(device=DEV).manual_seed(22))

    def run(graph):
        torch.manual_seed(0)
        m = resnet18(num_classes=10).to(DEV)
        opt = _sgd(m)
        x, y = batches[0][0].clone(), batches[0][1].clone()

        def step():
            opt.zero_grad()
            loss = cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss

        cs = CapturedStep(step, warmup=2, inputs=(x, y), enabled=graph)
        evals = []
        for k, (bx, by) in enumerate(batches):
            cs.set_inputs(bx, by)
            cs()
            if k in (3, 5, 7):   # eager evaluation between replays
                m.eval()
                with torch.no_grad():
                    evals.append(m(xe).float().clone())
                m.train()
        torch.cuda.synchronize()
        return evals

    ref, got = run(False), run(True)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_failed_capture_falls_back_to_eager():
    """an error inside the capture (here a host synchronisation in the middle of
    the step, which a capturing stream refuses -- like an uncapturable collective) must not kill the
    run: CapturedStep reports it, drops the graph, replaces the streams the capture left stuck and
    runs every step eagerly, in the same process, bit-identical to an all-eager run."""
    batches = _cifar_batches(6, 23)

    def run(inject):
        torch.manual_seed(0)
        m = resnet18(num_classes=10).to(DEV)
        m.engine_setup(DEV)
        m._be.aux_min_pixels = 0   # branch + side streams on: the capture forks them before failing
        opt = _sgd(m)
        x, y = batches[0][0].clone(), batches[0][1].clone()

        def step():
            opt.zero_grad()
            loss = cross_entropy(m(x), y)
            if inject and torch.cuda.is_current_stream_capturing():
                float(loss)   # device -> host copy + sync: refused while capturing
            loss.backward()
            opt.step()
            return loss

        cs = CapturedStep(step, warmup=2, inputs=(x, y), enabled=inject)
        losses = []
        for bx, by in batches:
            cs.set_inputs(bx, by)
            losses.append(cs().clone())
        torch.cuda.synchronize()
        if inject:
            assert cs.graph is None and not cs.enabled and cs.capture_error is not None
            torch.randn(8, device=DEV)   # the device's torch RNG still works after the failed capture
        return torch.stack(losses), [p.detach().clone() for p in list(m.parameters()) + list(m.buffers())]

    l1, p1 = run(False)
    l2, p2 = run(True)
    assert torch.equal(l1, l2), (l1, l2)
    for a, b in zip(p1, p2):
        assert torch.equal(a, b)


def test_failed_capture_inside_backward_drops_queued_reductions():
    """a capture that fails INSIDE the engine backward (here a host sync after the 6th
    weight gradient, with the side stream on) leaves weight-gradient split reductions queued whose
    slabs were never computed.  They must be dropped -- not flushed into the gradients of the eager
    fallback step -- and deferral turned off: every step bit-identical to an all-eager run."""
    from deeplearning_mpi_amd._ext import native

    C = native()
    batches = _cifar_batches(5, 31)

    def run(inject):
        torch.manual_seed(0)
        m = resnet18(num_classes=10).to(DEV)
        m.engine_setup(DEV)
        m._be.aux_min_pixels = 0   # side stream on: the reductions queue there
        be = m._be
        orig = be.conv_wgrad
        calls, seen = [0], []

        def conv_wgrad(*a, **k):
            orig(*a, **k)
            if inject and torch.cuda.is_current_stream_capturing():
                calls[0] += 1
            if calls[0] == 6 and torch.cuda.is_current_stream_capturing():
                seen.append(C.wgrad_pending())   # reductions queued when the capture dies
                float(torch.ones(1, device=DEV).sum())   # refused while capturing

        be.conv_wgrad = conv_wgrad
        opt = _sgd(m)
        x, y = batches[0][0].clone(), batches[0][1].clone()

        def step():
            opt.zero_grad()
            loss = cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss

        cs = CapturedStep(step, warmup=2, inputs=(x, y), enabled=inject)
        losses = []
        for bx, by in batches:
            cs.set_inputs(bx, by)
            losses.append(cs().clone())
        torch.cuda.synchronize()
        if inject:
            assert cs.graph is None and not cs.enabled and cs.capture_error is not None
            assert seen and seen[0] > 0, seen
        assert C.wgrad_pending() == 0
        return torch.stack(losses), [p.detach().clone() for p in list(m.parameters()) + list(m.buffers())]

    l1, p1 = run(False)
    l2, p2 = run(True)
    assert torch.equal(l1, l2), (l1, l2)
    for a, b in zip(p1, p2):
        assert torch.equal(a, b)


def test_failed_capture_agreement_runs_on_reset_comm_stream():
    """with world_size > 1 the rank agreement after a failed capture is a collective on the
    communicator's stream -- a stream the failed capture had forked and left in capture mode.  The
    fake communicator below reports world_size 2 and runs both a step-internal collective and the
    agreement on such a stream; the fallback must replace that stream BEFORE the agreement, then run
    every step eagerly, bit-identical to an all-eager run."""
    from deeplearning_mpi_amd._ext import native

    C = native()

    class FakeRccl:   # the `c` of a communicator: its raw HIP stream + reset_stream_if_capturing
        def __init__(self):
            self.stream = torch.cuda.ExternalStream(C.create_stream())
            self.was_capturing = None

        def reset_stream_if_capturing(self):
            self.was_capturing = bool(C.stream_capturing(self.stream.cuda_stream))
            if self.was_capturing:
                self.stream = torch.cuda.ExternalStream(C.create_stream())

    class FakeComm:
        world_size = 2

        def __init__(self):
            self.c = FakeRccl()
            self.device = torch.device(DEV, torch.cuda.current_device())
            self.agreements = 0

        def _on_comm_stream(self, t):
            s = self.c.stream
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                t.mul_(1.0)
            torch.cuda.current_stream().wait_stream(s)

        def collective(self, t):   # a collective of the step (forked into the capture)
            self._on_comm_stream(t)

        def allreduce(self, t, op):   # the agreement: the simulated peer agrees with this rank
            assert op == "min"
            self.agreements += 1
            self._on_comm_stream(t)

    batches = _cifar_batches(5, 29)

    def run(inject):
        torch.manual_seed(0)
        m = resnet18(num_classes=10).to(DEV)
        m.engine_setup(DEV)
        opt = _sgd(m)
        comm = FakeComm()
        x, y = batches[0][0].clone(), batches[0][1].clone()

        def step():
            opt.zero_grad()
            loss = cross_entropy(m(x), y)
            comm.collective(loss)
            if inject and torch.cuda.is_current_stream_capturing():
                float(loss)   # refused while capturing: the capture fails after the comm stream joined it
            loss.backward()
            opt.step()
            return loss

        cs = CapturedStep(step, warmup=2, inputs=(x, y), enabled=inject, comm=comm)
        losses = []
        for bx, by in batches:
            cs.set_inputs(bx, by)
            losses.append(cs().clone())
        torch.cuda.synchronize()
        if inject:
            assert cs.graph is None and not cs.enabled and cs.capture_error is not None
            assert comm.agreements == 1
            # HIP ends capture mode on every joined stream when the origin's capture is torn down, so
            # the comm stream may or may not still be capturing when the reset runs; either way the
            # agreement must have run on a stream that is not capturing
            assert comm.c.was_capturing is not None, "the comm stream was not checked before the agreement"
            assert not C.stream_capturing(comm.c.stream.cuda_stream)
        return torch.stack(losses), [p.detach().clone() for p in m.parameters()]

    l1, p1 = run(False)
    l2, p2 = run(True)
    assert torch.equal(l1, l2), (l1, l2)
    for a, b in zip(p1, p2):
        assert torch.equal(a, b)
