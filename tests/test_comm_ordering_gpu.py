"""Stream ordering of the DDP communication path with collectives that CHANGE data in flight
(VERDICT r2 next 2d, weak 7).

With a world-size-1 RCCL communicator every collective is an identity, so a missing fence between
the compute streams and the comm stream is invisible.  Here a Python communicator runs each
collective on its own HIP stream as ``x *= 2; <5 ms delay kernel>; x /= 2`` -- exact in fp32, but
anyone who reads the buffer before the collective has finished sees doubled values, and a collective
that starts before the producer finished doubles a half-written buffer.  Both the K5 BatchNorm-buffer
broadcast (``broadcast_async`` joined by ``ParamArena.wait_buffers``) and the K6 gradient buckets
(``begin_bucket`` on the producing side stream, ``end_backward`` joining the compute stream) go
through it, eagerly and inside a captured hipGraph.  Results must be bit-identical to the
single-process run; a negative control without the end-of-backward join must NOT be.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
DELAY_MS = 5.0


def _slow_comm(join_at_end=True):
    from deeplearning_mpi_amd._ext import native
    from deeplearning_mpi_amd.parallel.bootstrap import LaunchInfo
    from deeplearning_mpi_amd.parallel.comm import SingleCommunicator

    C = native()

    class SlowComm(SingleCommunicator):
        def __init__(self):
            super().__init__(LaunchInfo("single", 0, 1, 0, 1), torch.device(DEV, 0))
            self.s = torch.cuda.Stream()
            self.n_bcast = 0
            self.n_bucket = 0

        def scramble(self, t):   # runs on self.s
            t.mul_(2)
            C.delay_ms(DELAY_MS)
            t.div_(2)

        def broadcast_async(self, t, src=0):
            self.n_bcast += 1
            self.s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.s):
                self.scramble(t)
            return lambda: torch.cuda.current_stream().wait_stream(self.s)

        def bucket_comm(self):
            outer = self

            class Buckets(C.CommBase):
                def begin_bucket(self):
                    outer.s.wait_stream(torch.cuda.current_stream())

                def allreduce_bucket(self, t, average):
                    outer.n_bucket += 1
                    with torch.cuda.stream(outer.s):
                        outer.scramble(t)

                def end_backward(self):
                    if join_at_end:
                        torch.cuda.current_stream().wait_stream(outer.s)

            return Buckets()

    return SlowComm()


def _train(model, comm, batches, graph):
    import deeplearning_mpi_amd as dl
    from deeplearning_mpi_amd.ops import cross_entropy
    from deeplearning_mpi_amd.optim import SGD
    from deeplearning_mpi_amd.utils.graphs import CapturedStep

    model.engine_setup(DEV)
    model._be.aux_min_pixels = 0   # weight-gradient side stream + branch stream on
    ddp = dl.DistributedDataParallel(model, comm=comm, _force_reducer=comm is not None)
    opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-5)
    x, y = batches[0][0].clone(), batches[0][1].clone()

    def step():
        opt.zero_grad()
        loss = cross_entropy(ddp(x), y)
        loss.backward()
        opt.step()
        return loss

    cs = CapturedStep(step, warmup=2, inputs=(x, y), enabled=graph)
    losses = []
    for bx, by in batches:
        cs.set_inputs(bx, by)
        losses.append(cs().clone())
    torch.cuda.synchronize()
    assert (cs.graph is not None) == graph
    return torch.stack(losses), [t.detach().clone() for t in list(model.parameters()) + list(model.buffers())]


def _setup():
    from deeplearning_mpi_amd.models import resnet50

    g = torch.Generator(device=DEV).manual_seed(11)
    batches = [(torch.randn(8, 3, 64, 64, device=DEV, generator=g),
                torch.randint(100, (8,), device=DEV, generator=g)) for _ in range(5)]
    torch.manual_seed(0)
    return resnet50(num_classes=100).to(DEV), batches


@pytest.mark.parametrize("graph", [False, True])
def test_inflight_collectives_are_fenced(graph):
    m0, batches = _setup()
    ref = _train(copy.deepcopy(m0), None, batches, graph=False)
    comm = _slow_comm()
    got = _train(copy.deepcopy(m0), comm, batches, graph=graph)
    assert comm.n_bucket >= 3 and comm.n_bcast >= 1   # both paths really went through the slow comm
    assert torch.equal(ref[0], got[0]), (ref[0], got[0])
    for a, b in zip(ref[1], got[1]):
        assert torch.equal(a, b)


def test_negative_control_missing_join_is_detected():
    """Without the end-of-backward join the optimizer reads doubled gradients: the check above must
    be able to see that."""
    m0, batches = _setup()
    ref = _train(copy.deepcopy(m0), None, batches[:2], graph=False)
    got = _train(copy.deepcopy(m0), _slow_comm(join_at_end=False), batches[:2], graph=False)
    assert not all(torch.equal(a, b) for a, b in zip(ref[1], got[1]))
