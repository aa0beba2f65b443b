"""hipGraph capture of a whole training step (the MI355X replacement for a tracing compiler).

The engine's schedules are plain code with no host synchronisation inside a step (BN statistics,
loss, gradient-norm clipping, the NaN/Inf skip decision and the optimizer all stay on the
device), so a complete step -- forward, loss, backward with the DDP bucket all-reduces, fused
optimizer update -- can be recorded once into a hipGraph and replayed with a single launch.
That removes the per-kernel host launch cost, which dominates small-batch / small-image runs
(e.g. the reference's ResNet-18 on 32x32 CIFAR, /root/reference/pytorch/resnet/main.py:123-132,
launches ~300 kernels per step of a few microseconds each).

Contract of :class:`CapturedStep`:

* ``step_fn()`` reads its inputs from fixed tensors (copy each new batch into them, e.g. with
  :meth:`CapturedStep.set_inputs`) and returns device tensors (e.g. the loss);
* python-side hyper-parameters (learning rate, momentum, clip norm) are baked in at capture time:
  call :meth:`recapture` after changing them (Adam's bias corrections read a device step count,
  so they stay correct across replays);
* the first ``warmup`` calls run eagerly on a side stream (allocator / autograd / kernel caches
  and weight-layout descriptors are set up outside the capture), the next call captures, later
  calls replay.
"""
from __future__ import annotations

import torch


class CapturedStep:
    def __init__(self, step_fn, warmup: int = 2, inputs=(), enabled: bool = True):
        self.step_fn = step_fn
        self.warmup = warmup
        self.inputs = tuple(inputs)
        self.enabled = enabled and torch.cuda.is_available()
        self.graph = None
        self.out = None
        self._calls = 0
        self._pool = None

    def set_inputs(self, *tensors):
        """Copy a new batch into the captured input tensors (same shapes / dtypes)."""
        for dst, src in zip(self.inputs, tensors):
            if dst.data_ptr() != src.data_ptr():   # device pipelines may write the inputs in place
                dst.copy_(src, non_blocking=True)

    def recapture(self):
        self.graph = None
        self._calls = self.warmup   # next call captures again (caches are already warm)

    def __call__(self):
        if not self.enabled:
            return self.step_fn()
        if self.graph is not None:
            self.graph.replay()
            return self.out
        self._calls += 1
        if self._calls <= self.warmup:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.step_fn()
            torch.cuda.current_stream().wait_stream(s)
            return out
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        # thread_local: the RCCL watchdog thread may poll events while this thread captures
        with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
            self.out = self.step_fn()
        self.graph = g
        # the capture only recorded the step: run it once so this call has the step's effect
        g.replay()
        return self.out
