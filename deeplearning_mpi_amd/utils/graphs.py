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
  calls replay;
* a replay changes parameters behind the host's back (the optimizer kernel writes the flat
  master buffer through raw pointers), so every replay bumps :data:`REPLAYS`; ``ParamArena``
  folds that counter into its version, and the next EAGER use of the model (evaluation, a ragged
  last batch) recasts its compute weights instead of reading copies from before the replays;
* a failed capture never kills the run: the error is reported, the graph dropped, and the step
  runs eagerly from then on, in the same process (no re-exec).  With a communicator (``comm``)
  the ranks agree first -- if ANY rank failed to capture, every rank runs eagerly -- so the
  collectives stay matched across ranks.  A rank whose capture failed replaces its stuck streams
  (the communicator's included) BEFORE that agreement collective, which runs on the comm stream.

Why the capture runs on a helper thread, on a stream of its own: HIP (ROCm 7.2) does not close an
invalidated capture -- ``hipStreamEndCapture`` fails and the stream, every stream forked into the
capture and the capturing thread's legacy default stream all stay in capture mode, refusing every
later launch (scripts/diag/capture_fail.py).  So the capture begins and ends on a short-lived
thread (its thread-local capture state dies with it), on a raw HIP stream that is abandoned if the
capture fails, and the auxiliary streams / RCCL comm stream that the capture had forked are
replaced by fresh raw streams (``ops.backend.replace_poisoned_aux_streams``,
``RcclComm.reset_stream_if_capturing``).  None of them is a torch pool stream, so a stuck stream
is never handed out again.
"""
from __future__ import annotations

import sys
import threading

import torch

REPLAYS = 0   # replays (and failed captures) of any captured step in this process; ParamArena._version reads it


def _note_replay():
    """Host-side state no longer describes the device: a replay ran kernels the host did not issue,
    or a failed capture recorded (and never ran) kernels the host believes it issued -- e.g. the
    weight recast of ``ParamArena.refresh``.  Bumping the counter makes the next eager use recast."""
    global REPLAYS
    REPLAYS += 1



def _release_generator():
    """A capture that failed inside ``torch.cuda.graph`` leaves the device's default generator marked as
    capturing (its capture epilogue never ran): every later torch RNG call on the device then raises
    "Offset increment outside graph capture".  An empty capture on a fresh stream runs the prologue /
    epilogue pair again and clears the mark (tests/test_graphs_gpu.py checks torch RNG afterwards)."""
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream(), capture_error_mode="thread_local"):
            pass
        del g
    except Exception:   # noqa: BLE001 -- best effort: the eager fallback does not depend on it
        pass

class CapturedStep:
    def __init__(self, step_fn, warmup: int = 2, inputs=(), enabled: bool = True, comm=None):
        self.step_fn = step_fn
        self.warmup = warmup
        self.inputs = tuple(inputs)
        self.enabled = enabled and torch.cuda.is_available()
        self.comm = comm
        self.graph = None
        self.out = None
        self.capture_error = None   # the exception of a failed capture (then enabled is False)
        self._calls = 0
        self._pool = None
        self._stream = None   # the capture stream (ours, so a failed capture can be ended on it)

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
            _note_replay()
            return self.out
        self._calls += 1
        if self._calls <= self.warmup:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.step_fn()
            torch.cuda.current_stream().wait_stream(s)
            return out
        g, err = self._capture()
        if err is not None:
            # before anything else touches a stream: the communicator's stream may be one the failed
            # capture forked and left in capture mode, and the agreement below runs on it
            self._reset_streams()
        if not self._agree(err is None):
            self._fall_back(err)
            return self.step_fn()
        self.graph = g
        # the capture only recorded the step: run it once so this call has the step's effect
        g.replay()
        _note_replay()
        return self.out

    # ------------------------------------------------------------------ capture / fallback
    def _capture(self):
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        if self._stream is None:
            from .._ext import native

            self._stream = torch.cuda.ExternalStream(native().create_stream())
        dev = torch.cuda.current_device()
        res = {}

        def body():
            try:
                torch.cuda.set_device(dev)
                # thread_local: the RCCL watchdog thread may poll events while this thread captures
                with torch.cuda.graph(g, pool=self._pool, stream=self._stream, capture_error_mode="thread_local"):
                    res["out"] = self.step_fn()
            except BaseException as e:   # noqa: BLE001 -- any capture failure degrades to eager
                res["err"] = e

        t = threading.Thread(target=body, name="dlmpi-graph-capture")
        t.start()
        t.join()
        if "err" in res:
            self.out = None
            return None, res["err"]
        self.out = res["out"]
        return g, None

    def _agree(self, ok: bool) -> bool:
        """True iff every rank captured (MIN over ranks of the local success flag)."""
        c = self.comm
        if c is None or getattr(c, "world_size", 1) == 1:
            return ok
        t = torch.tensor([1.0 if ok else 0.0], device=c.device)
        c.allreduce(t, "min")
        return bool(t.item() > 0.5)

    def _reset_streams(self):
        """Replace every stream a failed capture left in capture mode (module docstring): the engine's
        auxiliary streams, the communicator's stream, our capture stream; clear the sticky HIP error."""
        from ..ops.backend import replace_poisoned_aux_streams

        replace_poisoned_aux_streams()
        nc = getattr(getattr(self.comm, "inner", self.comm), "c", None)
        if nc is not None and hasattr(nc, "reset_stream_if_capturing"):
            nc.reset_stream_if_capturing()
        self._stream = None   # abandoned (possibly still in capture mode)
        from .._ext import has_native, native

        if has_native():
            native().wgrad_discard()   # reductions queued by a backward the failed capture cut short
            native().clear_hip_error()

    def _fall_back(self, err):
        self.capture_error = err if err is not None else RuntimeError("hipGraph capture failed on another rank")
        print(f"[dlmpi] hipGraph capture failed ({self.capture_error!r}); running the step eagerly from now on",
              file=sys.stderr, flush=True)
        if err is None:   # this rank captured fine (its graph is dropped): nothing is stuck here
            self._stream = None
        torch.cuda.synchronize()
        if err is not None:
            _release_generator()
        self.graph = None
        self.enabled = False
        _note_replay()
