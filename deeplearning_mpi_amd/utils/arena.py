"""ParamArena: flat, device-resident parameter / gradient / buffer storage.

Every parameter of a model is re-homed into ONE fp32 buffer (and its gradient into ONE fp32
gradient buffer) laid out in the order in which the backward pass produces the gradients: the
engine models declare that order (``EngineModule._grad_ready_names``, checked against the
recorded ``ready`` sequence by tests/test_engine_cpu.py), other modules get reverse registration
order.  Consequences (MI355X-first design):

* DDP gradient buckets are contiguous slices of the flat gradient: all-reduced in place over RCCL,
  no pack/unpack (the reference's torch DDP Reducer copies grads into bucket buffers);
* optimizers (SGD / Adam / grad-norm clip) are ONE kernel over the flat buffers;
* BatchNorm running statistics live in one flat buffer -> the per-step buffer broadcast of DDP
   is a single collective;
* conv weights are stored channels-last (memory order [K][R][S][C]) so the fp32 master already
  has the GEMM layout, and the kernels' weight-gradient output lands in it directly;
* bf16 compute copies (forward layout and transposed data-gradient layout, channel padded) are
  produced for all layers by ONE multi-tensor cast launch whenever the masters changed -- two when
  the model marks its first layer (``mark_cast_group``): that layer's copies on the current stream,
  the rest on the backend's side stream beside the first layer's forward (``launch_cast``, joined
  lazily by ``get_compute``), so the recast is off the step's critical path.

``nn.Parameter`` objects are kept (their ``.data`` is re-pointed into the arena), so
``state_dict()`` keys/shapes/dtypes are unchanged and foreign optimizers still work.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

_ARENAS = {}   # id(param) -> arena


def arena_of(param) -> "ParamArena | None":
    a = _ARENAS.get(id(param))
    if a is not None and a.owns(param):
        return a
    return None


def _conv_like(m):
    return isinstance(m, (nn.Conv2d, nn.ConvTranspose2d))


class ParamArena:
    ALIGN = 16   # elements (64 bytes): every tensor starts on a 64-B boundary

    def __init__(self, module: nn.Module, device, backend=None, order_names=None):
        self.device = torch.device(device)
        self.backend = backend
        named = []
        seen = set()
        for n, p in module.named_parameters():
            if id(p) in seen:
                continue
            seen.add(id(p))
            named.append((n, p))
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        self.index = {id(p): i for i, p in enumerate(self.params)}

        layout = {}
        for m in module.modules():
            if isinstance(m, nn.Conv2d) and m.weight.dim() == 4:
                layout[id(m.weight)] = "krsc"          # [K,C,R,S] stored as [K][R][S][C]
            elif isinstance(m, nn.ConvTranspose2d):
                layout[id(m.weight)] = "convT"         # [Cin,Cout,kh,kw] stored as [Cin][kh][kw][Cout]

        # flat layout in gradient-ready order: declared names first, the rest in reverse registration
        order = list(range(len(self.params)))[::-1]
        if order_names:
            pos = {n: i for i, n in enumerate(self.names)}
            first = [pos[n] for n in order_names if n in pos]
            if len(set(first)) != len(first):
                raise ValueError("ParamArena: duplicate names in order_names")
            taken = set(first)
            order = first + [i for i in order if i not in taken]
        self.offsets = [0] * len(self.params)
        off = 0
        for i in order:
            self.offsets[i] = off
            n = self.params[i].numel()
            off += (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.total = off
        self.dtype = backend.dt if backend is not None else torch.float32
        self.flat = torch.zeros(self.total, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(self.total, dtype=self.dtype, device=self.device)
        self.order = order

        for i, p in enumerate(self.params):
            kind = layout.get(id(p), "contig")
            shape = tuple(p.shape)
            strides = self._strides(shape, kind)
            view = self.flat.as_strided(shape, strides, self.offsets[i])
            with torch.no_grad():
                view.copy_(p.data)
            p.data = view
            p.grad = self.grad.as_strided(shape, strides, self.offsets[i])
            _ARENAS[id(p)] = self
        self.layouts = [layout.get(id(p), "contig") for p in self.params]

        # buffers: BN running stats (float) + num_batches_tracked (int64)
        fbufs, ibufs = [], []
        for m in module.modules():
            for bn, b in m._buffers.items():
                if b is None:
                    continue
                (fbufs if b.is_floating_point() else ibufs).append((m, bn, b))
        self.fbuf_total = sum(b.numel() for _, _, b in fbufs)
        self.fbuf = torch.zeros(max(1, self.fbuf_total), dtype=self.dtype, device=self.device)
        o = 0
        for m, bn, b in fbufs:
            v = self.fbuf[o:o + b.numel()].view(b.shape)
            v.copy_(b.to(self.device, self.dtype))
            m._buffers[bn] = v
            o += b.numel()
        self.ibuf_total = sum(b.numel() for _, _, b in ibufs)
        self.ibuf = torch.zeros(max(1, self.ibuf_total), dtype=torch.int64, device=self.device)
        o = 0
        for m, bn, b in ibufs:
            v = self.ibuf[o:o + b.numel()].view(b.shape)
            v.copy_(b.to(self.device))
            m._buffers[bn] = v
            o += b.numel()

        # compute copies
        self._entries = []
        self._compute_total = 0
        self.compute = None
        self._synced_version = None
        self.post_refresh = []      # callables run after every recast (derived weight layouts)
        self._cast_split = None     # (entries, post_refresh) counts of the first layer (mark_cast_group)
        self._cast_lists = None     # (first-layer entries, the rest), kept for the backend's cast cache
        self._cast_deferred = None  # split recast's second part, not yet issued: (entries, post_refresh index)
        self._cast_event = None     # side-stream recast in flight: (event, first offset it covers, REPLAYS)
        self._cast_waited = []      # streams that have waited for it
        self.split_casts = 0        # recasts that took the two-stream path (tests)
        self.hook = None            # reducer.mark_ready(param_index) during backward
        self.backward_end = None    # reducer.finalize() at the end of the engine backward
        self.buffer_fence = None    # joins an in-flight broadcast of fbuf (DDP K5) before its first use
        self.zero_pending = False

    @staticmethod
    def _strides(shape, kind):
        if kind == "krsc":
            K, C, R, S = shape
            return (R * S * C, 1, S * C, C)
        if kind == "convT":
            Ci, Co, R, S = shape
            return (R * S * Co, 1, S * Co, Co)
        st, acc = [], 1
        for d in reversed(shape):
            st.append(acc)
            acc *= d
        return tuple(reversed(st))

    # ------------------------------------------------------------------ params / grads
    def owns(self, p) -> bool:
        i = self.index.get(id(p))
        if i is None:
            return False
        return p.data_ptr() == self.flat.data_ptr() + self.flat.element_size() * self.offsets[i]

    def valid(self) -> bool:
        """Every parameter still views its arena slot (called every step by the engine and the
        optimizers: one data_ptr comparison per parameter against addresses computed once)."""
        base = self.flat.data_ptr()
        exp = getattr(self, "_expect", None)
        if exp is None or exp[0] != base:
            es = self.flat.element_size()
            exp = self._expect = (base, [base + es * o for o in self.offsets])
        return all(p.data_ptr() == e for p, e in zip(self.params, exp[1]))

    def param_flat(self, p) -> torch.Tensor:
        i = self.index[id(p)]
        return self.flat[self.offsets[i]:self.offsets[i] + p.numel()]

    def grad_flat(self, p) -> torch.Tensor:
        i = self.index[id(p)]
        return self.grad[self.offsets[i]:self.offsets[i] + p.numel()]

    def attach_grads(self):
        """Re-attach .grad views (a foreign optimizer's zero_grad(set_to_none=True) drops them)."""
        dropped = False
        for i, p in enumerate(self.params):
            g = p.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + self.flat.element_size() * self.offsets[i]:
                p.grad = self.grad.as_strided(tuple(p.shape), self._strides(tuple(p.shape), self.layouts[i]),
                                              self.offsets[i])
                dropped = True
        if dropped:
            self.zero_grad()

    def zero_grad(self):
        """One launch of our fill kernel (reference backend / non-fp32: torch)."""
        be = self.backend
        if be is not None and hasattr(be, "fill_") and self.grad.dtype == torch.float32:
            be.fill_(self.grad, 0.0)
        else:
            self.grad.zero_()

    def ready(self, *ps):
        if self.hook is not None:
            for p in ps:
                if p is not None:
                    self.hook(self.index[id(p)])

    def wait_buffers(self):
        """Make the current stream wait for an in-flight update of the BN buffers (once)."""
        f = self.buffer_fence
        if f is not None:
            self.buffer_fence = None
            f()

    def end_backward(self):
        if self.backward_end is not None:
            self.backward_end()

    # ------------------------------------------------------------------ compute copies
    def add_compute(self, p, dims, valid, src_dims):
        """Register a compute copy of parameter ``p``: destination dims (4-D, contiguous), how many
        indices of each destination dim are valid (rest zero padding) and, for each destination dim,
        which source dim of ``p`` it walks (None = broadcast a size-1 dim).  Returns a handle."""
        st_p = p.data.stride()
        st = tuple(0 if s is None else st_p[s] for s in src_dims)
        off = self._compute_total
        n = dims[0] * dims[1] * dims[2] * dims[3]
        self._entries.append((p.data, off, tuple(dims), tuple(valid), st))
        self._compute_total += (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.compute = None
        return (off, n, tuple(dims))

    def mark_cast_group(self):
        """Called by a model right after registering its first layer's compute copies (and derived
        layouts): those are recast on the current stream, everything registered later on the side
        stream (``refresh``).  Only the first call counts."""
        if self._cast_split is None and os.environ.get("DLMPI_SPLIT_CAST", "1") != "0":   # (0: one launch, A/B)
            self._cast_split = (len(self._entries), len(self.post_refresh))

    def get_compute(self, handle) -> torch.Tensor:
        off, n, dims = handle
        if self._cast_deferred is not None and off >= self._cast_deferred[0][0][1]:
            self.launch_cast()
        ev = self._cast_event
        if ev is not None and off >= ev[1]:
            self.join_cast()
        return self.compute[off:off + n]

    def launch_cast(self):
        """Issue the deferred part of a split recast (every compute copy after the first layer's) on
        the backend's side stream, ordered after the current stream's work so far; the consumers join
        it in ``get_compute``.  A no-op without a deferred part."""
        d = self._cast_deferred
        if d is None:
            return
        self._cast_deferred = None
        rest, p1 = d
        side = getattr(self.backend, "side_stream", None)
        if side is None:   # (the auxiliary streams were turned off meanwhile)
            self.backend.cast_weights(rest, self._compute_total, self.compute)
            for fn in self.post_refresh[p1:]:
                fn()
            return
        cur = torch.cuda.current_stream(self.device)
        side.wait_stream(cur)   # the masters are final (optimizer step) and the old copies read
        torch.cuda.set_stream(side)
        try:
            self.backend.cast_weights(rest, self._compute_total, self.compute)
            for fn in self.post_refresh[p1:]:
                fn()
            ev = torch.cuda.Event()
            ev.record(side)
        finally:
            torch.cuda.set_stream(cur)
        from . import graphs

        self._cast_event = (ev, rest[0][1], graphs.REPLAYS)
        self._cast_waited = []
        self.split_casts += 1

    def join_cast(self):
        """Order the current stream after the side-stream recast (a no-op once it has waited).
        The engine forward joins on its own stream at its end.  A recast from before a hipGraph
        replay or a failed capture (``graphs.REPLAYS`` moved on) is dropped, never waited for: the
        next recast, queued behind it on the same side stream, supersedes it."""
        ev = self._cast_event
        if ev is None:
            return
        from . import graphs

        if ev[2] != graphs.REPLAYS:
            self._cast_event = None
            self._cast_waited = []
            return
        cur = torch.cuda.current_stream(self.device)
        if cur not in self._cast_waited:
            cur.wait_event(ev[0])
            self._cast_waited.append(cur)

    def end_cast(self):
        """Join the recast on the current stream and forget it (end of the engine forward)."""
        self.launch_cast()
        if self._cast_event is not None:
            self.join_cast()
            self._cast_event = None
            self._cast_waited = []

    def _split_lists(self, sp):
        lists = self._cast_lists
        if lists is None or sum(map(len, lists)) != len(self._entries):
            lists = self._cast_lists = (self._entries[:sp[0]], self._entries[sp[0]:])
        return lists

    def _version(self):
        # hipGraph replays update the masters without touching any host-side version counter
        from . import graphs

        return (sum(p._version for p in self.params) + self.flat._version, graphs.REPLAYS)

    def refresh(self, force=False, split=False):
        """Recast all compute copies if any master parameter changed (one kernel launch).  split (the
        engine forward): with a marked first layer and a side stream, only that layer's copies now,
        the rest at ``launch_cast`` on the side stream."""
        if self.compute is None:
            dt = self.backend.act_dtype if self.backend is not None else torch.bfloat16
            self.compute = torch.zeros(max(1, self._compute_total), dtype=dt, device=self.device)
            force = True
        v = self._version()
        if force or v != self._synced_version:
            self.end_cast()   # (a recast still in flight: ordered before this one)
            side = getattr(self.backend, "side_stream", None)
            sp = self._cast_split
            if not split or side is None or sp is None or not 0 < sp[0] < len(self._entries):
                self.backend.cast_weights(self._entries, self._compute_total, self.compute)
                for fn in self.post_refresh:   # derived layouts built from the compute copies
                    fn()
            elif torch.cuda.is_current_stream_capturing():
                # inside a hipGraph capture: both parts on the capturing stream (a capture that failed
                # after forking the side stream into it crashed HIP in the eager fallback; captured
                # steps are the launch-bound ones anyway), with the descriptors the eager steps cached
                # (building one would copy host memory, which a capture refuses)
                lists = self._split_lists(sp)
                self.backend.cast_weights(lists[0], self._compute_total, self.compute)
                for fn in self.post_refresh[:sp[1]]:
                    fn()
                self.backend.cast_weights(lists[1], self._compute_total, self.compute)
                for fn in self.post_refresh[sp[1]:]:
                    fn()
            else:
                lists = self._split_lists(sp)
                self.backend.cast_weights(lists[0], self._compute_total, self.compute)
                for fn in self.post_refresh[:sp[1]]:
                    fn()
                # the rest goes out at launch_cast(): the model calls it where the side-stream recast
                # overlaps compute-bound work (beside the memory-bound input preparation it cost
                # as much as it saved, profiles/r6_recast)
                self._cast_deferred = (lists[1], sp[1])
            self._synced_version = v

    def mark_updated(self):
        self._synced_version = None

    # ------------------------------------------------------------------ buckets
    def buckets(self, first_cap_bytes, cap_bytes, last_cap_bytes=None):
        """Contiguous gradient buckets over the flat buffer (in flat = reverse-registration order).
        Returns (list of (start, end) element ranges, param -> bucket index list).

        first_cap_bytes: the first bucket closes early (its all-reduce starts while most of the
        backward is still ahead).  last_cap_bytes: the tail of the flat order (the network's first
        layers, whose gradients are written last) is split off into a bucket of at most this size,
        so the collective left exposed after the backward pass ends is small."""
        bounds = []
        pb = [0] * len(self.params)
        start = 0
        cur = 0
        cap = first_cap_bytes
        ends = []
        for i in self.order:
            end = self.offsets[i] + self.params[i].numel()
            end = (end + self.ALIGN - 1) // self.ALIGN * self.ALIGN
            ends.append((i, end))
            cur = end
            if (cur - start) * 4 >= cap:
                bounds.append((start, cur))
                start = cur
                cap = cap_bytes
        if cur > start or not bounds:
            bounds.append((start, max(cur, start)))
        if last_cap_bytes and len(ends) > 1:
            s0, e0 = bounds[-1]
            if (e0 - s0) * 4 > last_cap_bytes:
                # smallest parameter boundary inside the last bucket leaving <= last_cap behind it
                cut = next((e for _, e in ends if s0 < e < e0 and (e0 - e) * 4 <= last_cap_bytes), None)
                if cut is not None:
                    bounds[-1] = (s0, cut)
                    bounds.append((cut, e0))
        b = 0
        for i, end in ends:   # bucket of a parameter = the bucket holding its (aligned) end
            while end > bounds[b][1] and b + 1 < len(bounds):
                b += 1
            pb[i] = b
        return bounds, pb
