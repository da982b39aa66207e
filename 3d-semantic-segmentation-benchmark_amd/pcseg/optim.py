"""Adam on flat buffers: one HIP launch per step for the whole model (pcs_adam).

The gradients already live in one flat fp32 buffer (pcseg.ddp.FlatGradAllReduce);
FlatAdam moves the parameters into a second flat buffer with the same layout (every
`param.data` becomes a view into it) and keeps the two moment estimates likewise, so
an optimizer step is a single memory-bound kernel instead of torch.optim.Adam's
~10 foreach launches per parameter group.  Same update and fp32 operation order as
torch.optim.Adam's default path (the reference trains with Adam, lr 1e-3:
Training/train_model.py:263, models/dgcnn/train.py:79).  The step count lives on the device
(pcs_adam_dev derives the bias corrections there), so a training step captured in a HIP
graph (pcseg.graphs) replays with the right corrections.
"""
from __future__ import annotations

import collections
import time

import torch

from ._lib import call, ptr, stream_ptr
from .engine import lane_join


class FlatAdam:
    def __init__(self, grads, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_inflight: int = 3):
        """grads: a pcseg.ddp.FlatGradAllReduce over the model's trainable parameters.

        max_inflight: training steps the host may enqueue ahead of the GPU (0: unbounded).  A
        step's buffers read by the side streams (the wgrad lane, the geometry stream) are held
        by the caching allocator until those streams pass the point where they were freed, so
        a host running N steps ahead holds N steps of them: DGCNN 5 GiB per step, until an
        allocation fails and the allocator frees its whole cache (a multi-second stall,
        profiles/r04_host_runahead.txt).  Each step() waits for the step max_inflight back,
        which leaves the GPU that many steps of queued work."""
        self.grads = grads
        self.max_inflight = int(max_inflight)
        self._inflight: collections.deque = collections.deque()
        self.wait_s = 0.0                        # host seconds spent waiting on the bound
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), tuple(betas), float(eps), float(weight_decay)
        flat_g = grads.flat
        self.flat = torch.zeros_like(flat_g)       # (alignment pads between parameters stay 0)
        base = flat_g.storage_offset()
        with torch.no_grad():
            for p in grads.params:
                off = grads.views[p].storage_offset() - base
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        # {int64 t; float step; float bc2_sqrt} (pcs_adam_dev)
        self.state = torch.zeros(2, dtype=torch.int64, device=self.flat.device)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.grads.zero_grad()

    @property
    def t(self) -> int:
        """Steps taken (a device read: synchronises)."""
        return int(self.state[0])

    @torch.no_grad()
    def step(self) -> None:
        b1, b2 = self.betas
        # the engine's deferred weight gradients are joined at the end of every backward; join
        # again here so no path (e.g. a backward that raised before its final callbacks ran)
        # lets the update read partial gradients
        lane_join(self.flat.device)
        call('pcs_adam_dev', ptr(self.flat), ptr(self.grads.flat), ptr(self.exp_avg), ptr(self.exp_avg_sq),
             self.flat.numel(), 1 - b1, b2, 1 - b2, self.lr, b1, b2, self.eps, self.weight_decay, ptr(self.state),
             stream_ptr(self.flat.device))
        if self.max_inflight > 0 and not torch.cuda.is_current_stream_capturing():
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.device))
            self._inflight.append(ev)
            if len(self._inflight) > self.max_inflight:
                t0 = time.perf_counter()
                while len(self._inflight) > self.max_inflight:
                    self._inflight.popleft().synchronize()
                self.wait_s += time.perf_counter() - t0
