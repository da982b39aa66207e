"""Data-parallel training over RCCL (torch.distributed backend "nccl" on ROCm).

S3DIS blocks are independent samples, so the only exchange step is the
gradient all-reduce after backward.  Gradients live in ONE flat
fp32 buffer (every `param.grad` is a view into it), split into a few
contiguous buckets that are all-reduced as soon as autograd has produced every
gradient in them -- overlapping the collective with the rest of backward on
RCCL's own stream.  BatchNorm statistics are computed locally per rank (DDP's
default; the reference has no SyncBN); parameters are broadcast from rank 0 once and,
as DDP's `broadcast_buffers=True` does, rank 0's buffers (BN running statistics) are
broadcast to every rank at the start of each training forward -- coalesced into one
flat buffer per dtype, so that is one or two collectives per step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import wgrad_lane, lane_join


def broadcast_model(model: torch.nn.Module, src: int = 0) -> None:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src)


def _align(n: int) -> int:
    return (n + 63) // 64 * 64


class FlatBuffers:
    """Every buffer of a model (BN running mean / var, num_batches_tracked) rebound as a view
    of one flat tensor per dtype, so rank 0's buffers reach every rank in one broadcast per
    dtype (DDP `broadcast_buffers` semantics).  The HIP engine updates running statistics in
    place through their pointers, which the views keep."""

    def __init__(self, model: torch.nn.Module):
        groups: dict = {}
        for mod in model.modules():
            for name, b in mod._buffers.items():
                if b is not None:
                    groups.setdefault(b.dtype, []).append((mod, name, b))
        self.flats = []
        for dtype, items in groups.items():
            flat = torch.empty(sum(b.numel() for _, _, b in items), dtype=dtype, device=items[0][2].device)
            off = 0
            for mod, name, b in items:
                n = b.numel()
                view = flat[off:off + n].view_as(b)
                view.copy_(b)
                mod._buffers[name] = view
                off += n
            self.flats.append(flat)

    def broadcast(self, src: int = 0) -> None:
        for f in self.flats:
            dist.broadcast(f, src)


class FlatGradAllReduce:
    """Flat gradient buffer + bucketed, backward-overlapped all-reduce (mean)."""

    def __init__(self, model: torch.nn.Module, bucket_bytes: int = 4 << 20, overlap: bool = True,
                 broadcast_buffers: bool = True, collectives_at_world_1: bool = False):
        """collectives_at_world_1: run the bucket all-reduces even in a world of one process (an
        identity there: the sum of one rank's buffer, divided by 1) -- exercises RCCL's stream
        ordering against the engine's wgrad lane on a single GPU (tests/test_gpu_rccl.py)."""
        self.params = [p for p in model.parameters() if p.requires_grad]
        # every parameter (and its gradient) starts on a 256-B boundary of the flat buffers: the
        # wide GEMMs stage weights by 16-B LDS-DMA and take only aligned operands
        total = sum(_align(p.numel()) for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.collective = self.world > 1 or (collectives_at_world_1 and dist.is_initialized())
        # buckets are laid out in REVERSE parameter order: backward produces the
        # last layers' gradients first, so the first bucket completes earliest.
        order = list(reversed(self.params))
        self.views = {}
        off = 0
        self.buckets: list[tuple[int, int, list[torch.nn.Parameter]]] = []
        cur_start, cur = 0, []
        for p in order:
            n = p.numel()
            self.views[p] = self.flat[off:off + n].view_as(p)
            cur.append(p)
            off += _align(n)
            if (off - cur_start) * 4 >= bucket_bytes:
                self.buckets.append((cur_start, off, cur))
                cur_start, cur = off, []
        if cur:
            self.buckets.append((cur_start, off, cur))
        self._bucket_of = {p: i for i, (_, _, ps) in enumerate(self.buckets) for p in ps}
        self._pending = [len(ps) for _, _, ps in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._seen: set[int] = set()
        self._handles: list = []
        self.overlap = overlap and self.collective
        self.buffers = None
        if broadcast_buffers and self.world > 1 and any(True for _ in model.buffers()):
            # DDP broadcast_buffers: rank 0's buffers at the start of every training forward
            self.buffers = FlatBuffers(model)
            model.register_forward_pre_hook(self._pre_forward)
        self.attach()
        if self.overlap:
            for p in self.params:
                # autograd-accumulated params fire the post-accumulate hook; params whose
                # gradients the HIP engine writes in place call _pcs_grad_ready instead
                p.register_post_accumulate_grad_hook(self._hook)
                p._pcs_grad_ready = self._hook

    def _pre_forward(self, module, inputs) -> None:
        if module.training and torch.is_grad_enabled():
            self.buffers.broadcast()

    def attach(self) -> None:
        """(Re)bind every param.grad to its view of the flat buffer."""
        for p in self.params:
            p.grad = self.views[p]

    def _reset(self) -> None:
        self._pending = [len(ps) for _, _, ps in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._seen = set()
        self._handles = []

    def zero_grad(self) -> None:
        self.flat.zero_()
        self.attach()
        self._reset()

    def _hook(self, p: torch.Tensor) -> None:
        # A parameter may be announced twice: by the HIP engine (which writes .grad in place)
        # and by autograd's post-accumulate hook, which still fires for it with an undefined
        # gradient.  Count each parameter once per step.
        if id(p) in self._seen:
            return
        self._seen.add(id(p))
        b = self._bucket_of[p]
        self._pending[b] -= 1
        if self._pending[b] == 0 and not self._launched[b]:
            s, e, _ = self.buckets[b]
            self._launched[b] = True
            lane = wgrad_lane(self.flat.device) if self.flat.is_cuda else None
            if lane is None:
                self._handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))
            else:
                # the bucket's weight gradients may still be running on the engine's wgrad lane
                # (pcs_mlp_backward_deferred): issue the reduction behind both the lane and the
                # current stream, without making the current stream wait for the lane
                lane.wait_stream(torch.cuda.current_stream(self.flat.device))
                with torch.cuda.stream(lane):
                    self._handles.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, async_op=True))

    def synchronize(self) -> None:
        """Finish all bucket reductions and average (call before optimizer.step())."""
        if self.flat.is_cuda:
            lane_join(self.flat.device)      # every deferred weight gradient is written
        if not self.collective:
            return
        if self.overlap:
            for h in self._handles:
                h.wait()
            # any bucket not launched from backward (unused params) is reduced now
            for b, (s, e, _) in enumerate(self.buckets):
                if not self._launched[b]:
                    dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM)
        else:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
        if self.world > 1:
            self.flat.div_(self.world)
        self._reset()
