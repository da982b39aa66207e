"""A whole training step captured in HIP graphs and replayed: one hipGraphLaunch per step
instead of ~250 kernel launches from Python.

Eager, the PointNet++ step's host enqueue (Python + ctypes + ~250 launches, 3.5-5.8 ms on
the boxes measured) is as long as its GPU time, so a slower host makes the step host-bound.
A replay of the captured step costs the host well under a millisecond
(scripts/graph_pieces.py), and the GPU then runs the step back to back.

What capture needs from the step, and how it is provided here:
  * every step-dependent scalar on the device: Adam's bias corrections (FlatAdam keeps its
    step count on the device, pcs_adam_dev), FPS start draws (torch.randint on the device:
    Philox offsets advance per replay), Dropout masks (a fused dropout's host-drawn seed would
    be baked into the graph, so under capture the module's nn.Dropout runs instead);
  * static buffers: the caller's input tensors are read in place (copy the next batch into
    them before `step()`); parameters, gradients, optimizer state and BN statistics are
    updated in place;
  * the next step's neighbour search (FPS / ball query / 3-NN / inverse maps) still runs
    under this step's backward: TWO graphs alternate, graph k consuming geometry plan k and
    computing plan 1-k into that plan's tensors (GeometryPlan(into=...)), so no copies;
  * all side-stream work (geometry stream, wgrad lane) is joined into the capturing stream
    before each capture ends.
Single process only: with torch.distributed, run the step eagerly (the bucketed all-reduce
is issued from backward hooks).
"""
from __future__ import annotations

import torch

from .common import side_stream


class CapturedStep:
    """step() = loss_fn(model(x), labels, lengths).backward(); grads.synchronize(); opt.step()
    -- replayed from HIP graphs.  `grads` is a pcseg.ddp.FlatGradAllReduce (world size 1) and
    `opt` a pcseg.optim.FlatAdam over it.  Returns the step's loss tensor (graph-owned: read
    it before the next step)."""

    def __init__(self, model, x, labels, lengths, grads, opt, loss_fn, logits_of=None, warmup: int = 2,
                 prefetch: bool = True, geometry: str = 'graph'):
        """geometry: 'graph' -- the next step's neighbour search is captured with the step (one
        launch per step); 'eager' -- it is enqueued eagerly on the side stream after each replay
        (the graphs then hold the main-stream work and the wgrad lane only)."""
        if grads.world != 1:
            raise RuntimeError('CapturedStep: single process only (multi-GPU steps run eagerly)')
        self.model, self.x, self.labels, self.lengths = model, x, labels, lengths
        self.grads, self.opt, self.loss_fn = grads, opt, loss_fn
        self.logits_of = logits_of or (lambda o: o[0] if isinstance(o, tuple) else o)
        dev = x.device
        self.dev = dev
        self.prefetch = prefetch and hasattr(model, 'prefetch_geometry')
        if geometry not in ('graph', 'eager'):
            raise ValueError(f"geometry must be 'graph' or 'eager', got {geometry!r}")
        self.geo_eager = self.prefetch and geometry == 'eager'
        main = torch.cuda.current_stream(dev)
        warm = torch.cuda.Stream(dev)
        warm.wait_stream(main)
        with torch.cuda.stream(warm):
            for _ in range(max(warmup, 1)):
                self._eager_step()
            self.plans = []
            if self.prefetch:
                for _ in range(2):          # the two alternating geometry buffers
                    model.prefetch_geometry(x)
                    self.plans.append(model._pcs_prefetched[2])
                model._pcs_prefetched = None
        main.wait_stream(warm)
        torch.cuda.synchronize(dev)
        for p in self.plans:
            p.settle()                       # complete: no cross-graph event waits
        self.captured_lr = opt.lr
        pool = torch.cuda.graph_pool_handle()
        self.graphs, self.losses = [], []
        for k in range(2 if self.prefetch else 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                loss = self._body(k)
            self.graphs.append(g)
            self.losses.append(loss)
        torch.cuda.synchronize(dev)
        self.k = 0
        if self.geo_eager:
            self.prev_done = torch.cuda.Event()
            self.geo_ready = [torch.cuda.Event(), torch.cuda.Event()]
            for e in self.geo_ready:
                e.record(main)

    def _eager_step(self):
        self.grads.zero_grad()
        loss = self.loss_fn(self.logits_of(self.model(self.x)), self.labels, self.lengths)
        loss.backward()
        self.grads.synchronize()
        self.opt.step()
        return loss

    def _body(self, k):
        m, x = self.model, self.x
        if self.prefetch:
            m._pcs_prefetched = (x, x._version, self.plans[k])
        self.grads.zero_grad()
        loss = self.loss_fn(self.logits_of(m(x)), self.labels, self.lengths)
        if self.prefetch and not self.geo_eager:
            # the other buffer's geometry for the next replay, under this backward
            m.prefetch_geometry(x, into=self.plans[1 - k])
        loss.backward()
        self.grads.synchronize()
        self.opt.step()
        if self.prefetch:
            m._pcs_prefetched = None
        if self.prefetch and not self.geo_eager:
            # join the geometry stream the captured prefetch forked (the wgrad lane joins in backward)
            torch.cuda.current_stream(self.dev).wait_stream(side_stream(self.dev))
        return loss

    def step(self) -> torch.Tensor:
        # the captured pcs_adam_dev launch holds the learning rate of capture time: a scheduler
        # that changed opt.lr since would be silently ignored by the replay
        if self.opt.lr != self.captured_lr:
            raise RuntimeError(f'CapturedStep: opt.lr changed from {self.captured_lr} to {self.opt.lr} after '
                               'capture (the replayed Adam step bakes it in); capture a new CapturedStep')
        k = self.k
        if not self.geo_eager:
            self.graphs[k].replay()
            self.k = (k + 1) % len(self.graphs)
            return self.losses[k]
        main = torch.cuda.current_stream(self.dev)
        side = side_stream(self.dev)
        self.prev_done.record(main)                 # the previous replay (the last reader of plan 1-k)
        main.wait_event(self.geo_ready[k])          # this replay's plan, computed under the last one
        self.graphs[k].replay()
        side.wait_event(self.prev_done)
        with torch.cuda.stream(side):
            self.model.prefetch_geometry(self.x, into=self.plans[1 - k])
            self.geo_ready[1 - k].record(side)
        self.model._pcs_prefetched = None
        self.k = 1 - k
        return self.losses[k]
