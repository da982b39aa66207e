"""Point-op library and PointNet++ building blocks -- drop-in for the reference's
`models/utils/common.py` (same function/class names, signatures, parameter
names, return conventions), executed by the gfx950 HIP kernels in libpcseg.so.

Internally every activation is point-major rows (rows, channels); the
reference's channel-first permutes become views at the module boundary.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .engine import shared_mlp, pad_rows, module_cache
from ._lib import call, stream_ptr
from .replay import active as _replay


# --------------------------------------------------------------------------- functional API
def _fps_start(B: int, N: int, device) -> torch.Tensor:
    rp = _replay()
    if rp is not None and rp.fps_starts:
        return rp.fps_starts.pop(0).to(device=device, dtype=torch.int32)
    # the reference draws its start exactly like this (common.py:22)
    return torch.randint(0, N, (B,), dtype=torch.int, device=device)


def sample_indices(coords: torch.Tensor, C: int, out=None):
    """FPS -> (idx (B,C) int32, centroid coords (B,C,3)); out = (idx, centroids) to write into."""
    B, N, _ = coords.shape
    start = _fps_start(B, N, coords.device)
    idx, cent = ops.fps(coords, C, start, out=out)
    rp = _replay()
    if rp is not None:
        rp.rec_fps_starts.append(start.detach().cpu())
        rp.rec_fps_idx.append(idx.detach().cpu())
    return idx, cent


def sample(coords: torch.Tensor, C: int) -> torch.Tensor:
    """Reference `sample` (common.py:6-34): farthest point sampling, returns (B, C, 3)."""
    return sample_indices(coords, C)[1]


def _ball(cent, coords, r, K, out=None):
    idx = ops.ball_query(cent, coords, r, K, out=out)
    rp = _replay()
    if rp is not None:
        rp.rec_group_idx.append(idx.detach().cpu())
    return idx


def group(centroid_coords: torch.Tensor, coords: torch.Tensor, features: torch.Tensor, r: float, K: int,
          normalize: bool = False) -> torch.Tensor:
    """Reference `group` (common.py:37-71) -> (B, C, K, 3+D)."""
    B, C, _ = centroid_coords.shape
    idx = _ball(centroid_coords, coords, r, K)
    rows = ops.group_rows(coords, features, centroid_coords, idx, r, normalize)
    D = features.shape[2] if features is not None else 0
    return rows.view(B, C, K, rows.shape[1])[..., :3 + D]


def reduce(x: torch.Tensor, type: str) -> torch.Tensor:
    """Reference `reduce` (common.py:74-91).  x (B, C, K, D') -> (B, C, D')."""
    if type == 'max':
        B, C, K, D = x.shape
        return ops.maxk(x.reshape(B * C * K, D), K).view(B, C, D)
    if type == 'avg':
        # kept bug-compatible with the reference (common.py:89 indexes [0] after the mean)
        return torch.mean(x, dim=2)[0]
    raise ValueError(f"'{type}' pooling not supported; use 'max' or 'avg'.")


def interpolate(points: torch.Tensor, coords_1: torch.Tensor, coords_2: torch.Tensor, k: int = 3) -> torch.Tensor:
    """Reference `interpolate` (common.py:94-122) -> (B, N, D).  k == 3 as in the reference's callers."""
    if k != 3:
        raise ValueError('pcseg interpolate supports k=3 (the reference default)')
    B, N, _ = coords_1.shape
    idx, dist = ops.knn_select(coords_1, coords_2, 3)
    rp = _replay()
    if rp is not None:
        rp.rec_interp_idx.append(idx.detach().cpu())
    return ops.interp_cat_rows(None, points, idx, dist).view(B, N, points.shape[2])


# --------------------------------------------------------------------------- geometry on a side stream
_side_streams: dict = {}
_plan_ws: dict = {}          # native geometry plan workspace bytes per plan structure
_events: dict = {}           # device -> ring of event sets for the native plans


def _event_set(dev, side, L):
    """L + 1 torch events (per level + after the 3-NN) from a small per-device ring, created and
    recorded once so that their raw handles exist; the native plan re-records them.  A plan's
    waits are enqueued by the forward that consumes it, before the ring comes round again."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ring = _events.get(key)
    if ring is None or len(ring[0][0]) < L + 1:
        sets = []
        for _ in range(4):
            evs = [torch.cuda.Event() for _ in range(max(L, 6) + 1)]
            for e in evs:
                e.record(side)
            sets.append(evs)
        ring = _events[key] = [sets, 0]
    sets, i = ring
    ring[1] = (i + 1) % len(sets)
    return sets[i]


def side_stream(device) -> torch.cuda.Stream:
    """One long-lived side stream per device for the neighbour-search work: the library's
    geometry stream (pcs_geometry_stream), at normal priority -- below the bench's high-priority
    step stream, so the queue scheduler hands free compute units to the step's kernels first
    (the lowest priority measured neutral, profiles/r05_ab_geometry_blocks.txt)."""
    import ctypes
    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _side_streams.get(key)
    if st is None:
        out = ctypes.c_void_p(0)
        with torch.cuda.device(key):
            call('pcs_geometry_stream', ctypes.byref(out))
        st = torch.cuda.ExternalStream(out.value, device=torch.device('cuda', key))
        _side_streams[key] = st
    return st


class GeometryPlan:
    """All neighbour structure of one PointNet++-family forward, enqueued up front
    on a side stream so it overlaps the shared-MLP work of the main stream.

    The geometry depends on coordinates only: level l's centroids are FPS of
    level l-1's (reference SetAbstraction.forward, common.py:204-206), its ball
    queries group them against level l-1 (SA) or against themselves (InvResMLP,
    common.py:288), and FeaturePropagation's 3-NN pairs adjacent levels
    (common.py:107-114).  `levels` = [(C, [(r, K, on_self), ...]), ...] in the
    reference's call order, so FPS start draws and replay records keep the
    reference's sequence.  Consumers wait on the per-level event before reading.
    """

    def __init__(self, coords: torch.Tensor, levels, interp: bool = True, inverse: bool = True,
                 into: 'GeometryPlan | None' = None):
        """into: a plan of the same structure whose tensors this one writes into (no allocation:
        the double-buffered plans of a HIP-graph-captured training step, pcseg.graphs)."""
        dev = coords.device
        main = torch.cuda.current_stream(dev)
        side = side_stream(dev)
        side.wait_stream(main)
        self.coords = [coords]
        self.balls, self.events, self.nn = [], [], []
        made = []
        self.inverse = inverse
        self.fps_idx = []
        # the native plan builds every inverse map after the last 3-NN when it has both: the
        # level events then do not cover the ball queries' maps, nn_event does (see sa())
        self._maps_late = _replay() is None and bool(interp) and bool(inverse)
        if _replay() is None:
            # one native call (pcs_geometry_plan): same kernels, same order, same RNG draws
            self._build_native(coords, levels, interp, inverse, into, main, side)
            return
        with torch.cuda.stream(side):
            prev = coords
            for lv, (C, queries) in enumerate(levels):
                fo = (into.fps_idx[lv], into.coords[lv + 1]) if into is not None else None
                fidx, cent = sample_indices(prev, C, out=fo)
                self.fps_idx.append(fidx)
                bl = []
                for q, (r, K, on_self) in enumerate(queries):
                    src = cent if on_self else prev
                    ib, iv = into.balls[lv][q] if into is not None else (None, None)
                    idx = _ball(cent, src, r, K, out=ib)
                    # inverse map for the atomic-free backward of the feature gather
                    inv = ops.inverse_index(idx, src.shape[1], out=iv) if inverse else None
                    bl.append((idx, inv))
                    made += [idx, *(inv or ())]
                ev = torch.cuda.Event()
                ev.record(side)
                self.coords.append(cent)
                self.balls.append(bl)
                self.events.append(ev)
                made += [fidx, cent]
                prev = cent
            if interp:
                nn_ = []
                for lv in range(len(levels) - 1, -1, -1):      # FP_L ... FP_1, the reference's order
                    no = into.nn[lv] if into is not None else (None, None, None)
                    idx, dist = ops.knn_select(self.coords[lv], self.coords[lv + 1], 3,
                                               out=(no[0], no[1]) if into is not None else None)
                    rp = _replay()
                    if rp is not None:
                        rp.rec_interp_idx.append(idx.detach().cpu())
                    inv = ops.inverse_index(idx, self.coords[lv + 1].shape[1], out=no[2]) if inverse else None
                    nn_.append((idx, dist, inv))
                    made += [idx, dist, *(inv or ())]
                self.nn = nn_[::-1]                             # nn[lv] pairs level lv with lv + 1
                self.nn_event = torch.cuda.Event()
                self.nn_event.record(side)
        if not torch.cuda.is_current_stream_capturing():
            # eager: tell the caching allocator about the cross-stream uses (under graph capture
            # the tensors are the `into` plan's, which outlives the graphs)
            coords.record_stream(side)
            for t in made:
                t.record_stream(main)

    def _build_native(self, coords, levels, interp, inverse, into, main, side):
        import ctypes
        from ._lib import GeoLevel, QMAX
        dev = coords.device
        if coords.dtype != torch.float32 or not coords.is_contiguous():
            coords = coords.float().contiguous()
            self.coords[0] = coords
        B, N, _ = coords.shape
        L = len(levels)
        if L > 6 or any(len(q) > QMAX for _, q in levels):
            raise ValueError('GeometryPlan: at most 6 levels of at most 4 ball queries')
        recs = (GeoLevel * L)()
        sizes = []                       # every output, int32 units, in a fixed order
        prev = N
        for l, (C, queries) in enumerate(levels):
            r = recs[l]
            r.C, r.nq = C, len(queries)
            sizes += [B * C, B * C * 3]
            for q, (rad, K, on_self) in enumerate(queries):
                r.r2[q] = ops.radius_sq_f32(rad)
                r.K[q], r.on_self[q] = K, int(bool(on_self))
                src = C if on_self else prev
                sizes += [B * C * K] + ([B * src + 1, B * C * K] if inverse else [])
            if interp:
                sizes += [B * prev * 3, B * prev * 3] + ([B * C + 1, B * prev * 3] if inverse else [])
            prev = C
        key = (B, N, tuple((C, tuple(qs)) for C, qs in levels), bool(interp), bool(inverse))
        nws = _plan_ws.get(key)
        if nws is None:
            out = ctypes.c_size_t(0)
            call('pcs_geometry_plan_workspace', B, N, recs, L, int(interp), int(inverse), ctypes.byref(out))
            nws = _plan_ws[key] = int(out.value)
        offs, o = [], 0
        for n in sizes:
            offs.append(o)
            o += (n + 63) // 64 * 64
        wso = o
        if into is None:
            buf = torch.empty(wso + (nws + 3) // 4, dtype=torch.int32, device=dev)
        else:
            # the plan's native scratch (inverse-map counters) lives as long as the plan it writes
            # into: under HIP-graph capture a block freed at the end of this call would be handed
            # to the step's later main-stream allocations while the side branch still writes it
            buf = into.__dict__.get('_pcs_scratch')
            if buf is None or buf.numel() < (nws + 3) // 4:
                buf = into._pcs_scratch = torch.empty((nws + 3) // 4, dtype=torch.int32, device=dev)
        parts = iter(zip(offs, sizes))
        evs = _event_set(dev, side, L)

        def take():
            off, n = next(parts)
            return buf[off:off + n]
        prev = N
        for l, (C, queries) in enumerate(levels):
            r = recs[l]
            if into is None:
                fidx, cent = take().view(B, C), take().view(torch.float32).view(B, C, 3)
            else:
                fidx, cent = into.fps_idx[l], into.coords[l + 1]
            r.fps_idx, r.cent = fidx.data_ptr(), cent.data_ptr()
            bl = []
            for q, (rad, K, on_self) in enumerate(queries):
                src = C if on_self else prev
                if into is None:
                    idx = take().view(B, C, K)
                    inv = (take(), take()) if inverse else None
                else:
                    idx, inv = into.balls[l][q]
                r.ball[q] = idx.data_ptr()
                if inv is not None:
                    r.ball_off[q], r.ball_ent[q] = inv[0].data_ptr(), inv[1].data_ptr()
                bl.append((idx, inv))
            if interp:
                if into is None:
                    nidx, ndist = take().view(B, prev, 3), take().view(torch.float32).view(B, prev, 3)
                    ninv = (take(), take()) if inverse else None
                else:
                    nidx, ndist, ninv = into.nn[l]
                r.nn_idx, r.nn_dist = nidx.data_ptr(), ndist.data_ptr()
                if ninv is not None:
                    r.nn_off, r.nn_ent = ninv[0].data_ptr(), ninv[1].data_ptr()
                self.nn.append((nidx, ndist, ninv))
            r.event = evs[l].cuda_event
            self.fps_idx.append(fidx)
            self.coords.append(cent)
            self.balls.append(bl)
            self.events.append(evs[l])
            prev = C
        if interp:
            self.nn_event = evs[L]
        with torch.cuda.stream(side):
            # the FPS starts: one torch.randint per level, as sample_indices draws them
            npts = [N] + [C for C, _ in levels[:-1]]
            starts = torch.stack([_fps_start(B, n, dev) for n in npts])
            call('pcs_geometry_plan', coords.data_ptr(), B, N, starts.data_ptr(), recs, L, int(interp),
                 int(inverse), evs[L].cuda_event if interp else None, buf.data_ptr() + 4 * (wso if into is None else 0),
                 nws, stream_ptr(dev))
        if not torch.cuda.is_current_stream_capturing():
            # buf is allocated on the main stream and WRITTEN by the side stream: a plan that is
            # dropped unread (a stale prefetch) must not hand buf back to the main stream's pool
            # while the side stream's kernels still write it
            coords.record_stream(side)
            if into is None:
                buf.record_stream(side)

    @staticmethod
    def _wait(ev):
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    def tensors(self) -> list:
        """Every tensor of the plan, in a fixed order (same structure -> same list layout)."""
        out = list(self.coords)
        for bl in self.balls:
            for idx, inv in bl:
                out += [idx, *(inv or ())]
        for idx, dist, inv in self.nn:
            out += [idx, dist, *(inv or ())]
        return out

    def settle(self) -> None:
        """Forget the side-stream events once the plan is known complete (after a device
        synchronize): a plan built outside a HIP-graph capture can then be read inside one."""
        self.events = [None] * len(self.events)
        if hasattr(self, 'nn_event'):
            self.nn_event = None

    def copy_from(self, other: 'GeometryPlan') -> None:
        """Overwrite this plan's tensors with `other`'s (same levels and sizes) on the current
        stream, after other's side-stream work: the double buffer of a graph-captured step,
        whose forward reads this plan while it computes the next one."""
        for ev in other.events:
            self._wait(ev)
        self._wait(getattr(other, 'nn_event', None))
        mine, theirs = self.tensors(), other.tensors()
        if len(mine) != len(theirs) or any(a.shape != b.shape for a, b in zip(mine, theirs)):
            raise ValueError('GeometryPlan.copy_from: plans of different structure')
        for a, b in zip(mine, theirs):
            a.copy_(b)

    def sa(self, level: int, q: int = 0):
        """(centroids, ball idx, inverse map or None) of level >= 1 for its q-th query.  Waits for
        the level's event, which covers the centroids and the ball idx.  The inverse map is read
        only by the gather's backward; where the native plan builds the maps after every 3-NN
        (interp and inverse, geometry.hip) the level event does not cover it, so it comes as
        (offsets, entries, event) with the event that does (nn_event), and ops.GroupFn's backward
        waits on that event before reading it.  Otherwise it is (offsets, entries)."""
        self._wait(self.events[level - 1])
        idx, inv = self.balls[level - 1][q]
        if inv is not None and self._maps_late:
            inv = (inv[0], inv[1], self.nn_event)
        return self.coords[level], idx, inv

    def fp(self, level: int):
        """(idx, dist, inverse map or None) of the 3-NN from level `level` into level `level + 1`."""
        self._wait(self.nn_event)
        return self.nn[level]


class GeometryPrefetch:
    """Mixin: `model.prefetch_geometry(x)` enqueues the GeometryPlan of a future
    forward(x) now (e.g. before the previous step's backward), so FPS / ball
    query / 3-NN of the next batch overlap that backward.  The next forward with
    the same, unmodified tensor consumes it; anything else recomputes."""

    def prefetch_geometry(self, x: torch.Tensor, into: GeometryPlan | None = None) -> None:
        """into: write the plan into an existing plan's tensors (see GeometryPlan)."""
        self._pcs_prefetched = (x, x._version, self._plan_for(self._coords_of(x), into=into))

    def prefetch_geometry_in_backward(self, x: torch.Tensor) -> None:
        """Arm a prefetch for the NEXT forward: it hooks the gradient of a mid-network
        activation (the input of the last FeaturePropagation) so that prefetch_geometry(x) is
        enqueued from the backward, once the head's and FP1's backward GEMMs are already queued
        on the GPU.  Enqueued between the loss and backward() instead, the ~25 Python-level
        geometry launches leave the GPU idle: the forward has drained its queue by then."""
        self._pcs_prefetch_armed = x

    def prefetch_geometry_at_start(self, x: torch.Tensor) -> None:
        """Arm a prefetch for the NEXT forward that is enqueued as soon as THIS forward has taken
        its own (prefetched) plan: the next batch's FPS then runs under this forward and backward."""
        self._pcs_prefetch_next = x

    def _prefetch_point(self, t: torch.Tensor) -> torch.Tensor:
        x = getattr(self, '_pcs_prefetch_armed', None)
        if x is not None and torch.is_grad_enabled() and t.requires_grad:
            self._pcs_prefetch_armed = None
            dev = t.device

            def hook(_grad, x=x):
                with torch.cuda.device(dev):
                    self.prefetch_geometry(x)
            t.register_hook(hook)
        return t

    def _geometry(self, x: torch.Tensor, coords: torch.Tensor) -> GeometryPlan:
        pf = getattr(self, '_pcs_prefetched', None)
        self._pcs_prefetched = None
        if pf is not None and pf[0] is x and pf[1] == x._version:
            plan = pf[2]
        else:
            # the inverse maps serve only the backward of the gathers: none under no_grad (eval)
            plan = self._plan_for(coords, inverse=torch.is_grad_enabled())
        nxt = getattr(self, '_pcs_prefetch_next', None)
        if nxt is not None:
            self._pcs_prefetch_next = None
            self.prefetch_geometry(nxt)
        return plan

    @staticmethod
    def _coords_of(x: torch.Tensor) -> torch.Tensor:
        return x[:, :, :3].contiguous()


# --------------------------------------------------------------------------- MLP blocks
class MiniPointNet(nn.Module):
    """Reference common.py:125-150 (Conv2d 1x1 -> BatchNorm2d -> ReLU)."""

    def __init__(self, in_channels: int, mlps: list[int]):
        super().__init__()
        self.conv = nn.ModuleList()
        self.batch = nn.ModuleList()
        prev = in_channels
        for m in mlps:
            self.conv.append(nn.Conv2d(prev, m, (1, 1)))
            self.batch.append(nn.BatchNorm2d(m))
            prev = m
        self.bwd_fuse = 0           # backward kernel choice (pcseg.engine.set_bwd_fuse)

    def forward_rows(self, x: torch.Tensor, kin: int | None = None, pool_k: int = 0, dx_from: int = 0) -> torch.Tensor:
        """rows (M, ld) -> (M, C_L), or (M/pool_k, C_L) max-pooled over consecutive groups of pool_k rows.
        dx_from: the first input column whose gradient is wanted (3 for grouped rows: their relative
        coordinates need none)."""
        return shared_mlp(x, kin or x.shape[1], self.conv, self.batch, 'relu', 0.0, pool_k, bwd_fuse=self.bwd_fuse,
                          cache=module_cache(self), dx_from=dx_from)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, Cin, H, W = x.shape
        rows = x.permute(0, 2, 3, 1).reshape(B * H * W, Cin)
        return self.forward_rows(pad_rows(rows), Cin).view(B, H, W, -1).permute(0, 3, 1, 2)


class UnitPointNet(nn.Module):
    """Reference common.py:153-178 (Conv1d 1x1 -> BatchNorm1d -> ReLU)."""

    def __init__(self, in_channels: int, mlps: list[int]):
        super().__init__()
        self.conv = nn.ModuleList()
        self.batch = nn.ModuleList()
        prev = in_channels
        for m in mlps:
            self.conv.append(nn.Conv1d(prev, m, 1))
            self.batch.append(nn.BatchNorm1d(m))
            prev = m
        self.bwd_fuse = 0           # backward kernel choice (pcseg.engine.set_bwd_fuse)

    def forward_rows(self, x: torch.Tensor, kin: int | None = None, dropout: tuple | None = None,
                     dx_from: int = 0) -> torch.Tensor:
        """dropout = (p, seed): a training-mode Dropout after the stack, fused into its output.
        dx_from: the first input column whose gradient is wanted (pcs_mlp_layer.dx_col0)."""
        return shared_mlp(x, kin or x.shape[1], self.conv, self.batch, 'relu', 0.0, 0, dropout=dropout,
                          bwd_fuse=self.bwd_fuse, cache=module_cache(self), dx_from=dx_from)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, Cin, N = x.shape
        rows = x.permute(0, 2, 1).reshape(B * N, Cin)
        return self.forward_rows(pad_rows(rows), Cin).view(B, N, -1).permute(0, 2, 1)


class SetAbstraction(nn.Module):
    """Reference common.py:180-214: FPS -> ball query + group -> shared MLP -> max over K."""

    def __init__(self, C: int, radius: float, in_channels: int, mlps: list[int], K: int = 32,
                 pooling_type: str = 'max', grouping_norm: bool = False):
        super().__init__()
        self.point_net = MiniPointNet(in_channels, mlps)
        self.C = C
        self.radius = radius
        self.K = K
        self.pooling_type = pooling_type
        self.grouping_norm = grouping_norm

    def forward(self, coords: torch.Tensor, features: torch.Tensor,
                geo: tuple | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        """geo = (centroids, ball idx) precomputed by a GeometryPlan, else computed here."""
        B = coords.shape[0]
        inv = None
        if geo is None:
            _, cent = sample_indices(coords, self.C)
            idx = _ball(cent, coords, self.radius, self.K)
        else:
            cent, idx = geo[0], geo[1]
            inv = geo[2] if len(geo) > 2 else None
        rows = ops.group_rows(coords, features, cent, idx, self.radius, self.grouping_norm, inv)
        kin = 3 + features.shape[2]
        if self.pooling_type == 'max':
            out = self.point_net.forward_rows(rows, kin, pool_k=self.K, dx_from=3).view(B, self.C, -1)
        else:
            act = self.point_net.forward_rows(rows, kin, dx_from=3)
            out = reduce(act.view(B, self.C, self.K, -1), self.pooling_type)
        return cent, out


class FeaturePropagation(nn.Module):
    """Reference common.py:217-243: 3-NN IDW interpolation, concat skip, shared MLP."""

    def __init__(self, in_channels: int, mlps: list[int]):
        super().__init__()
        self.point_net = UnitPointNet(in_channels, mlps)

    def forward(self, coords_1: torch.Tensor, coords_2: torch.Tensor, features_1: torch.Tensor | None,
                features_2: torch.Tensor, geo: tuple | None = None, dropout: tuple | None = None) -> torch.Tensor:
        """geo = (3-NN idx, squared dist) precomputed by a GeometryPlan, else computed here;
        dropout = (p, seed): the model head's training-mode Dropout, fused into the MLP output."""
        B, N, _ = coords_1.shape
        inv = None
        if geo is None:
            idx, dist = ops.knn_select(coords_1, coords_2, 3)
            rp = _replay()
            if rp is not None:
                rp.rec_interp_idx.append(idx.detach().cpu())
        else:
            idx, dist = geo[0], geo[1]
            inv = geo[2] if len(geo) > 2 else None
        rows = ops.interp_cat_rows(features_1, features_2, idx, dist, inv)
        return self.point_net.forward_rows(rows, dropout=dropout).view(B, N, -1)


class InvResMLP(nn.Module):
    """Reference common.py:246-301: group (C=N, normalised) -> 1-layer MLP -> max -> 2-layer MLP -> + residual."""

    def __init__(self, radius: int, in_channels: int, mlp_size: int, K: int, pooling_type: str = 'max'):
        super().__init__()
        self.radius = radius
        self.K = K
        self.pooling_type = pooling_type
        self.neighbour_features_mlp = MiniPointNet(in_channels, [mlp_size])
        self.point_features_mlp = UnitPointNet(mlp_size, [4 * mlp_size, mlp_size])

    def forward(self, centroid_coords: torch.Tensor, coords: torch.Tensor,
                features: torch.Tensor, geo=None) -> tuple[torch.Tensor, torch.Tensor]:
        """geo = ball idx (or (idx, inverse map)) precomputed by a GeometryPlan, else computed here."""
        B, C, _ = centroid_coords.shape
        inv = None
        if geo is None:
            idx = _ball(centroid_coords, coords, self.radius, self.K)
        elif isinstance(geo, torch.Tensor):
            idx = geo
        else:
            idx, inv = geo
        rows = ops.group_rows(coords, features, centroid_coords, idx, self.radius, True, inv)
        kin = 3 + features.shape[2]
        if self.pooling_type == 'max':
            pooled = self.neighbour_features_mlp.forward_rows(rows, kin, pool_k=self.K, dx_from=3)
        else:
            act = self.neighbour_features_mlp.forward_rows(rows, kin, dx_from=3)
            pooled = reduce(act.view(B, C, self.K, -1), self.pooling_type).reshape(B * C, -1)
        out = self.point_features_mlp.forward_rows(pooled).view(B, C, -1)
        return centroid_coords, out + features
