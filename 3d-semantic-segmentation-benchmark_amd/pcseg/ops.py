"""Tensor-level wrappers (torch.autograd.Function) over the HIP C ABI.

Every op runs on the current HIP stream of the input's device and is
allocation-light (outputs come from PyTorch's caching allocator).  Shapes and
devices are validated here, mirroring the reference's ValueError style; a
non-zero ABI status raises RuntimeError with the library's message.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr, check_cuda
from .replay import record_pool_arg


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def radius_sq_f32(r: float) -> float:
    """float32(r ** 2): the threshold the reference compares against (common.py:58)."""
    return float(np.float32(r ** 2))


# ------------------------------------------------------------------ neighbour search (no grad)
def _out(out, shape, dtype, dev):
    """`out` (a preallocated tensor of that shape / dtype, e.g. a graph-resident buffer) or a new one."""
    if out is None:
        return torch.empty(shape, dtype=dtype, device=dev)
    if tuple(out.shape) != tuple(shape) or out.dtype != dtype or not out.is_contiguous():
        raise ValueError(f'out: expected a contiguous {dtype} tensor of shape {tuple(shape)}, got {out.dtype} '
                         f'{tuple(out.shape)}')
    return out


def fps(xyz: torch.Tensor, C: int, start: torch.Tensor, out=None):
    """xyz (B,N,3) -> (idx (B,C) int32, centroids (B,C,3)); out = (idx, centroids) to write into."""
    check_cuda(xyz)
    xyz = _c(xyz.float())
    B, N, _ = xyz.shape
    start = _c(start.to(device=xyz.device, dtype=torch.int32))
    idx = _out(out[0] if out else None, (B, C), torch.int32, xyz.device)
    cent = _out(out[1] if out else None, (B, C, 3), torch.float32, xyz.device)
    call('pcs_fps', ptr(xyz), B, N, C, ptr(start), ptr(idx), ptr(cent), stream_ptr(xyz.device))
    return idx, cent


def ball_query(cent: torch.Tensor, xyz: torch.Tensor, r: float, K: int, out=None) -> torch.Tensor:
    check_cuda(cent, xyz)
    cent, xyz = _c(cent.float()), _c(xyz.float())
    B, C, _ = cent.shape
    N = xyz.shape[1]
    if K > N:
        raise RuntimeError(f'selected index k out of range (K={K} > N={N})')
    out = _out(out, (B, C, K), torch.int32, xyz.device)
    call('pcs_ball_query', ptr(cent), ptr(xyz), B, C, N, radius_sq_f32(r), K, ptr(out), stream_ptr(xyz.device))
    return out


def knn_select(query: torch.Tensor, ref: torch.Tensor, k: int = 3, out=None):
    """(idx (B,N,k) int32, squared dist (B,N,k)) of the k nearest ref points; out = (idx, dist)."""
    check_cuda(query, ref)
    query, ref = _c(query.float()), _c(ref.float())
    B, N, _ = query.shape
    M = ref.shape[1]
    if k > M:
        raise RuntimeError(f'selected index k out of range (k={k} > M={M})')
    idx = _out(out[0] if out else None, (B, N, k), torch.int32, query.device)
    dist = _out(out[1] if out else None, (B, N, k), torch.float32, query.device)
    call('pcs_knn_select', ptr(query), ptr(ref), B, N, M, k, ptr(idx), ptr(dist), stream_ptr(query.device))
    return idx, dist


def knn_order(xyz: torch.Tensor) -> torch.Tensor:
    """Morton order (B, N) int32 of each cloud's points by their first three features (the xyz
    graph's input): the scan order of knn(..., order=)."""
    check_cuda(xyz)
    xyz = _c(xyz.float())
    B, N, Fd = xyz.shape
    order = torch.empty((B, N), dtype=torch.int32, device=xyz.device)
    call('pcs_knn_order', ptr(xyz), B, N, Fd, ptr(order), stream_ptr(xyz.device))
    return order


def knn(x: torch.Tensor, k: int, seeds: torch.Tensor | None = None,
        order: torch.Tensor | None = None) -> torch.Tensor:
    """DGCNN feature-space kNN; x point-major (B,N,F) -> idx (B,N,k) int32.  seeds (B,N,ks)
    int32 (the previous graph) and order (B,N) int32 (knn_order of the cloud's xyz: candidate
    tiles are scanned nearest first and the provably farther ones skipped) only speed the
    search up: the lists are the same."""
    check_cuda(x)
    x = _c(x.float())
    B, N, Fd = x.shape
    out = torch.empty((B, N, k), dtype=torch.int32, device=x.device)
    if seeds is not None:
        if seeds.dtype != torch.int32 or seeds.shape[:2] != (B, N) or seeds.device != x.device:
            raise ValueError(f'knn seeds must be int32 (B, N, ks) on {x.device}, got {seeds.dtype} '
                             f'{tuple(seeds.shape)} on {seeds.device}')
        seeds = _c(seeds)
    if order is not None:
        if order.dtype != torch.int32 or tuple(order.shape) != (B, N) or order.device != x.device:
            raise ValueError(f'knn order must be int32 (B, N) on {x.device}, got {order.dtype} '
                             f'{tuple(order.shape)} on {order.device}')
        order = _c(order)
        nbytes = ctypes.c_size_t()
        call('pcs_knn_pruned_workspace', B, N, Fd, ctypes.byref(nbytes))
        ws = torch.empty(((nbytes.value + 3) // 4,), dtype=torch.float32, device=x.device)
        call('pcs_knn_pruned', ptr(x), B, N, Fd, k, ptr(order), ptr(seeds) if seeds is not None else None,
             seeds.shape[2] if seeds is not None else 0, ptr(out), ptr(ws), ws.numel() * 4, stream_ptr(x.device))
        return out
    ws = torch.empty((B * N + 64,), dtype=torch.float32, device=x.device)    # per-point squared norms
    if seeds is not None:
        call('pcs_knn_seeded', ptr(x), B, N, Fd, k, ptr(seeds), seeds.shape[2], ptr(out), ptr(ws), ws.numel() * 4,
             stream_ptr(x.device))
        return out
    call('pcs_knn_ws', ptr(x), B, N, Fd, k, ptr(out), ptr(ws), ws.numel() * 4, stream_ptr(x.device))
    return out


def inverse_index(idx: torch.Tensor, targets: int, out=None):
    """CSR inverse of a neighbour table idx (B, S, k) int32 with values in [0, targets):
    (offsets (B*targets+1,), entries (B*S*k,)) int32 -- the slots reading each source point,
    ascending.  Feeds the atomic-free, fixed-order gather backward.  out = (offsets, entries)."""
    check_cuda(idx)
    if idx.dtype != torch.int32:
        idx = idx.to(torch.int32)
    idx = _c(idx)
    B = idx.shape[0]
    per = idx[0].numel()
    n, T = B * per, B * targets
    # pcs_inverse_index_workspace: the scatter scratch (n ints) + T counters, each 256-B aligned
    nws = (n * 4 + 255) // 256 * 256 + (T * 4 + 255) // 256 * 256
    if out is None:
        # one int32 allocation: [offsets (T+1) | entries (n) | workspace], 256-B aligned parts
        o_ent = (T + 1 + 63) // 64 * 64
        o_ws = (o_ent + n + 63) // 64 * 64
        buf = torch.empty(o_ws + nws // 4, dtype=torch.int32, device=idx.device)
        offsets, entries, wsp = buf[:T + 1], buf[o_ent:o_ent + n], buf.data_ptr() + 4 * o_ws
    else:
        offsets = _out(out[0], (T + 1,), torch.int32, idx.device)
        entries = _out(out[1], (n,), torch.int32, idx.device)
        ws = torch.empty(nws, dtype=torch.uint8, device=idx.device)
        wsp = ws.data_ptr()
    call('pcs_inverse_index', ptr(idx), B, per, targets, ptr(offsets), ptr(entries), wsp, nws,
         stream_ptr(idx.device))
    return offsets, entries


def inverse_index_batch(tables) -> list:
    """Inverse maps of several neighbour tables in one native call (pcs_inverse_index_batch: 3
    launches for all maps of <= 8192 targets).  tables = [(idx (B, S, k) int32, targets), ...],
    one B for all; returns [(offsets, entries), ...] as inverse_index would, all views of one
    int32 allocation on the current stream."""
    import ctypes
    from ._lib import InverseMap
    B = tables[0][0].shape[0]
    dev = tables[0][0].device
    idxs = []
    for idx, _ in tables:
        check_cuda(idx)
        if idx.shape[0] != B:
            raise ValueError('inverse_index_batch: one batch size for all tables')
        idxs.append(_c(idx if idx.dtype == torch.int32 else idx.to(torch.int32)))
    maps = (InverseMap * len(tables))()
    sizes, o = [], 0
    for i, (idx, (_, T)) in enumerate(zip(idxs, tables)):
        per = idx[0].numel()
        maps[i].per_batch, maps[i].targets = per, T
        sizes.append((o, B * T + 1))
        o += (B * T + 1 + 63) // 64 * 64
        sizes.append((o, B * per))
        o += (B * per + 63) // 64 * 64
    nws = ctypes.c_size_t(0)
    call('pcs_inverse_index_batch_workspace', maps, len(tables), B, ctypes.byref(nws))
    buf = torch.empty(o + (nws.value + 3) // 4, dtype=torch.int32, device=dev)
    out = []
    for i, idx in enumerate(idxs):
        (oo, no), (oe, ne) = sizes[2 * i], sizes[2 * i + 1]
        off, ent = buf[oo:oo + no], buf[oe:oe + ne]
        maps[i].idx, maps[i].offsets, maps[i].entries = idx.data_ptr(), off.data_ptr(), ent.data_ptr()
        out.append((off, ent))
    call('pcs_inverse_index_batch', maps, len(tables), B, buf.data_ptr() + 4 * o, nws.value, stream_ptr(dev))
    return out


# ------------------------------------------------------------------ differentiable gathers
def ld4(n: int) -> int:
    return (n + 3) // 4 * 4


class GroupFn(torch.autograd.Function):
    """(B*C*K, ld) rows [ (xyz[idx]-c) (/r), feats[idx], 0-pad ], ld = 3+D rounded up to 4;
    grad flows to feats only (coords never require grad in the reference)."""

    @staticmethod
    def forward(ctx, xyz, feats, cent, idx, r, normalize, inv=None):
        B, N, _ = xyz.shape
        C, K = idx.shape[1], idx.shape[2]
        D = feats.shape[2] if feats is not None else 0
        ld = ld4(3 + D)
        out = torch.empty((B * C * K, ld), dtype=torch.float32, device=xyz.device)
        call('pcs_group_fwd', ptr(xyz), ptr(feats), ptr(cent), ptr(idx), B, N, C, K, D, float(np.float32(r)),
             int(bool(normalize)), ptr(out), ld, stream_ptr(xyz.device))
        # inv = (offsets, entries) or (offsets, entries, event): the event that covers the map
        # when it is still being built on the geometry stream (GeometryPlan.sa)
        ctx.save_for_backward(idx, *(inv[:2] if inv is not None else ()))
        ctx.inv_event = inv[2] if inv is not None and len(inv) > 2 else None
        ctx.dims = (B, N, C, K, D, ld)
        ctx.has_feats = feats is not None
        ctx.has_inv = inv is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        idx = saved[0]
        B, N, C, K, D, ld = ctx.dims
        gfeats = None
        if ctx.has_feats and ctx.needs_input_grad[1]:
            gout = _c(gout)
            # gather over the inverse map (built here when the forward was not handed one)
            off, ent = saved[1:3] if ctx.has_inv else inverse_index(idx, N)
            if ctx.inv_event is not None:
                torch.cuda.current_stream(gout.device).wait_event(ctx.inv_event)
            gfeats = torch.empty((B, N, D), dtype=torch.float32, device=gout.device)
            call('pcs_group_bwd_csr', ptr(gout), ld, ptr(off), ptr(ent), B, N, D, B * C * K, ptr(gfeats),
                 stream_ptr(gout.device))
        return None, gfeats, None, None, None, None, None


def group_rows(xyz, feats, cent, idx, r, normalize, inv=None):
    """inv: optional inverse_index(idx, N) for the atomic-free backward, optionally with the event
    that covers it as a third element (waited on by the backward before it reads the map)."""
    check_cuda(xyz, cent, idx)
    xyz, cent = _c(xyz.float()), _c(cent.float())
    feats = _c(feats.float()) if feats is not None else None
    return GroupFn.apply(xyz, feats, cent, _c(idx), r, normalize, inv)


class MaxKFn(torch.autograd.Function):
    """x (G*K, Ch) -> (G, Ch) max over K; backward routes to the first argmax."""

    @staticmethod
    def forward(ctx, x, K):
        x = _c(x)
        GK, Ch = x.shape
        G = GK // K
        out = torch.empty((G, Ch), dtype=torch.float32, device=x.device)
        arg = torch.empty((G, Ch), dtype=torch.uint8, device=x.device)
        call('pcs_maxk_fwd', ptr(x), G, K, Ch, ptr(out), ptr(arg), stream_ptr(x.device))
        record_pool_arg(arg)
        ctx.save_for_backward(arg)
        ctx.K = K
        ctx.mark_non_differentiable(arg)
        return out

    @staticmethod
    def backward(ctx, gout):
        (arg,) = ctx.saved_tensors
        gout = _c(gout)
        G, Ch = gout.shape
        gx = torch.empty((G * ctx.K, Ch), dtype=torch.float32, device=gout.device)
        call('pcs_maxk_bwd', ptr(gout), ptr(arg), G, ctx.K, Ch, ptr(gx), stream_ptr(gout.device))
        return gx, None


def maxk(x, K):
    check_cuda(x)
    if x.shape[0] % K:
        raise ValueError('maxk: rows not divisible by K')
    if K > 256:
        raise ValueError('maxk: K > 256 not supported')
    return MaxKFn.apply(x.float(), K)


class InterpCatFn(torch.autograd.Function):
    """rows (B*N, D1+D2) = [f1, IDW-interpolate(f2)] (reference FeaturePropagation.forward)."""

    @staticmethod
    def forward(ctx, f1, f2, idx, dist, inv=None):
        B, M, D2 = f2.shape
        N = idx.shape[1]
        D1 = f1.shape[2] if f1 is not None else 0
        W = D1 + D2
        out = torch.empty((B * N, W), dtype=torch.float32, device=f2.device)
        if D1 % 4 == 0 and D2 % 4 == 0:        # skip copy + interpolation in one pass
            call('pcs_interp_cat_fwd', ptr(f1), D1, ptr(f2), ptr(idx), ptr(dist), B, N, M, D2, ptr(out), W,
                 stream_ptr(f2.device))
        else:
            if f1 is not None:
                out.view(B, N, W)[:, :, :D1].copy_(f1)
            call('pcs_interp_fwd', ptr(f2), ptr(idx), ptr(dist), B, N, M, D2, ptr(out), W, D1, stream_ptr(f2.device))
        ctx.save_for_backward(idx, dist, *(inv if inv is not None else ()))
        ctx.dims = (B, N, M, D1, D2)
        ctx.has_f1 = f1 is not None
        ctx.has_inv = inv is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        idx, dist = saved[0], saved[1]
        B, N, M, D1, D2 = ctx.dims
        gout = _c(gout)
        W = D1 + D2
        g1 = gout.view(B, N, W)[:, :, :D1] if (ctx.has_f1 and ctx.needs_input_grad[0]) else None
        g2 = None
        if ctx.needs_input_grad[1]:
            # gather over the inverse map (built here when the forward was not handed one)
            off, ent = saved[2:4] if ctx.has_inv else inverse_index(idx, M)
            g2 = torch.empty((B, M, D2), dtype=torch.float32, device=gout.device)
            call('pcs_interp_bwd_csr', ptr(gout), W, D1, ptr(dist), ptr(off), ptr(ent), B, M, D2, 3 * B * N,
                 ptr(g2), stream_ptr(gout.device))
        return g1, g2, None, None, None


def interp_cat_rows(f1, f2, idx, dist, inv=None):
    """inv: optional inverse_index(idx, M) for the atomic-free backward."""
    check_cuda(f2, idx, dist)
    f1 = _c(f1.float()) if f1 is not None else None
    return InterpCatFn.apply(f1, _c(f2.float()), _c(idx), _c(dist), inv)


class EdgeFn(torch.autograd.Function):
    """rows (B*N*k, ld) = [x_j - x_i, x_i, 0-pad] (reference get_graph_feature, dgcnn.py:41-53)."""

    @staticmethod
    def forward(ctx, x, idx):
        B, N, D = x.shape
        k = idx.shape[2]
        ld = ld4(2 * D)
        out = torch.empty((B * N * k, ld), dtype=torch.float32, device=x.device)
        call('pcs_edge_fwd', ptr(x), ptr(idx), B, N, k, D, ptr(out), ld, stream_ptr(x.device))
        ctx.save_for_backward(idx)
        ctx.dims = (B, N, k, D, ld)
        return out

    @staticmethod
    def backward(ctx, gout):
        (idx,) = ctx.saved_tensors
        B, N, k, D, ld = ctx.dims
        gout = _c(gout)
        off, ent = inverse_index(idx, N)
        gx = torch.empty((B, N, D), dtype=torch.float32, device=gout.device)
        call('pcs_edge_bwd', ptr(gout), ld, ptr(off), ptr(ent), B, N, k, D, ptr(gx), stream_ptr(gout.device))
        return gx, None


def edge_rows(x, idx):
    check_cuda(x, idx)
    return EdgeFn.apply(_c(x.float()), _c(idx))
