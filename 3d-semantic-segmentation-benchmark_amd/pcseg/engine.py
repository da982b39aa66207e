"""Shared-MLP engine: a stack of (1x1 conv -> training-mode BN -> ReLU/LeakyReLU)
layers on point-major rows, optionally max-pooled over groups of K rows, run
entirely by the HIP kernels of csrc/mlp.hip (MFMA fp32 GEMMs with fused BN
statistics / BN-apply / pooling, fp64 statistics).

Reference semantics: MiniPointNet / UnitPointNet (models/utils/common.py:125-178)
followed by `reduce(..., 'max')` (common.py:211-212), EdgeConv
(models/dgcnn/dgcnn.py:67-76), DGCNN conv5..conv7 (dgcnn.py:188-207).

Only pre-BN activations Z are kept for backward; the BN-applied activation of
layer l is recomputed inside layer l+1's GEMM A-load, so it never touches HBM.
Backward mirrors it: a layer's dZ (the BatchNorm-backward of its output
gradient) is rebuilt on load by both consumers (weight-gradient and data-
gradient GEMMs) from the output gradient and Z, so it is never stored either.
"""
from __future__ import annotations

import collections
import ctypes
import math
import struct
import time

import torch

from ._lib import call, load, ptr, stream_ptr, Operand, OP_PLAIN, OP_BNACT, OP_BNBWD, OP_POOLBWD
from .replay import record_pool_arg, record_act_mask, recording

ACT = {'relu': 0, 'lrelu': 1, 'none': 2}


def ld4(n: int) -> int:
    return (n + 3) // 4 * 4


def pad_rows(x: torch.Tensor) -> torch.Tensor:
    """(M, C) -> contiguous rows with a stride that is a multiple of 4 (zero pad)."""
    M, C = x.shape
    ld = ld4(C)
    if ld == C and x.is_contiguous():
        return x
    out = torch.zeros((M, ld), dtype=torch.float32, device=x.device)
    out[:, :C] = x
    return out


def grad_target(p: torch.Tensor | None) -> torch.Tensor | None:
    """The buffer the engine accumulates p's gradient into (p.grad itself, created zeroed if absent).

    The engine writes parameter gradients directly (fp32 atomics / accumulate flag) instead
    of returning them, so autograd issues no AccumulateGrad add (and no zero fill) per
    parameter; hooks registered through `_pcs_grad_ready` (pcseg.ddp) are called after.
    """
    if p is None or not p.requires_grad:
        return None
    g = p.grad
    if g is None:
        g = torch.zeros_like(p, memory_format=torch.contiguous_format)
        p.grad = g
    elif not g.is_contiguous() or g.dtype != torch.float32:
        raise RuntimeError('pcseg engine: parameter .grad must be a contiguous fp32 tensor')
    return g


def grad_targets(params) -> list:
    """grad_target of every parameter, the missing gradients created as views of ONE zeroed
    buffer (one fill launch per stack call instead of one per parameter: an optimizer's
    zero_grad(set_to_none=True), the harness default, leaves every .grad None each step)."""
    need = [p for p in params if p is not None and p.requires_grad and p.grad is None]
    if len(need) > 1:
        flat = torch.zeros(sum(p.numel() for p in need), dtype=torch.float32, device=need[0].device)
        off = 0
        for p in need:
            if p.dtype != torch.float32:
                raise RuntimeError('pcseg engine: parameters must be fp32')
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
    return [grad_target(p) for p in params]


def notify_grad_ready(params) -> None:
    for p in params:
        if p is not None:
            cb = getattr(p, '_pcs_grad_ready', None)
            if cb is not None:
                cb(p)


# --------------------------------------------------------------------------- launch probe
class KernelProbe:
    """Bracket every engine GEMM launch with HIP events on the stream it runs on.

    Inside `with KernelProbe() as kp:` each pcs_gemm_rows / pcs_wgrad launch -- also
    those issued natively inside pcs_mlp_forward / pcs_mlp_backward -- is recorded by
    the library's launch probe (csrc/probe.cpp) as (kernel name as rocprof reports it,
    algorithmic flops, algorithmic bytes, elapsed time).  Used by bench.py's roofline.
    """

    def __enter__(self):
        call('pcs_probe_begin')
        self.n = 0
        return self

    def __exit__(self, *exc):
        self.n = load().pcs_probe_end()
        return False

    def records(self, with_stream: bool = False):
        """[(name, flops, bytes, seconds[, stream handle])] (waits for the launches)."""
        out = []
        buf = ctypes.create_string_buffer(128)
        fl, by, ms = ctypes.c_double(), ctypes.c_double(), ctypes.c_float()
        sp = ctypes.c_void_p()
        for i in range(self.n):
            call('pcs_probe_get', i, buf, 128, ctypes.byref(fl), ctypes.byref(by), ctypes.byref(ms))
            rec = (buf.value.decode(), fl.value, by.value, ms.value * 1e-3)
            if with_stream:
                call('pcs_probe_stream', i, ctypes.byref(sp))
                rec += (sp.value or 0,)
            out.append(rec)
        return out

    def timeline(self):
        """[(name, flops, stream handle, start s, end s)] with starts / ends relative to the
        first record's start (pcs_probe_times; waits for the launches)."""
        out = []
        buf = ctypes.create_string_buffer(128)
        fl, by, ms = ctypes.c_double(), ctypes.c_double(), ctypes.c_float()
        sp, t0, t1 = ctypes.c_void_p(), ctypes.c_double(), ctypes.c_double()
        for i in range(self.n):
            call('pcs_probe_get', i, buf, 128, ctypes.byref(fl), ctypes.byref(by), ctypes.byref(ms))
            call('pcs_probe_stream', i, ctypes.byref(sp))
            call('pcs_probe_times', i, ctypes.byref(t0), ctypes.byref(t1))
            out.append((buf.value.decode(), fl.value, sp.value or 0, t0.value * 1e-3, t1.value * 1e-3))
        return out

    def replay(self, name: str, reps: int = 20) -> float:
        """Average seconds per launch of kernel `name`, its recorded launches re-issued
        back to back (pcs_probe_replay; comparable with rocprofv3's AverageNs)."""
        us, n = ctypes.c_float(), ctypes.c_int()
        call('pcs_probe_replay', name.encode(), reps, ctypes.byref(us), ctypes.byref(n))
        return us.value * 1e-6

    def summary(self, stream=None, exclude: bool = False):
        """{kernel: (launches, flops, bytes, seconds)} (synchronises); with `stream` (a raw
        handle) only the launches on that stream, or with exclude=True only the others."""
        out = {}
        for name, fl, by, sec, sh in self.records(with_stream=True):
            if stream is not None and (sh == stream) == exclude:
                continue
            n, f, b, t = out.get(name, (0, 0, 0, 0.0))
            out[name] = (n + 1, f + fl, b + by, t + sec)
        return out


def operand(data, ld, mode=OP_PLAIN, s=None, t=None, act=0, slope=0.0, z=None, ldz=0, mean=None, inv=None,
            alpha=None, kb=None, arg=None, pool_k=0) -> Operand:
    """pcs_operand for a tensor and its on-load transform (the tensors must outlive the launch)."""
    return Operand(ptr(data), ld, mode, ptr(s), ptr(t), act, float(slope), ptr(z), ldz, ptr(mean), ptr(inv),
                   ptr(alpha), ptr(kb), ptr(arg), pool_k)


def gemm_rows(a: Operand, M, K, W, ldw, bias, C, ldc, N, stats=None, epi: Operand | None = None, bstats=None,
              st=None):
    """C[M,N] = T(A)[M,K] . W^T (+bias) with optional BN-stat / BN-backward partials."""
    call('pcs_gemm_rows', a, M, K, ptr(W), ldw, ptr(bias), ptr(C), ldc, N, ptr(stats), epi, ptr(bstats), st)


def gemm_rows_kmajor(a: Operand, M, K, W, ldw, C, ldc, N, epi: Operand | None = None, bstats=None, st=None):
    """C[M,N] = T(A)[M,K] . W with W row-major K x N (the data-gradient GEMM, no transpose)."""
    call('pcs_gemm_rows_kmajor', a, M, K, ptr(W), ldw, ptr(C), ldc, N, epi, ptr(bstats), st)


def gemm_rows_kmajor_variant(a: Operand, M, K, W, ldw, C, ldc, N, variant, epi: Operand | None = None,
                             bstats=None, st=None):
    """gemm_rows_kmajor with its kernel forced for this call: -1 the register-staged row GEMM, 0 the
    policy, 1 / 2 / 3 the LDS-DMA kernel as 64x3 / 128x2 / 128x3 (column tile x ring stages)."""
    call('pcs_gemm_rows_kmajor_variant', a, M, K, ptr(W), ldw, ptr(C), ldc, N, epi, ptr(bstats), variant, st)


def wgrad_workspace(N, K, M) -> int:
    """Bytes of pcs_wgrad's partial-tile workspace for an N x K gradient over M rows."""
    key = ('wgrad', N, K, M)
    n = _ws_cache.get(key)
    if n is None:
        out = ctypes.c_size_t(0)
        call('pcs_wgrad_workspace', N, K, M, ctypes.byref(out))
        n = _ws_cache[key] = int(out.value)
    return n


def wgrad(x: Operand, N, y: Operand, K, M, dW, db, st, ws=None):
    """dW[N,K] += T(X)^T . T(Y) over M rows, db += colsum(T(X)) (deterministic: per-split
    partial tiles in `ws`, allocated here when not given, added in a fixed order)."""
    nws = wgrad_workspace(N, K, M)
    if ws is None:
        ws = torch.empty((nws,), dtype=torch.uint8, device=dW.device)
    call('pcs_wgrad', x, N, y, K, M, ptr(dW), ptr(db), ptr(ws), ws.numel(), st)


def _f64(shape, dev):
    return torch.empty(shape, dtype=torch.float64, device=dev)


def _f32(shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


# pcs_mlp_layer (include/pcseg.h): 25 little-endian 8-byte slots (200 bytes)
_REC = struct.Struct('<QqqqQQQQQQddqqdQQQQQQdqqq')  # ... dW db dgamma dbeta drop_p drop_seed bwd_fuse dx_col0
_ws_cache: dict = {}


# --------------------------------------------------------------------------- wgrad lane
# A stack's weight gradients run on the device's wgrad lane (a native side stream).  With
# pcs_mlp_backward_deferred they keep running after the stack's backward returns, under the
# next autograd nodes, and one join per backward pass (an autograd engine callback) makes
# the caller's stream wait for them before anything reads the gradients (FlatAdam.step and
# FlatGradAllReduce.synchronize join again, unconditionally).
_lanes: dict = {}
_join_queued: dict = {}      # device index -> autograd graph task whose backward has a join queued
# Backward passes the host may run ahead of the GPU (0: unbounded).  The lane's inputs are
# record_stream'ed, so the caching allocator holds them until the lane passes their free point:
# a host N backward passes ahead holds N passes of them (DGCNN ~5 GiB each) until an allocation
# fails and the allocator drops its whole cache, a multi-second stall
# (profiles/r04_host_runahead.txt).  The join waits for the pass MAX_INFLIGHT_BACKWARDS back.
MAX_INFLIGHT_BACKWARDS = 3
_inflight: dict = {}         # device index -> deque of join events
inflight_wait_s = [0.0]      # host seconds spent in those waits (bench.py reports it apart)

BWD_FUSE = {'default': 0, 'off': 1, 'all': 2}   # pcs_mlp_layer.bwd_fuse (include/pcseg.h)


def wgrad_lane(dev: torch.device):
    """torch.cuda.ExternalStream of the device's wgrad lane (None if the library has none)."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _lanes:
        out = ctypes.c_void_p(0)
        with torch.cuda.device(idx):
            call('pcs_wgrad_lane', ctypes.byref(out))
        _lanes[idx] = torch.cuda.ExternalStream(out.value, device=torch.device('cuda', idx)) if out.value else None
    return _lanes[idx]


def _queue_lane_join(dev: torch.device) -> None:
    """Queue one lane join at the end of the CURRENT backward pass (graph task).  The dedup is
    keyed on the graph task id: if a backward raises after queueing, its final callbacks never
    run, and the next backward (a new task id) still queues its own join."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    task = torch._C._current_graph_task_id()
    if task >= 0 and _join_queued.get(idx) == task:
        return
    _join_queued[idx] = task

    def join():
        if _join_queued.get(idx) == task:
            del _join_queued[idx]
        with torch.cuda.device(idx):
            call('pcs_wgrad_lane_join', stream_ptr(torch.device('cuda', idx)))
            if MAX_INFLIGHT_BACKWARDS > 0 and not torch.cuda.is_current_stream_capturing():
                ev = torch.cuda.Event()
                ev.record()
                q = _inflight.setdefault(idx, collections.deque())
                q.append(ev)
                if len(q) > MAX_INFLIGHT_BACKWARDS:
                    t0 = time.perf_counter()
                    while len(q) > MAX_INFLIGHT_BACKWARDS:
                        q.popleft().synchronize()
                    inflight_wait_s[0] += time.perf_counter() - t0
    torch.autograd.Variable._execution_engine.queue_callback(join)


def lane_join(dev: torch.device) -> None:
    """Make the current stream wait for every weight gradient pending on the device's lane."""
    with torch.cuda.device(dev):
        call('pcs_wgrad_lane_join', stream_ptr(dev))


def module_cache(m: torch.nn.Module) -> dict:
    """The per-module dict shared_mlp keeps a stack's static layer records in (host cost)."""
    c = m.__dict__.get('_pcs_cache')
    if c is None:
        c = m.__dict__['_pcs_cache'] = {}
    return c


def set_bwd_fuse(module: torch.nn.Module, policy: str = 'default') -> None:
    """Per-module backward kernel choice of every shared-MLP stack under `module`
    (pcs_mlp_layer.bwd_fuse): 'default' fuses a thin layer's data + weight gradient into one
    launch only over >= 2^19 rows, 'off' never, 'all' for every eligible layer."""
    v = BWD_FUSE[policy]
    for m in module.modules():
        if hasattr(m, 'bwd_fuse'):
            m.bwd_fuse = v


def set_edge_inverse(module: torch.nn.Module, where: str = 'side') -> None:
    """Where every fused EdgeConv under `module` builds its backward's inverse kNN map: 'side' (on
    the side stream as soon as its forward is enqueued: it then competes with the next layer's kNN),
    'backward' (on the caller's stream when the backward needs it), or 'deferred' (the model
    enqueues all of them on the side stream once its EdgeConvs are done: EdgeInverseBatch)."""
    if where not in ('side', 'backward', 'deferred'):
        raise ValueError(f"edge inverse must be 'side', 'backward' or 'deferred', got {where!r}")
    for m in module.modules():
        if hasattr(m, 'edge_inverse'):
            m.edge_inverse = where


def _workspace(lib, key, M, kin, ldx, recs, nl, pool_k, backward):
    n = _ws_cache.get(key)
    if n is None:
        out = ctypes.c_size_t(0)
        rc = lib.pcs_mlp_workspace(M, kin, ldx, recs, nl, pool_k, backward, ctypes.byref(out))
        if rc:
            raise RuntimeError(f'pcs_mlp_workspace failed ({rc}): {lib.pcs_last_error().decode()}')
        n = int(out.value)
        _ws_cache[key] = n
    return n


def _nz(p) -> int:
    return 0 if p is None else p.data_ptr()


_STATIC = struct.Struct('<QqqqQQQQQQddqqd')     # pcs_mlp_layer fields W .. slope
_DYN = struct.Struct('<QQQQQQdqqq')              # Z coef dW db dgamma dbeta drop_p drop_seed bwd_fuse dx_col0
assert _STATIC.size + _DYN.size == _REC.size


def _layer_statics(Kin, bns, acts, params, couts, dev):
    """([static record bytes per layer], [weight matrices as the kernels read them], cacheable):
    the pcs_mlp_layer fields that do not change from call to call.  Not cacheable when a weight
    needs a padded copy (refreshed every call) or a BN momentum is None (cumulative average)."""
    statics, Wms = [], []
    cacheable = True
    cin = Kin
    for li, bn in enumerate(bns):
        W, b, g, be = params[4 * li:4 * li + 4]
        C = couts[li]
        if C % 4:
            raise ValueError(f'engine: layer width {C} must be a multiple of 4')
        # a DETACHED alias: a view of the parameter made here (autograd.Function.forward runs in
        # no-grad mode) and saved for backward is rejected once an optimizer updates the parameter
        # in place (torch.optim.Adam in the unchanged harness, Training/training.py:60)
        Wm = W.detach().reshape(C, -1)
        if Wm.shape[1] % 4 and li > 0:    # 16-B weight rows (the pad columns are zero)
            Wp = torch.zeros((C, ld4(Wm.shape[1])), dtype=torch.float32, device=dev)
            Wp[:, :Wm.shape[1]] = Wm
            Wm = Wp
            cacheable = False
        elif not Wm.is_contiguous():        # (an unpadded first layer is read as is)
            Wm = Wm.contiguous()
            cacheable = False
        Wms.append(Wm)
        use_batch = bn.training or bn.running_mean is None
        track = use_batch and bn.training and bn.track_running_stats and bn.running_mean is not None
        momentum = 0.0
        if track:
            if bn.momentum is None:
                cacheable = False
                momentum = 1.0 / float(bn.num_batches_tracked + 1)
            else:
                momentum = bn.momentum
        rm = bn.running_mean if (track or not use_batch) else None
        rv = bn.running_var if (track or not use_batch) else None
        nbt = bn.num_batches_tracked if track else None
        act, slope = acts[li]
        statics.append(_STATIC.pack(Wm.data_ptr(), Wm.shape[1], cin, C, _nz(b), _nz(g), _nz(be), _nz(rm), _nz(rv),
                                    _nz(nbt), float(momentum), float(bn.eps), int(use_batch), act, slope))
        cin = C
    return statics, Wms, cacheable


def _workspace_probe(lib, key, M, Kin, ldx, params, bns, nl, pool_K, couts, acts):
    """pcs_mlp_workspace for a stack (sizes only: the records carry non-null placeholder pointers)."""
    recs = []
    cin = Kin
    for li in range(nl):
        W = params[4 * li]
        C = couts[li]
        ldw = W.reshape(C, -1).shape[1]
        if ldw % 4 and li > 0:
            ldw = ld4(ldw)
        bn = bns[li]
        use_batch = bn.training or bn.running_mean is None
        recs.append(_REC.pack(16, ldw, cin, C, 0, 0, 0, 16, 16, 0, 0.0, 1e-5, int(use_batch), acts[li][0],
                              acts[li][1], 16, 16, 0, 0, 0, 0, 0.0, 0, 0, 0))
        cin = C
    return _workspace(lib, key, M, Kin, ldx, b''.join(recs), nl, pool_K, 0)


class SharedMLPFn(torch.autograd.Function):
    """rows X (M, ld) with Kin logical channels -> pooled (M/pool_K, C_L) or activation (M, C_L).

    The whole stack runs in ONE native call each way (pcs_mlp_forward / pcs_mlp_backward,
    csrc/engine.hip); Python only allocates the outputs and packs one pcs_mlp_layer
    record per layer."""

    @staticmethod
    def forward(ctx, X, Kin, pool_K, acts, bns, dest, drop, bwd_fuse, cache, dx_from, *params):
        dev = X.device
        st = stream_ptr(dev)
        lib = load()
        M = X.shape[0]
        ldx = X.stride(0)       # X may be a column block of a wider buffer (row stride > width)
        nl = len(bns)
        couts = [params[4 * li].shape[0] for li in range(nl)]
        tot = sum(couts)
        key = (M, Kin, ldx, tuple(couts), pool_K, 0)
        nws = _ws_cache.get(key)
        # ONE allocation per stack call: [pre-BN Z of every layer | BN coefficients | workspace]
        zc = M * tot + 4 * tot
        wsoff = (zc + 63) // 64 * 64                      # 256-B aligned workspace
        buf = _f32((wsoff + ((nws or 0) + 3) // 4,), dev) if nws is not None else None
        if buf is None:                                   # first call with this shape: size the workspace
            nws = _workspace_probe(lib, key, M, Kin, ldx, params, bns, nl, pool_K, couts, acts)
            buf = _f32((wsoff + (nws + 3) // 4,), dev)
        Zbuf = buf[:M * tot]
        coef = buf[M * tot:zc]
        # the per-layer static record fields (W .. slope): cached on the calling module (`cache`,
        # e.g. a MiniPointNet's dict) while the parameters' storage and the BN modes are unchanged
        ent = None
        if cache is not None:
            # everything _layer_statics bakes into the records: parameter storage, the BN modes and
            # hyper-parameters, and the running-statistics buffers (pcseg.ddp.FlatBuffers rebinds them)
            key = (Kin, acts, tuple(_nz(p) for p in params),
                   tuple((bn.training, bn.track_running_stats, bn.momentum, bn.eps, _nz(bn.running_mean),
                          _nz(bn.running_var), _nz(bn.num_batches_tracked)) for bn in bns))
            ent = cache.get('static')
            if ent is not None and ent[0] != key:
                ent = None
        if ent is None:
            statics, Wms, cacheable = _layer_statics(Kin, bns, acts, params, couts, dev)
            if cache is not None and cacheable:
                cache['static'] = (key, statics, Wms)
        else:
            statics, Wms = ent[1], ent[2]
        zc_ptr, cf_ptr = Zbuf.data_ptr(), coef.data_ptr()
        zptrs, off = [], 0
        for C in couts:
            zptrs.append((zc_ptr + 4 * M * off, cf_ptr + 16 * off))
            off += C
        # drop = (p, seed): the training-mode Dropout after the stack, fused into its output
        dp, dseed = drop if drop is not None else (0.0, 0)
        recs = b''.join(statics[li] + _DYN.pack(zp, cp, 0, 0, 0, 0, dp if li == nl - 1 else 0.0,
                                                  dseed if li == nl - 1 else 0, bwd_fuse, 0)
                        for li, (zp, cp) in enumerate(zptrs))
        CL = couts[-1]
        ldo = 0
        if pool_K:
            G = M // pool_K
            out = _f32((G, CL), dev)
            arg = torch.empty((G, CL), dtype=torch.uint8, device=dev)
            ctx.mark_non_differentiable(arg)
        elif dest is not None:
            out = dest[0]           # (M, CL) column block of a caller buffer (see storage_alias)
            ldo = out.stride(0)
            arg = None
        else:
            out = _f32((M, CL), dev)
            arg = None
        call('pcs_mlp_forward', ptr(X), ldx, Kin, M, recs, nl, pool_K, ptr(out), ldo, ptr(arg),
             buf.data_ptr() + 4 * wsoff, nws, st)
        if arg is not None:
            record_pool_arg(arg)
        if recording():
            # the kernels' activation decision y = z*s + t > 0 (unfused, as in the BNACT load,
            # pool_finalize and bn_act), per layer in stack order (replay into the fp64 oracle)
            off = 0
            for li, C in enumerate(couts):
                if acts[li][0] != ACT['none']:
                    Z = Zbuf[M * off:M * (off + C)].view(M, C)
                    cf = coef[4 * off:4 * off + 2 * C]
                    record_act_mask(Z * cf[:C] + cf[C:] > 0)
                off += C
        ctx.save_for_backward(X, Zbuf, coef, *Wms, *([arg] if arg is not None else []))
        ctx.meta = (Kin, pool_K, nl, statics, zptrs, couts, arg is not None)
        ctx.drop = drop
        ctx.bwd_fuse = bwd_fuse
        ctx.dx_from = dx_from
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, gout):
        Kin, pool_K, nl, statics, zptrs, couts, has_arg = ctx.meta
        saved = ctx.saved_tensors
        X = saved[0]
        arg = saved[3 + nl] if has_arg else None
        params = ctx.params
        dev = gout.device
        st = stream_ptr(dev)
        lib = load()
        M, ldx = X.shape[0], X.stride(0)
        # a row-strided gradient (e.g. a column slice of a concatenation's gradient) is read
        # in place; anything else is made dense
        if not (gout.dim() == 2 and gout.stride(1) == 1 and gout.stride(0) % 4 == 0 and gout.data_ptr() % 16 == 0
                and (pool_K == 0 or gout.is_contiguous())):
            gout = gout.contiguous()
        ldg = gout.stride(0)
        gt = grad_targets(params)
        # the fused dropout's backward runs inside the engine (its mask recomputed from the seed,
        # applied where the top layer's gradient is read): the top record carries (p, seed)
        dp, ds = (float(ctx.drop[0]), int(ctx.drop[1])) if ctx.drop is not None else (0.0, 0)
        recs = b''.join(statics[li] + _DYN.pack(zp, cp, _nz(gt[4 * li]), _nz(gt[4 * li + 1]), _nz(gt[4 * li + 2]),
                                                  _nz(gt[4 * li + 3]), dp if li == nl - 1 else 0.0,
                                                  ds if li == nl - 1 else 0, ctx.bwd_fuse,
                                                  ctx.dx_from if li == 0 else 0)
                        for li, (zp, cp) in enumerate(zptrs))
        dX = None
        if ctx.needs_input_grad[0]:
            dX = _f32((M, X.shape[1]), dev)       # dense, X's width (its pad columns zeroed)
        key = (M, Kin, ldx, tuple(couts), pool_K, 1, dp > 0.0)
        nws = _workspace(lib, key, M, Kin, ldx, recs, nl, pool_K, 1)
        ws = torch.empty((nws,), dtype=torch.uint8, device=dev)
        lane = wgrad_lane(dev)
        if lane is None:
            call('pcs_mlp_backward', ptr(X), ldx, Kin, M, recs, nl, pool_K, ptr(arg), ptr(gout), ldg, ptr(dX),
                 X.shape[1], ptr(ws), nws, st)
        else:
            call('pcs_mlp_backward_deferred', ptr(X), ldx, Kin, M, recs, nl, pool_K, ptr(arg), ptr(gout), ldg,
                 ptr(dX), X.shape[1], ptr(ws), nws, st)
            # the lane still reads these: the caching allocator must not hand them out before it is done
            for t in (X, saved[1], saved[2], gout, ws, *([arg] if arg is not None else [])):
                t.record_stream(lane)
            _queue_lane_join(dev)
        notify_grad_ready(params)
        return (dX, None, None, None, None, None, None, None, None, None, *([None] * len(params)))


def _edge_ws(B, N, C, Cout, backward, dev):
    key = ('edge', B, N, C, Cout, backward)
    n = _ws_cache.get(key)
    if n is None:
        out = ctypes.c_size_t(0)
        call('pcs_edgeconv_workspace', B, N, C, Cout, backward, ctypes.byref(out))
        n = int(out.value)
        _ws_cache[key] = n
    return torch.empty((n,), dtype=torch.uint8, device=dev)


class EdgeConvFn(torch.autograd.Function):
    """Fused EdgeConv (dgcnn.py:60-77) in training mode: point rows X (B*N, ld) with C logical
    channels and the kNN table idx (B, N, k) int32 -> pooled (B*N, Cout).  The (B, 2C, N, k)
    edge tensor is never formed: z_(i,j) = (Y_j - Y_i) + P_i with Y = X W1^T, P = X W2^T
    (csrc/edgeconv.hip); the backward gathers over the CSR inverse of idx."""

    @staticmethod
    def forward(ctx, X, idx, C, slope, bn, W, gamma, beta, inverse_side=True, holder=None, also=None):
        dev = X.device
        st = stream_ptr(dev)
        B, N, k = idx.shape
        M, ldx = X.shape
        Cout = W.shape[0]
        Wm = W.detach().reshape(Cout, 2 * C)      # detached alias (see _layer_statics)
        if not Wm.is_contiguous():
            Wm = Wm.contiguous()
        Y, PQ, S, out = (_f32((M, Cout), dev) for _ in range(4))
        pz = _f32((M, Cout), dev)                 # the one pooled extreme per channel (edgeconv.hip)
        pa = torch.empty((M, Cout), dtype=torch.uint8, device=dev)
        arg = torch.empty((M, Cout), dtype=torch.uint8, device=dev)
        coef = _f32((4 * Cout,), dev)
        track = bn.track_running_stats and bn.running_mean is not None
        momentum = 0.0
        if track:
            momentum = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked + 1)
        ws = _edge_ws(B, N, C, Cout, 0, dev)
        call('pcs_edgeconv_fwd', ptr(X), ldx, C, ptr(idx), B, N, k, ptr(Wm), Cout, ptr(gamma), ptr(beta),
             ptr(bn.running_mean) if track else None, ptr(bn.running_var) if track else None,
             ptr(bn.num_batches_tracked) if track else None, float(momentum), float(bn.eps), float(slope),
             ptr(Y), ptr(PQ), ptr(S), ptr(pz), ptr(pa), ptr(coef), ptr(out), ptr(arg),
             ptr(also[0]) if also is not None else None, also[0].stride(0) if also is not None else 0,
             ptr(ws), ws.numel(), st)
        record_pool_arg(arg)
        if recording():
            record_act_mask(out > 0)          # LeakyReLU keeps the sign: out > 0 <=> y > 0 at the argmax
        ctx.inv = None
        ctx.holder = holder if any(ctx.needs_input_grad) else None
        if ctx.holder is not None:
            ctx.holder.append((idx, N))          # built later on the side stream (EdgeInverseBatch)
        elif inverse_side and any(ctx.needs_input_grad):
            # the backward's inverse map of idx depends on idx only: build it now on the side
            # stream, under the rest of the forward, instead of on the backward's critical path
            from . import ops
            from .common import side_stream
            main, side = torch.cuda.current_stream(dev), side_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                off, ent = ops.inverse_index(idx, N)
                ev = torch.cuda.Event()
                ev.record(side)
            idx.record_stream(side)
            ctx.inv = (off, ent, ev)
        ctx.save_for_backward(X, idx, Wm, Y, PQ, S, pz, arg, coef)
        ctx.meta = (C, float(slope))
        ctx.params = (W, gamma, beta)
        return out

    @staticmethod
    def backward(ctx, gout):
        from . import ops
        X, idx, Wm, Y, Q, S, pz, arg, coef = ctx.saved_tensors
        C, slope = ctx.meta
        W, gamma, beta = ctx.params
        dev = gout.device
        st = stream_ptr(dev)
        B, N, k = idx.shape
        M, ldx = X.shape
        Cout = Wm.shape[0]
        # a row-strided gradient (DGCNN: the EdgeConv's column block of the head's concatenation
        # gradient) is read in place; anything else is made dense
        if not (gout.dim() == 2 and gout.stride(1) == 1 and gout.stride(0) >= Cout and gout.stride(0) % 4 == 0
                and gout.data_ptr() % 16 == 0):
            gout = gout.contiguous()
        if ctx.inv is None and ctx.holder is not None and len(ctx.holder) == 3:
            ctx.inv = tuple(ctx.holder)
        ctx.holder = None
        if ctx.inv is not None:
            off, ent, ev = ctx.inv
            torch.cuda.current_stream(dev).wait_event(ev)
            off.record_stream(torch.cuda.current_stream(dev))
            ent.record_stream(torch.cuda.current_stream(dev))
            ctx.inv = None
        else:
            off, ent = ops.inverse_index(idx, N)
        dX = _f32((M, ldx), dev) if ctx.needs_input_grad[0] else None
        if dX is not None and ldx != C:
            dX.zero_()
        ws = _edge_ws(B, N, C, Cout, 1, dev)
        dW, dg, db = grad_targets((W, gamma, beta))
        call('pcs_edgeconv_bwd', ptr(X), ldx, C, ptr(off), ptr(ent), B, N, k, ptr(Wm), Cout, ptr(Y), ptr(Q), ptr(S),
             ptr(pz), ptr(arg), ptr(coef), slope, ptr(gout), gout.stride(0), ptr(dX), ldx, ptr(dW), ptr(dg), ptr(db),
             ptr(ws),
             ws.numel(), st)
        notify_grad_ready((W, gamma, beta))
        return dX, None, None, None, None, None, None, None, None, None, None


def edgeconv_fused_ok(conv, bn, cin: int) -> bool:
    """The fused EdgeConv covers training-mode BN (eval-mode BN uses the materialised-edge path)."""
    return (bn.training and conv.weight.shape[0] % 4 == 0 and conv.bias is None
            and (cin % 4 == 0 or cin < 4))


def edgeconv(x_rows: torch.Tensor, cin: int, idx: torch.Tensor, conv, bn, slope: float,
             inverse_side: bool = True, holder: list | None = None, also: torch.Tensor | None = None) -> torch.Tensor:
    """x_rows (B*N, ld) point rows, idx (B, N, k) int32 -> pooled (B*N, Cout).  inverse_side: build
    the backward's inverse map of idx on the side stream during the forward (else in the backward).
    also: an (B*N, Cout) row block (e.g. a storage_alias column block of a concatenation buffer)
    that receives a second copy of the pooled rows, written by the same kernel -- not an autograd
    output: the caller connects it (models._CopyColumns with the part marked as written)."""
    if not x_rows.is_cuda:
        raise RuntimeError('pcseg ops run only on the GPU (no CPU fallback); got a CPU tensor')
    if x_rows.shape[1] % 4 or not x_rows.is_contiguous():
        x_rows = pad_rows(x_rows[:, :cin])
    if also is not None:
        Cout = conv.weight.shape[0]
        if (also.dim() != 2 or tuple(also.shape) != (x_rows.shape[0], Cout) or also.stride(1) != 1
                or also.stride(0) % 4 or also.data_ptr() % 16 or also.device != x_rows.device):
            raise ValueError(f'edgeconv: `also` must be a 16-B aligned ({x_rows.shape[0]}, {Cout}) row block '
                             f'with unit column stride, got {tuple(also.shape)} strides {also.stride()}')
    return EdgeConvFn.apply(x_rows, idx.contiguous(), cin, slope, bn, conv.weight, bn.weight, bn.bias, inverse_side,
                            holder, (also,) if also is not None else None)


class EdgeInverseBatch:
    """Deferred inverse kNN maps of a forward's EdgeConvs: each fused EdgeConv that needs a
    backward registers (idx, N) in its holder; `flush()` -- called by the model once its last
    EdgeConv is enqueued, so the maps do not compete with the later kNN searches -- builds them
    all on the side stream (after everything enqueued so far on the caller's stream), where
    they run under the head's GEMMs."""

    def __init__(self):
        self.holders = []

    def holder(self) -> list:
        h = []
        self.holders.append(h)
        return h

    def flush(self) -> None:
        from . import ops
        from .common import side_stream
        pend = [h for h in self.holders if len(h) == 1]
        self.holders = []
        if not pend:
            return
        dev = pend[0][0][0].device
        side = side_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            tabs = [h.pop() for h in pend]
            maps = ops.inverse_index_batch(tabs)       # one native call, 3 launches for all
            ev = torch.cuda.Event()
            ev.record(side)
            for h, (idx, _), (off, ent) in zip(pend, tabs, maps):
                idx.record_stream(side)
                h.extend((off, ent, ev))


def storage_alias(base: torch.Tensor, col0: int, ncol: int) -> torch.Tensor:
    """Columns [col0, col0 + ncol) of the row-major (M, ld) buffer `base` as an (M, ncol)
    tensor with row stride ld that shares base's storage WITHOUT being an autograd view of it:
    several custom Functions can each write their output into their own column block of one
    buffer (a zero-copy concatenation) without autograd's view+in-place checks firing."""
    t = torch.empty(0, dtype=base.dtype, device=base.device)
    t.set_(base.untyped_storage(), base.storage_offset() + col0, (base.shape[0], ncol), (base.stride(0), 1))
    return t


def _rows_ok(x: torch.Tensor) -> bool:
    """(M, W) rows the engine reads in place: unit column stride, 16-B aligned rows, W % 4 == 0."""
    return (x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.stride(0) >= x.shape[1]
            and x.shape[1] % 4 == 0 and x.data_ptr() % 16 == 0)


def shared_mlp(x_rows: torch.Tensor, kin: int, convs, bns, act='relu', slope=0.0,
               pool_k: int = 0, out: torch.Tensor | None = None, dropout: tuple | None = None,
               bwd_fuse: int = 0, cache: dict | None = None, dx_from: int = 0) -> torch.Tensor:
    """Run a conv/BN/act stack on rows.  x_rows (M, W) with `kin` logical channels, W % 4 == 0,
    dense or a column block of a wider buffer (row stride >= W).  `act` / `slope` are one value
    for every layer or a sequence with one per layer ('relu', 'lrelu', 'none').  `out`: an
    (M, cout) row block (storage_alias) the un-pooled activation is written into.  `dropout` =
    (p, seed): a training-mode nn.Dropout(p) after the stack, fused into its output
    (pcs_mlp_layer.drop_p; backward pcs_dropout_bwd recomputes the mask from the seed).
    `bwd_fuse`: the stack's backward kernel choice (BWD_FUSE values, pcs_mlp_layer.bwd_fuse).
    `cache`: a dict owned by the calling module, where the stack's static layer records are
    kept between calls (host enqueue cost).  `dx_from`: the first input column whose gradient
    is wanted (pcs_mlp_layer.dx_col0): grouped rows start with 3 relative-coordinate columns
    whose gradient no caller reads; the returned gradient's columns before it are undefined."""
    if not x_rows.is_cuda:
        raise RuntimeError('pcseg ops run only on the GPU (no CPU fallback); got a CPU tensor')
    if not _rows_ok(x_rows):
        x_rows = pad_rows(x_rows[:, :kin])
    if out is not None and (pool_k or not _rows_ok(out) or out.shape != (x_rows.shape[0], convs[-1].weight.shape[0])):
        raise ValueError('shared_mlp: out must be an un-pooled (M, cout) row block')
    nl = len(convs)
    names = [act] * nl if isinstance(act, str) else list(act)
    slopes = [slope] * nl if isinstance(slope, (int, float)) else list(slope)
    if len(names) != nl or len(slopes) != nl:
        raise ValueError('shared_mlp: one act/slope per layer')
    acts = tuple((ACT[a], float(sl)) for a, sl in zip(names, slopes))
    params = []
    for conv, bn in zip(convs, bns):
        params += [conv.weight, conv.bias, bn.weight, bn.bias]
    if dropout is not None and (pool_k or not 0.0 < float(dropout[0]) < 1.0):
        raise ValueError('shared_mlp: dropout needs an un-pooled output and 0 < p < 1')
    return SharedMLPFn.apply(x_rows, kin, pool_k, acts, list(bns), None if out is None else (out,), dropout,
                             int(bwd_fuse), cache, int(dx_from), *params)


class RowLinearFn(torch.autograd.Function):
    """A bare 1x1 convolution (no BN) on rows, e.g. the segmentation heads
    (PointNetpp.py:25,45 `self.conv`, dgcnn.py:210 `conv8`): out = X W^T + b on the
    engine GEMM; backward = one dgrad GEMM + one wgrad."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        dev = x.device
        M, K = x.shape
        N = weight.shape[0]
        Wm = weight.detach().reshape(N, -1)       # detached alias (see _layer_statics)
        if Wm.shape[1] != K or K % 4:
            raise ValueError(f'row linear: x has {K} channels, weight expects {Wm.shape[1]} (need a multiple of 4)')
        Wm = Wm.contiguous()
        out = _f32((M, N), dev)
        gemm_rows(operand(x, K), M, K, Wm, K, bias, out, N, N, st=stream_ptr(dev))
        ctx.save_for_backward(x, Wm)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        x, Wm = ctx.saved_tensors
        dev = gout.device
        st = stream_ptr(dev)
        M, K = x.shape
        N = Wm.shape[0]
        N4 = ld4(N)
        if N4 == N and gout.is_contiguous():
            gp = gout
        else:                                   # pad the class dimension to a 16-B row stride
            gp = torch.zeros((M, N4), dtype=torch.float32, device=dev)
            gp[:, :N] = gout
        gop = operand(gp, N4)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _f32((M, K), dev)
            # dgrad B[k=class][n=cin] = Wm[class][cin], read k-major
            gemm_rows_kmajor(gop, M, N, Wm, K, dx, K, K, st=st)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dwp = torch.zeros((N4, K), dtype=torch.float32, device=dev)
            dbp = torch.zeros((N4,), dtype=torch.float32, device=dev) if ctx.has_bias else None
            wgrad(gop, N4, operand(x, K), K, M, dwp, dbp, st)
            dw = dwp[:N]
            db = dbp[:N] if dbp is not None else None
        return dx, dw, db


def linear_rows(x: torch.Tensor, conv) -> torch.Tensor:
    """x (M, Cin) -> (M, Cout) for a 1x1 Conv1d/Conv2d holder, on the engine GEMM."""
    if not x.is_cuda:
        raise RuntimeError('pcseg ops run only on the GPU (no CPU fallback); got a CPU tensor')
    x = x.contiguous()
    out = RowLinearFn.apply(x, conv.weight.reshape(conv.weight.shape[0], -1), conv.bias)
    return out
