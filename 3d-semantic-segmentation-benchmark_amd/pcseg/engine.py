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

import math

import torch

from ._lib import call, load, ptr, stream_ptr, Operand, OP_PLAIN, OP_BNACT, OP_BNBWD, OP_POOLBWD

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


def notify_grad_ready(params) -> None:
    for p in params:
        if p is not None:
            cb = getattr(p, '_pcs_grad_ready', None)
            if cb is not None:
                cb(p)


# --------------------------------------------------------------------------- launch probe
_probe: list | None = None


class KernelProbe:
    """Bracket every engine GEMM launch with HIP events on the stream it runs on.

    Inside `with KernelProbe() as kp:` each pcs_gemm_rows / pcs_wgrad launch is
    recorded as (kernel name as rocprof reports it, algorithmic flops,
    algorithmic bytes, start event, end event).  Used by bench.py's roofline.
    """

    def __enter__(self):
        global _probe
        self.records = []
        _probe = self.records
        return self

    def __exit__(self, *exc):
        global _probe
        _probe = None
        return False

    def summary(self):
        """{kernel: (launches, flops, bytes, seconds)} (synchronises)."""
        out = {}
        for name, fl, by, e0, e1 in self.records:
            e1.synchronize()
            n, f, b, t = out.get(name, (0, 0, 0, 0.0))
            out[name] = (n + 1, f + fl, b + by, t + e0.elapsed_time(e1) * 1e-3)
        return out


def _gemm_tile(M: int, N: int) -> tuple[int, int, int, int]:
    """(BM, BN, WM, WN) of the row GEMM -- mirrors gemm_tile() in csrc/mlp.hip (used for naming only)."""
    if N <= 32:
        return 128, 32, 4, 1
    cands = [(128, 128, 2, 2), (64, 128, 2, 2), (64, 64, 2, 2), (32, 128, 1, 4)] if N > 64 else \
        [(128, 64, 4, 1), (64, 64, 2, 2)]
    best, pick = -1, cands[0]
    for c in cands:
        blocks = -(-M // c[0]) * -(-N // c[1])
        if blocks >= 512:
            return c
        if blocks > best:
            best, pick = blocks, c
    return pick


def _launch(name, fl, by, fn, *args):
    if _probe is None:
        call(fn, *args)
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call(fn, *args)
    e1.record()
    _probe.append((name, fl, by, e0, e1))


def operand(data, ld, mode=OP_PLAIN, s=None, t=None, act=0, slope=0.0, z=None, ldz=0, mean=None, inv=None,
            alpha=None, kb=None, arg=None, pool_k=0) -> Operand:
    """pcs_operand for a tensor and its on-load transform (the tensors must outlive the launch)."""
    return Operand(ptr(data), ld, mode, ptr(s), ptr(t), act, float(slope), ptr(z), ldz, ptr(mean), ptr(inv),
                   ptr(alpha), ptr(kb), ptr(arg), pool_k)


def _operand_bytes(op: Operand, M: int, K: int) -> int:
    if op.mode == OP_POOLBWD:
        return 4 * M * K                      # Z (the pooled gradient and argmax are M/pool_k rows)
    return 4 * M * K * (2 if op.mode == OP_BNBWD else 1)


def gemm_rows(a: Operand, M, K, W, ldw, bias, C, ldc, N, stats=None, epi: Operand | None = None, bstats=None,
              st=None):
    """C[M,N] = T(A)[M,K] . W^T (+bias) with optional BN-stat / BN-backward partials."""
    bm, bn, wm, wn = _gemm_tile(M, N)
    by = _operand_bytes(a, M, K) + 4 * M * N + (4 * M * N if bstats is not None else 0)
    _launch(f'pcs::gemm_rows_kernel<{bm}, {bn}, {wm}, {wn}, {a.mode}>', 2 * M * K * N, by, 'pcs_gemm_rows',
            a, M, K, ptr(W), ldw, ptr(bias), ptr(C), ldc, N, ptr(stats), epi, ptr(bstats), st)


def wgrad(x: Operand, N, y: Operand, K, M, dW, db, st):
    """dW[N,K] += T(X)^T . T(Y) over M rows, db += colsum(T(X))."""
    name = f'pcs::wgrad_kernel<{128 if N > 64 else 64}, {128 if K > 64 else 64}, {x.mode}, {y.mode}>'
    _launch(name, 2 * M * N * K, _operand_bytes(x, M, N) + _operand_bytes(y, M, K), 'pcs_wgrad',
            x, N, y, K, M, ptr(dW), ptr(db), st)


def _f64(shape, dev):
    return torch.empty(shape, dtype=torch.float64, device=dev)


def _f32(shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


class SharedMLPFn(torch.autograd.Function):
    """rows X (M, ld) with Kin logical channels -> pooled (M/pool_K, C_L) or activation (M, C_L)."""

    @staticmethod
    def forward(ctx, X, Kin, pool_K, acts, bns, *params):
        dev = X.device
        st = stream_ptr(dev)
        M, lda = X.shape
        A, lda_cur, K_cur, s_prev, t_prev = X, lda, Kin, None, None
        Zs, stats = [], []
        nl = len(bns)
        for li in range(nl):
            W, b, g, be = params[4 * li:4 * li + 4]
            bn = bns[li]
            Cout = W.shape[0]
            Wm = W.reshape(Cout, -1)
            if Wm.shape[1] % 4:                 # 16-B weight rows (the pad columns are zero)
                Wp = torch.zeros((Cout, ld4(Wm.shape[1])), dtype=torch.float32, device=dev)
                Wp[:, :Wm.shape[1]] = Wm
                Wm = Wp
            elif not Wm.is_contiguous():
                Wm = Wm.contiguous()
            if Cout % 4:
                raise ValueError(f'engine: layer width {Cout} must be a multiple of 4')
            Z = _f32((M, Cout), dev)
            a_op = operand(A, lda_cur) if s_prev is None else \
                operand(A, lda_cur, OP_BNACT, s_prev, t_prev, *acts[li - 1])
            use_batch = bn.training or bn.running_mean is None
            s, t, mean, inv = (_f32((Cout,), dev) for _ in range(4))
            if use_batch:
                nb = load().pcs_gemm_row_blocks(M, Cout)
                part = _f64((2, Cout, nb), dev)
                gemm_rows(a_op, M, K_cur, Wm, Wm.shape[1], b, Z, Cout, Cout, part, st=st)
                momentum = 0.0
                rm = rv = None
                if bn.training and bn.track_running_stats and bn.running_mean is not None:
                    bn.num_batches_tracked.add_(1)
                    momentum = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
                    rm, rv = bn.running_mean, bn.running_var
                call('pcs_bn_finalize', ptr(part), nb, Cout, M, ptr(g), ptr(be), float(bn.eps), float(momentum),
                     ptr(rm), ptr(rv), ptr(s), ptr(t), ptr(mean), ptr(inv), st)
            else:
                gemm_rows(a_op, M, K_cur, Wm, Wm.shape[1], b, Z, Cout, Cout, None, st=st)
                with torch.no_grad():
                    inv.copy_(torch.rsqrt(bn.running_var + bn.eps))
                    mean.copy_(bn.running_mean)
                    s.copy_((g if g is not None else 1.0) * inv)
                    t.copy_((be if be is not None else 0.0) - mean * s)
            Zs.append(Z)
            stats.append((s, t, mean, inv, use_batch))
            A, lda_cur, K_cur, s_prev, t_prev = Z, Cout, Cout, s, t
        CL = Zs[-1].shape[1]
        s, t = stats[-1][0], stats[-1][1]
        if pool_K:
            G = M // pool_K
            out = _f32((G, CL), dev)
            arg = torch.empty((G, CL), dtype=torch.uint8, device=dev)
            call('pcs_pool_fwd', ptr(Zs[-1]), CL, G, pool_K, ptr(s), ptr(t), *acts[-1], ptr(out), ptr(arg), st)
            ctx.mark_non_differentiable(arg)
        else:
            out = _f32((M, CL), dev)
            arg = None
            call('pcs_bn_act', ptr(Zs[-1]), CL, M, CL, ptr(s), ptr(t), *acts[-1], ptr(out), CL, st)
        ctx.save_for_backward(X, *Zs, *[x for st_ in stats for x in st_[:4]], *(p for p in params if p is not None),
                              *([arg] if arg is not None else []))
        ctx.meta = (Kin, pool_K, acts, nl, [st_[4] for st_ in stats],
                    [p is not None for p in params], arg is not None)
        return out

    @staticmethod
    def backward(ctx, gout):
        Kin, pool_K, acts, nl, use_batch, present, has_arg = ctx.meta
        saved = list(ctx.saved_tensors)
        X = saved[0]
        Zs = saved[1:1 + nl]
        flat = saved[1 + nl:1 + nl + 4 * nl]
        stats = [tuple(flat[4 * i:4 * i + 4]) for i in range(nl)]
        rest = saved[1 + nl + 4 * nl:]
        params = []
        it = iter(rest)
        for pr in present:
            params.append(next(it) if pr else None)
        arg = next(it) if has_arg else None
        dev = gout.device
        st = stream_ptr(dev)
        lib = load()
        M, lda = X.shape
        gout = gout.contiguous()
        CL = Zs[-1].shape[1]
        s, t, mean, inv = stats[-1]
        grads = [None] * len(params)

        # ---- top layer: BN-backward sums and dZ
        if pool_K:
            G = M // pool_K
            nb = lib.pcs_pool_bwd_reduce_blocks(G)
            part = _f64((2, CL, nb), dev)
            call('pcs_pool_bwd_reduce', ptr(gout), ptr(arg), ptr(Zs[-1]), CL, G, pool_K, ptr(s), ptr(t), ptr(mean),
                 ptr(inv), *acts[-1], ptr(part), st)
        else:
            nb = lib.pcs_bn_bwd_reduce_blocks(M)
            part = _f64((2, CL, nb), dev)
            call('pcs_bn_bwd_reduce', ptr(gout), CL, ptr(Zs[-1]), CL, M, CL, ptr(s), ptr(t), ptr(mean), ptr(inv),
                 *acts[-1], ptr(part), st)
        kB, alpha = _f32((CL,), dev), _f32((CL,), dev)
        gg, gb = grad_target(params[4 * (nl - 1) + 2]), grad_target(params[4 * (nl - 1) + 3])
        call('pcs_bn_bwd_finalize', ptr(part), nb, CL, M, ptr(s), ptr(inv), ptr(gg), ptr(gb), ptr(kB), ptr(alpha), 1,
             st)
        if not use_batch[-1]:
            kB.zero_()
            alpha.zero_()
        # dZ of the top layer is never materialised: its consumers rebuild it on load
        if pool_K:
            xop = operand(gout, CL, OP_POOLBWD, s, t, *acts[-1], Zs[-1], CL, mean, None, alpha, kB, arg, pool_K)
        else:
            xop = operand(gout, CL, OP_BNBWD, s, t, *acts[-1], Zs[-1], CL, mean, None, alpha, kB)
        keep = [gout, kB, alpha]
        dX = None
        for li in range(nl - 1, -1, -1):
            W, b = params[4 * li], params[4 * li + 1]
            Cout = W.shape[0]
            Wm = W.reshape(Cout, -1)
            Cin = Wm.shape[1]
            Wt = Wm.t().contiguous()          # (Cin x Cout): dgrad B[k=cout][n=cin] = Wt[n][k]
            dW = grad_target(W)
            db = grad_target(b)
            if dW is not None:
                if li > 0:
                    sp, tp, mp, ip = stats[li - 1]
                    yop = operand(Zs[li - 1], Cin, OP_BNACT, sp, tp, *acts[li - 1])
                    wgrad(xop, Cout, yop, Cin, M, dW, db, st)
                else:
                    wgrad(xop, Cout, operand(X, lda), Kin, M, dW, db, st)
            if li > 0:
                sp, tp, mp, ip = stats[li - 1]
                dA = _f32((M, Cin), dev)
                nbg = lib.pcs_gemm_row_blocks(M, Cin)
                bpart = _f64((2, Cin, nbg), dev)
                epi = operand(None, 0, OP_BNBWD, sp, tp, *acts[li - 1], Zs[li - 1], Cin, mp, ip)
                gemm_rows(xop, M, Cout, Wt, Cout, None, dA, Cin, Cin, None, epi, bpart, st=st)
                kB2, alpha2 = _f32((Cin,), dev), _f32((Cin,), dev)
                g2, b2 = grad_target(params[4 * (li - 1) + 2]), grad_target(params[4 * (li - 1) + 3])
                call('pcs_bn_bwd_finalize', ptr(bpart), nbg, Cin, M, ptr(sp), ptr(ip), ptr(g2), ptr(b2), ptr(kB2),
                     ptr(alpha2), 1, st)
                if not use_batch[li - 1]:
                    kB2.zero_()
                    alpha2.zero_()
                xop = operand(dA, Cin, OP_BNBWD, sp, tp, *acts[li - 1], Zs[li - 1], Cin, mp, None, alpha2, kB2)
                keep += [dA, kB2, alpha2]
            elif ctx.needs_input_grad[0]:
                dX = torch.zeros((M, lda), dtype=torch.float32, device=dev) if lda != Kin else _f32((M, lda), dev)
                gemm_rows(xop, M, Cout, Wt, Cout, None, dX, lda, Kin, st=st)
        notify_grad_ready(params)
        return (dX, None, None, None, None, *grads)


def shared_mlp(x_rows: torch.Tensor, kin: int, convs, bns, act='relu', slope=0.0,
               pool_k: int = 0) -> torch.Tensor:
    """Run a conv/BN/act stack on rows.  x_rows (M, ld) with `kin` logical channels, ld % 4 == 0.
    `act` / `slope` are one value for every layer or a sequence with one per layer
    ('relu', 'lrelu', 'none')."""
    if not x_rows.is_cuda:
        raise RuntimeError('pcseg ops run only on the GPU (no CPU fallback); got a CPU tensor')
    if x_rows.shape[1] % 4 or not x_rows.is_contiguous():
        x_rows = pad_rows(x_rows[:, :kin])
    nl = len(convs)
    names = [act] * nl if isinstance(act, str) else list(act)
    slopes = [slope] * nl if isinstance(slope, (int, float)) else list(slope)
    if len(names) != nl or len(slopes) != nl:
        raise ValueError('shared_mlp: one act/slope per layer')
    acts = tuple((ACT[a], float(sl)) for a, sl in zip(names, slopes))
    params = []
    for conv, bn in zip(convs, bns):
        params += [conv.weight, conv.bias, bn.weight, bn.bias]
    return SharedMLPFn.apply(x_rows, kin, pool_k, acts, list(bns), *params)


class RowLinearFn(torch.autograd.Function):
    """A bare 1x1 convolution (no BN) on rows, e.g. the segmentation heads
    (PointNetpp.py:25,45 `self.conv`, dgcnn.py:210 `conv8`): out = X W^T + b on the
    engine GEMM; backward = one dgrad GEMM + one wgrad."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        dev = x.device
        M, K = x.shape
        N = weight.shape[0]
        Wm = weight.reshape(N, -1)
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
            Wt = torch.zeros((K, N4), dtype=torch.float32, device=dev)     # dgrad B[k=n][n=cin] = Wt[cin][n]
            Wt[:, :N] = Wm.t()
            dx = _f32((M, K), dev)
            gemm_rows(gop, M, N, Wt, N4, None, dx, K, K, st=st)
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
