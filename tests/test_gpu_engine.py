"""Engine GEMMs (pcs_gemm_rows / pcs_wgrad) against a float64 torch reference of the
same op, for every operand transform (PLAIN, BNACT, BNBWD, POOLBWD), the fused
BN-statistics / BN-backward epilogues and ragged M / K / N; the weight gradient's
determinism (identical calls give bitwise-identical dW / db).

Tolerance: fp32 MFMA accumulation vs the fp64 reference, norm-relative 2e-6 * sqrt(K)
(plus 1e-5 absolute slack for the near-zero BN-backward sums)."""
import math

import pytest
import torch

from pcseg._lib import load, stream_ptr, OP_PLAIN, OP_BNACT, OP_BNBWD, OP_POOLBWD
from pcseg.engine import operand, gemm_rows, gemm_rows_kmajor, wgrad, ld4

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def act(v, slope):
    return torch.where(v > 0, v, v * slope)


def dact(v, slope):
    return torch.where(v > 0, torch.ones_like(v), torch.full_like(v, slope))


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


class Xform:
    """Inputs of one operand transform and its float64 evaluation."""

    def __init__(self, mode, M, K, ld, slope, pool_k=0, g=None):
        self.mode, self.M, self.K, self.ld, self.slope, self.pool_k = mode, M, K, ld, slope, pool_k
        rows = M // pool_k if mode == OP_POOLBWD else M
        self.data = torch.randn(rows, ld, device=DEV, generator=g)
        self.s = (torch.rand(K, device=DEV, generator=g) + 0.5)
        self.t = torch.randn(K, device=DEV, generator=g) * 0.3
        self.z = torch.randn(M, ld, device=DEV, generator=g)
        self.mean = torch.randn(K, device=DEV, generator=g) * 0.1
        self.alpha = torch.randn(K, device=DEV, generator=g) * 0.05
        self.kb = torch.randn(K, device=DEV, generator=g) * 0.05
        self.arg = torch.randint(0, max(pool_k, 1), (rows, ld), device=DEV, dtype=torch.uint8, generator=g)

    def op(self):
        if self.mode == OP_PLAIN:
            return operand(self.data, self.ld)
        if self.mode == OP_BNACT:
            return operand(self.data, self.ld, OP_BNACT, self.s, self.t, 1, self.slope)
        return operand(self.data, self.ld, self.mode, self.s, self.t, 1, self.slope, self.z, self.ld, self.mean,
                       None, self.alpha, self.kb, self.arg if self.mode == OP_POOLBWD else None, self.pool_k)

    def value(self):
        K = self.K
        d = self.data.double()[:, :K]
        if self.mode == OP_PLAIN:
            return d
        s, t = self.s.double(), self.t.double()
        if self.mode == OP_BNACT:
            return act(d * s + t, self.slope)
        if self.mode == OP_POOLBWD:
            r = torch.arange(self.M, device=DEV)
            gsel = r // self.pool_k
            kk = (r % self.pool_k).to(torch.uint8)
            d = torch.where(self.arg[gsel, :K] == kk[:, None], d[gsel], torch.zeros_like(d[gsel]))
        z = self.z.double()[:, :K]
        # the activation-derivative branch is decided on the fp32 pre-activation, as the kernel
        # (and the reference's fp32 autograd) does: at large M * K a few z*s+t sit within fp32
        # rounding of 0, and an fp64 decision there flips dact between 1 and the slope
        pre32 = (self.z[:, :K] * self.s + self.t).double()
        dy = d * dact(pre32, self.slope)
        return s * dy - self.kb.double() - self.alpha.double() * (z - self.mean.double())


SHAPES = [  # M, K, N
    (1000, 9, 32), (4099, 32, 64), (2048, 67, 64), (3000, 128, 128), (515, 259, 256), (777, 384, 512),
    (128, 1408, 96), (64, 20, 36), (131073, 32, 64), (70001, 128, 128), (300000, 12, 32),
    (65537, 384, 256),   # data-gradient modes: the wide-tile regime (N >= 256 over >= 64K rows)
]


@pytest.mark.parametrize('M,K,N', SHAPES)
@pytest.mark.parametrize('mode', [OP_PLAIN, OP_BNACT, OP_BNBWD, OP_POOLBWD])
def test_gemm_rows_vs_fp64(M, K, N, mode):
    if mode != OP_PLAIN and K % 4:
        pytest.skip('transform modes need K % 4 == 0')
    pool_k = 0
    if mode == OP_POOLBWD:
        pool_k = 16 if M % 16 == 0 else (4 if M % 4 == 0 else 1)
    g = torch.Generator(device=DEV).manual_seed(M * 7 + K * 3 + N + mode)
    lda = ld4(K)
    x = Xform(mode, M, K, lda, 0.2, pool_k, g)
    W = torch.zeros(N, lda, device=DEV)
    W[:, :K] = torch.randn(N, K, device=DEV, generator=g) / math.sqrt(K)
    bias = torch.randn(N, device=DEV, generator=g)
    C = torch.full((M, N), float('nan'), device=DEV)
    nb = (load().pcs_gemm_row_blocks_dgrad if mode >= OP_BNBWD else load().pcs_gemm_row_blocks)(M, N)
    part = torch.empty(2, N, nb, dtype=torch.float64, device=DEV)
    st = stream_ptr(torch.device(DEV))
    gemm_rows(x.op(), M, K, W, lda, bias, C, N, N, part, st=st)
    ref = x.value() @ W.double()[:, :K].t() + bias.double()
    tol = 2e-6 * math.sqrt(K)
    assert rel(C, ref) <= tol
    if K % 4:
        # unpadded weight rows (ldw = K, scalar B loads) give the same bits as the padded copy
        Wu = W[:, :K].contiguous()
        Cu = torch.full((M, N), float('nan'), device=DEV)
        gemm_rows(x.op(), M, K, Wu, K, bias, Cu, N, N, None, st=stream_ptr(torch.device(DEV)))
        assert torch.equal(Cu, C)
    sums = part.sum(-1)
    assert rel(sums[0], ref.sum(0)) <= tol + 1e-6
    assert rel(sums[1], (ref * ref).sum(0)) <= tol

    # dgrad form: same A operand, BN-backward epilogue of a layer whose pre-BN output is ze
    if N % 4 == 0:
        ze = torch.randn(M, N, device=DEV, generator=g)
        se, te = torch.rand(N, device=DEV, generator=g) + 0.5, torch.randn(N, device=DEV, generator=g) * 0.3
        me, ie = torch.randn(N, device=DEV, generator=g) * 0.1, torch.rand(N, device=DEV, generator=g) + 0.5
        epi = operand(None, 0, OP_BNBWD, se, te, 1, 0.2, ze, N, me, ie)
        bpart = torch.empty(2, N, nb, dtype=torch.float64, device=DEV)
        C2 = torch.empty(M, N, device=DEV)
        gemm_rows(x.op(), M, K, W, lda, None, C2, N, N, None, epi, bpart, st=st)
        ref2 = x.value() @ W.double()[:, :K].t()
        assert rel(C2, ref2) <= tol
        dy = ref2 * dact((ze * se + te).double(), 0.2)     # the kernel's fp32 gate
        xh = (ze.double() - me.double()) * ie.double()
        bs = bpart.sum(-1)
        assert rel(bs[0], dy.sum(0)) <= tol + 1e-5
        assert rel(bs[1], (dy * xh).sum(0)) <= tol + 1e-5


KSHAPES = [  # M, K (= cout of the layer), N (= its cin): the data-gradient GEMM on k-major W
    (1000, 32, 12), (4099, 64, 32), (3000, 128, 128), (515, 256, 260), (777, 512, 384), (64, 36, 20),
    (70001, 128, 128), (2000, 13, 128), (300000, 32, 12),
    (65536, 512, 384), (66001, 256, 260),   # wide-tile regime (DGCNN conv5-7 shapes)
]


@pytest.mark.parametrize('M,K,N', KSHAPES)
@pytest.mark.parametrize('mode', [OP_PLAIN, OP_BNBWD, OP_POOLBWD])
def test_gemm_rows_kmajor_vs_fp64(M, K, N, mode):
    """pcs_gemm_rows_kmajor: B[k][n] = W[k*ldw + n] (W read in place, no transpose), with the
    fused BN-backward epilogue; LDS engine only."""
    if mode != OP_PLAIN and K % 4:
        pytest.skip('transform modes need K % 4 == 0')
    pool_k = 0
    if mode == OP_POOLBWD:
        pool_k = 16 if M % 16 == 0 else (4 if M % 4 == 0 else 1)
    g = torch.Generator(device=DEV).manual_seed(M * 5 + K * 3 + N + mode)
    lda, ldw = ld4(K), ld4(N)
    x = Xform(mode, M, K, lda, 0.2, pool_k, g)
    W = torch.randn(K, ldw, device=DEV, generator=g) / math.sqrt(K)    # pad columns hold junk: never read into C
    C = torch.full((M, N), float('nan'), device=DEV)
    st = stream_ptr(torch.device(DEV))
    tol = 2e-6 * math.sqrt(K)
    if N % 4 == 0:
        nb = load().pcs_gemm_row_blocks_dgrad(M, N)          # k-major: always the data-gradient grid
        ze = torch.randn(M, N, device=DEV, generator=g)
        se, te = torch.rand(N, device=DEV, generator=g) + 0.5, torch.randn(N, device=DEV, generator=g) * 0.3
        me, ie = torch.randn(N, device=DEV, generator=g) * 0.1, torch.rand(N, device=DEV, generator=g) + 0.5
        epi = operand(None, 0, OP_BNBWD, se, te, 1, 0.2, ze, N, me, ie)
        bpart = torch.empty(2, N, nb, dtype=torch.float64, device=DEV)
        gemm_rows_kmajor(x.op(), M, K, W, ldw, C, N, N, epi, bpart, st=st)
    else:
        gemm_rows_kmajor(x.op(), M, K, W, ldw, C, N, N, st=st)
    ref = x.value() @ W.double()[:, :N]
    assert rel(C, ref) <= tol
    if N % 4 == 0:
        dy = ref * dact((ze * se + te).double(), 0.2)      # the kernel's fp32 gate
        xh = (ze.double() - me.double()) * ie.double()
        bs = bpart.sum(-1)
        assert rel(bs[0], dy.sum(0)) <= tol + 1e-5
        assert rel(bs[1], (dy * xh).sum(0)) <= tol + 1e-5


WSHAPES = [  # M rows, N (dZ channels), K (input channels)
    (5000, 32, 9), (4099, 64, 32), (3000, 128, 67), (2100, 256, 128), (1030, 512, 259), (640, 96, 1408),
    (100, 36, 20), (70001, 32, 32), (300000, 32, 12), (9000, 96, 32), (4100, 32, 96), (4100, 40, 24),
]


@pytest.mark.parametrize('M,N,K', WSHAPES)
@pytest.mark.parametrize('xmode,ymode', [(OP_PLAIN, OP_PLAIN), (OP_BNBWD, OP_BNACT), (OP_POOLBWD, OP_BNACT),
                                         (OP_BNBWD, OP_PLAIN)])
def test_wgrad_vs_fp64(M, N, K, xmode, ymode):
    if ymode == OP_BNACT and K % 4:
        pytest.skip('BNACT needs K % 4 == 0')
    pool_k = 0
    if xmode == OP_POOLBWD:
        pool_k = 20 if M % 20 == 0 else (4 if M % 4 == 0 else 1)
    g = torch.Generator(device=DEV).manual_seed(M + 11 * N + 5 * K + xmode * 3 + ymode)
    x = Xform(xmode, M, N, ld4(N), 0.2, pool_k, g)
    y = Xform(ymode, M, K, ld4(K), 0.0, 0, g)
    dW = torch.zeros(N, K, device=DEV)
    db = torch.zeros(N, device=DEV)
    wgrad(x.op(), N, y.op(), K, M, dW, db, stream_ptr(torch.device(DEV)))
    X, Y = x.value(), y.value()
    tol = 2e-6 * math.sqrt(M)
    assert rel(dW, X.t() @ Y) <= tol
    assert rel(db, X.sum(0)) <= tol
    # deterministic: the same call again gives the same bits (no float atomics)
    dW2 = torch.zeros(N, K, device=DEV)
    db2 = torch.zeros(N, device=DEV)
    wgrad(x.op(), N, y.op(), K, M, dW2, db2, stream_ptr(torch.device(DEV)))
    assert torch.equal(dW, dW2) and torch.equal(db, db2)


@pytest.mark.parametrize('K,act', [(32, 'relu'), (16, 'lrelu'), (20, 'relu'), (32, 'lrelu')])
def test_stack_pooling_matches_max_of_activation(K, act):
    """A pooled stack (SA / EdgeConv: conv -> BN -> act -> max over K) against the same stack
    unpooled followed by torch's max over K.  K = 16 / 32 take the GEMM-epilogue z-space
    max/min + pool_finalize path; K = 20 the separate pooling kernel.  Negative and zero BN
    scales exercise the min / first-index branches."""
    from pcseg.engine import shared_mlp
    torch.manual_seed(K)
    G, kin, widths = 777, 9, [32, 48]

    def stack():
        convs = torch.nn.ModuleList([torch.nn.Conv2d(kin, widths[0], 1), torch.nn.Conv2d(widths[0], widths[1], 1)])
        bns = torch.nn.ModuleList([torch.nn.BatchNorm2d(w) for w in widths])
        with torch.no_grad():
            bns[1].weight[::3] = -0.7
            bns[1].weight[1] = 0.0
        return convs.to(DEV), bns.to(DEV).train()
    c1, b1 = stack()
    c2, b2 = stack()
    c2.load_state_dict(c1.state_dict())
    b2.load_state_dict(b1.state_dict())
    x = torch.randn(G * K, 12, device=DEV)
    x[:, 9:] = 0
    x.view(G, K, 12)[:, 5] = x.view(G, K, 12)[:, 2]            # duplicated rows: exact ties in z
    slope = 0.2 if act == 'lrelu' else 0.0
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    pooled = shared_mlp(xa, kin, list(c1), list(b1), act, slope, pool_k=K)
    full = shared_mlp(xb, kin, list(c2), list(b2), act, slope, pool_k=0)
    ref = full.view(G, K, -1).max(dim=1).values
    assert torch.equal(pooled, ref)
    w = torch.randn_like(pooled)
    (pooled * w).sum().backward()
    (ref * w).sum().backward()
    assert rel(xa.grad, xb.grad) <= 1e-5
    # (pre-BN conv biases have an analytically zero gradient: compare on the scale of the stack's gradients)
    scale = max(float(q.grad.abs().max()) for q in list(c2.parameters()) + list(b2.parameters()))
    for p, q in zip(list(c1.parameters()) + list(b1.parameters()), list(c2.parameters()) + list(b2.parameters())):
        assert float((p.grad - q.grad).abs().max()) <= 1e-5 * scale


# ---------------------------------------------------------------- DGCNN conv5-7 at BASELINE config 2
# B = 32 x N = 4096 -> M = 131 072 rows (models/dgcnn/dgcnn.py:188-207, colour model: x_cat 384,
# emb 1024, conv6 input 1408): the LDS-DMA wide GEMMs of gemm_big.hip, each identified by the
# launch probe's kernel name, against an fp64 product on the GPU.
def _rel_dev(a, b):
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-30))


WIDE = [  # M, K (contraction), N (outputs), ldc, BN statistics, kernel the dispatch must pick
    (131072, 1024, 384, 1408, False, 'pcs::gemm_nt_kernel<128, 4, 2, false>'),   # conv5 dgrad into the head buffer
    (131072, 512, 1408, 1408, False, 'pcs::gemm_nt_kernel<128, 4, 2, false>'),   # conv6 dgrad
    (131072, 256, 512, 512, False, 'pcs::gemm_nt_kernel<256, 2, 4, false>'),     # conv7 dgrad
    (131072, 384, 1024, 1408, True, 'pcs::gemm_nt_kernel<256, 2, 4, true>'),     # conv5 forward
    (131072, 1408, 512, 512, True, 'pcs::gemm_nt_kernel<256, 2, 4, true>'),      # conv6 forward
    (65601, 64, 300, 300, False, 'pcs::gemm_nt_kernel<128, 4, 2, false>'),       # ragged M and N
    (65601, 96, 512, 516, True, 'pcs::gemm_nt_kernel<256, 2, 4, true>'),         # ragged M, stats
]


@pytest.mark.parametrize('M,K,N,ldc,stats,kernel', WIDE)
def test_wide_gemm_nt_vs_fp64(M, K, N, ldc, stats, kernel):
    from pcseg.engine import KernelProbe
    g = torch.Generator(device=DEV).manual_seed(M + 3 * K + 7 * N)
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / math.sqrt(K)
    bias = torch.randn(N, device=DEV, generator=g) if stats else None
    C = torch.full((M, ldc), float('nan'), device=DEV)
    part = None
    if stats:
        nb = load().pcs_gemm_row_blocks(M, N)
        assert nb == load().pcs_gemm_nt_row_tiles(M)
        part = torch.empty(2, N, nb, dtype=torch.float64, device=DEV)
    with KernelProbe() as kp:
        gemm_rows(operand(A, K), M, K, W, K, bias, C, ldc, N, part, st=stream_ptr(torch.device(DEV)))
    assert [r[0] for r in kp.records()] == [kernel]
    ref = A.double() @ W.double().t()
    if bias is not None:
        ref += bias.double()
    tol = 2e-6 * math.sqrt(K)
    assert _rel_dev(C[:, :N], ref) <= tol
    assert torch.isnan(C[:, N:]).all()                      # the row stride's pad columns are not written
    if stats:
        sums = part.sum(-1)
        assert _rel_dev(sums[0], ref.sum(0)) <= tol + 1e-6
        assert _rel_dev(sums[1], (ref * ref).sum(0)) <= tol


WIDE_W = [  # M rows, N (dZ channels), K (input channels), Y operand mode, kernel the dispatch must pick
    (131072, 256, 512, OP_PLAIN, 'pcs::wgrad_nt_kernel<128, 4, 2>'),            # conv7 weight gradient
    (131072, 1024, 384, OP_PLAIN, 'pcs::wgrad_kernel<128, 128, 0, 0, 1>'),      # conv5 (row-split wgrad)
    (131072, 512, 1408, OP_PLAIN, 'pcs::wgrad_kernel<128, 128, 0, 0, 1>'),      # conv6
    (131072, 256, 512, OP_BNACT, 'pcs::wgrad_kernel<128, 128, 0, 1, 1>'),       # conv7 over a BN+act input
    (65568, 256, 256, OP_PLAIN, 'pcs::wgrad_nt_kernel<128, 4, 2>'),             # M % 32 == 0, not a split multiple
]


@pytest.mark.parametrize('M,N,K,ymode,kernel', WIDE_W)
def test_wide_wgrad_vs_fp64(M, N, K, ymode, kernel):
    """dW = dZ^T . X for the wide layers (no bias: conv5-7 have bias=False), plain dZ (the
    materialised top-layer gradient), fp64 reference on the GPU; deterministic."""
    from pcseg.engine import KernelProbe
    g = torch.Generator(device=DEV).manual_seed(M + 11 * N + 5 * K + ymode)
    x = Xform(OP_PLAIN, M, N, ld4(N), 0.2, 0, g)
    y = Xform(ymode, M, K, ld4(K), 0.2, 0, g)
    st = stream_ptr(torch.device(DEV))
    dW = torch.zeros(N, K, device=DEV)
    with KernelProbe() as kp:
        wgrad(x.op(), N, y.op(), K, M, dW, None, st)
    names = [r[0] for r in kp.records()]
    assert names == [kernel], names
    ref = x.value().t() @ y.value()
    assert _rel_dev(dW, ref) <= 3e-5
    dW2 = torch.zeros(N, K, device=DEV)
    wgrad(x.op(), N, y.op(), K, M, dW2, None, st)
    assert torch.equal(dW, dW2)


def test_lane_join_after_a_backward_that_raised(monkeypatch):
    """A backward that raises after a deferred stack backward queued its wgrad-lane join never
    runs its final callbacks; the next backward (a new graph task) must queue and run its own
    join, and its gradients must be those of a clean run."""
    import pcseg
    import pcseg.engine as E
    joins = []
    orig = E.call

    def counting(name, *a):
        if name == 'pcs_wgrad_lane_join':
            joins.append(1)
        return orig(name, *a)
    monkeypatch.setattr(E, 'call', counting)

    class Boom(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return t.clone()

        @staticmethod
        def backward(ctx, gr):
            raise RuntimeError('boom')

    torch.manual_seed(3)
    mods = [pcseg.MiniPointNet(32, [64, 64]).to(DEV).train() for _ in range(2)]
    mods[1].load_state_dict(mods[0].state_dict())
    x = torch.randn(8192, 32, device=DEV, requires_grad=True)
    y = mods[0].forward_rows(Boom.apply(x), 32)
    with pytest.raises(RuntimeError, match='boom'):
        y.square().sum().backward()
    torch.cuda.synchronize()
    n0 = len(joins)
    for m in mods:
        m.zero_grad(set_to_none=True)
        m.forward_rows(x.detach(), 32).square().sum().backward()
    torch.cuda.synchronize()
    assert len(joins) >= n0 + 2                             # both backwards joined the lane
    for (k, a), (_, b) in zip(mods[0].named_parameters(), mods[1].named_parameters()):
        assert torch.equal(a.grad, b.grad), k
