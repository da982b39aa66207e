"""The LDS-DMA forward GEMM (csrc/fwd_dma.hip, round 5) against the register-staged row GEMM it
replaces for the inner layers (gemm_rows_kernel, forced by pcs_gemm_rows_variant(-1) /
pcs_set_kernel_variant(-1)) and against float64: PLAIN and BNACT operands, bias, the fp64 BN
partials, ragged M and N, several column tiles, and the fused pooling epilogue through whole
stacks (pool_k 16 / 32, negative and zero BN scales).  The two kernels sum a slab's 32 k in the
same order but split the tile differently, so they agree to fp32 rounding, not bit for bit; each is
held to the fp64 tolerance of tests/test_gpu_engine.py (2e-6 sqrt(K) norm-relative)."""
import math

import pytest
import torch

from pcseg._lib import call, load, stream_ptr, OP_PLAIN, OP_BNACT
from pcseg.engine import operand, ld4, KernelProbe

pytestmark = pytest.mark.gpu
DEV = 'cuda'

# M, K, N: PointNet++ inner layers (SA1 .. SA4, FP1) and ragged / multi-tile shapes
SHAPES = [(1048576, 32, 32), (1048576, 32, 64), (262144, 64, 128), (65536, 128, 256), (16384, 256, 512),
          (131072, 128, 128), (4099, 64, 36), (515, 96, 260), (70001, 32, 64)]


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _gemm(x, M, K, W, ldw, bias, C, N, stats, variant):
    call('pcs_gemm_rows_variant', x, M, K, W.data_ptr(), ldw, bias.data_ptr(), C.data_ptr(), N, N,
         stats.data_ptr() if stats is not None else None, variant, stream_ptr(torch.device(DEV)))


@pytest.mark.parametrize('M,K,N', SHAPES, ids=lambda v: str(v))
@pytest.mark.parametrize('mode', [OP_PLAIN, OP_BNACT])
def test_fwd_dma_vs_row_gemm_and_fp64(M, K, N, mode):
    g = torch.Generator(device=DEV).manual_seed(M + 3 * K + 7 * N + mode)
    a = torch.randn(M, K, device=DEV, generator=g)
    s, t = torch.rand(K, device=DEV, generator=g) + 0.5, torch.randn(K, device=DEV, generator=g) * 0.3
    x = operand(a, K) if mode == OP_PLAIN else operand(a, K, OP_BNACT, s, t, 1, 0.2)
    W = torch.randn(N, K, device=DEV, generator=g) / math.sqrt(K)
    bias = torch.randn(N, device=DEV, generator=g)
    nb = load().pcs_gemm_row_blocks(M, N)
    out = {}
    for v in (-1, 1):
        C = torch.full((M, N), float('nan'), device=DEV)
        part = torch.full((2, N, nb), float('nan'), dtype=torch.float64, device=DEV)
        with KernelProbe() as kp:
            _gemm(x, M, K, W, K, bias, C, N, part, v)
        torch.cuda.synchronize()
        out[v] = (C, part, [r[0] for r in kp.records()])
    if mode == OP_PLAIN and out[-1][2][0].startswith('pcs::gemm_nt_kernel<'):
        assert out[1][2] == out[-1][2]        # plain operands of the wide regime: gemm_big.hip either way
    else:
        assert all(n.startswith('pcs::gemm_rows_kernel<') for n in out[-1][2]), out[-1][2]
        assert out[1][2] and all(n.startswith('pcs::fwd_dma_kernel<') for n in out[1][2]), out[1][2]
    # the product's policy: the DMA kernel for > 64 outputs over >= 8192 rows
    with KernelProbe() as kp:
        _gemm(x, M, K, W, K, bias, torch.empty(M, N, device=DEV), N, None, 0)
    torch.cuda.synchronize()
    pol = [r[0] for r in kp.records()]
    if not pol[0].startswith('pcs::gemm_nt_kernel<'):
        assert pol[0].startswith('pcs::fwd_dma_kernel<' if N > 64 and M >= 8192 else 'pcs::gemm_rows_kernel<'), pol
    A = a.double() if mode == OP_PLAIN else torch.where(a * s + t > 0, a * s + t, (a * s + t) * 0.2).double()
    ref = A @ W.double().t() + bias.double()
    tol = 2e-6 * math.sqrt(K)
    for v in (-1, 1):
        C, part, _ = out[v]
        assert not torch.isnan(C).any() and not torch.isnan(part).any()
        assert rel(C, ref) <= tol, v
        sums = part.sum(-1)
        assert rel(sums[0], ref.sum(0)) <= tol + 1e-6, v
        assert rel(sums[1], (ref * ref).sum(0)) <= tol, v
    assert rel(out[1][0], out[-1][0]) <= tol


@pytest.mark.parametrize('pool_k', [16, 32])
@pytest.mark.parametrize('widths', [[64, 64, 128], [128, 128, 256], [128, 256, 512]])
def test_fwd_dma_pooled_stack_vs_row_gemm(pool_k, widths):
    """A SetAbstraction-shaped stack (first layer on the row GEMM, inner layers on the DMA kernel,
    the top one with the fused pooling epilogue) against the same stack on the row GEMMs only:
    pooled outputs, argmax slots (away from near-ties) and BN running statistics."""
    from pcseg.engine import shared_mlp
    torch.manual_seed(pool_k + widths[0])
    G, kin = 2048, 67

    def stack():
        convs, bns, c = [], [], kin
        for w in widths:
            convs.append(torch.nn.Conv2d(c, w, 1))
            bns.append(torch.nn.BatchNorm2d(w))
            c = w
        convs, bns = torch.nn.ModuleList(convs).to(DEV), torch.nn.ModuleList(bns).to(DEV).train()
        with torch.no_grad():
            bns[-1].weight[::3] = -0.7
            bns[-1].weight[1] = 0.0
        return convs, bns
    c1, b1 = stack()
    c2, b2 = stack()
    c2.load_state_dict(c1.state_dict())
    b2.load_state_dict(b1.state_dict())
    x = torch.zeros(G * pool_k, 68, device=DEV)
    x[:, :kin] = torch.randn(G * pool_k, kin, device=DEV)
    lib = load()
    try:
        lib.pcs_set_kernel_variant(-1)
        ref = shared_mlp(x, kin, list(c2), list(b2), 'relu', 0.0, pool_k=pool_k)
        torch.cuda.synchronize()
    finally:
        lib.pcs_set_kernel_variant(0)
    got = shared_mlp(x, kin, list(c1), list(b1), 'relu', 0.0, pool_k=pool_k)
    torch.cuda.synchronize()
    assert rel(got, ref) <= 1e-5
    for p, q in zip(b1, b2):
        assert rel(p.running_mean, q.running_mean) <= 1e-5
        assert rel(p.running_var, q.running_var) <= 1e-5
