"""The LDS-DMA data-gradient kernel (csrc/dgrad.hip) against the register-staged row GEMM it
replaces (gemm_rows_kernel<64, 64, 2, 2, PLAIN | BNBWD | POOLBWD, true, EPI>): BITWISE equal
outputs and BN-backward partials, with and without the fused epilogue, on the PointNet++ dgrad
shapes and ragged ones (M not a multiple of 64, N not a multiple of 64, several column tiles),
for every ring variant.  pcs_gemm_rows_kmajor_variant forces the kernel for one call (-1 = the row
GEMM), and the launch probe names the kernel that ran.  Values against fp64 are covered by
tests/test_gpu_engine.py::test_gemm_rows_kmajor_vs_fp64 (on this kernel), and the pooled form by
the model three-way tests (SetAbstraction's top layer)."""
import math

import pytest
import torch

from pcseg._lib import load, stream_ptr, OP_BNBWD, OP_PLAIN, OP_POOLBWD
from pcseg.engine import operand, gemm_rows_kmajor_variant, ld4, KernelProbe

pytestmark = pytest.mark.gpu

# M, K (the layer's cout: contraction), N (its cin: outputs)
SHAPES = [(131072, 128, 128), (262144, 64, 64), (65536, 256, 128), (4099, 64, 64), (515, 256, 260),
          (1000, 32, 36), (70001, 128, 128)]
# pooled top layers: M, K, N, pool_k (SA2 / SA3 of PointNet++ B=32, MSG's 16-row groups, one-group
# tiles, ragged M and N)
POOL_SHAPES = [(262144, 128, 64, 32), (65536, 256, 128, 32), (65536, 128, 64, 16), (1040, 64, 36, 16),
               (4480, 128, 128, 64), (1152, 64, 260, 128), (2080, 96, 64, 32)]
VARIANTS = {1: '64, 3', 2: '128, 2', 3: '128, 3'}


def _case(M, K, N, mode, pk=0):
    dev = torch.device('cuda')
    g = torch.Generator(device='cuda').manual_seed(M + 3 * K + 7 * N + pk)
    r = lambda *s: torch.randn(*s, device=dev, generator=g)
    lda, ldw = ld4(K), ld4(N)
    z = r(M, lda)
    s, t = torch.rand(K, device=dev, generator=g) + 0.5, r(K) * 0.3
    mean, alpha, kb = r(K) * 0.1, r(K) * 0.05, r(K) * 0.05
    keep = [z, s, t, mean, alpha, kb]
    if mode == 'plain':
        dy = r(M, lda)
        x = operand(dy, lda, OP_PLAIN)
    elif mode == 'bnbwd':
        dy = r(M, lda)
        x = operand(dy, lda, OP_BNBWD, s, t, 1, 0.0, z, lda, mean, None, alpha, kb)
    else:
        G = M // pk
        dy = r(G, K)
        arg = torch.randint(0, pk, (G, K), device=dev, generator=g, dtype=torch.uint8)
        keep.append(arg)
        x = operand(dy, K, OP_POOLBWD, s, t, 1, 0.0, z, lda, mean, None, alpha, kb, arg, pk)
    keep.append(dy)
    W = r(K, ldw) / math.sqrt(K)
    ze = r(M, N)
    se, te = torch.rand(N, device=dev, generator=g) + 0.5, r(N) * 0.3
    me, ie = r(N) * 0.1, torch.rand(N, device=dev, generator=g) + 0.5
    keep += [W, ze, se, te, me, ie]
    epi = operand(None, 0, OP_BNBWD, se, te, 1, 0.0, ze, N, me, ie)
    return x, W, ldw, epi, keep


def _run(x, M, K, N, W, ldw, epi, variant):
    st = stream_ptr(torch.device('cuda'))
    nb = load().pcs_gemm_row_blocks_dgrad(M, N)
    C1 = torch.full((M, N), float('nan'), device='cuda')
    C2 = torch.full((M, N), float('nan'), device='cuda')
    bp = torch.full((2, N, nb), float('nan'), dtype=torch.float64, device='cuda')
    with KernelProbe() as kp:
        gemm_rows_kmajor_variant(x, M, K, W, ldw, C1, N, N, variant, epi, bp, st=st)
        gemm_rows_kmajor_variant(x, M, K, W, ldw, C2, N, N, variant, st=st)
    torch.cuda.synchronize()
    return (C1, C2, bp), [rr[0] for rr in kp.records()]


def _check(shape, mode, pk=0):
    M, K, N = shape
    x, W, ldw, epi, keep = _case(M, K, N, mode, pk)
    old, names_old = _run(x, M, K, N, W, ldw, epi, -1)
    opm = {'plain': 0, 'bnbwd': 2, 'pool': 3}[mode]
    xm = {'plain': 0, 'bnbwd': 1, 'pool': 2}[mode]
    assert all(n.startswith(f'pcs::gemm_rows_kernel<64, 64, 2, 2, {opm}, true') for n in names_old), names_old
    for v, tile in VARIANTS.items():
        new, names_new = _run(x, M, K, N, W, ldw, epi, v)
        tile = '64, 3' if N <= 64 else tile
        assert names_new == [f'pcs::dgrad_kernel<true, {tile}, {xm}>', f'pcs::dgrad_kernel<false, {tile}, {xm}>'], \
            (shape, v, names_new)
        for a, b, what in zip(new, old, ('c_epi', 'c', 'partials')):
            assert not torch.isnan(a).any(), (shape, v, what)
            assert torch.equal(a, b), (shape, v, what)
    del keep


@pytest.mark.parametrize('mode', ['bnbwd', 'plain'])
@pytest.mark.parametrize('shape', SHAPES, ids=lambda s: 'x'.join(map(str, s)))
def test_dgrad_dma_bitwise_equal_to_row_gemm(shape, mode):
    _check(shape, mode)


@pytest.mark.parametrize('shape', POOL_SHAPES, ids=lambda s: 'x'.join(map(str, s)))
def test_dgrad_dma_pooled_bitwise_equal_to_row_gemm(shape):
    """The pooled top layer's data gradient (A = POOLBWD: the pooled gradient routed to each
    group's argmax row, then the BN backward) on the DMA ring (round 5)."""
    M, K, N, pk = shape
    _check((M, K, N), 'pool', pk)


def test_dgrad_policy_picks_dma_for_pooled_operand():
    """The product's policy call (variant 0) runs the DMA kernel for the SA2 / SA3 shapes."""
    for M, K, N, pk in POOL_SHAPES[:2]:
        x, W, ldw, epi, keep = _case(M, K, N, 'pool', pk)
        _, names = _run(x, M, K, N, W, ldw, epi, 0)
        tile = '64, 3' if N <= 64 else '128, 2'
        assert names == [f'pcs::dgrad_kernel<true, {tile}, 2>', f'pcs::dgrad_kernel<false, {tile}, 2>'], names
