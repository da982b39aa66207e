"""Isolated timing of the BN-backward data gradient (pcs_gemm_rows_kmajor, BNBWD operand, fused
BN-backward epilogue) on the PointNet++ dgrad shapes, for every kernel variant of
pcs_gemm_rows_kmajor_variant (-1 = the register-staged row GEMM, 1 / 2 / 3 = the LDS-DMA kernel with
64x3 / 128x2 / 128x3 column tile x ring stages); argv[1] == "plain": a materialised (plain) dZ
operand.  Prints us per launch and algorithmic GB/s."""
import math, os, sys
import torch
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd')]
from pcseg._lib import load, stream_ptr, OP_BNBWD, OP_PLAIN
from pcseg.engine import operand, gemm_rows_kmajor_variant, ld4

plain = len(sys.argv) > 1 and sys.argv[1] == 'plain'
st = stream_ptr(torch.device('cuda'))
for var, (M, K, N) in [(v, s) for v in (-1, 1, 2, 3) for s in [(131072, 128, 128), (262144, 64, 64), (65536, 256, 128), (65536, 128, 128), (32768, 256, 256)]]:
    tag = f'variant {var}' + (' plain' if plain else ' bnbwd')
    g = torch.Generator(device='cuda').manual_seed(1)
    r = lambda *s: torch.randn(*s, device='cuda', generator=g)
    lda, ldw = ld4(K), ld4(N)
    x = operand(r(M, lda), lda, OP_PLAIN) if plain else operand(
        r(M, lda), lda, OP_BNBWD, torch.rand(K, device='cuda') + 0.5, r(K) * 0.3, 1, 0.0, r(M, lda), lda,
        r(K) * 0.1, None, r(K) * 0.05, r(K) * 0.05)
    W = r(K, ldw) / math.sqrt(K)
    epi = operand(None, 0, OP_BNBWD, torch.rand(N, device='cuda') + 0.5, r(N) * 0.3, 1, 0.0, r(M, N), N, r(N) * 0.1,
                  torch.rand(N, device='cuda') + 0.5)
    nb = load().pcs_gemm_row_blocks_dgrad(M, N)
    C = torch.empty(M, N, device='cuda')
    bp = torch.empty(2, N, nb, dtype=torch.float64, device='cuda')
    for _ in range(3):
        gemm_rows_kmajor_variant(x, M, K, W, ldw, C, N, N, var, epi, bp, st=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        gemm_rows_kmajor_variant(x, M, K, W, ldw, C, N, N, var, epi, bp, st=st)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    e0.record()
    for _ in range(20):
        gemm_rows_kmajor_variant(x, M, K, W, ldw, C, N, N, var, st=st)
    e1.record(); torch.cuda.synchronize()
    us0 = e0.elapsed_time(e1) / 20 * 1e3
    gb = (8.0 * M * K + 8.0 * M * N) / us * 1e-3
    print(f'dma={tag} M={M} K={K} N={N}: {us:7.1f} us  {gb:6.0f} GB/s  {2.0 * M * K * N / us * 1e-6:5.1f} TF/s'
          f'  | no epilogue {us0:7.1f} us', flush=True)
