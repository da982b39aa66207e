"""Isolated timing of the BN-backward data gradient (pcs_gemm_rows_kmajor, BNBWD operand, fused
BN-backward epilogue) on the PointNet++ dgrad shapes; PCS_DGRAD_DMA=0 selects the register-staged
row GEMM, PCS_DGRAD_VAR the DMA kernel's column tile x ring depth, PCS_DGRAD_MODE=plain a
materialised (plain) dZ operand (run the script once per setting).  Prints us per launch and algorithmic GB/s."""
import math, os, sys
import torch
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd')]
from pcseg._lib import load, stream_ptr, OP_BNBWD, OP_PLAIN
from pcseg.engine import operand, gemm_rows_kmajor, ld4

plain = os.environ.get('PCS_DGRAD_MODE') == 'plain'
tag = os.environ.get('PCS_DGRAD_DMA', '1') + ' var=' + os.environ.get('PCS_DGRAD_VAR', '128x2') + (' plain' if plain else ' bnbwd')
st = stream_ptr(torch.device('cuda'))
for (M, K, N) in [(131072, 128, 128), (262144, 64, 64), (65536, 256, 128), (65536, 128, 128), (32768, 256, 256)]:
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
        gemm_rows_kmajor(x, M, K, W, ldw, C, N, N, epi, bp, st=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        gemm_rows_kmajor(x, M, K, W, ldw, C, N, N, epi, bp, st=st)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    e0.record()
    for _ in range(20):
        gemm_rows_kmajor(x, M, K, W, ldw, C, N, N, st=st)
    e1.record(); torch.cuda.synchronize()
    us0 = e0.elapsed_time(e1) / 20 * 1e3
    gb = (8.0 * M * K + 8.0 * M * N) / us * 1e-3
    print(f'dma={tag} M={M} K={K} N={N}: {us:7.1f} us  {gb:6.0f} GB/s  {2.0 * M * K * N / us * 1e-6:5.1f} TF/s'
          f'  | no epilogue {us0:7.1f} us', flush=True)
