"""Compare pcs_gemm_rows_kmajor with pcs_gemm_rows on W^T (same dgrad), bitwise and stats."""
import math, os, sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '3d-semantic-segmentation-benchmark_amd')]
import torch
from pcseg._lib import load, stream_ptr, OP_BNBWD
from pcseg.engine import operand, gemm_rows, gemm_rows_kmajor
dev = 'cuda'
st = stream_ptr(torch.device(dev))
for (M, K, N) in [(300000, 32, 12), (300000, 32, 16), (1000, 32, 12), (100000, 32, 12), (300000, 32, 32)]:
    g = torch.Generator(device=dev).manual_seed(1)
    A = torch.randn(M, K, device=dev, generator=g)
    ldw = (N + 3) // 4 * 4
    W = torch.randn(K, ldw, device=dev, generator=g)
    Wt = W[:, :N].t().contiguous()
    Wt = torch.nn.functional.pad(Wt, (0, 0, 0, 0))
    nb = load().pcs_gemm_row_blocks(M, N)
    ze = torch.randn(M, N, device=dev, generator=g)
    se, te = torch.rand(N, device=dev, generator=g) + 0.5, torch.randn(N, device=dev, generator=g) * 0.3
    me, ie = torch.randn(N, device=dev, generator=g) * 0.1, torch.rand(N, device=dev, generator=g) + 0.5
    epi = operand(None, 0, OP_BNBWD, se, te, 1, 0.2, ze, N, me, ie)
    res = []
    for mode in ('k', 'n'):
        C = torch.empty(M, N, device=dev)
        bp = torch.zeros(2, N, nb, dtype=torch.float64, device=dev)
        if mode == 'k':
            gemm_rows_kmajor(operand(A, K), M, K, W, ldw, C, N, N, epi, bp, st=st)
        else:
            gemm_rows(operand(A, K), M, K, Wt, K, None, C, N, N, None, epi, bp, st=st)
        res.append((C, bp))
    torch.cuda.synchronize()
    ref = A.double() @ W.double()[:, :N]
    dy = ref * torch.where(ze.double() * se.double() + te.double() > 0, 1.0, 0.2)
    for (C, bp), nm in zip(res, ('kmajor', 'nmajor')):
        s0 = bp.sum(-1)[0]
        print(M, K, N, nm, 'C rel', float((C.double() - ref).norm() / ref.norm()),
              'sum rel', float((s0 - dy.sum(0)).norm() / dy.sum(0).norm()), 'nb', nb, flush=True)
    print('  C equal', torch.equal(res[0][0], res[1][0]), 'partials max diff', float((res[0][1] - res[1][1]).abs().max()))
