"""Per-shape timing of the engine GEMMs (pcs_gemm_rows fwd/dgrad, pcs_wgrad) on the GPU."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg._lib import stream_ptr, OP_BNACT, OP_BNBWD  # noqa: E402
from pcseg.engine import operand, gemm_rows, wgrad  # noqa: E402
from pcseg._lib import load  # noqa: E402

dev = 'cuda'
SHAPES = [  # (name, M, K, N)
    ('sa1.l1', 1048576, 9, 32), ('sa1.l2', 1048576, 32, 32), ('sa1.l3', 1048576, 32, 64),
    ('sa2.l1', 262144, 67, 64), ('sa2.l3', 262144, 64, 128),
    ('sa3.l1', 65536, 131, 128), ('sa3.l3', 65536, 128, 256),
    ('sa4.l1', 16384, 259, 256), ('sa4.l3', 16384, 256, 512),
    ('fp3.l1', 8192, 384, 256), ('fp2.l1', 32768, 320, 256), ('fp1.lx', 131072, 128, 128),
    ('dg.e2', 2621440, 128, 64), ('dg.c5', 131072, 384, 1024), ('dg.c6', 131072, 1408, 512),
]


REPS = int(os.environ.get('GEMM_REPS', '10'))
_only = os.environ.get('GEMM_SHAPES')
if _only:
    SHAPES = [sh for sh in SHAPES if any(sh[0].startswith(p) for p in _only.split(','))]


def timeit(fn, reps=REPS):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


st = stream_ptr(torch.device(dev))
for name, M, K, N in SHAPES:
    lda = (K + 3) // 4 * 4
    A = torch.randn(M, lda, device=dev)
    W = torch.zeros(N, lda, device=dev)
    W[:, :K] = torch.randn(N, K, device=dev)
    s = torch.rand(K, device=dev) + 0.5
    t = torch.randn(K, device=dev) * 0.1
    b = torch.randn(N, device=dev)
    C = torch.empty(M, N, device=dev)
    part = torch.empty(2, N, load().pcs_gemm_row_blocks(M, N), dtype=torch.float64, device=dev)
    aop = operand(A, lda, OP_BNACT, s, t, 0, 0.0) if K % 4 == 0 else operand(A, lda)
    fwd = lambda: gemm_rows(aop, M, K, W, lda, b, C, N, N, part, st=st)  # noqa
    ms = timeit(fwd)
    fl = 2.0 * M * K * N
    by = 4.0 * M * (lda + N)
    dW = torch.zeros(N, K, device=dev)  # noqa
    db = torch.zeros(N, device=dev)
    Z = torch.randn(M, N, device=dev)
    sN, tN = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
    mN, aN, kN = torch.randn(N, device=dev), torch.randn(N, device=dev) * 1e-3, torch.randn(N, device=dev) * 1e-3
    xop = operand(C, N, OP_BNBWD, sN, tN, 0, 0.0, Z, N, mN, None, aN, kN)
    wg = lambda: wgrad(xop, N, aop, K, M, dW, db, st)  # noqa
    ms2 = timeit(wg)
    # dgrad: dA (M x K) = dZ(M x N, rebuilt from C and Z) . W, epilogue = previous layer's BN-backward sums
    if K % 4 == 0:
        Wt = W[:, :K].t().contiguous()
        dA = torch.empty(M, K, device=dev)
        ZK = torch.randn(M, K, device=dev)
        bpart = torch.empty(2, K, load().pcs_gemm_row_blocks_dgrad(M, K), dtype=torch.float64, device=dev)
        epi = operand(None, 0, OP_BNBWD, s, t, 0, 0.0, ZK, K, torch.randn(K, device=dev), torch.rand(K, device=dev))
        dg = lambda: gemm_rows(xop, M, N, Wt, N, None, dA, K, K, None, epi, bpart, st=st)  # noqa
        ms3 = timeit(dg)
        dgs = f'{ms3*1e3:8.1f} us {fl/ms3/1e9:6.1f} TF/s'
    else:
        dgs = '       -'
    print(f'{name:8s} M={M:8d} K={K:5d} N={N:5d}  fwd {ms*1e3:8.1f} us {fl/ms/1e9:6.1f} TF/s {by/ms/1e6:6.0f} GB/s'
          f' | dgrad {dgs} | wgrad {ms2*1e3:8.1f} us {fl/ms2/1e9:6.1f} TF/s', flush=True)
