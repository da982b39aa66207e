"""Row-GEMM check + timing on the engine's shapes: forward (BNACT + BN stats), data gradient
(BNBWD / POOLBWD over k-major W + BN-backward epilogue), against an fp64 torch reference,
HIP-event timing.  (Round 2 used it to A/B an LDS-DMA pipelined variant against the
register-staged kernel: DESIGN.md section 8.)"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg._lib import stream_ptr, load, call, OP_BNACT, OP_BNBWD, OP_POOLBWD  # noqa: E402
from pcseg.engine import operand, gemm_rows, gemm_rows_kmajor  # noqa: E402

dev = 'cuda'
torch.manual_seed(0)
SHAPES = [  # (name, M, K, N, pool_k of the dgrad's A (0 = BNBWD))
    ('sa1.l2', 1048576, 32, 32, 0), ('sa1.l3', 1048576, 32, 64, 32),
    ('sa2.l2', 262144, 64, 64, 0), ('sa2.l3', 262144, 64, 128, 32),
    ('sa3.l2', 65536, 128, 128, 0), ('sa3.l3', 65536, 128, 256, 32),
    ('sa4.l3', 16384, 256, 512, 32), ('fp2.l1', 32768, 320, 256, 0), ('fp1.lx', 131072, 128, 128, 0),
    ('dg.c5', 131072, 384, 1024, 0), ('dg.c6', 131072, 1408, 512, 0), ('dg.c7', 131072, 512, 256, 0),
]
_only = os.environ.get('GEMM_SHAPES')
if _only:
    SHAPES = [sh for sh in SHAPES if any(sh[0].startswith(p) for p in _only.split(','))]
REPS = int(os.environ.get('GEMM_REPS', '10'))
st = stream_ptr(torch.device(dev))
lib = load()


def timeit(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / REPS * 1e3


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def act(y):
    return torch.relu(y)


for name, M, K, N, pk in SHAPES:
    # ---------------- forward: C = relu(A*s+t) W^T + b, stats of C
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev) / K ** 0.5
    s = torch.rand(K, device=dev) + 0.5
    t = torch.randn(K, device=dev) * 0.1
    b = torch.randn(N, device=dev)
    res = {}
    for impl in (0,):
        C = torch.empty(M, N, device=dev)
        nb = lib.pcs_gemm_row_blocks(M, N)
        part = torch.empty(2, N, nb, dtype=torch.float64, device=dev)
        aop = operand(A, K, OP_BNACT, s, t, 0, 0.0)
        fwd = lambda: gemm_rows(aop, M, K, W, K, b, C, N, N, part, st=st)  # noqa
        us = timeit(fwd)
        res[impl] = (us, C.clone(), part.sum(-1).clone())
    ref = (act(A.double() * s.double() + t.double()) @ W.double().t() + b.double())
    fl = 2.0 * M * K * N
    by = 4.0 * M * (K + N)
    line = f'{name:7s} M={M:8d} K={K:5d} N={N:5d} fwd  '
    for impl in (0,):
        us, C, ps = res[impl]
        line += (f'[{"engine"}] {us:8.1f} us {fl / us / 1e6:6.1f} TF {by / us / 1e3:6.0f} GB/s '
                 f'err {rel(C, ref):.1e} sum {rel(ps[0], ref.sum(0)):.1e}  ')
    print(line, flush=True)
    # ---------------- data gradient: dA = dZ . W  (W k-major N_out x K_in), dZ rebuilt
    # the layer has N outputs (dZ: M x N), the GEMM's K = N, output dA: M x K
    Z = torch.randn(M, N, device=dev)
    sN, tN = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
    mN = torch.randn(N, device=dev) * 0.1
    aN, kN = torch.randn(N, device=dev) * 1e-2, torch.randn(N, device=dev) * 1e-2
    if pk:
        G = M // pk
        dpool = torch.randn(G, N, device=dev)
        arg = torch.randint(0, pk, (G, N), dtype=torch.uint8, device=dev)
        xop = operand(dpool, N, OP_POOLBWD, sN, tN, 0, 0.0, Z, N, mN, None, aN, kN, arg, pk)
        rows = torch.arange(M, device=dev)
        dyfull = torch.where(arg.long().repeat_interleave(pk, 0) == (rows % pk).unsqueeze(1),
                             dpool.repeat_interleave(pk, 0), torch.zeros((), device=dev))
    else:
        dyfull = torch.randn(M, N, device=dev)
        xop = operand(dyfull, N, OP_BNBWD, sN, tN, 0, 0.0, Z, N, mN, None, aN, kN)
    ZK = torch.randn(M, K, device=dev)
    sK, tK = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
    mK, iK = torch.randn(K, device=dev) * 0.1, torch.rand(K, device=dev) + 0.5
    epi = operand(None, 0, OP_BNBWD, sK, tK, 0, 0.0, ZK, K, mK, iK)
    zd = Z.double()
    dy = dyfull.double() * ((zd * sN.double() + tN.double()) > 0).double()
    dZ = sN.double() * dy - kN.double() - aN.double() * (zd - mN.double())
    dref = dZ @ W.double()                      # (M x N) . (N x K)
    res = {}
    for impl in (0,):
        dA = torch.empty(M, K, device=dev)
        nb = lib.pcs_gemm_row_blocks_dgrad(M, K)
        bpart = torch.empty(2, K, nb, dtype=torch.float64, device=dev)
        dg = lambda: gemm_rows_kmajor(xop, M, N, W, K, dA, K, K, epi, bpart, st=st)  # noqa
        us = timeit(dg)
        res[impl] = (us, dA.clone(), bpart.sum(-1).clone())
    dyk = dref * ((ZK.double() * sK.double() + tK.double()) > 0).double()
    line = f'{name:7s} M={M:8d} K={N:5d} N={K:5d} dgr{"P" if pk else "B"} '
    by = 4.0 * M * (2 * N + 2 * K)
    for impl in (0,):
        us, dA, bs = res[impl]
        line += (f'[{"engine"}] {us:8.1f} us {fl / us / 1e6:6.1f} TF {by / us / 1e3:6.0f} GB/s '
                 f'err {rel(dA, dref):.1e} bsum {rel(bs[0], dyk.sum(0)):.1e}  ')
    print(line, flush=True)
    del A, Z, ZK, dyfull
    torch.cuda.empty_cache()
