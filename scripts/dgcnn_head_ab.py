"""DGCNN head GEMMs (conv5-7 at B=32, N=4096): forward vs data / weight gradient with the
layer's dZ rebuilt on load (BNBWD) or read materialised (PLAIN), HIP-event timing.
Decides whether wide layers should materialise dZ once instead of rebuilding it in every
column tile."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg._lib import stream_ptr, load, OP_BNBWD  # noqa: E402
from pcseg.engine import operand, gemm_rows, gemm_rows_kmajor, wgrad  # noqa: E402

dev = 'cuda'
torch.manual_seed(0)
M = 32 * 4096
SHAPES = [('conv5', 384, 1024), ('conv6', 1408, 512), ('conv7', 512, 256)]   # (name, cin, cout)
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


for name, K, N in SHAPES:
    fl = 2.0 * M * K * N
    X = torch.randn(M, K, device=dev)                   # layer input
    W = torch.randn(N, K, device=dev) / K ** 0.5
    Z = torch.empty(M, N, device=dev)
    nb = lib.pcs_gemm_row_blocks(M, N)
    part = torch.empty(2, N, nb, dtype=torch.float64, device=dev)
    us_f = timeit(lambda: gemm_rows(operand(X, K), M, K, W, K, None, Z, N, N, part, st=st))
    # the layer's output gradient dy and BN-backward coefficients
    dy = torch.randn(M, N, device=dev)
    s, t = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
    mean, al, kb = torch.randn(N, device=dev) * 0.1, torch.randn(N, device=dev) * 1e-2, torch.randn(N, device=dev) * 1e-2
    xb = operand(dy, N, OP_BNBWD, s, t, 1, 0.2, Z, N, mean, None, al, kb)
    dZ = torch.randn(M, N, device=dev)
    xp = operand(dZ, N)
    # previous layer's BN-backward epilogue (its Z and coefficients)
    ZK = torch.randn(M, K, device=dev)
    sK, tK = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
    epi = operand(None, 0, OP_BNBWD, sK, tK, 1, 0.2, ZK, K, torch.randn(K, device=dev), torch.rand(K, device=dev))
    dA = torch.empty(M, K, device=dev)
    nbg = lib.pcs_gemm_row_blocks_dgrad(M, K)
    bpart = torch.empty(2, K, nbg, dtype=torch.float64, device=dev)
    res = {}
    for tag, xo in (('rebuilt', xb), ('plain', xp)):
        res[f'dgrad {tag}+epi'] = timeit(lambda: gemm_rows_kmajor(xo, M, N, W, K, dA, K, K, epi, bpart, st=st))
        res[f'dgrad {tag}'] = timeit(lambda: gemm_rows_kmajor(xo, M, N, W, K, dA, K, K, st=st))
        dW = torch.zeros(N, K, device=dev)
        ws = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
        res[f'wgrad {tag}'] = timeit(lambda: wgrad(xo, N, operand(X, K), K, M, dW, None, st, ws))
    if os.environ.get('HEAD_TORCH', '1') == '1':     # vendor fp32 GEMM (hipBLASLt/rocBLAS) as a ceiling reference
        torch.backends.cuda.matmul.allow_tf32 = False
        res['torch fwd'] = timeit(lambda: torch.mm(X, W.t(), out=Z))
        res['torch dgrad'] = timeit(lambda: torch.mm(dZ, W, out=dA))
        dWt = torch.empty(N, K, device=dev)
        res['torch wgrad'] = timeit(lambda: torch.mm(dZ.t(), X, out=dWt))
    line = f'{name} M={M} K={K} N={N}: fwd {us_f:7.0f} us {fl / us_f / 1e6:5.1f} TF'
    for k, us in res.items():
        line += f' | {k} {us:7.0f} us {fl / us / 1e6:5.1f} TF'
    print(line, flush=True)
    del X, Z, dy, dZ, ZK, dA
    torch.cuda.empty_cache()
