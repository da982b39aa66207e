"""One data-gradient GEMM launch shape, repeated (for rocprofv3 --pmc passes on a single kernel):
SA2 layer 3's dgrad at B=32 (M = 262144 rows, dZ 128 wide rebuilt from dy and Z, cin = 64,
k-major W, BN-backward epilogue)."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg._lib import stream_ptr, load, OP_BNBWD  # noqa: E402
from pcseg.engine import operand, gemm_rows_kmajor  # noqa: E402

M, C, K = int(os.environ.get('DG_M', 1 << 18)), int(os.environ.get('DG_C', 128)), int(os.environ.get('DG_K', 64))
dev = 'cuda'
st = stream_ptr(torch.device(dev))
W = torch.randn(C, K, device=dev)
dy, Z = torch.randn(M, C, device=dev), torch.randn(M, C, device=dev)
xo = operand(dy, C, OP_BNBWD, torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1, 0, 0.0, Z, C,
             torch.randn(C, device=dev) * 0.1, None, torch.randn(C, device=dev) * 1e-2,
             torch.randn(C, device=dev) * 1e-2)
ZK = torch.randn(M, K, device=dev)
epi = operand(None, 0, OP_BNBWD, torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev), 0, 0.0, ZK, K,
              torch.randn(K, device=dev), torch.rand(K, device=dev))
dA = torch.empty(M, K, device=dev)
bpart = torch.empty(2, K, load().pcs_gemm_row_blocks_dgrad(M, K), dtype=torch.float64, device=dev)
for _ in range(int(os.environ.get('DG_REPS', 10))):
    gemm_rows_kmajor(xo, M, C, W, K, dA, K, K, epi, bpart, st=st)
torch.cuda.synchronize()
print('done', flush=True)
