"""Pruned kNN diagnostics (PCS_LIB=.../libpcseg_kdiag.so): per graph of DGCNNWithColor's forward
(B=32, N=4096, k=20), the candidate tiles each wave scanned (mean / max fraction, and the mean over
4-wave blocks of their slowest wave: what a block's LDS residency costs), its running merges and
the s_memtime cycles of its setup, scan and final merge (100 MHz... see the wall-clock note in the
output: s_memtime counts the shader clock on gfx950)."""
import ctypes
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg import _lib, ops  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

B, N, k = 32, 4096, 20
torch.manual_seed(0)
m = pcseg.DGCNNWithColor(14).cuda().train()
pts, _, _ = make_batch(B, N, seed=3)
x = pts[:, :, :6].contiguous().transpose(1, 2).cuda()
feats, graphs = [], []
orig = pcseg.models.EdgeConv.forward_graph


def rec(self, xp, seeds=None, **kw):
    out, idx = orig(self, xp, seeds, **kw)
    feats.append(xp.detach().clone())
    graphs.append(idx)
    return out, idx


pcseg.models.EdgeConv.forward_graph = rec
with torch.no_grad():
    m(x)
pcseg.models.EdgeConv.forward_graph = orig
lib = _lib.load()
nt = N // 32
od = ops.knn_order(feats[0])
for i in range(4):
    sd = None if i == 0 else graphs[i - 1]
    ops.knn(feats[i], k, seeds=sd, order=od)
    torch.cuda.synchronize()
    buf = (ctypes.c_int * (8 * B * nt))()
    lib.pcs_knn_diag(buf, 8 * B * nt)
    d = np.frombuffer(buf, dtype=np.int32).reshape(B, nt, 8)
    c = d[..., 0] / nt
    blk = c.reshape(B, nt // 4, 4).max(-1).mean()
    cyc = d[..., 2:5].astype(np.float64)
    print(f'graph {i + 1}: scanned mean {c.mean():.3f} max {c.max():.3f} block-max mean {blk:.3f} '
          f'p90 {np.percentile(c, 90):.3f} | merges/wave {d[..., 1].mean():.1f} | kcycles/wave setup '
          f'{cyc[..., 0].mean() / 1e3:.1f} scan {cyc[..., 1].mean() / 1e3:.1f} final {cyc[..., 2].mean() / 1e3:.1f} '
          f'| scan kcycles per scanned tile {(cyc[..., 1] / np.maximum(d[..., 0], 1)).mean() / 1e3:.2f} '
          f'| setup split: seeds {d[..., 5].mean() / 1e3:.1f} bounds {d[..., 6].mean() / 1e3:.1f}', flush=True)
