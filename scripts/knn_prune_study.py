"""Offline study (CPU, numpy) for a tile-pruned kNN: on DGCNN's own kNN inputs
(scripts/knn_dump.py), points ordered by the Morton code of their xyz, 32-point tiles; for each
32-row query block and candidate tile, can the tile be skipped because even its closest possible
point is farther than every row's k-th neighbour bound?  Bounds: bounding spheres (centroid +
radius) and axis-aligned boxes.  Row thresholds: the exact k-th neighbour distance (best case) and
the seed bound the kernel starts from (graph 1: the k-th over the 20 Morton neighbours; graphs 2-4:
over the previous graph's lists).  Prints the fraction of (block, tile) pairs that must be computed."""
import sys

import numpy as np

d = np.load(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/knn_feats.npz')
K, T = 20, 32


def morton(xyz):
    lo, hi = xyz.min(0), xyz.max(0)
    q = ((xyz - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64)
    key = np.zeros(len(xyz), np.int64)
    for b in range(10):
        for a in range(3):
            key |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return np.argsort(key, kind='stable')


for c in range(d['xyz'].shape[0]):
    xyz = d['xyz'][c].astype(np.float64)
    order = morton(xyz)
    for gi in range(4):
        f = d[f'f{gi}'][c].astype(np.float64)
        n = len(f)
        D = ((f[:, None, :] - f[None, :, :]) ** 2).sum(-1)
        kth = np.sort(D, 1)[:, K - 1]
        if gi == 0:
            pos = np.empty(n, np.int64)
            pos[order] = np.arange(n)
            nb = np.array([order[np.clip(np.arange(p - 10, p + 11), 0, n - 1)] for p in pos])
            seedb = np.sort(np.take_along_axis(D, nb, 1), 1)[:, K - 1]
        else:
            g = d[f'g{gi - 1}'][c]
            seedb = np.sort(np.take_along_axis(D, g.astype(np.int64), 1), 1)[:, K - 1]
        fo = f[order]
        nt = n // T
        tiles = fo.reshape(nt, T, -1)
        cen = tiles.mean(1)
        rad = np.sqrt(((tiles - cen[:, None]) ** 2).sum(-1)).max(1)
        lo, hi = tiles.min(1), tiles.max(1)
        cd = np.sqrt(((cen[:, None] - cen[None]) ** 2).sum(-1))
        sph = np.maximum(cd - rad[:, None] - rad[None], 0) ** 2
        gap = np.maximum(0, np.maximum(lo[:, None] - hi[None], lo[None] - hi[:, None]))
        box = (gap ** 2).sum(-1)
        lb = np.maximum(sph, box)
        for name, thr in (('exact', kth), ('seed', seedb)):
            tb = thr[order].reshape(nt, T).max(1)         # the block's loosest row
            keep = (lb <= tb[:, None] * (1 + 1e-4)).mean()
            keep_s = (sph <= tb[:, None] * (1 + 1e-4)).mean()
            print(f'cloud {c} graph {gi + 1} (F={f.shape[1]}): {name:5s} threshold -> compute '
                  f'{keep:.3f} of tiles (spheres only {keep_s:.3f})', flush=True)
