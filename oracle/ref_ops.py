"""PyTorch-CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).

This is the oracle every HIP kernel is checked against and the `cpu_baseline`
leg of `bench.py`.  It restates the reference algorithm op for op, on the CPU,
with the same ATen calls wherever the result depends on them (topk tie
resolution, vector_norm rounding), so it reproduces the reference bit for bit
on identical inputs.  It is pinned against fixtures captured from the
reference itself (tests/golden/make_golden.py, tests/test_oracle_golden.py).

Deviations from the reference, all test hooks:
  * FPS start indices and DGCNN kNN indices can be injected / recorded through
    `Replay` (the reference draws `torch.randint` inside `sample`,
    models/utils/common.py:22, and recomputes kNN in every EdgeConv,
    models/dgcnn/dgcnn.py:34).
  * `get_graph_feature` uses the input's device instead of
    `'cuda' if available` (dgcnn.py:39) -- this oracle only runs on the CPU.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# replay / record of the random and rounding-sensitive choices
# --------------------------------------------------------------------------
class Replay:
    """Queues of FPS starts / kNN indices consumed in call order, plus records."""

    def __init__(self, fps_starts=None, knn_idx=None, fps_idx=None, group_idx=None, interp_idx=None,
                 pool_arg=None, act_mask=None):
        self.fps_starts = list(fps_starts) if fps_starts is not None else None
        self.knn_idx = list(knn_idx) if knn_idx is not None else None
        # full index replay (used to run the oracle in float64 on the float32 run's neighbour choices)
        self.fps_idx = list(fps_idx) if fps_idx is not None else None
        self.group_idx = list(group_idx) if group_idx is not None else None
        self.interp_idx = list(interp_idx) if interp_idx is not None else None
        # max-pool argmax decisions of another run (SA / InvResMLP reduce, EdgeConv max over k),
        # (groups, channels) in forward order: the pool takes the value at that index instead of
        # re-deciding near-ties (test hook; the reference always takes torch.max)
        self.pool_arg = list(pool_arg) if pool_arg is not None else None
        # activation decisions of another run (y > 0 of every engine-site ReLU / LeakyReLU, rows x
        # channels, forward order): ReLU / LeakyReLU take that sign decision instead of their own
        self.act_mask = list(act_mask) if act_mask is not None else None
        self.rec_fps_starts: list[torch.Tensor] = []
        self.rec_fps_idx: list[torch.Tensor] = []
        self.rec_group_idx: list[torch.Tensor] = []
        self.rec_interp_idx: list[torch.Tensor] = []
        self.rec_knn_idx: list[torch.Tensor] = []


_ACTIVE: list[Replay] = []


@contextlib.contextmanager
def replay(rp: Replay):
    _ACTIVE.append(rp)
    try:
        yield rp
    finally:
        _ACTIVE.pop()


def _rp():
    return _ACTIVE[-1] if _ACTIVE else None


# --------------------------------------------------------------------------
# a1  farthest point sampling            (models/utils/common.py:6-34)
# --------------------------------------------------------------------------
def fps_indices(coords: torch.Tensor, C: int, start: torch.Tensor | None = None) -> torch.Tensor:
    """Indices (B, C) int32 picked by the reference's iterative FPS.

    Same ops as common.py:17-31: running min of `vector_norm` with a strict
    `<` mask, next = first argmax.  `start` replaces the `torch.randint` draw
    of common.py:22.
    """
    B, N, _ = coords.shape
    if start is None:
        start = torch.randint(0, N, (B,), dtype=torch.int)
    far = start.to(torch.int64)
    out = torch.zeros((B, C), dtype=torch.int)
    best = torch.full((B, N), torch.inf)
    rows = torch.arange(B)
    for i in range(C):
        out[:, i] = far.to(torch.int)
        c = coords[rows, far, :].view(B, 1, 3)
        d = torch.linalg.vector_norm(coords - c, dim=-1)
        m = d < best
        best[m] = d[m]
        _, far = torch.max(best, -1)
    return out


def sample(coords: torch.Tensor, C: int) -> torch.Tensor:
    """Reference `sample` (common.py:6-34): returns centroid coordinates (B, C, 3)."""
    rp = _rp()
    start = None
    if rp is not None and rp.fps_starts is not None:
        start = rp.fps_starts.pop(0)
    B, N, _ = coords.shape
    if rp is not None and rp.fps_idx:
        idx = rp.fps_idx.pop(0)
        start = idx[:, 0].clone()
    else:
        if start is None:
            start = torch.randint(0, N, (B,), dtype=torch.int)
        idx = fps_indices(coords, C, start)
    if rp is not None:
        rp.rec_fps_starts.append(start.clone())
        rp.rec_fps_idx.append(idx.clone())
    rows = torch.arange(B).view(B, 1).expand(B, C)
    return coords[rows, idx.long(), :]


# --------------------------------------------------------------------------
# a2  ball query + group                 (common.py:37-71)
# --------------------------------------------------------------------------
def ball_query(centroids: torch.Tensor, coords: torch.Tensor, r: float, K: int) -> torch.Tensor:
    """(B, C, K) int64 neighbour indices exactly as common.py:54-61 selects them."""
    B, C, _ = centroids.shape
    N = coords.shape[1]
    diff = coords.unsqueeze(1).expand(B, C, N, 3) - centroids.unsqueeze(2).expand(B, C, N, 3)
    d = (diff ** 2).sum(dim=-1)
    d[~(d <= r ** 2)] = torch.inf
    return torch.topk(d, K, dim=-1, largest=False, sorted=True)[1]


def group(centroid_coords, coords, features, r, K, normalize=False):
    """Reference `group` (common.py:37-71) -> (B, C, K, 3+D)."""
    B, N, _ = features.shape
    C = centroid_coords.shape[1]
    rp = _rp()
    if rp is not None and rp.group_idx:
        idx = rp.group_idx.pop(0).long()
    else:
        idx = ball_query(centroid_coords, coords, r, K)
    if rp is not None:
        rp.rec_group_idx.append(idx.clone())
    bi = torch.arange(B).view(B, 1, 1).expand(B, C, K)
    gc = coords[bi, idx]
    gf = features[bi, idx]
    gc = gc - centroid_coords.view(B, C, 1, 3)
    if normalize:
        gc = gc / r
    return torch.cat([gc, gf], dim=-1)


# --------------------------------------------------------------------------
# a3  reduce                             (common.py:74-91)
# --------------------------------------------------------------------------
def _replayed_arg(shape_bcd):
    rp = _rp()
    if rp is not None and rp.pool_arg:
        return rp.pool_arg.pop(0).long().reshape(shape_bcd)
    return None


def act(y: torch.Tensor, slope: float = 0.0, layout: str = 'points') -> torch.Tensor:
    """F.relu (slope 0) / LeakyReLU(slope) of an engine-site activation; with a replayed sign
    decision (Replay.act_mask, rows x channels in the product's point-major layout) the
    branch is taken from it.  layout: 'points' y (B, C, N) <- rows (B*N, C); 'grouped'
    y (B, C, G, K) <- rows (B*G*K, C)."""
    rp = _rp()
    if rp is None or not rp.act_mask:
        return F.relu(y) if slope == 0.0 else F.leaky_relu(y, slope)
    m = rp.act_mask.pop(0)
    if layout == 'grouped':
        B, C, G, K = y.shape
        m = m.reshape(B, G, K, C).permute(0, 3, 1, 2)
    else:
        B, C, N = y.shape
        m = m.reshape(B, N, C).permute(0, 2, 1)
    return torch.where(m, y, y * slope)


def _seq_act(seq, x):
    """Sequential(Conv1d, BatchNorm1d, LeakyReLU[, Dropout]) (dgcnn.py:188-210) with the
    activation through `act`."""
    y = act(seq[1](seq[0](x)), seq[2].negative_slope, 'points')
    for mod in list(seq)[3:]:
        y = mod(y)
    return y


def reduce(x: torch.Tensor, type: str) -> torch.Tensor:
    if type == 'max':
        arg = _replayed_arg((x.shape[0], x.shape[1], x.shape[3]))
        if arg is not None:
            return x.gather(2, arg.unsqueeze(2)).squeeze(2)
        return torch.max(x, dim=2)[0]
    if type == 'avg':
        # the reference indexes [0] after the mean (common.py:89); kept as is.
        return torch.mean(x, dim=2)[0]
    raise ValueError(f"'{type}' pooling not supported; use 'max' or 'avg'.")


# --------------------------------------------------------------------------
# a4  3-NN inverse-distance interpolation (common.py:94-122)
# --------------------------------------------------------------------------
def three_nn(coords_1, coords_2, k=3):
    B, N, _ = coords_1.shape
    M = coords_2.shape[1]
    diff = coords_2.unsqueeze(1).expand(B, N, M, 3) - coords_1.unsqueeze(2).expand(B, N, M, 3)
    d = (diff ** 2).sum(dim=-1)
    return torch.topk(d, k, dim=-1, largest=False, sorted=True)


def interpolate(points, coords_1, coords_2, k=3):
    B, N, _ = coords_1.shape
    rp = _rp()
    if rp is not None and rp.interp_idx:
        idx = rp.interp_idx.pop(0).long()
        bj = torch.arange(B).view(B, 1, 1).expand_as(idx)
        dist = ((coords_2[bj, idx] - coords_1.unsqueeze(2)) ** 2).sum(dim=-1)
    else:
        dist, idx = three_nn(coords_1, coords_2, k)
    if rp is not None:
        rp.rec_interp_idx.append(idx.clone())
    bi = torch.arange(B).view(B, 1, 1).expand(B, N, k)
    p = points[bi, idx]
    w = 1.0 / (dist.view(B, N, k, 1) + 1e-9)
    norm = torch.sum(w, dim=2, keepdim=True)
    return torch.sum(p * w / norm, dim=2)


# --------------------------------------------------------------------------
# a12/a13  DGCNN kNN + graph feature      (models/dgcnn/dgcnn.py:7-57)
# --------------------------------------------------------------------------
def knn(x, k):
    inner = -2 * torch.matmul(x.transpose(2, 1), x)
    xx = torch.sum(x ** 2, dim=1, keepdim=True)
    pd = -xx - inner - xx.transpose(2, 1)
    return pd.topk(k=k, dim=-1)[1]


def get_graph_feature(x, k=20, idx=None, dim9=False):
    B = x.size(0)
    N = x.size(2)
    x = x.view(B, -1, N)
    if idx is None:
        rp = _rp()
        if rp is not None and rp.knn_idx is not None:
            idx = rp.knn_idx.pop(0)
        elif dim9:
            idx = knn(x[:, 6:], k=k)
        else:
            idx = knn(x, k=k)
        if rp is not None:
            rp.rec_knn_idx.append(idx.clone())
    base = torch.arange(0, B, device=x.device).view(-1, 1, 1) * N
    flat = (idx + base).view(-1)
    Cd = x.size(1)
    xt = x.transpose(2, 1).contiguous()
    feat = xt.view(B * N, -1)[flat, :].view(B, N, k, Cd)
    xr = xt.view(B, N, 1, Cd).repeat(1, 1, k, 1)
    if dim9:
        return torch.cat((feat - xr, xr, xr), dim=3).permute(0, 3, 1, 2).contiguous()
    return torch.cat((feat - xr, xr), dim=3).permute(0, 3, 1, 2).contiguous()


# --------------------------------------------------------------------------
# a5..a11 building blocks and models (same parameter names as the reference)
# --------------------------------------------------------------------------
class MiniPointNet(nn.Module):           # common.py:125-150
    def __init__(self, in_channels, mlps):
        super().__init__()
        self.conv = nn.ModuleList()
        self.batch = nn.ModuleList()
        prev = in_channels
        for m in mlps:
            self.conv.append(nn.Conv2d(prev, m, (1, 1)))
            self.batch.append(nn.BatchNorm2d(m))
            prev = m

    def forward(self, x):
        for c, b in zip(self.conv, self.batch):
            x = act(b(c(x)), 0.0, 'grouped')
        return x


class UnitPointNet(nn.Module):           # common.py:153-178
    def __init__(self, in_channels, mlps):
        super().__init__()
        self.conv = nn.ModuleList()
        self.batch = nn.ModuleList()
        prev = in_channels
        for m in mlps:
            self.conv.append(nn.Conv1d(prev, m, 1))
            self.batch.append(nn.BatchNorm1d(m))
            prev = m

    def forward(self, x):
        for c, b in zip(self.conv, self.batch):
            x = act(b(c(x)), 0.0, 'points')
        return x


class SetAbstraction(nn.Module):         # common.py:180-214
    def __init__(self, C, radius, in_channels, mlps, K=32, pooling_type='max', grouping_norm=False):
        super().__init__()
        self.point_net = MiniPointNet(in_channels, mlps)
        self.C, self.radius, self.K = C, radius, K
        self.pooling_type, self.grouping_norm = pooling_type, grouping_norm

    def forward(self, coords, features):
        cc = sample(coords, self.C)
        f = group(cc, coords, features, self.radius, self.K, self.grouping_norm)
        f = self.point_net(f.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
        return cc, reduce(f, self.pooling_type)


class FeaturePropagation(nn.Module):     # common.py:217-243
    def __init__(self, in_channels, mlps):
        super().__init__()
        self.point_net = UnitPointNet(in_channels, mlps)

    def forward(self, coords_1, coords_2, features_1, features_2):
        f2 = interpolate(features_2, coords_1, coords_2)
        f = torch.cat([features_1, f2], dim=-1) if features_1 is not None else f2
        return self.point_net(f.permute(0, 2, 1)).permute(0, 2, 1)


class InvResMLP(nn.Module):              # common.py:246-301
    def __init__(self, radius, in_channels, mlp_size, K, pooling_type='max'):
        super().__init__()
        self.radius, self.K, self.pooling_type = radius, K, pooling_type
        self.neighbour_features_mlp = MiniPointNet(in_channels, [mlp_size])
        self.point_features_mlp = UnitPointNet(mlp_size, [4 * mlp_size, mlp_size])

    def forward(self, centroid_coords, coords, features):
        g = group(centroid_coords, coords, features, self.radius, self.K, True)
        f = self.neighbour_features_mlp(g.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
        f = reduce(f, self.pooling_type)
        f = self.point_features_mlp(f.permute(0, 2, 1)).permute(0, 2, 1)
        return centroid_coords, f + features


class PointNetpp(nn.Module):             # models/PointNetpp/PointNetpp.py:6-48
    def __init__(self, part_classes):
        super().__init__()
        self.sa1 = SetAbstraction(1024, 0.1, 9, [32, 32, 64])
        self.sa2 = SetAbstraction(256, 0.2, 64 + 3, [64, 64, 128])
        self.sa3 = SetAbstraction(64, 0.4, 128 + 3, [128, 128, 256])
        self.sa4 = SetAbstraction(16, 0.8, 256 + 3, [256, 256, 512])
        self.fp4 = FeaturePropagation(512 + 256, [256, 256])
        self.fp3 = FeaturePropagation(256 + 128, [256, 256])
        self.fp2 = FeaturePropagation(256 + 64, [256, 128])
        self.fp1 = FeaturePropagation(128, [128, 128, 128, 128])
        self.drop = nn.Dropout(0.5)
        self.conv = nn.Conv1d(128, part_classes, 1)

    def forward(self, x):
        c0, f0 = x[:, :, :3], x[:, :, 3:]
        c1, f1 = self.sa1(c0, f0)
        c2, f2 = self.sa2(c1, f1)
        c3, f3 = self.sa3(c2, f2)
        c4, f4 = self.sa4(c3, f3)
        f3 = self.fp4(c3, c4, f3, f4)
        f2 = self.fp3(c2, c3, f2, f3)
        f1 = self.fp2(c1, c2, f1, f2)
        f0 = self.fp1(c0, c1, None, f1)
        y = self.drop(f0).permute(0, 2, 1)
        return self.conv(y).permute(0, 2, 1)


class PointNetppMSG(nn.Module):
    """PointNet++ MSG (BASELINE.json config 4).  NOT in the reference: composed here from the
    reference's own blocks -- `sample` (common.py:6-34) once per level, then per radius
    `group` (common.py:37-71) -> MiniPointNet (common.py:125-150) -> `reduce` max
    (common.py:74-91), the branches concatenated in radius order; FeaturePropagation
    (common.py:217-243) as in PointNetpp.py:19-22, 42-45 -- with the standard sem-seg MSG
    widths of SURVEY.md section 8(d).  Same module tree / state_dict keys as pcseg.PointNetppMSG."""

    CFG = [  # (C, radii, Ks, [mlp per scale])
        (1024, (0.05, 0.1), (16, 32), ([16, 16, 32], [32, 32, 64])),
        (256, (0.1, 0.2), (16, 32), ([64, 64, 128], [64, 96, 128])),
        (64, (0.2, 0.4), (16, 32), ([128, 196, 256], [128, 196, 256])),
        (16, (0.4, 0.8), (16, 32), ([256, 256, 512], [256, 384, 512])),
    ]

    def __init__(self, part_classes):
        super().__init__()
        self.levels = nn.ModuleList()
        d, skips = 6, [6]
        for C, radii, Ks, mlps in self.CFG:
            self.levels.append(nn.ModuleList([SetAbstraction(C, r, d + 3, m, K=k)
                                              for r, k, m in zip(radii, Ks, mlps)]))
            d = sum(m[-1] for m in mlps)
            skips.append(d)
        self.fp4 = FeaturePropagation(skips[4] + skips[3], [256, 256])
        self.fp3 = FeaturePropagation(256 + skips[2], [256, 256])
        self.fp2 = FeaturePropagation(256 + skips[1], [256, 128])
        self.fp1 = FeaturePropagation(128, [128, 128, 128])
        self.drop = nn.Dropout(0.5)
        self.conv = nn.Conv1d(128, part_classes, 1)

    @staticmethod
    def _level(branches, coords, feats):
        cc = sample(coords, branches[0].C)                 # one centroid set shared by the scales
        outs = []
        for sa in branches:
            f = group(cc, coords, feats, sa.radius, sa.K, sa.grouping_norm)
            f = sa.point_net(f.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
            outs.append(reduce(f, sa.pooling_type))
        return cc, torch.cat(outs, dim=-1)

    def forward(self, x):
        cs, fs = [x[:, :, :3]], [x[:, :, 3:]]
        for branches in self.levels:
            c, f = self._level(branches, cs[-1], fs[-1])
            cs.append(c)
            fs.append(f)
        f3 = self.fp4(cs[3], cs[4], fs[3], fs[4])
        f2 = self.fp3(cs[2], cs[3], fs[2], f3)
        f1 = self.fp2(cs[1], cs[2], fs[1], f2)
        f0 = self.fp1(cs[0], cs[1], None, f1)
        y = self.drop(f0).permute(0, 2, 1)
        return self.conv(y).permute(0, 2, 1)


class PointNeXt(nn.Module):              # models/PointNeXt/PointNeXt.py:17-147
    def __init__(self, part_classes, version='b'):
        super().__init__()
        self.num_classes = part_classes
        self.mlp = UnitPointNet(9, [32])
        self.sa1 = SetAbstraction(1024, 0.1, 32 + 3, [32, 32, 64], grouping_norm=True)
        self.irmlp1 = InvResMLP(0.1, 64 + 3, 64, 32)
        self.sa2 = SetAbstraction(256, 0.2, 64 + 3, [64, 64, 128], grouping_norm=True)
        self.irmlp2 = InvResMLP(0.1, 128 + 3, 128, 32)
        self.irmlp2_1 = InvResMLP(0.2, 128 + 3, 128, 32)
        self.sa3 = SetAbstraction(64, 0.4, 128 + 3, [128, 128, 256], grouping_norm=True)
        self.irmlp3 = InvResMLP(0.4, 256 + 3, 256, 32)
        self.sa4 = SetAbstraction(16, 0.8, 256 + 3, [256, 256, 512], grouping_norm=True)
        self.irmlp4 = InvResMLP(0.8, 512 + 3, 512, 16)
        self.fp4 = FeaturePropagation(512 + 256, [256, 256])
        self.fp3 = FeaturePropagation(256 + 128, [256, 256])
        self.fp2 = FeaturePropagation(256 + 64, [256, 128])
        self.fp1 = FeaturePropagation(128 + 32, [128, 128, 128, 128])
        self.drop = nn.Dropout(0.5)
        self.conv = nn.Conv1d(128, part_classes, 1)

    def forward(self, x):
        x = x.permute(0, 2, 1)
        f0 = self.mlp(x).permute(0, 2, 1)
        c0 = x[:, :3, :].permute(0, 2, 1)
        c1, f1 = self.sa1(c0, f0)
        c1, f1 = self.irmlp1(c1, c1, f1)
        c2, f2 = self.sa2(c1, f1)
        c2, f2 = self.irmlp2(c2, c2, f2)
        c2, f2 = self.irmlp2_1(c2, c2, f2)
        c3, f3 = self.sa3(c2, f2)
        c3, f3 = self.irmlp3(c3, c3, f3)
        c4, f4 = self.sa4(c3, f3)
        c4, f4 = self.irmlp4(c4, c4, f4)
        f3 = self.fp4(c3, c4, f3, f4)
        f2 = self.fp3(c2, c3, f2, f3)
        f1 = self.fp2(c1, c2, f1, f2)
        f0 = self.fp1(c0, c1, f0, f1)
        y = self.drop(f0).permute(0, 2, 1)
        return self.conv(y).permute(0, 2, 1)


class EdgeConv(nn.Module):               # models/dgcnn/dgcnn.py:60-77
    def __init__(self, in_channels, out_channels, k=20):
        super().__init__()
        self.k = k
        self.conv = nn.Sequential(
            nn.Conv2d(in_channels * 2, out_channels, kernel_size=1, bias=False),
            nn.BatchNorm2d(out_channels),
            nn.LeakyReLU(negative_slope=0.2))

    def forward(self, x):
        rp = _rp()
        if rp is not None and (rp.pool_arg or rp.act_mask):
            # replayed decisions: max_k act(y_k) = act(y at the argmax) (act is monotone)
            e = self.conv[1](self.conv[0](get_graph_feature(x, k=self.k)))      # (B, Cout, N, k)
            arg = _replayed_arg((e.shape[0], e.shape[2], e.shape[1]))           # (B*N, Cout) -> (B, N, Cout)
            y = e.gather(3, arg.permute(0, 2, 1).unsqueeze(3)).squeeze(3) if arg is not None else e.max(-1)[0]
            return act(y, self.conv[2].negative_slope, 'points')
        return self.conv(get_graph_feature(x, k=self.k)).max(dim=-1, keepdim=False)[0]


def _head(cin, cout, dropout):
    return nn.Sequential(nn.Conv1d(cin, cout, kernel_size=1, bias=False), nn.BatchNorm1d(cout),
                         nn.LeakyReLU(negative_slope=0.2), nn.Dropout(dropout))


class DGCNN(nn.Module):                  # dgcnn.py:80-162
    def __init__(self, num_classes=13, k=20, emb_dims=1024, dropout=0.5):
        super().__init__()
        self.k, self.num_classes = k, num_classes
        self.conv1 = EdgeConv(3, 64, k)
        self.conv2 = EdgeConv(64, 64, k)
        self.conv3 = EdgeConv(64, 64, k)
        self.conv4 = EdgeConv(64, 128, k)
        self.conv5 = nn.Sequential(nn.Conv1d(320, emb_dims, kernel_size=1, bias=False),
                                   nn.BatchNorm1d(emb_dims), nn.LeakyReLU(negative_slope=0.2))
        self.conv6 = _head(emb_dims + 320, 512, dropout)
        self.conv7 = _head(512, 256, dropout)
        self.conv8 = nn.Conv1d(256, num_classes, kernel_size=1)

    def forward(self, x):
        xyz = x[:, :3, :] if x.size(1) == 6 else x
        x1 = self.conv1(xyz)
        x2 = self.conv2(x1)
        x3 = self.conv3(x2)
        x4 = self.conv4(x3)
        xc = torch.cat((x1, x2, x3, x4), dim=1)
        x5 = _seq_act(self.conv5, xc)
        x7 = _seq_act(self.conv7, _seq_act(self.conv6, torch.cat((xc, x5), dim=1)))
        return self.conv8(x7).transpose(2, 1).contiguous(), x5, None


class DGCNNWithColor(nn.Module):         # dgcnn.py:165-257
    def __init__(self, num_classes=13, k=20, emb_dims=1024, dropout=0.5):
        super().__init__()
        self.k, self.num_classes = k, num_classes
        self.conv1 = EdgeConv(3, 64, k)
        self.conv2 = EdgeConv(64, 64, k)
        self.conv3 = EdgeConv(64, 64, k)
        self.conv4 = EdgeConv(64, 128, k)
        self.color_conv = nn.Sequential(nn.Conv1d(3, 64, kernel_size=1, bias=False),
                                        nn.BatchNorm1d(64), nn.LeakyReLU(negative_slope=0.2))
        self.conv5 = nn.Sequential(nn.Conv1d(384, emb_dims, kernel_size=1, bias=False),
                                   nn.BatchNorm1d(emb_dims), nn.LeakyReLU(negative_slope=0.2))
        self.conv6 = _head(emb_dims + 384, 512, dropout)
        self.conv7 = _head(512, 256, dropout)
        self.conv8 = nn.Conv1d(256, num_classes, kernel_size=1)

    def forward(self, x):
        if x.size(1) != 6:
            raise ValueError("DGCNNWithColor expects 6-channel input (xyz + rgb)")
        xyz, rgb = x[:, :3, :], x[:, 3:6, :]
        x1 = self.conv1(xyz)
        x2 = self.conv2(x1)
        x3 = self.conv3(x2)
        x4 = self.conv4(x3)
        xc = torch.cat((x1, x2, x3, x4, _seq_act(self.color_conv, rgb)), dim=1)
        x5 = _seq_act(self.conv5, xc)
        x7 = _seq_act(self.conv7, _seq_act(self.conv6, torch.cat((xc, x5), dim=1)))
        return self.conv8(x7).transpose(2, 1).contiguous(), x5, None


class TNet(nn.Module):                   # models/PointNet/PointNet.py:6-38
    def __init__(self, k=9):
        super().__init__()
        self.k = k
        self.conv1, self.conv2, self.conv3 = nn.Conv1d(k, 64, 1), nn.Conv1d(64, 128, 1), nn.Conv1d(128, 1024, 1)
        self.fc1, self.fc2, self.fc3 = nn.Linear(1024, 512), nn.Linear(512, 256), nn.Linear(256, k * k)
        self.bn1, self.bn2, self.bn3 = nn.BatchNorm1d(64), nn.BatchNorm1d(128), nn.BatchNorm1d(1024)
        self.bn4, self.bn5 = nn.BatchNorm1d(512), nn.BatchNorm1d(256)

    def forward(self, x):
        B = x.size(0)
        x = act(self.bn1(self.conv1(x)))
        x = act(self.bn2(self.conv2(x)))
        x = act(self.bn3(self.conv3(x)))
        x = torch.max(x, 2, keepdim=False)[0]
        x = F.relu(self.bn4(self.fc1(x)))
        x = F.relu(self.bn5(self.fc2(x)))
        eye = torch.eye(self.k, device=x.device).view(1, self.k * self.k).repeat(B, 1)
        return (self.fc3(x) + eye).view(B, self.k, self.k)


class PointNetEncoder(nn.Module):        # PointNet.py:41-90
    def __init__(self, global_feat=True, feature_transform=False, k=9):
        super().__init__()
        self.stn = TNet(k=k)
        self.conv1, self.bn1 = nn.Conv1d(k, 64, 1), nn.BatchNorm1d(64)
        self.feature_transform = feature_transform
        if feature_transform:
            self.fstn = TNet(k=64)
        self.conv2, self.bn2 = nn.Conv1d(64, 128, 1), nn.BatchNorm1d(128)
        self.conv3, self.bn3 = nn.Conv1d(128, 1024, 1), nn.BatchNorm1d(1024)
        self.global_feat = global_feat

    def forward(self, x):
        B, _, N = x.size()
        trans = self.stn(x)
        x = torch.bmm(x.transpose(2, 1), trans).transpose(2, 1)
        x = act(self.bn1(self.conv1(x)))
        trans_feat = None
        if self.feature_transform:
            trans_feat = self.fstn(x)
            x = torch.bmm(x.transpose(2, 1), trans_feat).transpose(2, 1)
        pf = x
        x = act(self.bn2(self.conv2(x)))
        x = self.bn3(self.conv3(x))
        x = torch.max(x, 2, keepdim=False)[0]
        if self.global_feat:
            return x, trans, trans_feat
        return torch.cat([x.view(B, 1024, 1).repeat(1, 1, N), pf], 1), trans, trans_feat


class PointNetSeg(nn.Module):            # PointNet.py:119-150
    def __init__(self, part_classes=13, feature_transform=False):
        super().__init__()
        self.feature_transform = feature_transform
        self.feat = PointNetEncoder(global_feat=False, feature_transform=feature_transform)
        self.conv1, self.bn1 = nn.Conv1d(1088, 512, 1), nn.BatchNorm1d(512)
        self.conv2, self.bn2 = nn.Conv1d(512, 256, 1), nn.BatchNorm1d(256)
        self.conv3, self.bn3 = nn.Conv1d(256, 128, 1), nn.BatchNorm1d(128)
        self.conv4 = nn.Conv1d(128, part_classes, 1)

    def forward(self, x):
        x, _, _ = self.feat(torch.transpose(x, -1, -2))
        x = act(self.bn1(self.conv1(x)))
        x = act(self.bn2(self.conv2(x)))
        x = act(self.bn3(self.conv3(x)))
        x = self.conv4(x).transpose(2, 1).contiguous()
        x = torch.exp(x)
        return x / torch.sum(x, keepdim=True, dim=-1)


# --------------------------------------------------------------------------
# a17 masked one-hot cross entropy         (Training/train_model.py:15-57)
# --------------------------------------------------------------------------
def masked_onehot_cross_entropy(logits, targets_onehot, pad_starts, eps=1e-9):
    B, L, C = logits.shape
    lp = F.log_softmax(logits, dim=-1)
    tok = -torch.sum(targets_onehot * lp, dim=-1)
    pos = torch.arange(L, device=logits.device).unsqueeze(0).expand(B, L)
    mask = (pos < pad_starts.to(logits.device).long().unsqueeze(1)).float()
    total = mask.sum()
    if total.item() == 0:
        return torch.tensor(0.0, device=logits.device, requires_grad=True)
    return (tok * mask).sum() / total


# --------------------------------------------------------------------------
# section 8(f) row 4: sliding-window scene inference  (models/dgcnn/utils.py:67-131)
# --------------------------------------------------------------------------
def predict_single_scene(model, points, batch_size=4096, overlap=512):
    model.eval()
    n = points.shape[0]
    if n <= batch_size:
        with torch.no_grad():
            logits = model(points.T.unsqueeze(0))[0].squeeze(0)
        return torch.argmax(logits, dim=1), torch.softmax(logits, dim=1).max(dim=1)[0]
    step = batch_size - overlap
    all_logits = torch.zeros(n, model.num_classes)
    counts = torch.zeros(n)
    with torch.no_grad():
        for s in range(0, n, step):                              # :112-127
            e = min(s + batch_size, n)
            all_logits[s:e] += model(points[s:e].T.unsqueeze(0))[0].squeeze(0)
            counts[s:e] += 1
    all_logits = all_logits / counts.unsqueeze(1)
    return torch.argmax(all_logits, dim=1), torch.softmax(all_logits, dim=1).max(dim=1)[0]


# --------------------------------------------------------------------------
# section 8(f) row 2: harness-B batch builder  (Training/train_model.py:89-171)
# --------------------------------------------------------------------------
def preprocess_batch_to_train_format(x, y, mapping, cut=None, sampling=None):
    if sampling is not None:
        if not (0 < sampling <= 1.0):
            raise ValueError(f"sampling must be in (0,1], got {sampling}")
        xs, ys = [], []
        for xi, yi in zip(x, y):                                 # :122-133
            perm = torch.randperm(xi.shape[0], device=xi.device)[:max(int(xi.shape[0] * sampling), 1)]
            xs.append(xi[perm])
            ys.append([yi[j] for j in perm.cpu().tolist()])
        x, y = xs, ys
    lengths = torch.tensor([xi.shape[0] for xi in x], dtype=torch.int32)   # :136
    L = int(lengths.max().item())
    if cut is not None:
        L = min(L, cut)
    B, D, C = len(x), x[0].shape[-1], len(mapping)
    out = torch.zeros((B, L, D), device=x[0].device, dtype=x[0].dtype)
    for i, xi in enumerate(x):                                   # :146-149
        n = min(xi.shape[0], L)
        out[i, :n] = xi[:n]
    label = torch.zeros((B, L, C), dtype=torch.float32, device=out.device)
    for i, yi in enumerate(y):                                   # :152-159
        for j, name in enumerate(yi):
            if j >= L:
                break
            label[i, j, mapping.index(name)] = 1.0
    if cut is not None:
        lengths = torch.clamp(lengths, max=cut)
    return out.transpose(1, 2), label, lengths, B > 1


# --------------------------------------------------------------------------
# section 8(f) row 3: segmentation metrics       (Training/metrics.py:3-142)
# predictions (B, N, C) probabilities, labels (B, N, C) one-hot, mask (B,) lengths
# --------------------------------------------------------------------------
def overall_accuracy(predictions, labels, mask):                      # metrics.py:3-25
    correct, total = update_accuracy(predictions, labels, mask)
    return correct / total


def update_accuracy(predictions, labels, mask):                       # metrics.py:28-51
    B = labels.shape[0]
    correct = 0
    for b in range(B):
        n = mask[b]
        correct += (labels[b, :n].argmax(-1) == predictions[b, :n].argmax(-1)).sum().item()
    return correct, mask.sum().item()


def confusion_matrix(predictions, labels, mask):                      # metrics.py:53-79
    B, _, C = labels.shape
    matrix = torch.zeros((C, C), dtype=torch.int64)
    for b in range(B):
        n = mask[b]
        pc = predictions[b, :n].argmax(-1)
        lc = labels[b, :n].argmax(-1)
        for i in range(C):
            pi = pc[lc == i]
            for j in range(C):
                matrix[i, j] += (pi == j).sum().item()
    return matrix


def update_intersection_over_union(predictions, labels, mask):        # metrics.py:113-142
    B, _, C = labels.shape
    inter = torch.zeros((C,), dtype=torch.float32)
    union = torch.zeros((C,), dtype=torch.float32)
    for c in range(C):
        for b in range(B):
            n = mask[b]
            lm = labels[b, :n, c] == 1
            pm = predictions[b, :n].argmax(-1) == c
            inter[c] += torch.logical_and(lm, pm).sum().item()
            union[c] += torch.logical_or(lm, pm).sum().item()
    return inter, union


def intersection_over_union(predictions, labels, mask):               # metrics.py:82-110
    B, _, C = labels.shape
    eps = 1e-6
    ious = torch.zeros((C,), dtype=torch.float32)
    for c in range(C):
        inter = union = 0
        for b in range(B):
            n = mask[b]
            lm = labels[b, :n, c] == 1
            pm = predictions[b, :n].argmax(-1) == c
            inter += torch.logical_and(lm, pm).sum().item()
            union += torch.logical_or(lm, pm).sum().item()
        ious[c] = (inter + eps) / (union + eps)
    return ious.mean().item(), ious


# --------------------------------------------------------------------------
# deterministic, key-ordered parameter init shared by oracle and product
# --------------------------------------------------------------------------
def seeded_init_(model: nn.Module, seed: int) -> nn.Module:
    """Fill every parameter/buffer from a generator seeded once, in key order.

    Conv/Linear weights ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)), biases likewise;
    BN weight ~ U(0.5, 1.5), bias ~ U(-0.1, 0.1).  Running stats left at
    (0, 1).  Product models have identical state_dict keys, so loading this
    state_dict into them gives bit-identical weights.
    """
    g = torch.Generator().manual_seed(seed)
    sd = model.state_dict()
    with torch.no_grad():
        for key in sorted(sd.keys()):
            t = sd[key]
            if not t.is_floating_point():
                continue
            if key.endswith('running_mean') or key.endswith('running_var'):
                continue
            mod_key = key.rsplit('.', 1)[0]
            is_bn = any(k.startswith(mod_key + '.running_mean') for k in sd.keys())
            if is_bn:
                if key.endswith('weight'):
                    t.copy_(torch.rand(t.shape, generator=g) + 0.5)
                else:
                    t.copy_((torch.rand(t.shape, generator=g) - 0.5) * 0.2)
            else:
                w = sd.get(mod_key + '.weight')
                fan_in = max(1, w[0].numel()) if w is not None and w.dim() > 1 else max(1, t.numel())
                bound = 1.0 / fan_in ** 0.5
                t.copy_((torch.rand(t.shape, generator=g) * 2 - 1) * bound)
    model.load_state_dict(sd)
    return model
