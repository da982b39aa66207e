"""Segmentation models with the reference's constructors, forward signatures,
return conventions and state_dict keys.

  PointNetpp        models/PointNetpp/PointNetpp.py:6-48     (B,N,9) -> (B,N,classes)
  PointNetppMSG     (not in the reference; composed from the same SA/FP blocks)
  PointNeXt         models/PointNeXt/PointNeXt.py:17-147     (B,N,9) -> (B,N,classes)
  DGCNN             models/dgcnn/dgcnn.py:80-162             (B,3|6,N) -> (logits, x5, None)
  DGCNNWithColor    models/dgcnn/dgcnn.py:165-257            (B,6,N)   -> (logits, x5, None)
  get_model/get_loss models/dgcnn/dgcnn.py:260-280
  PointNetSeg       models/PointNet/PointNet.py:119-150      (B,N,9) -> probabilities
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .common import SetAbstraction, FeaturePropagation, InvResMLP, UnitPointNet, GeometryPlan, GeometryPrefetch
from .engine import (shared_mlp, pad_rows, linear_rows, edgeconv, edgeconv_fused_ok, storage_alias, module_cache,
                     EdgeInverseBatch)
from .replay import active as _replay
from ._lib import call, ptr, stream_ptr


def _head_rows(x_rows: torch.Tensor, drop: nn.Module | None, conv: nn.Module) -> torch.Tensor:
    return linear_rows(drop(x_rows) if drop is not None else x_rows, conv)


def _fused_dropout(drop: nn.Module):
    """(p, seed) for a training-mode Dropout the engine fuses into the preceding stack's output
    (one 64-bit mask seed from torch's CPU generator), else None.  Under HIP-graph capture the
    seed would be baked into the graph as a kernel argument (every replay the same mask), so
    there the module's own nn.Dropout runs instead: torch's Philox offset advances per replay."""
    if drop.training and 0.0 < drop.p < 1.0 and not torch.cuda.is_current_stream_capturing():
        return float(drop.p), int(torch.randint(0, 2 ** 62, (1,)).item())
    return None


class PointNetpp(GeometryPrefetch, nn.Module):
    """PointNet++ SSG semantic segmentation (reference PointNetpp.py:6-48)."""

    def __init__(self, part_classes: int):
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

    def _plan_for(self, c0, inverse=True, into=None):
        return GeometryPlan(c0, [(sa.C, [(sa.radius, sa.K, False)]) for sa in (self.sa1, self.sa2, self.sa3, self.sa4)],
                            inverse=inverse, into=into)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, N, _ = x.shape
        c0 = self._coords_of(x)
        f0 = x[:, :, 3:].contiguous()
        geo = self._geometry(x, c0)
        c0 = geo.coords[0]
        c1, f1 = self.sa1(c0, f0, geo=geo.sa(1))
        c2, f2 = self.sa2(c1, f1, geo=geo.sa(2))
        c3, f3 = self.sa3(c2, f2, geo=geo.sa(3))
        c4, f4 = self.sa4(c3, f3, geo=geo.sa(4))
        f3 = self.fp4(c3, c4, f3, f4, geo=geo.fp(3))
        f2 = self.fp3(c2, c3, f2, f3, geo=geo.fp(2))
        f1 = self._prefetch_point(self.fp2(c1, c2, f1, f2, geo=geo.fp(1)))
        dz = _fused_dropout(self.drop)       # the head's Dropout, fused into FP1's output
        f0 = self.fp1(c0, c1, None, f1, geo=geo.fp(0), dropout=dz)
        return _head_rows(f0.reshape(B * N, -1), None if dz else self.drop, self.conv).view(B, N, -1)


class PointNetppMSG(GeometryPrefetch, nn.Module):
    """PointNet++ MSG (multi-scale grouping) segmentation.

    Not in the reference (BASELINE.json config 4 names it); composed from the
    reference's own SetAbstraction / FeaturePropagation semantics with the
    standard semantic-segmentation MSG widths: each level
    samples its centroids ONCE and groups them at two radii, concatenating the
    two pooled branches.
    """

    CFG = [  # (C, radii, Ks, [mlp per scale])
        (1024, (0.05, 0.1), (16, 32), ([16, 16, 32], [32, 32, 64])),
        (256, (0.1, 0.2), (16, 32), ([64, 64, 128], [64, 96, 128])),
        (64, (0.2, 0.4), (16, 32), ([128, 196, 256], [128, 196, 256])),
        (16, (0.4, 0.8), (16, 32), ([256, 256, 512], [256, 384, 512])),
    ]

    def __init__(self, part_classes: int):
        super().__init__()
        self.levels = nn.ModuleList()
        d = 6
        skips = [6]
        for C, radii, Ks, mlps in self.CFG:
            branches = nn.ModuleList([SetAbstraction(C, r, d + 3, m, K=k) for r, k, m in zip(radii, Ks, mlps)])
            self.levels.append(branches)
            d = sum(m[-1] for m in mlps)
            skips.append(d)
        self.fp4 = FeaturePropagation(skips[4] + skips[3], [256, 256])
        self.fp3 = FeaturePropagation(256 + skips[2], [256, 256])
        self.fp2 = FeaturePropagation(256 + skips[1], [256, 128])
        self.fp1 = FeaturePropagation(128, [128, 128, 128])
        self.drop = nn.Dropout(0.5)
        self.conv = nn.Conv1d(128, part_classes, 1)

    def _plan_for(self, c0, inverse=True, into=None):
        return GeometryPlan(c0, [(br[0].C, [(sa.radius, sa.K, False) for sa in br]) for br in self.levels],
                            inverse=inverse, into=into)

    def _sa_level(self, branches, coords, feats, geo, level):
        C = branches[0].C
        B = coords.shape[0]
        outs = []
        for q, sa in enumerate(branches):
            cent, idx, inv = geo.sa(level, q)
            rows = ops.group_rows(coords, feats, cent, idx, sa.radius, sa.grouping_norm, inv)
            outs.append(sa.point_net.forward_rows(rows, 3 + feats.shape[2], pool_k=sa.K, dx_from=3).view(B, C, -1))
        return cent, torch.cat(outs, dim=-1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, N, _ = x.shape
        c0 = self._coords_of(x)
        geo = self._geometry(x, c0)
        cs, fs = [geo.coords[0]], [x[:, :, 3:].contiguous()]
        for lv, branches in enumerate(self.levels, start=1):
            c, f = self._sa_level(branches, cs[-1], fs[-1], geo, lv)
            cs.append(c)
            fs.append(f)
        f3 = self.fp4(cs[3], cs[4], fs[3], fs[4], geo=geo.fp(3))
        f2 = self.fp3(cs[2], cs[3], fs[2], f3, geo=geo.fp(2))
        f1 = self._prefetch_point(self.fp2(cs[1], cs[2], fs[1], f2, geo=geo.fp(1)))
        dz = _fused_dropout(self.drop)       # the head's Dropout, fused into FP1's output
        f0 = self.fp1(cs[0], cs[1], None, f1, geo=geo.fp(0), dropout=dz)
        return _head_rows(f0.reshape(B * N, -1), None if dz else self.drop, self.conv).view(B, N, -1)


class PointNeXt(GeometryPrefetch, nn.Module):
    """PointNeXt(-B-like) segmentation (reference PointNeXt.py:17-147)."""

    def __init__(self, part_classes: int, version: str = 'b'):
        super().__init__()
        self.num_classes = part_classes
        self.mlp = UnitPointNet(9, [32])
        mlp_last = self.mlp.conv[-1].out_channels
        self.sa1 = SetAbstraction(1024, 0.1, mlp_last + 3, [32, 32, 64], grouping_norm=True)
        sa1 = self.sa1.point_net.conv[-1].out_channels
        self.irmlp1 = InvResMLP(0.1, sa1 + 3, sa1, 32)
        self.sa2 = SetAbstraction(256, 0.2, sa1 + 3, [64, 64, 128], grouping_norm=True)
        sa2 = self.sa2.point_net.conv[-1].out_channels
        self.irmlp2 = InvResMLP(0.1, sa2 + 3, sa2, 32)
        self.irmlp2_1 = InvResMLP(0.2, sa2 + 3, sa2, 32)
        self.sa3 = SetAbstraction(64, 0.4, sa2 + 3, [128, 128, 256], grouping_norm=True)
        sa3 = self.sa3.point_net.conv[-1].out_channels
        self.irmlp3 = InvResMLP(0.4, sa3 + 3, sa3, 32)
        self.sa4 = SetAbstraction(16, 0.8, sa3 + 3, [256, 256, 512], grouping_norm=True)
        sa4 = self.sa4.point_net.conv[-1].out_channels
        self.irmlp4 = InvResMLP(0.8, sa4 + 3, sa4, 16)
        self.fp4 = FeaturePropagation(sa4 + sa3, [256, 256])
        fp4 = self.fp4.point_net.conv[-1].out_channels
        self.fp3 = FeaturePropagation(fp4 + sa2, [256, 256])
        fp3 = self.fp3.point_net.conv[-1].out_channels
        self.fp2 = FeaturePropagation(fp3 + sa1, [256, 128])
        fp2 = self.fp2.point_net.conv[-1].out_channels
        self.fp1 = FeaturePropagation(fp2 + mlp_last, [128, 128, 128, 128])
        fp1 = self.fp1.point_net.conv[-1].out_channels
        self.drop = nn.Dropout(0.5)
        self.conv = nn.Conv1d(fp1, part_classes, 1)

    def _plan_for(self, c0, inverse=True, into=None):
        def q(m, on_self):
            return (m.radius, m.K, on_self)
        return GeometryPlan(c0, [
            (self.sa1.C, [q(self.sa1, False), q(self.irmlp1, True)]),
            (self.sa2.C, [q(self.sa2, False), q(self.irmlp2, True), q(self.irmlp2_1, True)]),
            (self.sa3.C, [q(self.sa3, False), q(self.irmlp3, True)]),
            (self.sa4.C, [q(self.sa4, False), q(self.irmlp4, True)])], inverse=inverse, into=into)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, N, Cin = x.shape
        c0 = self._coords_of(x)
        geo = self._geometry(x, c0)          # FPS etc. start on the side stream before the stem MLP
        c0 = geo.coords[0]
        x = x.contiguous()
        f0 = self.mlp.forward_rows(pad_rows(x.view(B * N, Cin)), Cin).view(B, N, -1)
        c1, f1 = self.sa1(c0, f0, geo=geo.sa(1, 0))
        c1, f1 = self.irmlp1(c1, c1, f1, geo=geo.sa(1, 1)[1:])
        c2, f2 = self.sa2(c1, f1, geo=geo.sa(2, 0))
        c2, f2 = self.irmlp2(c2, c2, f2, geo=geo.sa(2, 1)[1:])
        c2, f2 = self.irmlp2_1(c2, c2, f2, geo=geo.sa(2, 2)[1:])
        c3, f3 = self.sa3(c2, f2, geo=geo.sa(3, 0))
        c3, f3 = self.irmlp3(c3, c3, f3, geo=geo.sa(3, 1)[1:])
        c4, f4 = self.sa4(c3, f3, geo=geo.sa(4, 0))
        c4, f4 = self.irmlp4(c4, c4, f4, geo=geo.sa(4, 1)[1:])
        f3 = self.fp4(c3, c4, f3, f4, geo=geo.fp(3))
        f2 = self.fp3(c2, c3, f2, f3, geo=geo.fp(2))
        f1 = self._prefetch_point(self.fp2(c1, c2, f1, f2, geo=geo.fp(1)))
        dz = _fused_dropout(self.drop)       # the head's Dropout, fused into FP1's output
        f0 = self.fp1(c0, c1, f0, f1, geo=geo.fp(0), dropout=dz)
        return _head_rows(f0.reshape(B * N, -1), None if dz else self.drop, self.conv).view(B, N, -1)


# ------------------------------------------------------------------------- DGCNN
def _seq_rows(x_rows: torch.Tensor, seq: nn.Sequential, kin: int | None = None,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """Conv1d(bias=False) -> BN1d -> LeakyReLU [-> Dropout] on rows (HIP shared-MLP engine);
    `out`: a row block the activation is written into (no Dropout after it)."""
    # training-mode Dropout fused into the stack's output
    drop = _fused_dropout(seq[3]) if len(seq) > 3 and out is None else None
    y = shared_mlp(x_rows, kin or x_rows.shape[1], [seq[0]], [seq[1]], 'lrelu', seq[2].negative_slope, 0, out=out,
                   dropout=drop, cache=module_cache(seq))
    if len(seq) > 3 and drop is None:
        y = seq[3](y)
    return y


def knn(x: torch.Tensor, k: int) -> torch.Tensor:
    """Reference `knn` (dgcnn.py:7-21): x (B, F, N) -> idx (B, N, k) int64, k largest of
    -|xi|^2 + 2 xi.xj - |xj|^2 (self included).  HIP kernel: F in {3, 64}."""
    return ops.knn(x.transpose(1, 2).contiguous(), k).long()


def get_graph_feature(x: torch.Tensor, k: int = 20, idx: torch.Tensor | None = None,
                      dim9: bool = False) -> torch.Tensor:
    """Reference `get_graph_feature` (dgcnn.py:24-57): x (B, C, N) ->
    (B, 2C, N, k) = [x_j - x_i, x_i] (dim9: [x_j - x_i, x_i, x_i], kNN on channels 6:)."""
    B, N = x.size(0), x.size(2)
    xp = x.reshape(B, -1, N).transpose(1, 2).contiguous()          # (B, N, C)
    C = xp.shape[2]
    if idx is None:
        idx = ops.knn(xp[:, :, 6:].contiguous() if dim9 else xp, k)
    k = idx.shape[2]
    rows = ops.edge_rows(xp, idx.to(device=xp.device, dtype=torch.int32).contiguous())
    feat = rows[:, :2 * C]
    if dim9:
        feat = torch.cat((feat, rows[:, C:2 * C]), dim=1)
    return feat.reshape(B, N, k, -1).permute(0, 3, 1, 2).contiguous()


class EdgeConv(nn.Module):
    """Reference dgcnn.py:60-77.  forward takes/returns the reference's (B, C, N) layout."""

    def __init__(self, in_channels, out_channels, k=20):
        super().__init__()
        self.k = k
        self.conv = nn.Sequential(
            nn.Conv2d(in_channels * 2, out_channels, kernel_size=1, bias=False),
            nn.BatchNorm2d(out_channels),
            nn.LeakyReLU(negative_slope=0.2))
        self.edge_inverse = 'deferred'  # where the backward's inverse kNN map is built (engine.set_edge_inverse)

    def forward_points(self, xp: torch.Tensor) -> torch.Tensor:
        """xp point-major (B, N, C) -> (B, N, Cout)."""
        return self.forward_graph(xp)[0]

    def forward_graph(self, xp: torch.Tensor, seeds: torch.Tensor | None = None, inv_batch=None,
                      also: torch.Tensor | None = None, order: torch.Tensor | None = None):
        """(output (B, N, Cout), this layer's kNN graph (B, N, k) int32).  seeds: the previous
        EdgeConv's graph -- its neighbours' distances in this layer's feature space bound the
        search threshold from the start (same graph, less merge work).  order: ops.knn_order of
        the cloud's xyz -- the kNN scans candidate tiles nearest first and skips the provably
        farther ones (same graph).  also: a (B*N, Cout) row block that receives a copy of the
        output (the fused kernel writes both; DGCNN's head concatenation), not connected to
        autograd here."""
        B, N, _ = xp.shape
        rp = _replay()
        if rp is not None and rp.knn_idx:
            idx = rp.knn_idx.pop(0).to(device=xp.device, dtype=torch.int32).contiguous()
        else:
            idx = ops.knn(xp, self.k, seeds=seeds, order=order)
        if rp is not None:
            rp.rec_knn_idx.append(idx.detach().cpu())
        C = xp.shape[2]
        if edgeconv_fused_ok(self.conv[0], self.conv[1], C):
            holder = inv_batch.holder() if (inv_batch is not None and self.edge_inverse == 'deferred') else None
            pooled = edgeconv(xp.reshape(B * N, C), C, idx, self.conv[0], self.conv[1], self.conv[2].negative_slope,
                              inverse_side=self.edge_inverse == 'side', holder=holder, also=also)
            return pooled.view(B, N, -1), idx
        rows = ops.edge_rows(xp, idx)
        pooled = shared_mlp(rows, 2 * C, [self.conv[0]], [self.conv[1]], 'lrelu',
                            self.conv[2].negative_slope, pool_k=self.k)
        if also is not None:
            with torch.no_grad():
                also.copy_(pooled)
        return pooled.view(B, N, -1), idx

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward_points(x.transpose(1, 2).contiguous()).transpose(1, 2)


class _CopyColumns(torch.autograd.Function):
    """parts (B, N, C_i) side by side in the (B*N, sum C_i) row block dest[0] (torch.cat(parts,
    dim=-1) of dgcnn.py:200 / :245, into a wider buffer): copied here unless dest[1] marks the
    part as already written there by its producer (the EdgeConv kernel's second output, the colour
    branch's GEMM epilogue).  Backward: each part gets its column slice of the gradient."""

    @staticmethod
    def forward(ctx, dest, *parts):
        out = dest[0]
        written = dest[1] if len(dest) > 1 else (False,) * len(parts)
        off = 0
        for p, done in zip(parts, written):
            c = p.shape[-1]
            if done:
                off += c
                continue
            src = p.reshape(-1, c)
            blk = out[:, off:off + c]
            if (src.stride(1) == 1 and src.stride(0) % 4 == 0 and c % 4 == 0 and out.stride(0) % 4 == 0
                    and src.data_ptr() % 16 == 0 and blk.data_ptr() % 16 == 0):
                # one float4 copy kernel per block (torch's strided copy_ runs at ~2 TB/s)
                call('pcs_copy_cols', ptr(src), src.stride(0), src.shape[0], c, ptr(blk), out.stride(0),
                     stream_ptr(out.device))
            else:
                blk.copy_(src)
            off += c
        ctx.shapes = [p.shape for p in parts]
        return out

    @staticmethod
    def backward(ctx, g):
        grads, off = [], 0
        for shp in ctx.shapes:
            c = shp[-1]
            grads.append(g[:, off:off + c].view(shp))
            off += c
        return (None, *grads)


class _ColumnConcat(torch.autograd.Function):
    """torch.cat(blocks, dim=1) of row blocks that already sit side by side in one buffer
    (equal row stride, consecutive columns): the result aliases them, nothing is copied; the
    backward hands each block its column slice of the gradient (row-strided, read in place)."""

    @staticmethod
    def forward(ctx, *blocks):
        first = blocks[0]
        off = 0
        for b in blocks:
            if (b.data_ptr() != first.data_ptr() + 4 * off or b.stride(0) != first.stride(0) or b.stride(1) != 1
                    or b.shape[0] != first.shape[0]):
                raise RuntimeError('_ColumnConcat: blocks are not adjacent column blocks of one buffer')
            off += b.shape[1]
        ctx.widths = [b.shape[1] for b in blocks]
        return storage_alias(first, 0, off)

    @staticmethod
    def backward(ctx, g):
        grads, off = [], 0
        for w in ctx.widths:
            grads.append(g[:, off:off + w])
            off += w
        return tuple(grads)


def _head_buffer(self, M: int, widths: list[int], dev):
    """conv6 reads cat((x1..x4 [, colour], x5), 1) (dgcnn.py:203-206 / :248-251): one (B*N,
    cxr + emb) buffer H holds it.  The EdgeConv kernels write their outputs into its first
    columns as a second copy (their dense outputs feed the next kNN / EdgeConv), the colour
    branch and conv5 write their activations straight into their blocks, and the concatenation
    is an alias: no copy kernel and no 0.7 GB cat.  -> (H, the parts' column blocks)."""
    emb = self.conv5[0].weight.shape[0]
    H = torch.empty((M, sum(widths) + emb), dtype=torch.float32, device=dev)
    blocks, off = [], 0
    for w in widths:
        blocks.append(storage_alias(H, off, w))
        off += w
    return H, blocks


def _dgcnn_head(self, parts: list[torch.Tensor], B: int, N: int, H: torch.Tensor | None = None):
    # H: _head_buffer's, the parts already written into its first columns (else copied here)
    M = B * N
    cxr = sum(p.shape[-1] for p in parts)
    emb = self.conv5[0].weight.shape[0]
    written = H is not None
    if H is None:
        H = torch.empty((M, cxr + emb), dtype=torch.float32, device=parts[0].device)
    xr = _CopyColumns.apply((storage_alias(H, 0, cxr), (written,) * len(parts)), *parts)  # (B*N, 320|384), stride 1344|1408
    x5 = _seq_rows(xr, self.conv5, out=storage_alias(H, cxr, emb))        # (B*N, emb)
    x6 = _seq_rows(_ColumnConcat.apply(xr, x5), self.conv6)
    x7 = _seq_rows(x6, self.conv7)
    logits = linear_rows(x7, self.conv8).view(B, N, -1)
    # the reference returns x5 as a contiguous (B, emb, N); a transposed view of
    # the point-major rows has the same shape and values without a 0.5 GB copy
    return logits, x5.view(B, N, -1).transpose(1, 2), None


def _head_seq(cin, cout, dropout):
    return nn.Sequential(nn.Conv1d(cin, cout, kernel_size=1, bias=False), nn.BatchNorm1d(cout),
                         nn.LeakyReLU(negative_slope=0.2), nn.Dropout(dropout))


# Graphs 1-3 of a DGCNN forward take the pruned kNN (ops.knn(order=): candidate tiles of the
# Morton-ordered cloud scanned nearest first, the provably farther ones skipped; the same lists).
# The fourth graph is built on conv3's features, which follow the geometry least: the pruned scan
# still reads 0.57 of its tiles (block-max; 0.25-0.34 for graphs 1-3) and measured no faster than
# the seeded full scan (956 vs 953 us at B=32, profiles/r06_knn_pruned.txt).


class DGCNN(nn.Module):
    """Reference dgcnn.py:80-162 (xyz graph; 6-channel input uses xyz only)."""

    def __init__(self, num_classes=13, k=20, emb_dims=1024, dropout=0.5):
        super().__init__()
        self.k = k
        self.num_classes = num_classes
        self.conv1 = EdgeConv(3, 64, k)
        self.conv2 = EdgeConv(64, 64, k)
        self.conv3 = EdgeConv(64, 64, k)
        self.conv4 = EdgeConv(64, 128, k)
        self.conv5 = nn.Sequential(nn.Conv1d(320, emb_dims, kernel_size=1, bias=False),
                                   nn.BatchNorm1d(emb_dims), nn.LeakyReLU(negative_slope=0.2))
        self.conv6 = _head_seq(emb_dims + 320, 512, dropout)
        self.conv7 = _head_seq(512, 256, dropout)
        self.conv8 = nn.Conv1d(256, num_classes, kernel_size=1)

    def forward(self, x):
        B, _, N = x.shape
        xyz = x[:, :3, :] if x.size(1) == 6 else x
        xp = xyz.transpose(1, 2).contiguous()
        ib = EdgeInverseBatch()
        convs = (self.conv1, self.conv2, self.conv3, self.conv4)
        H, blk = _head_buffer(self, B * N, [c.conv[0].weight.shape[0] for c in convs], xp.device)
        od = ops.knn_order(xp)                           # one Morton order for graphs 1-3
        x1, g = self.conv1.forward_graph(xp, None, inv_batch=ib, also=blk[0], order=od)
        x2, g = self.conv2.forward_graph(x1, g, inv_batch=ib, also=blk[1], order=od)
        x3, g = self.conv3.forward_graph(x2, g, inv_batch=ib, also=blk[2], order=od)
        x4, _ = self.conv4.forward_graph(x3, g, inv_batch=ib, also=blk[3])       # full scan (note above DGCNN)
        ib.flush()
        return _dgcnn_head(self, [x1, x2, x3, x4], B, N, H)


class DGCNNWithColor(nn.Module):
    """Reference dgcnn.py:165-257 (xyz graph + per-point colour branch)."""

    def __init__(self, num_classes=13, k=20, emb_dims=1024, dropout=0.5):
        super().__init__()
        self.k = k
        self.num_classes = num_classes
        self.conv1 = EdgeConv(3, 64, k)
        self.conv2 = EdgeConv(64, 64, k)
        self.conv3 = EdgeConv(64, 64, k)
        self.conv4 = EdgeConv(64, 128, k)
        self.color_conv = nn.Sequential(nn.Conv1d(3, 64, kernel_size=1, bias=False),
                                        nn.BatchNorm1d(64), nn.LeakyReLU(negative_slope=0.2))
        self.conv5 = nn.Sequential(nn.Conv1d(384, emb_dims, kernel_size=1, bias=False),
                                   nn.BatchNorm1d(emb_dims), nn.LeakyReLU(negative_slope=0.2))
        self.conv6 = _head_seq(emb_dims + 384, 512, dropout)
        self.conv7 = _head_seq(512, 256, dropout)
        self.conv8 = nn.Conv1d(256, num_classes, kernel_size=1)

    def forward(self, x):
        if x.size(1) != 6:
            raise ValueError("DGCNNWithColor expects 6-channel input (xyz + rgb)")
        B, _, N = x.shape
        xp = x.transpose(1, 2)                           # (B, N, 6) view of the (B,6,N) input
        xyz = xp[:, :, :3].contiguous()
        rgb = xp[:, :, 3:6].contiguous()
        ib = EdgeInverseBatch()
        convs = (self.conv1, self.conv2, self.conv3, self.conv4)
        H, blk = _head_buffer(self, B * N, [c.conv[0].weight.shape[0] for c in convs] +
                              [self.color_conv[0].weight.shape[0]], xp.device)
        od = ops.knn_order(xyz)                          # one Morton order for graphs 1-3
        x1, g = self.conv1.forward_graph(xyz, None, inv_batch=ib, also=blk[0], order=od)
        x2, g = self.conv2.forward_graph(x1, g, inv_batch=ib, also=blk[1], order=od)
        x3, g = self.conv3.forward_graph(x2, g, inv_batch=ib, also=blk[2], order=od)
        x4, _ = self.conv4.forward_graph(x3, g, inv_batch=ib, also=blk[3])       # full scan (note above DGCNN)
        ib.flush()
        # the colour branch's activation lands in its block directly (the head's only reader)
        color = _seq_rows(pad_rows(rgb.view(B * N, 3)), self.color_conv, 3, out=blk[4])
        return _dgcnn_head(self, [x1, x2, x3, x4, color], B, N, H)


def get_model(num_classes=13, use_color=True, **kwargs):
    """Reference dgcnn.py:260-273."""
    if use_color:
        return DGCNNWithColor(num_classes=num_classes, **kwargs)
    return DGCNN(num_classes=num_classes, **kwargs)


def get_loss():
    """Reference dgcnn.py:276-280."""
    return nn.CrossEntropyLoss(ignore_index=-1)


# ------------------------------------------------------------------------- PointNet (dense plumbing)
class TNet(nn.Module):
    """Reference PointNet.py:6-38."""

    def __init__(self, k=9):
        super().__init__()
        self.k = k
        self.conv1 = nn.Conv1d(k, 64, 1)
        self.conv2 = nn.Conv1d(64, 128, 1)
        self.conv3 = nn.Conv1d(128, 1024, 1)
        self.fc1 = nn.Linear(1024, 512)
        self.fc2 = nn.Linear(512, 256)
        self.fc3 = nn.Linear(256, k * k)
        self.bn1 = nn.BatchNorm1d(64)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(1024)
        self.bn4 = nn.BatchNorm1d(512)
        self.bn5 = nn.BatchNorm1d(256)

    def forward_points(self, xp):
        """xp (B, N, k) point-major."""
        B, N, _ = xp.shape
        r = pad_rows(xp.reshape(B * N, -1))
        r = shared_mlp(r, self.k, [self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3], 'relu')
        g = r.view(B, N, -1).max(dim=1)[0]
        g = F.relu(self.bn4(self.fc1(g)))
        g = F.relu(self.bn5(self.fc2(g)))
        eye = torch.eye(self.k, device=g.device).view(1, self.k * self.k).repeat(B, 1)
        return (self.fc3(g) + eye).view(B, self.k, self.k)

    def forward(self, x):
        return self.forward_points(x.transpose(1, 2))


class PointNetEncoder(nn.Module):
    """Reference PointNet.py:41-90."""

    def __init__(self, global_feat=True, feature_transform=False, k=9):
        super().__init__()
        self.stn = TNet(k=k)
        self.conv1 = nn.Conv1d(k, 64, 1)
        self.bn1 = nn.BatchNorm1d(64)
        self.feature_transform = feature_transform
        if feature_transform:
            self.fstn = TNet(k=64)
        self.conv2 = nn.Conv1d(64, 128, 1)
        self.bn2 = nn.BatchNorm1d(128)
        self.conv3 = nn.Conv1d(128, 1024, 1)
        self.bn3 = nn.BatchNorm1d(1024)
        self.global_feat = global_feat

    def forward_points(self, xp):
        B, N, _ = xp.shape
        trans = self.stn.forward_points(xp)
        xp = torch.bmm(xp, trans)
        r = shared_mlp(pad_rows(xp.reshape(B * N, -1)), xp.shape[2], [self.conv1], [self.bn1], 'relu')
        trans_feat = None
        if self.feature_transform:
            trans_feat = self.fstn.forward_points(r.view(B, N, -1))
            r = torch.bmm(r.view(B, N, -1), trans_feat).reshape(B * N, -1)
        pf = r.view(B, N, -1)
        # conv2 -> BN -> ReLU -> conv3 -> BN (no activation, PointNet.py:82-83) in one engine stack
        r = shared_mlp(r, 64, [self.conv2, self.conv3], [self.bn2, self.bn3], ('relu', 'none'))
        g = r.view(B, N, -1).max(dim=1)[0]
        if self.global_feat:
            return g, trans, trans_feat
        return torch.cat([g.view(B, 1, 1024).expand(B, N, 1024), pf], dim=2), trans, trans_feat

    def forward(self, x):
        out, trans, tf = self.forward_points(x.transpose(1, 2))
        if self.global_feat:
            return out, trans, tf
        return out.transpose(1, 2), trans, tf


class PointNetSeg(nn.Module):
    """Reference PointNet.py:119-150 ((B, N, 9) -> per-point class probabilities)."""

    def __init__(self, part_classes=13, feature_transform=False):
        super().__init__()
        self.feature_transform = feature_transform
        self.feat = PointNetEncoder(global_feat=False, feature_transform=feature_transform)
        self.conv1 = nn.Conv1d(1088, 512, 1)
        self.bn1 = nn.BatchNorm1d(512)
        self.conv2 = nn.Conv1d(512, 256, 1)
        self.bn2 = nn.BatchNorm1d(256)
        self.conv3 = nn.Conv1d(256, 128, 1)
        self.bn3 = nn.BatchNorm1d(128)
        self.conv4 = nn.Conv1d(128, part_classes, 1)

    def forward(self, x):
        B, N, _ = x.shape
        feat, _, _ = self.feat.forward_points(x)
        r = feat.reshape(B * N, -1)
        r = shared_mlp(r, r.shape[1], [self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3], 'relu')
        r = linear_rows(r, self.conv4).view(B, N, -1)
        e = torch.exp(r)
        return e / torch.sum(e, keepdim=True, dim=-1)
