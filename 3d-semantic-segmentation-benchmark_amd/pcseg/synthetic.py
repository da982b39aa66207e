"""Synthetic S3DIS-like blocks (no dataset ships in this environment).

Layout follows the reference's block format: 9 channels
`[x, y, z, r, g, b, nx, ny, nz]` (data_processing/preprocess_dataset.py:73-90)
with 14-class one-hot u8 labels and u64 lengths as `collate_blocks` returns
them (data_processing/block_datasets.py:5-29).

Geometry: a 1 m x 1 m footprint, z in [0, 3]: floor (30 %),
ceiling (25 %), wall x=0 (30 %), table top z=0.75 over [.3,.8]^2 (15 %), each
with N(0, 5 mm) noise; rgb are raw 0-255 integers stored as float; the last
three channels are xyz re-centred like `augment_points`.  `uniform=True`
gives the stress variant (uniform 1x1x3 m box; every ball underfull).
"""
from __future__ import annotations

import torch

NUM_CLASSES = 14


def make_block(n: int, gen: torch.Generator, uniform: bool = False) -> torch.Tensor:
    if uniform:
        xyz = torch.rand((n, 3), generator=gen) * torch.tensor([1.0, 1.0, 3.0])
    else:
        u = torch.rand((n,), generator=gen)
        a = torch.rand((n,), generator=gen)
        b = torch.rand((n,), generator=gen)
        xyz = torch.empty((n, 3))
        floor = u < 0.30
        ceil = (u >= 0.30) & (u < 0.55)
        wall = (u >= 0.55) & (u < 0.85)
        table = u >= 0.85
        xyz[floor] = torch.stack([a[floor], b[floor], torch.zeros_like(a[floor])], 1)
        xyz[ceil] = torch.stack([a[ceil], b[ceil], torch.full_like(a[ceil], 3.0)], 1)
        xyz[wall] = torch.stack([torch.zeros_like(a[wall]), a[wall], 3.0 * b[wall]], 1)
        xyz[table] = torch.stack([0.3 + 0.5 * a[table], 0.3 + 0.5 * b[table],
                                  torch.full_like(a[table], 0.75)], 1)
        xyz = xyz + torch.randn((n, 3), generator=gen) * 0.005
    rgb = torch.randint(0, 256, (n, 3), generator=gen).float()
    mn = xyz.min(0).values
    mx = xyz.max(0).values
    center = torch.stack([mn[0] + 0.5, mn[1] + 0.5, mn[2] + (mx[2] - mn[2]) / 2])
    return torch.cat([xyz, rgb, xyz - center], 1).float()


def make_batch(B: int, n: int, seed: int, uniform: bool = False):
    """(points (B,n,9) f32, labels (B,n,14) u8 one-hot, lengths (B,) u64)."""
    gen = torch.Generator().manual_seed(seed)
    pts = torch.stack([make_block(n, gen, uniform) for _ in range(B)])
    cls = torch.randint(0, NUM_CLASSES, (B, n), generator=gen)
    labels = torch.nn.functional.one_hot(cls, NUM_CLASSES).to(torch.uint8)
    lengths = torch.full((B,), n, dtype=torch.uint64)
    return pts, labels, lengths
