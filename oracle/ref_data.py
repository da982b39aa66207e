"""CPU restatement of the reference's block data path (TEST INFRASTRUCTURE ONLY).

Follows data_processing/block_datasets.py (piotr-bledowski/3D-Semantic-
Segmentation-Benchmark): `collate_blocks` (:5-31), the block index built from
file names (`BlockS3DISDataset._create_block_index`, :63-93), per-block
sampling (`__getitem__`, :118-128).  The on-disk block format is the one
`preprocess_dataset.py:134` writes: torch.save((points (n, 9) f32, labels
(n, 14) u8)) at area_{a}/room{rr:02d}_block{bbb:03d}.pt.
"""
from __future__ import annotations

import os

import torch


def collate_blocks(batch):
    """block_datasets.py:5-31: zero-pad to the longest block, lengths as uint64."""
    B = len(batch)
    N = max(x.shape[0] for x, _ in batch)
    pts = torch.zeros((B, N, 9), dtype=torch.float32)
    lab = torch.zeros((B, N, 14), dtype=torch.uint8)
    for i, (p, l) in enumerate(batch):
        pts[i, :p.shape[0]] = p
        lab[i, :p.shape[0]] = l
    return pts, lab, torch.tensor([x.shape[0] for x, _ in batch], dtype=torch.uint64)


def block_index(data_dir, included_areas):
    """block_datasets.py:63-93: sorted (area, room, block) triples from the file names."""
    blocks = []
    for a in sorted(included_areas):
        d = os.path.join(data_dir, f'area_{a}')
        if not os.path.exists(d):
            raise FileNotFoundError(f'Directory for area {a} does not exist.')
        idx = [f.replace('room', '').replace('block', '').replace('.pt', '').split('_') for f in os.listdir(d)]
        if not idx:
            raise FileNotFoundError(f'Directory for area {a} does not contain any blocks.')
        idx = sorted((a, int(r), int(b)) for r, b in idx)
        blocks += idx
    return torch.tensor(blocks, dtype=torch.uint16)


def load_block(data_dir, area, room, block):
    return torch.load(os.path.join(data_dir, f'area_{area}', f'room{room:02d}_block{block:03d}.pt'),
                      weights_only=True)


def sample_block(points, labels, sampling, perm_or_idx):
    """block_datasets.py:118-128 with the random draw supplied: randperm(n)[:S] when
    n > S, randint(n, (S,)) otherwise."""
    return points[perm_or_idx], labels[perm_or_idx]
