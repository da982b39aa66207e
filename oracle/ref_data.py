"""CPU restatement of the reference's block data path (TEST INFRASTRUCTURE ONLY).

Follows data_processing/block_datasets.py (piotr-bledowski/3D-Semantic-
Segmentation-Benchmark): `collate_blocks` (:5-29), the block index built from
file names (`BlockS3DISDataset._create_block_index`, :56-90), per-block
sampling (`__getitem__`, :104-130) and `create_block_dataloaders`' area split
and batching (:133-183).  The on-disk block format is the one
`preprocess_dataset.py:134` writes: torch.save((points (n, 9) f32, labels
(n, 14) u8)) at area_{a}/room{rr:02d}_block{bbb:03d}.pt.

Pinned by tests/golden/blocks.npz (captured from the reference by
tests/golden/make_golden.py::golden_blocks; tests/test_data.py).
"""
from __future__ import annotations

import os

import torch

AREAS = {1, 2, 3, 4, 5, 6}


def collate_blocks(batch):
    """block_datasets.py:5-29: zero-pad to the longest block, lengths as uint64."""
    B = len(batch)
    N = max(x.shape[0] for x, _ in batch)
    pts = torch.zeros((B, N, 9), dtype=torch.float32)
    lab = torch.zeros((B, N, 14), dtype=torch.uint8)
    for i, (p, l) in enumerate(batch):
        pts[i, :p.shape[0]] = p
        lab[i, :p.shape[0]] = l
    return pts, lab, torch.tensor([x.shape[0] for x, _ in batch], dtype=torch.uint64)


def block_index(data_dir, included_areas):
    """block_datasets.py:56-90: sorted (area, room, block) triples from the file names."""
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


def sample_rows(n: int, sampling: int) -> torch.Tensor:
    """block_datasets.py:119-125: the reference's own draw from the global RNG --
    randperm(n)[:S] when n > S, randint(n, (S,)) otherwise."""
    if n > sampling:
        return torch.randperm(n)[:sampling]
    return torch.randint(n, (sampling,))


def get_block(data_dir, blocks, i, sampling=None):
    """BlockS3DISDataset.__getitem__ (block_datasets.py:104-130)."""
    a, r, b = (int(v) for v in blocks[i])
    p, l = load_block(data_dir, a, r, b)
    if sampling is not None:
        rows = sample_rows(p.shape[0], sampling)
        p, l = p[rows], l[rows]
    return p, l


def block_splits(data_dir, test_areas):
    """create_block_dataloaders' split (block_datasets.py:161-164): train = the other areas."""
    return block_index(data_dir, AREAS - set(test_areas)), block_index(data_dir, set(test_areas))


def unshuffled_batches(data_dir, blocks, batch_size, sampling=None):
    """DataLoader(shuffle=False, collate_fn=collate_blocks) over a block list (:166-181)."""
    out = []
    for s in range(0, blocks.shape[0], batch_size):
        out.append(collate_blocks([get_block(data_dir, blocks, i, sampling)
                                   for i in range(s, min(s + batch_size, blocks.shape[0]))]))
    return out
