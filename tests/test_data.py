"""Block data path: index, collate and the HBM-resident
store against the CPU restatement of data_processing/block_datasets.py."""
import os

import pytest
import torch

import pcseg.data as D
from oracle import ref_data as RD


@pytest.fixture(scope='module')
def blockdir(tmp_path_factory):
    root = tmp_path_factory.mktemp('blocks')
    g = torch.Generator().manual_seed(3)
    sizes = {1: [(1, 1, 150), (1, 3, 40), (2, 2, 90), (10, 12, 64)], 3: [(1, 1, 33), (4, 7, 200)]}
    for area, blocks in sizes.items():
        os.makedirs(root / f'area_{area}')
        for room, block, n in blocks:
            pts = torch.randn(n, 9, generator=g)
            lab = torch.nn.functional.one_hot(torch.randint(0, 14, (n,), generator=g), 14).to(torch.uint8)
            torch.save((pts, lab), root / f'area_{area}' / f'room{room:02d}_block{block:03d}.pt')
    os.makedirs(root / 'area_2')                      # empty area
    return str(root)


def test_block_index_matches_reference(blockdir):
    assert torch.equal(D.block_index(blockdir, {1, 3}), RD.block_index(blockdir, {1, 3}))
    assert D.block_index(blockdir, {3}).tolist() == [[3, 1, 1], [3, 4, 7]]
    with pytest.raises(FileNotFoundError):
        D.block_index(blockdir, {2})
    with pytest.raises(FileNotFoundError):
        D.block_index(blockdir, {4})
    with pytest.raises(ValueError):
        D.block_index(blockdir, {7})


def test_collate_matches_reference(blockdir):
    idx = RD.block_index(blockdir, {1, 3}).tolist()
    batch = [RD.load_block(blockdir, *t) for t in idx[:4]]
    for a, b in zip(D.collate_blocks(batch), RD.collate_blocks(batch)):
        assert a.dtype == b.dtype and torch.equal(a, b)


@pytest.mark.gpu
def test_device_store_whole_blocks_equal_reference_collate(blockdir):
    store = D.DeviceBlockStore(blockdir, {1, 3}, sampling=None)
    idx = RD.block_index(blockdir, {1, 3}).tolist()
    ids = [5, 0, 2]
    pts, lab, lens = store.batch(ids)
    rp, rl, rn = RD.collate_blocks([RD.load_block(blockdir, *idx[i]) for i in ids])
    assert torch.equal(pts.cpu(), rp) and torch.equal(lab.cpu(), rl) and torch.equal(lens.cpu(), rn)


@pytest.mark.gpu
def test_device_store_sampling_semantics(blockdir):
    S = 64
    store = D.DeviceBlockStore(blockdir, {1, 3}, sampling=S)
    idx = RD.block_index(blockdir, {1, 3}).tolist()
    ids = list(range(len(idx)))
    torch.manual_seed(0)
    pts, lab, lens = store.batch(ids)
    assert pts.shape == (len(ids), S, 9) and lab.shape == (len(ids), S, 14)
    assert torch.equal(lens.cpu(), torch.full((len(ids),), S, dtype=torch.uint64))
    for b, i in enumerate(ids):
        p, l = RD.load_block(blockdir, *idx[i])
        n = p.shape[0]
        # every sampled row is a row of its own block, with its own label
        match = (pts[b].cpu().unsqueeze(1) == p.unsqueeze(0)).all(-1)          # (S, n)
        assert match.any(1).all()
        rows = match.float().argmax(1)
        assert torch.equal(lab[b].cpu(), l[rows])
        if n > S:                                                                  # randperm(n)[:S]: distinct
            assert rows.unique().numel() == S
