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


# ---------------------------------------------------------------- pinned by tests/golden/blocks.npz
@pytest.fixture(scope='module')
def golden_blocks(tmp_path_factory, golden):
    """The block directory golden_blocks() wrote (tests/golden/make_golden.py), rebuilt from the
    fixture, plus the fixture itself."""
    z = golden('blocks.npz')
    root = tmp_path_factory.mktemp('golden_blocks')
    for k in z.files:
        if k.startswith('file/') and k.endswith('/points'):
            _, a, r, b, _ = k.split('/')
            os.makedirs(root / f'area_{a}', exist_ok=True)
            torch.save((torch.from_numpy(z[k]), torch.from_numpy(z[k.replace('/points', '/labels')])),
                       root / f'area_{a}' / f'room{int(r):02d}_block{int(b):03d}.pt')
    return str(root), z


def _T(a):
    return torch.from_numpy(a)


def test_oracle_block_index_and_sampling_match_reference(golden_blocks):
    root, z = golden_blocks
    blocks = RD.block_index(root, {1, 3})
    assert torch.equal(blocks, _T(z['index_13']))
    for i in range(blocks.shape[0]):
        torch.manual_seed(1000 + i)                   # the reference's own global-RNG draw
        p, l = RD.get_block(root, blocks, i, sampling=64)
        assert torch.equal(p, _T(z[f'sample64/{i}/points'])) and torch.equal(l, _T(z[f'sample64/{i}/labels']))


def test_oracle_collate_and_split_match_reference(golden_blocks):
    root, z = golden_blocks
    whole = RD.block_index(root, {1, 3})
    cp, cl, cn = RD.collate_blocks([RD.get_block(root, whole, i) for i in (5, 0, 2)])
    assert torch.equal(cp, _T(z['collate/points'])) and torch.equal(cl, _T(z['collate/labels']))
    assert torch.equal(cn.to(torch.int64), _T(z['collate/lengths'])) and cn.dtype == torch.uint64
    train, test = RD.block_splits(root, {2, 5})
    assert torch.equal(train, _T(z['split/train'])) and torch.equal(test, _T(z['split/test']))
    for tag, blocks, bs in (('train', train, 3), ('test', test, 2)):
        for j, (p, l, n) in enumerate(RD.unshuffled_batches(root, blocks, bs)):
            assert torch.equal(p, _T(z[f'{tag}_batch/{j}/points']))
            assert torch.equal(l, _T(z[f'{tag}_batch/{j}/labels']))
            assert torch.equal(n.to(torch.int64), _T(z[f'{tag}_batch/{j}/lengths']))
        assert f'{tag}_batch/{j + 1}/points' not in z.files


def test_product_index_split_and_collate_match_reference(golden_blocks):
    root, z = golden_blocks
    assert torch.equal(D.block_index(root, {1, 3}), _T(z['index_13']))
    assert torch.equal(D.block_index(root, {1, 3, 4, 6}), _T(z['split/train']))
    batch = [RD.get_block(root, RD.block_index(root, {1, 3}), i) for i in (5, 0, 2)]
    for a, k in zip(D.collate_blocks(batch), ('points', 'labels', 'lengths')):
        assert torch.equal(a if k != 'lengths' else a.to(torch.int64), _T(z[f'collate/{k}']))


@pytest.mark.gpu
def test_device_loaders_unshuffled_match_reference_batches(golden_blocks):
    root, z = golden_blocks
    train, test = D.create_block_dataloaders(root, {2, 5}, train_batch_size=3, test_batch_size=2,
                                             num_workers=0, train_sampling=None, test_sampling=None,
                                             train_shuffle=False, test_shuffle=False)
    assert torch.equal(train.dataset.blocks, _T(z['split/train']))
    for tag, loader in (('train', train), ('test', test)):
        n = 0
        for j, (p, l, ln) in enumerate(loader):
            assert torch.equal(p.cpu(), _T(z[f'{tag}_batch/{j}/points']))
            assert torch.equal(l.cpu(), _T(z[f'{tag}_batch/{j}/labels']))
            assert torch.equal(ln.cpu().to(torch.int64), _T(z[f'{tag}_batch/{j}/lengths']))
            n += 1
        assert n == len(loader) and f'{tag}_batch/{n}/points' not in z.files


@pytest.mark.gpu
def test_device_loader_sampling_is_per_rank_and_reproducible(golden_blocks):
    root, _ = golden_blocks
    tr0, _ = D.create_block_dataloaders(root, {2, 5}, train_batch_size=2, train_sampling=64, seed=3, rank=0,
                                        world=2)
    tr1, _ = D.create_block_dataloaders(root, {2, 5}, train_batch_size=2, train_sampling=64, seed=3, rank=1,
                                        world=2)
    a = [p.cpu() for p, _, _ in tr0]
    b = [p.cpu() for p, _, _ in tr0]
    assert all(torch.equal(x, y) for x, y in zip(a, b))          # same (seed, rank, epoch): same draws
    tr0.set_epoch(1)
    c = [p.cpu() for p, _, _ in tr0]
    assert not all(torch.equal(x, y) for x, y in zip(a, c))      # a new epoch: new order and draws
    assert tr0.sampler.order() == tr1.sampler.order() or tr0.sampler.epoch != tr1.sampler.epoch
    assert len(tr0) == len(tr1) == 3                             # 9 train blocks -> 5 per rank (padded), B=2


# ---------------------------------------------------------------- distributed block sampler
@pytest.mark.parametrize('n,world,drop_last', [(13, 2, False), (12, 4, False), (13, 4, True), (3, 4, False)])
def test_sampler_shards_partition_each_epoch(n, world, drop_last):
    for epoch in range(3):
        shards = []
        for r in range(world):
            s = D.DistributedBlockSampler(n, rank=r, world=world, seed=11, drop_last=drop_last)
            s.set_epoch(epoch)
            shards.append(list(s))
            assert len(shards[-1]) == len(s)
        flat = [i for sh in shards for i in sh]
        if drop_last:
            assert len(set(flat)) == len(flat) == (n // world) * world
        else:
            assert set(flat) == set(range(n)) and len(flat) == -(-n // world) * world
            if n % world == 0:
                assert len(set(flat)) == n                          # disjoint when nothing is padded
    s0 = D.DistributedBlockSampler(n, rank=0, world=world, seed=11)
    s0.set_epoch(0)
    e0 = list(s0)
    s0.set_epoch(1)
    assert list(s0) != e0 or n <= world


@pytest.mark.parametrize('n,world', [(13, 2), (12, 4), (3, 4), (10, 3)])
def test_eval_sampler_shards_have_no_duplicates(n, world):
    """pad=False (the test loader's sampler): the union of the ranks' shards is every block
    exactly once, shard lengths differ by at most one."""
    for shuffle in (False, True):
        shards = []
        for r in range(world):
            s = D.DistributedBlockSampler(n, rank=r, world=world, seed=11, shuffle=shuffle, pad=False)
            shards.append(list(s))
            assert len(shards[-1]) == len(s)
        flat = [i for sh in shards for i in sh]
        assert sorted(flat) == list(range(n))
        assert max(map(len, shards)) - min(map(len, shards)) <= 1
    with pytest.raises(ValueError):
        D.DistributedBlockSampler(n, rank=0, world=world, drop_last=True, pad=False)


def _sampler_worker(rank, world, port, n, out):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        s = D.DistributedBlockSampler(n, seed=5)            # rank / world from the process group
        assert (s.rank, s.world) == (rank, world)
        res = []
        for epoch in range(2):
            s.set_epoch(epoch)
            mine = torch.tensor(list(s), dtype=torch.int64)
            got = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(got, mine)
            res.append(torch.stack(got))
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_sampler_world2_gloo_disjoint_and_covering():
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    n, world = 10, 2
    out = mp.Manager().dict()
    mp.spawn(_sampler_worker, args=(world, port, n, out), nprocs=world, join=True)
    for epoch in range(2):
        a, b = out[0][epoch], out[1][epoch]
        assert torch.equal(a, b)                             # every rank sees the same assignment
        assert set(a[0].tolist()).isdisjoint(a[1].tolist())
        assert sorted(a.reshape(-1).tolist()) == list(range(n))
    assert not torch.equal(out[0][0], out[0][1])             # a fresh permutation per epoch


def _eval_shard_worker(rank, world, port, n, out):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        s = D.DistributedBlockSampler(n, seed=5, pad=False)
        mine = torch.tensor(list(s), dtype=torch.int64)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([mine.numel()]))
        width = int(max(sizes))
        padded = torch.full((width,), -1, dtype=torch.int64)
        padded[:mine.numel()] = mine
        got = [torch.zeros_like(padded) for _ in range(world)]
        dist.all_gather(got, padded)
        out[rank] = torch.stack(got)
    finally:
        dist.destroy_process_group()


def test_eval_shards_world2_gloo_cover_each_block_once():
    """The test loader's shards over a world-2 gloo group: no block is evaluated twice."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    n, world = 11, 2
    out = mp.Manager().dict()
    mp.spawn(_eval_shard_worker, args=(world, port, n, out), nprocs=world, join=True)
    allb = out[0].reshape(-1)
    allb = allb[allb >= 0]
    assert sorted(allb.tolist()) == list(range(n))
