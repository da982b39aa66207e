"""HBM-resident S3DIS block store -- the data path in front of the hot path
(reference data_processing/block_datasets.py).

The reference loads one `.pt` file per block per step in DataLoader workers,
samples 4096 rows on the CPU and collates on the CPU (block_datasets.py:5-31,
:118-128).  A whole S3DIS split is a few GB, so `DeviceBlockStore` loads every
block of the split ONCE into two device arrays -- points (P, 9) f32 and
one-hot labels (P, 14) u8, 50 B per point -- and assembles each batch on the
GPU: the per-block row draw has the reference's distribution (a uniformly
random ordered subset via `randperm(n)[:S]` when n > S, `randint(n, (S,))`
otherwise), realised with one segmented sort of random keys, and the gather +
zero padding is one HIP kernel (`pcs_gather_blocks`).  No host work per step
beyond a few small launches.

`collate_blocks`, the block-index builder and the file format follow the
reference exactly (same names, errors and ordering).
"""
from __future__ import annotations

import os

import torch

from ._lib import call, check_cuda, ptr, stream_ptr


def collate_blocks(batch):
    """Reference `collate_blocks` (block_datasets.py:5-31): zero-pad a list of
    (points (n, 9), labels (n, 14)) to (B, N, 9) / (B, N, 14), lengths uint64."""
    B = len(batch)
    N = max(x.shape[0] for x, _ in batch)
    pts = torch.zeros((B, N, 9), dtype=torch.float32)
    lab = torch.zeros((B, N, 14), dtype=torch.uint8)
    for i, (p, l) in enumerate(batch):
        pts[i, :p.shape[0]] = p
        lab[i, :p.shape[0]] = l
    return pts, lab, torch.tensor([x.shape[0] for x, _ in batch], dtype=torch.uint64)


def block_index(data_dir: str, included_areas) -> torch.Tensor:
    """(area, room, block) uint16 triples in the reference's order
    (BlockS3DISDataset._create_block_index, block_datasets.py:63-93)."""
    if not os.path.exists(data_dir):
        raise FileNotFoundError(f'Data directory "{data_dir}" does not exist.')
    if any(a < 1 or a > 6 for a in included_areas):
        raise ValueError(f'Included areas can only contain values from the range [1, 6], got {included_areas}.')
    blocks = []
    for a in sorted(included_areas):
        d = os.path.join(data_dir, f'area_{a}')
        if not os.path.exists(d):
            raise FileNotFoundError(f'Directory for area {a} does not exist.')
        names = os.listdir(d)
        if not names:
            raise FileNotFoundError(f'Directory for area {a} does not contain any blocks.')
        idx = [n.replace('room', '').replace('block', '').replace('.pt', '').split('_') for n in names]
        blocks += sorted((a, int(r), int(b)) for r, b in idx)
    return torch.tensor(blocks, dtype=torch.uint16)


class DeviceBlockStore:
    """Every block of a split resident in HBM; `batch(ids)` assembles a padded,
    sampled batch on the device (see module docstring)."""

    def __init__(self, data_dir: str, included_areas, sampling: int | None = 4096, device='cuda'):
        self.blocks = block_index(data_dir, included_areas)
        self.sampling = sampling
        self.device = torch.device(device)
        pts, lab, lens = [], [], []
        for a, r, b in self.blocks.tolist():
            p, l = torch.load(os.path.join(data_dir, f'area_{a}', f'room{r:02d}_block{b:03d}.pt'),
                              weights_only=True)
            if p.ndim != 2 or p.shape[1] != 9 or l.shape != (p.shape[0], 14):
                raise ValueError(f'block area {a} room {r} block {b}: expected (n, 9) points and (n, 14) labels')
            pts.append(p.to(torch.float32))
            lab.append(l.to(torch.uint8))
            lens.append(p.shape[0])
        self.lengths = torch.tensor(lens, dtype=torch.int64)
        self.offsets = torch.zeros(len(lens) + 1, dtype=torch.int64)
        self.offsets[1:] = torch.cumsum(self.lengths, 0)
        self.points = torch.cat(pts).to(self.device)
        self.labels = torch.cat(lab).to(self.device)
        self._offsets_dev = self.offsets.to(self.device)
        self._lengths_dev = self.lengths.to(self.device)

    def __len__(self) -> int:
        return self.blocks.shape[0]

    def _rows(self, ids_host: torch.Tensor, generator=None) -> tuple[torch.Tensor, int, torch.Tensor]:
        """Store row per output row (B*N, -1 = padding), N, lengths (host ids: no device sync)."""
        dev = self.device
        ids = ids_host.to(dev, non_blocking=True)
        n = self._lengths_dev[ids]                                   # (B,)
        start = self._offsets_dev[ids]
        B = ids.numel()
        S = self.sampling
        if S is None:                                                 # whole blocks, padded to the longest
            N = int(self.lengths[ids_host].max())
            pos = torch.arange(N, device=dev).unsqueeze(0)
            rows = torch.where(pos < n.unsqueeze(1), start.unsqueeze(1) + pos, torch.full_like(pos, -1))
            return rows.reshape(-1), N, n.to(torch.uint64)
        # per block: n > S -> first S of a random permutation; else S draws with replacement
        tot = int(self.lengths[ids_host].sum())
        seg = torch.repeat_interleave(torch.arange(B, device=dev), n, output_size=tot)
        local = torch.arange(tot, device=dev) - torch.repeat_interleave(torch.cumsum(n, 0) - n, n, output_size=tot)
        key = torch.randint(0, 1 << 31, (tot,), device=dev, generator=generator, dtype=torch.int64)
        order = torch.argsort(seg * (1 << 31) + key)                  # random order inside each block
        first = (torch.cumsum(n, 0) - n)                               # segment starts in the sorted order
        take = first.unsqueeze(1) + torch.arange(S, device=dev).unsqueeze(0)
        perm_rows = local[order[take.clamp(max=tot - 1)]]             # (B, S) local row ids (valid where n > S)
        draw = (torch.rand((B, S), device=dev, generator=generator) * n.unsqueeze(1)).long()
        draw = torch.minimum(draw, (n - 1).unsqueeze(1))              # fp32 rounding can reach n
        local_rows = torch.where((n > S).unsqueeze(1), perm_rows, draw)
        rows = start.unsqueeze(1) + local_rows
        return rows.reshape(-1), S, torch.full((B,), S, dtype=torch.uint64, device=dev)

    def batch(self, ids, generator=None):
        """ids: block indices (list or tensor) -> points (B, N, 9) f32, labels (B, N, 14) u8,
        lengths (B,) uint64, all on the device (the reference's collate output)."""
        ids = torch.as_tensor(ids, dtype=torch.int64).cpu()
        rows, N, lengths = self._rows(ids, generator)
        return self.gather(rows, ids.numel(), N) + (lengths,)

    def gather(self, rows: torch.Tensor, B: int, N: int):
        check_cuda(self.points, rows)
        rows = rows.to(torch.int64).contiguous()
        pts = torch.empty((B, N, 9), dtype=torch.float32, device=self.device)
        lab = torch.empty((B, N, 14), dtype=torch.uint8, device=self.device)
        call('pcs_gather_blocks', ptr(self.points), ptr(self.labels), ptr(rows), rows.numel(), ptr(pts), ptr(lab),
             stream_ptr(self.device))
        return pts, lab


def _dist_rank_world(rank, world):
    import torch.distributed as dist
    if rank is None or world is None:
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
        return 0, 1
    return rank, world


class DistributedBlockSampler:
    """Block ids for one rank of a data-parallel job (SURVEY.md section 8(e) "Partitioning").

    Every epoch draws ONE permutation of all blocks from a generator seeded with
    (seed + epoch) -- identical on every rank without communication -- pads it by
    wrapping to a multiple of the world size (or drops the tail, `drop_last`) and
    hands rank r the entries r, r + world, r + 2*world, ...  So the ranks' shards of
    an epoch are disjoint and together cover every block (the reference's
    DataLoader(shuffle=True) draws one uniform permutation per epoch for its single
    process, block_datasets.py:166-173).  `shuffle=False` keeps the block order.

    `pad=False` (evaluation): no wrap padding and no dropping -- rank r takes entries r,
    r + world, ... of the permutation, so the shards have uneven lengths (they differ by at
    most one) and every block is evaluated exactly once across ranks, as the reference's
    single-process test loader does; a padded shard would count some blocks twice in
    aggregated metrics.
    """

    def __init__(self, num_blocks: int, rank: int | None = None, world: int | None = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False, pad: bool = True):
        self.n = int(num_blocks)
        self.rank, self.world = _dist_rank_world(rank, world)
        if not 0 <= self.rank < self.world:
            raise ValueError(f'rank {self.rank} out of range for world size {self.world}')
        if drop_last and not pad:
            raise ValueError('DistributedBlockSampler: drop_last and pad=False exclude each other')
        self.shuffle, self.seed, self.drop_last, self.pad = shuffle, int(seed), drop_last, pad
        self.epoch = 0
        if not pad:
            self.per_rank = len(range(self.rank, self.n, self.world))
        else:
            self.per_rank = self.n // self.world if drop_last else -(-self.n // self.world)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def order(self) -> list[int]:
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            perm = torch.randperm(self.n, generator=g).tolist()
        else:
            perm = list(range(self.n))
        if not self.pad:
            return perm
        total = self.per_rank * self.world
        if total > self.n:                                  # wrap-pad so every rank gets per_rank blocks
            perm = (perm * (-(-total // max(self.n, 1))))[:total]
        return perm[:total]

    def __iter__(self):
        return iter(self.order()[self.rank::self.world])

    def __len__(self) -> int:
        return self.per_rank


class DeviceBlockLoader:
    """Batches of one rank's blocks from a `DeviceBlockStore`: (points (B, N, 9) f32, labels
    (B, N, 14) u8, lengths (B,) uint64) on the device, as the reference's DataLoader with
    `collate_blocks` yields them (block_datasets.py:166-181).  The row sampling of each
    block draws from a per-rank device generator seeded with (seed, rank, epoch)."""

    def __init__(self, store: DeviceBlockStore, batch_size: int, sampler: DistributedBlockSampler, seed: int = 0):
        if batch_size < 1:
            raise ValueError(f'batch_size must be >= 1, got {batch_size}')
        self.store, self.batch_size, self.sampler, self.seed = store, int(batch_size), sampler, int(seed)

    @property
    def dataset(self):
        return self.store

    def set_epoch(self, epoch: int) -> None:
        self.sampler.set_epoch(epoch)

    def __len__(self) -> int:
        return -(-len(self.sampler) // self.batch_size)

    def __iter__(self):
        ids = list(self.sampler)
        gen = None
        if self.store.sampling is not None:
            gen = torch.Generator(device=self.store.device)
            gen.manual_seed((self.seed * 1_000_003 + self.sampler.rank * 7_919 + self.sampler.epoch) & ((1 << 62) - 1))
        for s in range(0, len(ids), self.batch_size):
            yield self.store.batch(ids[s:s + self.batch_size], generator=gen)


def create_block_dataloaders(data_dir: str, test_areas, train_batch_size: int = 4, test_batch_size: int = 4,
                             num_workers: int = 4, train_sampling: int | None = 4096,
                             test_sampling: int | None = None, train_shuffle: bool = True,
                             test_shuffle: bool = False, device='cuda', seed: int = 0, rank: int | None = None,
                             world: int | None = None):
    """Reference `create_block_dataloaders` (block_datasets.py:133-183): same arguments and
    area split (train = areas {1..6} minus `test_areas`), returning (train, test) loaders
    whose blocks are resident in HBM (`DeviceBlockStore`) and whose batches are assembled
    on the device.  `num_workers` is accepted for signature compatibility (no host workers
    are needed).  Under torch.distributed (or explicit rank/world) each loader yields only
    this rank's shard (`DistributedBlockSampler`): the train shards are padded to equal
    length, the test shards are not (every test block is evaluated exactly once)."""
    del num_workers
    areas = {1, 2, 3, 4, 5, 6}
    test_areas = set(test_areas)
    out = []
    for inc, bs, samp, shuf, pad in ((areas - test_areas, train_batch_size, train_sampling, train_shuffle, True),
                                     (test_areas, test_batch_size, test_sampling, test_shuffle, False)):
        store = DeviceBlockStore(data_dir, inc, sampling=samp, device=device)
        sampler = DistributedBlockSampler(len(store), rank, world, shuffle=shuf, seed=seed, pad=pad)
        out.append(DeviceBlockLoader(store, bs, sampler, seed=seed))
    return out[0], out[1]


def preprocess_batch_to_train_format(x, y, mapping, cut=None, sampling=None, device=None):
    """Reference `preprocess_batch_to_train_format` (Training/train_model.py:89-171),
    harness B's batch builder: optional per-sample random subsampling, zero padding to
    the longest sample (or `cut`), one-hot fp32 labels from per-point class names.

    Same arguments, RNG calls (one `torch.randperm(N_i, device=x_i.device)` per sample),
    errors and returns: (batch_input (B, D, L) -- a transposed view, as the reference's --,
    label (B, L, C) fp32, lengths (B,) int32 on the CPU, cont = B > 1).  The per-point
    Python `mapping.index` loop of the reference becomes one dictionary pass per sample
    (numpy); padding and one-hot encoding are one HIP launch (`pcs_pad_onehot`).  Outputs
    are on `device` (default: the first sample's device, or cuda when that is the CPU).
    """
    import numpy as np

    if sampling is not None:
        if not (0 < sampling <= 1.0):
            raise ValueError(f"sampling must be in (0,1], got {sampling}")
    xs, perms = [], []
    for xi in x:
        if sampling is not None:
            k = max(int(xi.shape[0] * sampling), 1)
            perm = torch.randperm(xi.shape[0], device=xi.device)[:k]
            xi = xi[perm]
            perms.append(perm.cpu().numpy())
        else:
            perms.append(None)
        xs.append(xi)
    lengths = torch.tensor([xi.shape[0] for xi in xs], dtype=torch.int32)
    max_length = int(lengths.max().item())
    if cut is not None:
        max_length = min(max_length, cut)
    B = len(xs)
    D = xs[0].shape[-1]
    C = len(mapping)
    dev = torch.device(device) if device is not None else xs[0].device
    if dev.type != 'cuda':
        dev = torch.device('cuda')
    used = torch.clamp(lengths, max=max_length)
    # class ids of the rows that are kept (the reference looks labels up only below
    # max_length, so an unknown name beyond the cut is not an error there either)
    lut = {}
    for i, name in enumerate(mapping):        # list.index returns the first occurrence
        lut.setdefault(name, i)
    ids = []
    for yi, perm, n in zip(y, perms, used.tolist()):
        sel = (yi[j] for j in perm[:n]) if perm is not None else (yi[j] for j in range(n))
        try:
            ids.append(np.fromiter((lut[v] for v in sel), dtype=np.int32, count=n))
        except KeyError as e:
            raise ValueError(f'{e.args[0]!r} is not in list') from None
    rows = [xi[:n] for xi, n in zip(xs, used.tolist())]
    pts = torch.cat([r.to(device=dev, dtype=torch.float32) for r in rows]).contiguous()
    cls = torch.from_numpy(np.concatenate(ids)).to(dev)
    offsets = torch.zeros(B, dtype=torch.int64)
    if B > 1:
        offsets[1:] = torch.cumsum(used[:-1].to(torch.int64), 0)
    offsets = offsets.to(dev)
    used_d = used.to(dev)
    batch_input = torch.empty((B, max_length, D), dtype=torch.float32, device=dev)
    label = torch.empty((B, max_length, C), dtype=torch.float32, device=dev)
    call('pcs_pad_onehot', ptr(pts), D, ptr(cls), ptr(offsets), ptr(used_d), B, max_length, C, ptr(batch_input),
         ptr(label), stream_ptr(dev))
    if cut is not None:
        lengths = torch.clamp(lengths, max=cut)
    return batch_input.transpose(1, 2), label, lengths, B > 1
