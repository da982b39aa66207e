"""Three-way precision check: GPU fp32 vs reference-algorithm CPU fp32 vs CPU fp64.

Training-mode BatchNorm makes many gradients sums with heavy cancellation
(the BN beta / pre-BN conv bias of a layer feeding another BN), so two
correct fp32 implementations that merely sum in different orders differ by
far more than 1e-3 on those tensors.  The float64 run of the same algorithm on
the SAME neighbour indices (FPS / ball query / 3-NN replayed from the fp32 run)
is the ground truth; a tensor passes when the GPU's error is within 1e-3 of the
truth's norm, or no worse than `factor` x the CPU fp32 reference's own error.
"""
from __future__ import annotations

import copy

import torch

import pcseg
from pcseg.synthetic import make_batch
from oracle import ref_ops as R


def _dropout_off(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()


def three_way(prod_ctor, ref_ctor, B, N, seed, uniform=False, pad=0, dev='cuda', chfirst=False,
              inputs=None, init_seed=None, fps_starts=None, knn_idx=None):
    """inputs=(x, labels, lengths) overrides the synthetic batch; fps_starts / knn_idx seed the
    fp32 oracle run (e.g. a golden fixture's recorded draws)."""
    if inputs is None:
        pts, labels, lengths = make_batch(B, N, seed=seed, uniform=uniform)
        if pad:
            lengths = torch.tensor([N - pad * (i % 2) for i in range(B)], dtype=torch.uint64)
            for i in range(B):
                pts[i, int(lengths[i]):] = 0.0
        x = pts[:, :, :6].contiguous().transpose(1, 2) if chfirst else pts
        lab = labels.float() if chfirst else labels
    else:
        x, lab, lengths = inputs
    ref32 = R.seeded_init_(ref_ctor(), seed if init_seed is None else init_seed)
    ref64 = copy.deepcopy(ref32).double()
    prod = prod_ctor()
    prod.load_state_dict(ref32.state_dict())
    prod = prod.to(dev)
    for m in (ref32, ref64, prod):
        m.train()
        _dropout_off(m)

    def logits_of(o):
        return o[0] if isinstance(o, tuple) else o

    rp = R.Replay(fps_starts=fps_starts, knn_idx=knn_idx)
    with R.replay(rp):
        l32 = logits_of(ref32(x))
    R.masked_onehot_cross_entropy(l32, lab, lengths).backward()
    rp64 = R.Replay(fps_idx=rp.rec_fps_idx, group_idx=rp.rec_group_idx, interp_idx=rp.rec_interp_idx,
                    knn_idx=rp.rec_knn_idx if rp.rec_knn_idx else None)
    with R.replay(rp64):
        l64 = logits_of(ref64(x.double()))
    R.masked_onehot_cross_entropy(l64, lab.double() if lab.is_floating_point() else lab, lengths).backward()
    rg = pcseg.Replay(fps_starts=rp.rec_fps_starts, knn_idx=rp.rec_knn_idx if rp.rec_knn_idx else None)
    with pcseg.replay(rg):
        lg = logits_of(prod(x.to(dev)))
    pcseg.masked_onehot_cross_entropy(lg, lab.to(dev), lengths.to(dev)).backward()

    # neighbour choices of the GPU run must equal the reference's (index-exact work)
    for lv, (a, b) in enumerate(zip(rg.rec_fps_idx, rp.rec_fps_idx)):
        if not torch.equal(a, b):
            bad = (a.long() != b.long()).nonzero()
            bb, ii = bad[0].tolist()
            raise AssertionError(f'FPS index mismatch at level {lv}: {bad.shape[0]} entries, first (batch {bb}, '
                                 f'step {ii}): gpu {a[bb, max(ii - 2, 0):ii + 3].tolist()} '
                                 f'ref {b[bb, max(ii - 2, 0):ii + 3].tolist()} starts {rp.rec_fps_starts[lv].tolist()}')
    for q, (a, b) in enumerate(zip(rg.rec_group_idx, rp.rec_group_idx)):
        sa, sb = a.long().sort(-1).values, b.sort(-1).values
        bad = (sa != sb).any(-1).nonzero()
        assert bad.numel() == 0, (f'ball-query set mismatch in query {q}: {bad.shape[0]} rows, first {bad[0].tolist()}: '
                                  f'gpu {sa[tuple(bad[0])].tolist()} ref {sb[tuple(bad[0])].tolist()}')
    for a, b in zip(rg.rec_interp_idx, rp.rec_interp_idx):
        assert torch.equal(a.long().sort(-1).values, b.sort(-1).values), '3-NN set mismatch'

    rows = []

    def add(name, g, c, t):
        g, c, t = g.detach().cpu().double(), c.detach().double(), t.detach().double()
        rows.append((name, float((g - t).norm()), float((c - t).norm()), float(t.norm())))
    add('logits', lg, l32, l64)
    for (k, pg), (_, p32), (_, p64) in zip(sorted(prod.named_parameters()), sorted(ref32.named_parameters()),
                                           sorted(ref64.named_parameters())):
        add(k, pg.grad, p32.grad, p64.grad)
    for (k, bg), (_, b32), (_, b64) in zip(sorted(prod.state_dict().items()), sorted(ref32.state_dict().items()),
                                           sorted(ref64.state_dict().items())):
        if 'running' in k:
            add(k, bg, b32, b64)
    return rows


def failures(rows, rtol=1e-3, factor=10.0, floor=1e-3):
    """A tensor passes when its GPU error vs the fp64 truth is
      <= rtol x its norm, or
      <= factor x the CPU fp32 reference's own error, or
      <= floor x the largest gradient norm in the same top-level module (sa3, fp1, conv2, ...):
         the survey's floor for sums that are pure cancellation (pre-BN conv biases,
         BN betas of pooled layers), whose value is decided by a handful of ReLU/argmax
         flips at |y| ~ 1e-7 in ANY fp32 evaluation order."""
    top = {}
    for name, _, _, n in rows:
        if name != 'logits' and 'running' not in name:
            key = name.split('.')[0]
            top[key] = max(top.get(key, 0.0), n)
    bad = []
    for name, eg, ec, n in rows:
        fl = floor * top.get(name.split('.')[0], 0.0) if 'running' not in name else 0.0
        if not (eg <= rtol * n or eg <= factor * ec or eg <= fl):
            bad.append((name, eg, ec, n))
    return bad
