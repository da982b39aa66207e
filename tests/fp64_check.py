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
              inputs=None, init_seed=None, fps_starts=None, knn_idx=None, label_classes=None,
              replay_pool_arg=True):
    """inputs=(x, labels, lengths) overrides the synthetic batch; fps_starts / knn_idx seed the
    fp32 oracle run (e.g. a golden fixture's recorded draws).  Order: CPU fp32 oracle (records
    its neighbour indices), GPU (same FPS starts / kNN graphs; records its discrete decisions:
    max-pool argmax, activation signs), then the CPU oracle in fp32 and in fp64 on those same
    indices and decisions.  Rows: (tensor, |GPU - fp64|, |CPU fp32 - fp64| on the same decisions,
    |fp64|, |CPU fp32 with its own decisions (= the reference's run) - fp64|)."""
    if inputs is None:
        pts, labels, lengths = make_batch(B, N, seed=seed, uniform=uniform)
        if pad:
            lengths = torch.tensor([N - pad * (i % 2) for i in range(B)], dtype=torch.uint64)
            for i in range(B):
                pts[i, int(lengths[i]):] = 0.0
        x = pts[:, :, :6].contiguous().transpose(1, 2) if chfirst else pts
        lab = labels.float() if chfirst else labels
        if label_classes is not None:
            lab = lab[..., :label_classes].contiguous()
    else:
        x, lab, lengths = inputs
    ref32 = R.seeded_init_(ref_ctor(), seed if init_seed is None else init_seed)
    ref32s = copy.deepcopy(ref32)           # fp32 again, on the GPU's decisions
    ref64 = copy.deepcopy(ref32).double()
    prod = prod_ctor()
    prod.load_state_dict(ref32.state_dict())
    prod = prod.to(dev)
    for m in (ref32, ref32s, ref64, prod):
        m.train()
        _dropout_off(m)

    def logits_of(o):
        return o[0] if isinstance(o, tuple) else o

    rp = R.Replay(fps_starts=fps_starts, knn_idx=knn_idx)
    with R.replay(rp):
        l32 = logits_of(ref32(x))
    R.masked_onehot_cross_entropy(l32, lab, lengths).backward()
    rg = pcseg.Replay(fps_starts=rp.rec_fps_starts, knn_idx=rp.rec_knn_idx if rp.rec_knn_idx else None)
    with pcseg.replay(rg):
        lg = logits_of(prod(x.to(dev)))
    pcseg.masked_onehot_cross_entropy(lg, lab.to(dev), lengths.to(dev)).backward()
    # the fp64 truth: same algorithm on the same neighbour indices (from the fp32 run) and the
    # same discrete decisions as the GPU run -- max-pool argmax and ReLU / LeakyReLU sign: a
    # near-tie at fp32 rounding level decided one way there is evaluated the same way here, so
    # the comparison stays a smooth one (one flipped sign among 1M activations moves a weight
    # gradient by ~1e-3 of its norm: measured on DGCNN conv6, scripts/diag/dgcnn_grad_trace.py)
    # (ball-query sets are checked equal below; the fp64 run takes them in the GPU's within-ball
    # order so the recorded per-row decisions line up with its grouped rows)
    def decisions():
        return R.Replay(fps_idx=rp.rec_fps_idx, group_idx=[g.long() for g in rg.rec_group_idx],
                        interp_idx=rp.rec_interp_idx, knn_idx=rp.rec_knn_idx if rp.rec_knn_idx else None,
                        pool_arg=rg.rec_pool_arg if replay_pool_arg else None,
                        act_mask=rg.rec_act_mask if replay_pool_arg else None)
    # the reference algorithm in fp32 once more, on the same decisions: its distance to the fp64
    # run is the rounding error of an fp32 evaluation of the same branch (the yardstick of the
    # 'ref-noise' clause)
    rp32s = decisions()
    with R.replay(rp32s):
        l32s = logits_of(ref32s(x))
    R.masked_onehot_cross_entropy(l32s, lab, lengths).backward()
    rp64 = decisions()
    with R.replay(rp64):
        l64 = logits_of(ref64(x.double()))
    R.masked_onehot_cross_entropy(l64, lab.double() if lab.is_floating_point() else lab, lengths).backward()
    l_rel = float((l32s.detach().double() - l64.detach()).norm() / l64.detach().norm())
    if l_rel > 2e-3:
        raise AssertionError(f'fp32 oracle logits {l_rel:.2e} from the fp64 run: the fp64 run is not the same '
                             'computation (replayed indices / decisions misaligned)')
    if replay_pool_arg and (rp64.pool_arg or rp64.act_mask):
        raise AssertionError(f'{len(rp64.pool_arg or [])} pool / {len(rp64.act_mask or [])} activation decisions '
                             'recorded on the GPU were not consumed by the oracle')

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

    def add(name, g, c, t, cf):
        g, c, t, cf = g.detach().cpu().double(), c.detach().double(), t.detach().double(), cf.detach().double()
        rows.append((name, float((g - t).norm()), float((c - t).norm()), float(t.norm()), float((cf - t).norm())))
    add('logits', lg, l32s, l64, l32)
    for (k, pg), (_, p32), (_, p64), (_, pf) in zip(sorted(prod.named_parameters()), sorted(ref32s.named_parameters()),
                                                    sorted(ref64.named_parameters()),
                                                    sorted(ref32.named_parameters())):
        add(k, pg.grad, p32.grad, p64.grad, pf.grad)
    for (k, bg), (_, b32), (_, b64), (_, bf) in zip(sorted(prod.state_dict().items()),
                                                    sorted(ref32s.state_dict().items()),
                                                    sorted(ref64.state_dict().items()),
                                                    sorted(ref32.state_dict().items())):
        if 'running' in k:
            add(k, bg, b32, b64, bf)
    return rows


def classify(rows, rtol=1e-3, factor=10.0, floor=1e-3):
    """{tensor: clause} -- the first clause a tensor passes by, or None when it fails:
      'rel'       GPU error vs the fp64 truth <= rtol x its norm;
      'ref-noise' <= factor x the CPU fp32 reference's own error;
      'floor'     <= floor x the largest gradient norm in the same top-level module (sa3, fp1,
                  conv2, ...): the survey's floor for sums that are pure cancellation (pre-BN
                  conv biases, BN betas of pooled layers), whose value is decided by a handful
                  of ReLU/argmax flips at |y| ~ 1e-7 in ANY fp32 evaluation order."""
    top = {}
    for name, _, _, n, *_ in rows:
        if name != 'logits' and 'running' not in name:
            key = name.split('.')[0]
            top[key] = max(top.get(key, 0.0), n)
    out = {}
    for name, eg, ec, n, *_ in rows:
        fl = floor * top.get(name.split('.')[0], 0.0) if 'running' not in name else 0.0
        out[name] = 'rel' if eg <= rtol * n else 'ref-noise' if eg <= factor * ec else 'floor' if eg <= fl else None
    return out


def is_weight(name: str) -> bool:
    """Conv / linear / BN-gamma weight gradients: no cancellation excuse applies to them."""
    return name.endswith('.weight')


def failures(rows, rtol=1e-3, factor=10.0, floor=1e-3, weight_factor=3.0):
    """Tensors that fail every clause, plus every WEIGHT tensor (conv / linear / BN gamma) whose
    GPU error is neither within rtol of the fp64 truth nor within weight_factor x the CPU fp32
    reference's own error: the module floor never excuses a weight, and the reference-noise
    clause only at 3x, not 10x.  (The reference's own fp32 weight gradients are not
    reproducible to 1e-3: on PointNet++ B=2..8, N=4096 they move by 1e-1 between 1 and 8 CPU
    threads and sit 3-4e-2 from the fp64 run -- DESIGN.md section 5.)"""
    cl = classify(rows, rtol, factor, floor)
    bad = []
    for name, eg, ec, n, *_ in rows:
        c = cl[name]
        if c is None or (is_weight(name) and not (eg <= rtol * n or eg <= weight_factor * ec)):
            bad.append((name, c, eg, ec, n))
        elif is_weight(name) and ec > 0.1 * n:
            # a reference this far from the truth means the truth is not the same computation
            # (mis-replayed decisions): the three-way comparison would pass vacuously
            bad.append((name, 'truth-unreliable', eg, ec, n))
    return bad


def report(rows, rtol=1e-3, factor=10.0, floor=1e-3):
    """Human-readable table: which clause each tensor passed by (printed by the GPU tests)."""
    cl = classify(rows, rtol, factor, floor)
    lines = []
    for name, eg, ec, n, *_ in rows:
        rel = eg / n if n else 0.0
        lines.append(f'{cl[name] or "FAIL":9s} gpu/truth {rel:9.2e}  cpu32/truth {ec / n if n else 0.0:9.2e}  {name}')
    counts = {k: sum(v == k for v in cl.values()) for k in ('rel', 'ref-noise', 'floor', None)}
    lines.append(f'clauses: {counts}')
    w = [(eg / ec if ec else float('inf'), eg / n if n else 0.0, name) for name, eg, ec, n, *_ in rows
         if is_weight(name) and n]
    if w:
        ratio = max(w)
        rel = max(w, key=lambda t: t[1])
        lines.append(f'worst weight: gpu/cpu32 error ratio {ratio[0]:.2f} ({ratio[2]}), '
                     f'gpu/truth {rel[1]:.2e} ({rel[2]})')
    return '\n'.join(lines)
