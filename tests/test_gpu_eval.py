"""Eval-mode parity of the PointNet++ family and PointNet on harness A's evaluation batches.

Harness A's `evaluate` (reference Training/training.py:80-111) runs `model.eval()` under
`torch.no_grad()` over the UNSAMPLED test loader, whose `collate_blocks`
(data_processing/block_datasets.py:5-29) zero-pads the blocks of a batch to the longest one:
e.g. (2, 3701, 9) with lengths [2780, 3701].  The pad rows are real
points at the origin for FPS, ball query, 3-NN and the BatchNorm-free (running-statistics)
MLPs; only the loss masks them.  This path runs the engine's eval-BN branch (use_batch = 0:
bn_eval_coef_kernel, csrc/engine.hip) that the training-mode tests never reach.

Checked per model, against the oracle (the reference algorithm on PyTorch-CPU) with the FPS
starts replayed and non-trivial running statistics (calibrated by one training-mode forward,
then perturbed):
  * geometry index-exact: every FPS index list, ball-query set and 3-NN set, including the
    921 duplicate pad points of sample 0;
  * logits / probabilities within north_star's 1e-3 (norm-relative) of the oracle's fp32
    output (and the fp64 evaluation of the same algorithm on the same indices is printed);
  * the masked loss within 1e-3; running statistics and num_batches_tracked untouched.
"""
import copy

import pytest
import torch

import pcseg
from pcseg.synthetic import make_batch
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
DEV = 'cuda'
RTOL = 1e-3

MODELS = {
    'pointnetpp': (lambda: pcseg.PointNetpp(14), lambda: R.PointNetpp(14), 201),
    'pointnext': (lambda: pcseg.PointNeXt(14), lambda: R.PointNeXt(14), 202),
    'msg': (lambda: pcseg.PointNetppMSG(14), lambda: R.PointNetppMSG(14), 203),
    'pointnet': (lambda: pcseg.PointNetSeg(part_classes=14), lambda: R.PointNetSeg(part_classes=14), 204),
}


def eval_batch(N=3701, lengths=(2780, 3701), seed=211):
    """A zero-padded harness-A test batch: sample i keeps lengths[i] points, the rest are zeros."""
    pts, labels, _ = make_batch(len(lengths), N, seed=seed)
    for i, n in enumerate(lengths):
        pts[i, n:] = 0.0
        labels[i, n:] = 0
    return pts, labels, torch.tensor(lengths, dtype=torch.uint64)


def calibrated(ref_ctor, seed):
    """Oracle model with seeded weights and realistic running statistics: one training-mode
    forward (momentum 1) on another batch, then a perturbation so that they are not batch
    statistics of anything the test evaluates."""
    ref = R.seeded_init_(ref_ctor(), seed)
    bns = [m for m in ref.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)]
    for m in bns:
        m.momentum = 1.0
    cal, _, _ = make_batch(6, 2048, seed=seed + 1)       # 6 samples: the TNet BN1d layers see a batch of 6
    ref.train()
    with torch.no_grad(), R.replay(R.Replay(fps_starts=[torch.tensor([5, 9, 1, 7, 3, 2], dtype=torch.int32)] * 4)):
        ref(cal)
    g = torch.Generator().manual_seed(seed + 2)
    with torch.no_grad():
        for m in bns:
            m.momentum = 0.1
            m.running_mean.add_(torch.randn(m.running_mean.shape, generator=g) * 0.05)
            m.running_var.mul_(torch.rand(m.running_var.shape, generator=g) * 0.4 + 0.8)
    return ref.eval()


def _rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize('name', list(MODELS))
def test_eval_forward_on_padded_test_batch_matches_oracle(name):
    prod_ctor, ref_ctor, seed = MODELS[name]
    ref = calibrated(ref_ctor, seed)
    prod = prod_ctor()
    prod.load_state_dict(ref.state_dict())
    prod = prod.to(DEV).eval()
    before = {k: v.detach().clone() for k, v in prod.state_dict().items()}
    x, labels, lengths = eval_batch()

    rp = R.Replay()
    with R.replay(rp), torch.no_grad():
        l32 = ref(x)
    rg = pcseg.Replay(fps_starts=rp.rec_fps_starts)
    with pcseg.replay(rg), torch.no_grad():
        lg = prod(x.to(DEV))
    torch.cuda.synchronize()
    assert not lg.requires_grad

    # neighbour structure index-exact (sets: the reference's own topk order is not a contract)
    assert len(rg.rec_fps_idx) == len(rp.rec_fps_idx)
    for lv, (a, b) in enumerate(zip(rg.rec_fps_idx, rp.rec_fps_idx)):
        assert torch.equal(a.long(), b.long()), f'FPS level {lv}'
    assert len(rg.rec_group_idx) == len(rp.rec_group_idx)
    for q, (a, b) in enumerate(zip(rg.rec_group_idx, rp.rec_group_idx)):
        assert torch.equal(a.long().sort(-1).values, b.sort(-1).values), f'ball query {q}'
    assert len(rg.rec_interp_idx) == len(rp.rec_interp_idx)
    for q, (a, b) in enumerate(zip(rg.rec_interp_idx, rp.rec_interp_idx)):
        assert torch.equal(a.long().sort(-1).values, b.sort(-1).values), f'3-NN {q}'

    # the same algorithm in fp64 on the same indices: how far fp32 evaluation itself is from exact
    ref64 = copy.deepcopy(ref).double()
    with R.replay(R.Replay(fps_idx=rp.rec_fps_idx, group_idx=rp.rec_group_idx, interp_idx=rp.rec_interp_idx)), \
            torch.no_grad():
        l64 = ref64(x.double())
    e_gpu, e_ref, e_64 = _rel(lg, l32), _rel(l32, l64), _rel(lg, l64)
    print(f'\n{name}: |gpu - oracle32| {e_gpu:.2e}  |oracle32 - fp64| {e_ref:.2e}  |gpu - fp64| {e_64:.2e}')
    assert e_gpu <= RTOL, e_gpu
    assert e_64 <= RTOL, e_64

    loss_g = pcseg.masked_onehot_cross_entropy(lg, labels.to(DEV), lengths.to(DEV))
    loss_r = R.masked_onehot_cross_entropy(l32, labels, lengths)
    assert abs(float(loss_g) - float(loss_r)) <= RTOL * abs(float(loss_r))

    # eval does not touch the running statistics / counters
    for k, v in prod.state_dict().items():
        assert torch.equal(v, before[k]), k


def test_eval_no_grad_builds_no_inverse_maps_and_matches_grad_mode():
    """Under no_grad the forward's geometry plan skips the backward-only inverse maps; the
    outputs equal an eval forward with grad mode on (same FPS starts)."""
    prod_ctor, ref_ctor, seed = MODELS['pointnetpp']
    ref = calibrated(ref_ctor, seed)
    prod = prod_ctor()
    prod.load_state_dict(ref.state_dict())
    prod = prod.to(DEV).eval()
    x, _, _ = eval_batch()
    xd = x.to(DEV)
    with torch.no_grad():
        plan = prod._geometry(xd, prod._coords_of(xd))
    assert all(inv is None for bl in plan.balls for _, inv in bl) and all(t[2] is None for t in plan.nn)
    starts = [torch.tensor([17, 3], dtype=torch.int32) for _ in range(4)]
    with pcseg.replay(pcseg.Replay(fps_starts=list(starts))), torch.no_grad():
        a = prod(xd)
    with pcseg.replay(pcseg.Replay(fps_starts=list(starts))):
        b = prod(xd).detach()
    assert torch.equal(a, b)
