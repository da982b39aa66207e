"""pcseg.graphs.CapturedStep: the training step replayed from two alternating HIP graphs must
give the same parameters, gradients, optimizer state and BN statistics, bit for bit, as the
same steps run eagerly -- with the FPS starts made deterministic and dropout off (under
capture the fused dropout falls back to nn.Dropout, a different random stream)."""
import pytest
import torch

import pcseg
from pcseg.ddp import FlatGradAllReduce
from pcseg.graphs import CapturedStep
from pcseg.optim import FlatAdam
from pcseg.synthetic import make_batch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _zero_starts(B, N, device):
    return torch.zeros(B, dtype=torch.int32, device=device)


def _setup(ctor, seed=0):
    torch.manual_seed(seed)
    m = ctor().to(DEV).train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    grads = FlatGradAllReduce(m)
    return m, grads, FlatAdam(grads, lr=1e-3)


@pytest.mark.parametrize('ctor', [lambda: pcseg.PointNetpp(14), lambda: pcseg.PointNeXt(14)],
                         ids=['pointnetpp', 'pointnext'])
def test_captured_step_matches_eager_steps(monkeypatch, ctor):
    monkeypatch.setattr(pcseg.common, '_fps_start', _zero_starts)
    pts, labels, lengths = make_batch(4, 4096, seed=21)
    x, lab, ln = pts.to(DEV), labels.to(DEV), lengths.to(DEV)
    ce = pcseg.masked_onehot_cross_entropy

    a, ga, oa = _setup(ctor)
    for _ in range(5):
        ga.zero_grad()
        ce(a(x), lab, ln).backward()
        ga.synchronize()
        oa.step()
    torch.cuda.synchronize()

    b, gb, ob = _setup(ctor)
    cs = CapturedStep(b, x, lab, ln, gb, ob, ce, warmup=2)
    assert cs.prefetch and len(cs.graphs) == 2
    losses = [float(cs.step()) for _ in range(3)]      # steps 3, 4, 5 (replays of graph 0, 1, 0)
    torch.cuda.synchronize()
    assert all(torch.isfinite(torch.tensor(losses)))
    assert ob.t == oa.t == 5
    for (k, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(p, q), k
        assert torch.equal(p.grad, q.grad), k
    for (k, u), v in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(u, v), k
    assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq)


def test_captured_step_draws_new_fps_starts_per_replay():
    """With the default device-side FPS draws, consecutive replays sample different centroids
    (the Philox offset advances per replay), as eager steps do."""
    pts, labels, lengths = make_batch(2, 4096, seed=22)
    x, lab, ln = pts.to(DEV), labels.to(DEV), lengths.to(DEV)
    b, gb, ob = _setup(lambda: pcseg.PointNetpp(14), seed=1)
    cs = CapturedStep(b, x, lab, ln, gb, ob, pcseg.masked_onehot_cross_entropy, warmup=1)
    seen = []
    for _ in range(4):
        cs.step()
        torch.cuda.synchronize()
        seen.append(torch.cat([t.reshape(-1).float() for t in cs.plans[cs.k].fps_idx]).clone())
    assert not torch.equal(seen[0], seen[2]) and not torch.equal(seen[1], seen[3])
