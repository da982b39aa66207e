"""Training-mode Dropout fused into a shared-MLP stack's output (DGCNN conv6 / conv7,
reference models/dgcnn/dgcnn.py:196-207: Conv1d -> BatchNorm1d -> LeakyReLU -> Dropout).

The mask comes from a counter-based hash of (seed, element) instead of torch's Philox
stream, so it is checked by its properties: every output is either 0 or exactly
activation / (1 - p); the kept fraction is 1 - p; one seed gives one mask, another seed a
different one; and the backward (pcs_dropout_bwd, mask recomputed) equals the stack's
backward fed with the masked, scaled gradient -- bitwise, as the engine is deterministic."""
import pytest
import torch
import torch.nn as nn

import pcseg
from pcseg.engine import shared_mlp

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _stack(cin=64, cout=128, seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Conv1d(cin, cout, 1, bias=False), nn.BatchNorm1d(cout),
                         nn.LeakyReLU(negative_slope=0.2)).to(DEV).train()


def _run(seq, x, dropout):
    return shared_mlp(x, x.shape[1], [seq[0]], [seq[1]], 'lrelu', 0.2, 0, dropout=dropout)


@pytest.mark.parametrize('p', [0.5, 0.2])
def test_fused_dropout_forward_properties(p):
    seq = _stack()
    x = torch.randn(65536, 64, device=DEV)
    y0 = _run(seq, x, None).detach()
    y = _run(seq, x, (p, 1234)).detach()
    scale = torch.tensor(1.0 / (1.0 - p), dtype=torch.float32)
    kept = y != 0
    assert torch.equal(y[kept], y0[kept] * scale.to(DEV))
    frac = float(kept.float().mean())
    assert abs(frac - (1.0 - p)) < 0.005, frac
    again = _run(seq, x, (p, 1234)).detach()
    assert torch.equal(y, again)
    other = _run(seq, x, (p, 99)).detach()
    assert not torch.equal(y != 0, other != 0)


@pytest.mark.parametrize('M,cin,cout,xgrad', [(32768, 64, 128, False),
                                              # a wide layer whose dZ is materialised (DGCNN conv7's
                                              # shape): the mask is applied on load by the BN-backward
                                              # reduce and the dZ pass, no masked copy
                                              (65536, 512, 256, True)])
def test_fused_dropout_backward_matches_masked_gradient(M, cin, cout, xgrad):
    p, seed = 0.5, 777
    seq_a, seq_b = _stack(cin, cout, seed=3), _stack(cin, cout, seed=3)
    xa = torch.randn(M, cin, device=DEV, requires_grad=xgrad)
    xb = xa.detach().clone().requires_grad_(xgrad)
    g = torch.randn(M, cout, device=DEV)
    y0 = _run(seq_b, xb, None)
    y = _run(seq_a, xa, (p, seed))
    kept = ((y != 0) | (y0 == 0)).float()
    y.backward(g)
    y0.backward(g * kept * 2.0)
    torch.cuda.synchronize()
    for a, b in zip(seq_a.parameters(), seq_b.parameters()):
        assert torch.equal(a.grad, b.grad)
    if xgrad:
        assert torch.equal(xa.grad, xb.grad)


def test_dgcnn_head_uses_fused_dropout():
    """DGCNNWithColor in training mode runs its conv6 / conv7 dropout inside the engine (no
    torch dropout kernel), and a seeded step is reproducible."""
    def step():
        torch.manual_seed(0)
        m = pcseg.DGCNNWithColor(num_classes=13, k=20).to(DEV).train()
        torch.manual_seed(1)
        x = torch.randn(2, 6, 1024, device=DEV)
        out = m(x)[0]
        out.square().mean().backward()
        return out.detach(), m.conv6[0].weight.grad.clone()
    o1, g1 = step()
    o2, g2 = step()
    assert torch.equal(o1, o2) and torch.equal(g1, g2)


@pytest.mark.parametrize('ctor', [lambda: pcseg.PointNetpp(14), lambda: pcseg.PointNetppMSG(14)])
def test_pointnet2_head_dropout_fused_and_reproducible(ctor):
    """PointNet++'s head Dropout (PointNetpp.py:44-45: drop -> conv) runs fused into FP1's
    output in training mode: the step is finite and, seeded, bitwise reproducible (the mask
    seed comes from torch's CPU generator)."""
    from pcseg.synthetic import make_batch

    def step():
        torch.manual_seed(0)
        m = ctor().to(DEV).train()
        pts, _, _ = make_batch(2, 2048, seed=4)
        torch.manual_seed(1)
        out = m(pts.to(DEV))
        out.square().mean().backward()
        return out.detach(), m.conv.weight.grad.clone()
    o1, g1 = step()
    o2, g2 = step()
    assert torch.isfinite(o1).all()
    assert torch.equal(o1, o2) and torch.equal(g1, g2)


def test_dropout_masks_differ_between_graph_replays():
    """A training step captured in a HIP graph: the Dropout after a DGCNN head stack must draw a
    new mask on every replay (the fused path's host-drawn seed would be baked into the graph,
    so under capture the module's nn.Dropout runs -- torch's Philox offset advances per replay)."""
    from pcseg.models import _seq_rows
    torch.manual_seed(0)
    seq = nn.Sequential(nn.Conv1d(64, 128, 1, bias=False), nn.BatchNorm1d(128), nn.LeakyReLU(negative_slope=0.2),
                        nn.Dropout(0.5)).to(DEV).train()
    x = torch.randn(8192, 64, device=DEV)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            _seq_rows(x, seq)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = _seq_rows(x, seq)
    g.replay()
    a = y.detach().clone()
    g.replay()
    b = y.detach().clone()
    torch.cuda.synchronize()
    za, zb = a == 0, b == 0
    assert not torch.equal(za, zb)
    for z in (za, zb):
        assert abs(float(z.float().mean()) - 0.5) < 0.01
