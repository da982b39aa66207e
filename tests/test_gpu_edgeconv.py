"""Fused EdgeConv (csrc/edgeconv.hip, pcs_edgeconv_fwd/bwd) against the reference EdgeConv
(models/dgcnn/dgcnn.py:60-77, restated in oracle/ref_ops.py) evaluated in float64 on the
CPU with the same kNN graph, and against pcseg's materialised-edge path (edge rows + engine
GEMM) on the GPU.

The fused path computes z_(i,j) = (Y_j - Y_i) + P_i (Y = X W1^T, P = X W2^T) instead of
W [x_j - x_i ; x_i]: the same value up to fp32 rounding, so the check is norm-relative:
forward output, running stats and every gradient within 1e-4 of the fp64 reference
(north_star: 1e-3 relative fp32); argmax ties are not expected on random features."""
import copy

import pytest
import torch

import pcseg
from pcseg import ops
from pcseg.engine import edgeconv, edgeconv_fused_ok
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
DEV = 'cuda'
TOL = 1e-4


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _case(C, Cout, B=2, N=512, k=20, seed=0, dup=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, N, generator=g)
    if dup:                                     # duplicate points: exact ties in z over k
        x[:, :, 1::2] = x[:, :, 0::2]
    idx = R.knn(x, k)
    ref = R.EdgeConv(C, Cout, k)
    R.seeded_init_(ref, seed + 1)
    prod = pcseg.EdgeConv(C, Cout, k)
    prod.load_state_dict(ref.state_dict())
    return x, idx, ref, prod


def _ref_fp64(x, idx, ref):
    r64 = copy.deepcopy(ref).double().train()
    xr = x.double().clone().requires_grad_(True)
    with R.replay(R.Replay(knn_idx=[idx])):
        out = r64(xr)                                        # (B, Cout, N)
    return r64, xr, out


@pytest.mark.parametrize('C,Cout', [(3, 64), (64, 64), (64, 128)])
def test_edgeconv_fused_matches_reference_fp64(C, Cout):
    x, idx, ref, prod = _case(C, Cout, seed=C + Cout)
    prod = prod.to(DEV).train()
    assert edgeconv_fused_ok(prod.conv[0], prod.conv[1], C)
    r64, xr, out64 = _ref_fp64(x, idx, ref)
    xd = x.to(DEV).requires_grad_(C != 3)
    with pcseg.replay(pcseg.Replay(knn_idx=[idx])):
        out = prod(xd)
    assert out.shape == out64.shape
    assert rel(out.detach(), out64.detach()) < TOL
    w = torch.randn(out64.shape, generator=torch.Generator().manual_seed(5), dtype=torch.float64)
    (out64 * w).sum().backward()
    (out * w.float().to(DEV)).sum().backward()
    for (name, p64), p in zip(r64.named_parameters(), prod.parameters()):
        assert rel(p.grad, p64.grad) < TOL, name
    if C != 3:
        assert rel(xd.grad, xr.grad) < TOL
    bn64, bn = r64.conv[1], prod.conv[1]
    assert rel(bn.running_mean, bn64.running_mean) < TOL
    assert rel(bn.running_var, bn64.running_var) < TOL
    assert int(bn.num_batches_tracked) == 1


def test_edgeconv_fused_negative_gamma():
    """BN scales of both signs (and a zero): the forward keeps the max over k where gamma >= 0
    and the min where gamma < 0; output, argmax routing and every gradient against fp64."""
    x, idx, ref, prod = _case(64, 64, seed=21)
    with torch.no_grad():
        w = ref.conv[1].weight
        w.copy_(w.abs() * torch.tensor([1.0, -1.0]).repeat(w.numel() // 2))
        w[5] = 0.0
    prod.load_state_dict(ref.state_dict())
    prod = prod.to(DEV).train()
    r64, xr, out64 = _ref_fp64(x, idx, ref)
    xd = x.to(DEV).requires_grad_(True)
    with pcseg.replay(pcseg.Replay(knn_idx=[idx])):
        out = prod(xd)
    assert rel(out.detach(), out64.detach()) < TOL
    g = torch.randn(out64.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    (out64 * g).sum().backward()
    (out * g.float().to(DEV)).sum().backward()
    assert rel(xd.grad, xr.grad) < TOL
    for (name, p64), p in zip(r64.named_parameters(), prod.parameters()):
        assert rel(p.grad, p64.grad) < TOL, name


def test_edgeconv_fused_equals_materialised_path():
    """Same module, same graph: the fused kernels and the edge-row engine path agree."""
    x, idx, _, prod = _case(64, 64, seed=3)
    prod = prod.to(DEV).train()
    other = copy.deepcopy(prod)
    xp = x.transpose(1, 2).contiguous().to(DEV)
    B, N, C = xp.shape
    i32 = idx.to(torch.int32).to(DEV)
    a_in = xp.reshape(B * N, C).clone().requires_grad_(True)
    a = edgeconv(a_in, C, i32, prod.conv[0], prod.conv[1], 0.2)
    b_in = xp.clone().requires_grad_(True)
    rows = ops.edge_rows(b_in, i32)
    b = pcseg.engine.shared_mlp(rows, 2 * C, [other.conv[0]], [other.conv[1]], 'lrelu', 0.2, pool_k=20)
    assert rel(a.detach(), b.detach()) < TOL
    gw = torch.randn(a.shape, device=DEV)
    (a * gw).sum().backward()
    (b * gw).sum().backward()
    assert rel(a_in.grad, b_in.grad.reshape(B * N, C)) < TOL
    for p, q in zip(prod.parameters(), other.parameters()):
        assert rel(p.grad, q.grad) < TOL


def test_edgeconv_fused_duplicate_points():
    """Duplicate points give exact ties over k: the first-index argmax rule of the reference
    (max over dim=-1) must route the gradient to the same slot."""
    x, idx, ref, prod = _case(64, 64, seed=9, dup=True)
    prod = prod.to(DEV).train()
    r64, xr, out64 = _ref_fp64(x, idx, ref)
    xd = x.to(DEV).requires_grad_(True)
    with pcseg.replay(pcseg.Replay(knn_idx=[idx])):
        out = prod(xd)
    assert rel(out.detach(), out64.detach()) < TOL
    w = torch.randn(out64.shape, generator=torch.Generator().manual_seed(6), dtype=torch.float64)
    (out64 * w).sum().backward()
    (out * w.float().to(DEV)).sum().backward()
    assert rel(xd.grad, xr.grad) < 1e-3
    for (name, p64), p in zip(r64.named_parameters(), prod.parameters()):
        assert rel(p.grad, p64.grad) < 1e-3, name


def test_edgeconv_eval_mode_uses_materialised_path():
    x, idx, ref, prod = _case(64, 64, seed=4)
    prod = prod.to(DEV).eval()
    assert not edgeconv_fused_ok(prod.conv[0], prod.conv[1], 64)
    ref = ref.eval()
    with torch.no_grad():
        with R.replay(R.Replay(knn_idx=[idx])):
            o_ref = ref(x)
        with pcseg.replay(pcseg.Replay(knn_idx=[idx])):
            o = prod(x.to(DEV))
    assert rel(o, o_ref) < TOL


@pytest.mark.parametrize('tail', [0, 64])
@pytest.mark.parametrize('C,Cout', [(64, 64), (3, 64)])
def test_edgeconv_weight_at_storage_end_in_nan_storage(C, Cout, tail):
    """Regression guard of the round-4 over-read (the row GEMM's B loads clamped to the weight's
    row STRIDE, so W + C -- the second half of the (Cout, 2C) EdgeConv weight, read as a column
    block -- ran up to C floats past the weight's end): the weight is a view into a NaN-filled
    storage, ending exactly at the storage's end (tail = 0) or followed by NaNs (tail = 64), with
    NaNs before it.  Any load outside the weight's logical extent reads NaN (or faults at the
    allocation's end), so outputs and every gradient must be finite and equal the fp64 oracle."""
    x, idx, ref, prod = _case(C, Cout, seed=11 + C)
    prod = prod.to(DEV).train()
    conv = prod.conv[0]
    w = conv.weight.detach()
    n = w.numel()
    store = torch.full((256 + n + tail,), float('nan'), device=DEV)
    view = store[256:256 + n].view_as(w)
    view.copy_(w)
    conv.weight = torch.nn.Parameter(view)
    assert conv.weight.data_ptr() + 4 * n == store.data_ptr() + 4 * (store.numel() - tail)
    r64, xr, out64 = _ref_fp64(x, idx, ref)
    xd = x.to(DEV).requires_grad_(C != 3)
    with pcseg.replay(pcseg.Replay(knn_idx=[idx])):
        out = prod(xd)
    g = torch.randn(out64.shape, generator=torch.Generator().manual_seed(6), dtype=torch.float64)
    (out64 * g).sum().backward()
    (out * g.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert rel(out.detach(), out64.detach()) < TOL
    for (name, p64), p in zip(r64.named_parameters(), prod.parameters()):
        assert torch.isfinite(p.grad).all(), name
        assert rel(p.grad, p64.grad) < TOL, name
    if C != 3:
        assert torch.isfinite(xd.grad).all()
        assert rel(xd.grad, xr.grad) < TOL
    # the NaN storage around the weight is untouched (nothing wrote outside the view either)
    assert torch.isnan(store[:256]).all() and torch.isnan(store[256 + n:]).all()


@pytest.mark.parametrize('C,Cout,ld,col0', [(64, 64, 1408, 0), (64, 128, 1408, 192), (3, 64, 388, 4)])
def test_edgeconv_second_output_into_row_block(C, Cout, ld, col0):
    """`also` (round 5, pcs_edgeconv_fwd's out2): the pooled rows land bit for bit in a column
    block of a wider buffer too, nothing else of that buffer is touched, and the dense output and
    every gradient are bitwise those of the call without it."""
    from pcseg.engine import storage_alias
    B, N, k = 2, 512, 20
    x, idx, _, prod = _case(C, Cout, B=B, N=N, k=k, seed=7)
    prod = prod.to(DEV).train()
    twin = copy.deepcopy(prod)
    xp = x.transpose(1, 2).contiguous().to(DEV)
    gi = idx.to(DEV, torch.int32)
    H = torch.full((B * N, ld), float('nan'), device=DEV)
    blk = storage_alias(H, col0, Cout)
    outs, grads = [], []
    for m, also in ((prod, blk), (twin, None)):
        # (a 3-channel input takes no gradient, as DGCNN's coordinates: the kernel's dX needs C % 4 == 0)
        xr = xp.reshape(B * N, C).clone().requires_grad_(C % 4 == 0)
        out = edgeconv(xr, C, gi, m.conv[0], m.conv[1], m.conv[2].negative_slope, also=also)
        (out * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
        outs.append(out.detach())
        grads.append(([xr.grad] if C % 4 == 0 else []) + [p.grad for p in m.parameters()])
    torch.cuda.synchronize()
    assert torch.equal(blk, outs[0])
    assert torch.equal(outs[0], outs[1])
    for a, b in zip(grads[0], grads[1]):
        assert torch.equal(a, b)
    rest = torch.cat([H[:, :col0], H[:, col0 + Cout:]], dim=1)
    assert torch.isnan(rest).all()


def test_dgcnn_head_buffer_equals_copied_concatenation():
    """DGCNN-colour with its parts written into the head buffer by their producers (round 5) against
    the same model taking the copy path (_dgcnn_head(H=None)): logits, x5 and every gradient bitwise."""
    import pcseg.models as PM
    torch.manual_seed(3)
    m1 = pcseg.DGCNNWithColor(13).to(DEV).train()
    m2 = copy.deepcopy(m1)
    x = torch.randn(2, 6, 1024, device=DEV)
    res = []
    fg, head = PM.EdgeConv.forward_graph, PM._dgcnn_head
    for m, old in ((m1, False), (m2, True)):
        if old:
            PM.EdgeConv.forward_graph = lambda self, xp, seeds=None, inv_batch=None, also=None, order=None: fg(
                self, xp, seeds, inv_batch=inv_batch, order=order)
            PM._dgcnn_head = lambda self, parts, B, N, H=None: head(self, parts, B, N, None)
        try:
            torch.manual_seed(11)           # the same dropout draws in both runs
            logits, x5, _ = m(x)
            (logits * torch.linspace(-1, 1, logits.numel(), device=DEV).view_as(logits)).sum().backward()
        finally:
            PM.EdgeConv.forward_graph, PM._dgcnn_head = fg, head
        res.append((logits.detach(), x5.detach(), [p.grad for p in m.parameters()]))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for a, b in zip(res[0][2], res[1][2]):
        assert torch.equal(a, b)
