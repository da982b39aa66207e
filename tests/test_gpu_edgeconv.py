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
