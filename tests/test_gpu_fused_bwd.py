"""Fused thin-layer backward (csrc/fused_bwd.hip): one launch gives an inner layer's data
gradient, its input layer's BN-backward sums and its weight/bias gradient from one read of
the rebuilt dZ.  Checked through MiniPointNet stacks (reference models/utils/common.py:125-150)
against the same stack evaluated in fp64 on the CPU, for every width pair the fused kernel
is built for (32 / 64 / 128), the pooled (POOLBWD) and plain (BNBWD) top layers and a ragged
row count, and for bitwise reproducibility.

The engine's default policy fuses only layers over >= 2^19 rows (SA1-sized: there the fused
launch beats the dgrad + side-lane wgrad pair, PointNet++ step -1.2 %; on the smaller 128-wide
layers the overlapped pair is faster).  So the width sweep sets the per-layer policy
(pcs_mlp_layer.bwd_fuse, pcseg.engine.set_bwd_fuse) to 'all' (every thin inner layer fused),
and one SA1-sized stack checks the default policy."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (REPO, os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import pcseg  # noqa: E402

pytestmark = pytest.mark.gpu


def _fp64_stack(mod, x, pool_k):
    """MiniPointNet forward in fp64 on the CPU with mod's parameters (training-mode BN)."""
    B, Cin, H, W = x.shape
    a = x.permute(0, 2, 3, 1).reshape(-1, Cin)
    for conv, bn in zip(mod.conv, mod.batch):
        w = conv.weight.detach().double().cpu().view(conv.weight.shape[0], -1).requires_grad_()
        b = conv.bias.detach().double().cpu().requires_grad_()
        g = bn.weight.detach().double().cpu().requires_grad_()
        be = bn.bias.detach().double().cpu().requires_grad_()
        z = a @ w.t() + b
        mean = z.mean(0)
        var = z.var(0, unbiased=False)
        a = torch.relu((z - mean) / torch.sqrt(var + bn.eps) * g + be)
        yield (w, b, g, be)
    if pool_k:
        a = a.view(-1, pool_k, a.shape[1]).max(1).values
    yield a


def _run(widths, cin, B, H, W, pool_k, seed, need_dx=True, fuse='all'):
    """need_dx=False: the stack's input takes no gradient (PointNet++ SA1's grouped rows), so
    its first layer runs the weight-gradient-only form."""
    torch.manual_seed(seed)
    mod = pcseg.MiniPointNet(cin, widths).cuda().train()
    pcseg.engine.set_bwd_fuse(mod, fuse)
    x = torch.randn(B, cin, H, W, dtype=torch.float32)
    xg = x.cuda().requires_grad_(need_dx)
    if pool_k:
        rows = xg.permute(0, 2, 3, 1).reshape(B * H * W, cin)
        out = mod.forward_rows(pcseg.engine.pad_rows(rows), cin, pool_k=pool_k)
    else:
        out = mod(xg).permute(0, 2, 3, 1).reshape(B * H * W, -1)
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed + 1))
    out.backward(gout.cuda())
    torch.cuda.synchronize()
    grads = [(c.weight.grad.view(c.weight.shape[0], -1).cpu(), c.bias.grad.cpu(), n.weight.grad.cpu(),
              n.bias.grad.cpu()) for c, n in zip(mod.conv, mod.batch)]
    return mod, x, gout, grads, xg.grad.cpu() if need_dx else None


def _rel(a, b):
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-30))


# (input width, widths, pooled group size): every fused (C, CI) pair appears as an inner layer
CASES = [
    (9, [32, 32, 64], 32),       # SA1: (32, 32), (64, 32), pooled top
    (67, [64, 64, 128], 32),     # SA2: (64, 64), (128, 64)
    (131, [128, 128, 256], 0),   # SA3-like inner (128, 128); the 256-wide top stays on two GEMMs
    (134, [128, 128, 128], 0),   # FP1: (128, 128) twice, plain top
    (16, [128, 32, 64], 16),     # (32, 128), (64, 32)
    (16, [32, 128, 64], 0),      # (128, 32), (64, 128)
]


def check_vs_fp64(cin, widths, pool_k, B=2, H=80, W=32, need_dx=True, fuse='all'):
    """M = B*H*W rows (default 5120 = 80 row tiles)."""
    mod, x, gout, grads, gx = _run(widths, cin, B, H, W, pool_k, seed=cin + len(widths), need_dx=need_dx,
                                   fuse=fuse)
    xd = x.double().requires_grad_()
    it = _fp64_stack(mod, xd, pool_k)
    params = [next(it) for _ in widths]
    out = next(it)
    out.backward(gout.double().view(out.shape))
    scale = max(float(p[0].grad.norm()) for p in params)
    for l, (got, ref) in enumerate(zip(grads, params)):
        dw, db, dg, dbe = got
        assert _rel(dw, ref[0].grad) < 1e-3, (l, 'dW', _rel(dw, ref[0].grad))
        assert _rel(dg, ref[2].grad) < 1e-3, (l, 'dgamma', _rel(dg, ref[2].grad))
        assert _rel(dbe, ref[3].grad) < 1e-3, (l, 'dbeta', _rel(dbe, ref[3].grad))
        # pre-BN conv bias: analytically zero under training-mode BN; its fp32 value is noise
        assert float((db.double() - ref[1].grad).abs().max()) < 1e-3 * scale, (l, 'db')
    if need_dx:
        assert _rel(gx, xd.grad) < 1e-3, ('dX', _rel(gx, xd.grad))


@pytest.mark.parametrize('case', CASES, ids=[f'{c[0]}-{"x".join(map(str, c[1]))}-{c[2]}' for c in CASES])
def test_fused_backward_width_sweep_vs_fp64(case):
    """Every width pair and the pooled / plain top layers with every thin inner layer fused
    (bwd_fuse = 'all'); first layers of <= 32 channels also in the weight-gradient-only form."""
    check_vs_fp64(*case)
    if case[0] <= 32:
        check_vs_fp64(*case, need_dx=False)


def test_fused_backward_ragged_and_bitwise():
    check_ragged_rows()
    check_bitwise_reproducible()


def test_bwd_fuse_policy_is_per_call():
    """Two stacks in one process with different policies: the 'all' stack's backward runs the
    fused kernel, the 'off' stack's does not (no process-global switch)."""
    from pcseg.engine import KernelProbe
    names = {}
    for fuse in ('all', 'off'):
        with KernelProbe() as kp:
            _run([64, 64], 64, 2, 40, 32, 0, seed=3, fuse=fuse)
        names[fuse] = {r[0] for r in kp.records()}
    assert any('fused_bwd_kernel' in n for n in names['all']), names['all']
    assert not any('fused_bwd_kernel' in n for n in names['off']), names['off']


def test_fused_backward_default_policy_sa1_sized():
    """SA1 of PointNet++ at batch 16: 16 x 1024 centroids x 32 neighbours = 2^19 rows, widths
    9 -> 32 -> 32 -> 64, pooled over 32 -- the layers the default policy fuses; the input takes
    no gradient, as in the model, so the first layer runs the weight-gradient-only form."""
    check_vs_fp64(9, [32, 32, 64], 32, B=16, H=1024, W=32, need_dx=False, fuse='default')


def check_ragged_rows():
    """M not a multiple of the 64-row tile: the last tile's missing rows contribute nothing."""
    B, H, W = 1, 2051, 1
    mod, x, gout, grads, gx = _run([64, 64], 64, B, H, W, 0, seed=5)   # 64 x 64 inner layer fused
    xd = x.double().requires_grad_()
    it = _fp64_stack(mod, xd, 0)
    params = [next(it) for _ in range(2)]
    out = next(it)
    out.backward(gout.double().view(out.shape))
    for l, (got, ref) in enumerate(zip(grads, params)):
        assert _rel(got[0], ref[0].grad) < 1e-3, (l, 'dW')
        assert _rel(got[2], ref[2].grad) < 1e-3, (l, 'dgamma')
    assert _rel(gx, xd.grad) < 1e-3


def check_bitwise_reproducible():
    a = _run([32, 64, 128], 64, 2, 64, 32, 32, seed=11)
    b = _run([32, 64, 128], 64, 2, 64, 32, 32, seed=11)
    for ga, gb in zip(a[3], b[3]):
        for ta, tb in zip(ga, gb):
            assert torch.equal(ta, tb)
    assert torch.equal(a[4], b[4])


@pytest.mark.parametrize('cin,widths,rows,pool_k', [(67, [64, 64, 128], 32768, 32), (131, [128, 128, 256], 16384, 32),
                                                     (259, [256, 256, 512], 8192, 32), (35, [32, 64], 5000, 0)])
def test_first_layer_dx_from_column3(cin, widths, rows, pool_k):
    """MiniPointNet.forward_rows(dx_from=3) (pcs_mlp_layer.dx_col0; SetAbstraction's grouped rows:
    no caller reads the gradient of their 3 relative-coordinate columns): the data gradient of
    columns [3, cin) -- a GEMM of cin - 3 outputs on W read k-major from column 3 with scalar loads
    (rows of 3 + D floats are unaligned) -- equals the full-width gradient's columns, and every
    weight gradient is unchanged."""
    torch.manual_seed(11)
    mod = pcseg.MiniPointNet(cin, widths).cuda().train()
    x = torch.randn(rows, cin, device='cuda')
    out_g = None
    res = []
    for dx_from in (0, 3):
        for p in mod.parameters():
            p.grad = None
        xg = pcseg.engine.pad_rows(x).requires_grad_()
        out = mod.forward_rows(xg, cin, pool_k=pool_k, dx_from=dx_from)
        if out_g is None:
            out_g = torch.randn(out.shape, device='cuda', generator=torch.Generator(device='cuda').manual_seed(5))
        out.backward(out_g)
        torch.cuda.synchronize()
        res.append((xg.grad[:, 3:cin].clone(), [p.grad.clone() for p in mod.parameters()]))
    (d0, g0), (d3, g3) = res
    assert float((d3 - d0).norm() / d0.norm()) <= 1e-6
    for a, b in zip(g0, g3):
        assert torch.equal(a, b)
