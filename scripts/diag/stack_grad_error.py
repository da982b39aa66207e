"""Diagnostic (GPU box): input-gradient error of one shared-MLP stack (GPU vs CPU fp32 oracle vs
CPU fp64) at the shapes of PointNeXt's small levels, where the end-to-end gradient error grows
most (scripts/diag/pointnext_grad_trace.py: irmlp4's backward, 16 points x 16 neighbours)."""
import copy
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd'), os.path.join(REPO, 'tests')]
import pcseg  # noqa: E402
import pcseg.common as PC  # noqa: E402
from oracle import ref_ops as R  # noqa: E402

torch.manual_seed(0)


def run(kind, cin, mlps, M, pool_k=None, mean=0.0):
    ref = R.seeded_init_((R.UnitPointNet if kind == 'unit' else R.MiniPointNet)(cin, mlps), 11)
    r64 = copy.deepcopy(ref).double()
    prod = (PC.UnitPointNet if kind == 'unit' else PC.MiniPointNet)(cin, mlps)
    prod.load_state_dict(ref.state_dict())
    prod = prod.cuda().train()
    x = torch.randn(M, cin) + mean
    G = M // pool_k if pool_k else M
    g = torch.randn(G, mlps[-1])
    res = {}
    for tag, m, dt in (('cpu', ref, torch.float32), ('f64', r64, torch.float64)):
        xi = x.to(dt).t().unsqueeze(0).contiguous().requires_grad_(True)      # (1, cin, M)
        if kind == 'unit':
            o = m(xi)                                                           # (1, C, M)
        else:
            o = m(xi.view(1, cin, G, pool_k)) if pool_k else m(xi.view(1, cin, M, 1))
            o = o.amax(-1) if o.dim() == 4 else o
        (o.reshape(mlps[-1], G).t() * g.to(dt)).sum().backward()
        res[tag] = (xi.grad[0].t().double(), {k: p.grad.double() for k, p in m.named_parameters()})
    xg = x.cuda().contiguous().requires_grad_(True)
    xr = pcseg.engine.pad_rows(xg)
    o = prod.forward_rows(xr, cin, pool_k=pool_k) if pool_k else prod.forward_rows(xr, cin)
    (o[:, :mlps[-1]] * g.cuda()).sum().backward()
    gp = (xg.grad.cpu().double(), {k: p.grad.cpu().double() for k, p in prod.named_parameters()})
    t = res['f64'][0]
    line = f'{kind:4s} cin {cin:4d} {mlps} M {M:6d} pool {pool_k} mean {mean:4.1f}: dX gpu {float((gp[0] - t).norm() / t.norm()):.2e} ' \
           f'cpu {float((res["cpu"][0] - t).norm() / t.norm()):.2e}'
    for k in res['f64'][1]:
        if k.endswith('weight') and 'conv' in k:
            tw = res['f64'][1][k]
            line += f' | {k} gpu {float((gp[1][k] - tw).norm() / tw.norm()):.1e} cpu {float((res["cpu"][1][k] - tw).norm() / tw.norm()):.1e}'
    print(line, flush=True)


for M in (32, 256, 4096):
    run('unit', 512, [2048, 512], M)
for M in (512, 8192):
    run('mini', 515, [512], M, pool_k=16)
run('unit', 256, [1024, 256], 128)
run('unit', 128, [512, 128], 512)
run('mini', 259, [256], 4096, pool_k=32)
run('unit', 64, [256, 64], 2048)
for mean in (0.0, 3.0):
    run('unit', 9, [32], 8192, mean=mean)
