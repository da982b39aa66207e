"""The fused 128-wide backward ring (bwd_ring.hip) on the PointNet++ FP1 / FP2 stack shapes:
its per-launch time (probe events, each launch alone on an idle GPU, replayed back to back) and
the whole stack backward per policy ('all' = the ring, opt-in; 'off' = dgrad + lane wgrad, as the default).
usage: python scripts/ring_ab.py            (PCS_LIB selects a library build)"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg.common import UnitPointNet  # noqa: E402
from pcseg.engine import KernelProbe, lane_join, set_bwd_fuse  # noqa: E402

dev = torch.device('cuda')
for name, M, kin, mlps in (('fp1', 131072, 128, [128, 128, 128]), ('fp2', 32768, 320, [256, 128])):
    torch.manual_seed(0)
    mod = UnitPointNet(kin, mlps).to(dev).train()
    ld = (kin + 3) // 4 * 4
    x = torch.zeros(M, ld, device=dev)
    x[:, :kin] = torch.randn(M, kin, device=dev)
    x.requires_grad_(True)
    res = []
    for pol in ('all', 'off'):
        set_bwd_fuse(mod, pol)
        mod.__dict__.pop('_pcs_cache', None)
        g = None
        times = []
        for it in range(8):
            y = mod.forward_rows(x, kin)
            if g is None:
                g = torch.randn_like(y)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y.backward(g)
            lane_join(dev)
            e1.record()
            e1.synchronize()
            if it >= 3:
                times.append(e0.elapsed_time(e1) * 1e3)
        times.sort()
        res.append(f'{pol} bwd {times[len(times) // 2]:7.1f} us')
        if pol == 'all':
            y = mod.forward_rows(x, kin)
            with KernelProbe() as kp:
                y.backward(g)
                lane_join(dev)
            torch.cuda.synchronize()
            for nm, (n, fl, by, sec) in kp.summary().items():
                if 'bwd_ring' in nm:
                    rep = kp.replay(nm, reps=20)
                    res.append(f'{nm} x{n}: in-call {sec / n * 1e6:6.1f} us, replayed {rep * 1e6:6.1f} us '
                               f'= {fl / n / rep / 1e12:5.1f} TF/s, {by / n / rep / 1e9:6.0f} GB/s')
    print(f'{name} M={M} {kin}->{mlps}: ' + ' | '.join(res), flush=True)
