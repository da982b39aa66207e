"""Ball queries on the introselect path (rows with K * 64 > N) at the PointNeXt-B and PointNet++
shapes below SA1 (HIP events, median of 20 per launch); PCS_LIB picks the library to time.
Also reports the share of rows whose ball is unambiguous (>= K in radius, no tie at the K-th)."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg import ops  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

dev = torch.device('cuda')


def timed(fn, reps=20):
    ts = []
    for _ in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts = sorted(ts[3:])
    return ts[len(ts) // 2]


def levels(B, N, Cs):
    pts, _, _ = make_batch(B, N, seed=5)
    c = pts[:, :, :3].contiguous().to(dev)
    out = [c]
    for C in Cs:
        start = torch.zeros(B, dtype=torch.int32, device=dev)
        _, c = ops.fps(c, C, start)
        out.append(c.contiguous())
    return out


def eligible(q, x, r, k):
    d = torch.cdist(q, x) ** 2
    ins = (d < r * r).sum(-1)
    return float((ins >= k).float().mean())


total = 0.0
for name, B, N, Cs, queries in (
        ('pointnext', 16, 24576, (1024, 256, 64, 16),
         ((1, 1, 0.1, 32), (2, 1, 0.2, 32), (2, 2, 0.1, 32), (2, 2, 0.2, 32), (3, 2, 0.4, 32), (3, 3, 0.4, 32),
          (4, 3, 0.8, 32), (4, 4, 0.8, 16))),
        ('pointnetpp', 32, 4096, (1024, 256, 64, 16),
         ((2, 1, 0.2, 32), (3, 2, 0.4, 32), (4, 3, 0.8, 32)))):
    lv = levels(B, N, Cs)
    for qi, xi, r, k in queries:
        q, x = lv[qi], lv[xi]
        t = timed(lambda: ops.ball_query(q, x, r, k))
        total += t
        print(f'{name}: q={q.shape[1]:5d} n={x.shape[1]:5d} r={r} k={k}: {t:7.1f} us  '
              f'(>= k in radius: {eligible(q, x, r, k):.2f})', flush=True)
print(f'sum {total:.1f} us', flush=True)
