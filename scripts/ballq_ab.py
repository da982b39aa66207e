"""Ball query alone at the SA1 shapes (HIP events, median of 10): PointNet++ (B=32, 4096 -> 1024,
r 0.1, k 32) and PointNeXt-B (B=16, 24 576 -> 1024, r 0.1, k 32), and the FPS launches before it."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg import ops  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

dev = torch.device('cuda')


def timed(fn, reps=10):
    ts = []
    for _ in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts = sorted(ts[2:])
    return ts[len(ts) // 2]


for name, B, N, C in (('pointnetpp sa1', 32, 4096, 1024), ('pointnext sa1', 16, 24576, 1024)):
    pts, _, _ = make_batch(B, N, seed=5)
    xyz = pts[:, :, :3].contiguous().to(dev)
    start = torch.zeros(B, dtype=torch.int32, device=dev)
    idx, cent = ops.fps(xyz, C, start)
    t_fps = timed(lambda: ops.fps(xyz, C, start))
    t_bq = timed(lambda: ops.ball_query(cent, xyz, 0.1, 32))
    print(f'{name}: B={B} N={N} C={C}: fps {t_fps:8.1f} us | ball query {t_bq:8.1f} us', flush=True)
