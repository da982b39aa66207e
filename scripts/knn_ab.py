"""DGCNN kNN timing at B=32, N=4096, k=20 (xyz graph F=3 and a 64-d feature graph), and
run-to-run bitwise equality of the neighbour lists."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
from pcseg import ops  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

B, N, k = 32, 4096, 20
pts, _, _ = make_batch(B, N, seed=3)
xyz = pts[:, :, :3].contiguous().cuda()
feat = torch.randn(B, N, 64, device='cuda')
from pcseg._lib import call, ptr, stream_ptr  # noqa: E402


def plain(x, k):      # pcs_knn: squared norms recomputed by every streaming wave
    o = torch.empty((x.shape[0], x.shape[1], k), dtype=torch.int32, device=x.device)
    call('pcs_knn', ptr(x), x.shape[0], x.shape[1], x.shape[2], k, ptr(o), stream_ptr(x.device))
    return o


for name, x in (('F=3', xyz), ('F=64', feat)):
    for path, fn in (('ws', ops.knn), ('plain', plain)):
        out = fn(x, k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            again = fn(x, k)
        e1.record()
        e1.synchronize()
        print(f'{name} {path}: {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us  repeat bitwise-equal {torch.equal(out, again)}'
              f'  equal to ws {torch.equal(out, ops.knn(x, k))}', flush=True)
