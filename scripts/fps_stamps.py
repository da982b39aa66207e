"""Per-segment cycles of one FPS step (diagnostic build pcseg/libpcseg_fps_stamps.so, built with
-DPCS_FPS_STAMPS: s_memtime stamps of wave 0 / block 0, summed over the steps of one launch)."""
import ctypes
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd')]
from pcseg.synthetic import make_batch  # noqa: E402

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd', 'pcseg')
lib = ctypes.CDLL(os.path.join(root, 'libpcseg_fps_stamps.so'))
vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
names = ['loop top', 'distances + local max', 'wave max', 'window/cand select', 'wave min + ballot',
         'slot write', 'barrier', 'block reduce + coords']
for B, N, C in [(32, 4096, 1024), (16, 24576, 1024)]:
    pts, _, _ = make_batch(B, N, seed=5)
    xyz = pts[:, :, :3].contiguous().cuda()
    start = torch.zeros(B, dtype=torch.int32, device='cuda')
    idx = torch.empty(B, C, dtype=torch.int32, device='cuda')
    cx = torch.empty(B, C, 3, device='cuda')
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        assert lib.pcs_fps(vp(xyz), B, N, C, vp(start), vp(idx), vp(cx), st) == 0
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 8)()
    assert lib.pcs_debug_fps_stamps(out) == 0
    tot = sum(out)
    print(f'B={B} N={N} C={C}: {tot / C:.0f} cycles/step')
    for k in range(8):
        print(f'  {names[k]:24s} {out[k] / C:8.1f} cycles/step')
