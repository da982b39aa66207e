"""A/B pcs_fps of libpcseg.so vs pcseg/libpcseg_fps_*.so (indices must match; HIP-event timing)."""
import ctypes, glob, os, sys
import torch
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd')]
from pcseg.synthetic import make_batch
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd', 'pcseg')
libs = [os.path.join(root, 'libpcseg.so')] + sorted(glob.glob(os.path.join(root, 'libpcseg_fps_*.so')))
st = torch.cuda.current_stream()
vp = lambda t: ctypes.c_void_p(t.data_ptr())
for B, N, C in [(32, 4096, 1024), (32, 1024, 256), (16, 24576, 1024), (3, 4000, 999)]:
    pts, _, _ = make_batch(B, N, seed=5)
    xyz = pts[:, :, :3].contiguous().cuda()
    start = torch.randint(0, N, (B,), dtype=torch.int32, device='cuda')
    ref = None
    for path in libs:
        lib = ctypes.CDLL(path)
        idx = torch.empty(B, C, dtype=torch.int32, device='cuda'); cx = torch.empty(B, C, 3, device='cuda')
        run = lambda: lib.pcs_fps(vp(xyz), B, N, C, vp(start), vp(idx), vp(cx), ctypes.c_void_p(st.cuda_stream))
        assert run() == 0; torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): run()
        e1.record(); torch.cuda.synchronize()
        same = 'ref' if ref is None else ('SAME' if torch.equal(idx, ref) else 'DIFF')
        ref = idx.clone() if ref is None else ref
        print(f'B={B} N={N} C={C} {os.path.basename(path):24s} {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us {same}', flush=True)
