"""Time diagnostic builds of pcs_knn (pcseg/libpcseg_knn_*.so) at B=32, N=4096, k=20."""
import ctypes, glob, os, sys, time
import torch
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd', 'pcseg')
B, N, k = 32, 4096, 20
dev = 'cuda'
xs = {3: torch.rand(B, N, 3, device=dev), 64: torch.randn(B, N, 64, device=dev)}
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for path in [os.path.join(root, 'libpcseg.so')] + sorted(glob.glob(os.path.join(root, 'libpcseg_knn_*.so'))):
    lib = ctypes.CDLL(path)
    for F, x in xs.items():
        out = torch.empty((B, N, k), dtype=torch.int32, device=dev)
        def run():
            rc = lib.pcs_knn(ctypes.c_void_p(x.data_ptr()), B, N, F, k, ctypes.c_void_p(out.data_ptr()), st)
            assert rc == 0
        run(); run(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20): run()
        torch.cuda.synchronize()
        print(f'{os.path.basename(path):28s} F={F:2d}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms', flush=True)
        if 'COUNT' in path:
            o = out.view(-1, k).float()
            print(f'   merges/row {o[:, 0].mean():.2f}  survivors/row {(o[:, 1] + o[:, 2]).mean():.1f}  '
                  f'tiles with merges/wave {o[:, 3].mean():.1f}', flush=True)
