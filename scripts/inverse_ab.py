"""Inverse-map microbenchmark: ops.inverse_index alone on the bench's map shapes (PointNet++ B=32
ball-query and interpolation maps, DGCNN B=32 kNN maps), HIP-event timing, plus a checksum so
variants (env A/B switches, separate processes) can be compared for identical output."""
import os, sys
import torch
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd')]
from pcseg import ops

tag = sys.argv[1] if len(sys.argv) > 1 else ''
g = torch.Generator(device='cuda').manual_seed(3)
# (name, B, S, k, targets): PointNet++ SA1..SA4 ball maps, FP interp maps; DGCNN kNN maps
shapes = [('pnpp_sa1', 32, 1024, 32, 4096), ('pnpp_sa2', 32, 256, 32, 1024), ('pnpp_sa3', 32, 64, 32, 256),
          ('pnpp_sa4', 32, 16, 32, 64), ('pnpp_fp1', 32, 4096, 3, 1024), ('pnpp_fp2', 32, 1024, 3, 256),
          ('dgcnn_knn', 32, 4096, 20, 4096)]
tot = 0.0
for name, B, S, k, T in shapes:
    idx = torch.randint(0, T, (B, S, k), generator=g, device='cuda', dtype=torch.int32)
    for _ in range(3):
        off, ent = ops.inverse_index(idx, T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        off, ent = ops.inverse_index(idx, T)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    tot += us
    ck = int((ent.long() * torch.arange(1, ent.numel() + 1, device='cuda') % 1000003).sum()) + int(off.long().sum())
    print(f'{tag:8s} {name:10s} B={B} S={S} k={k} T={T}: {us:8.1f} us  checksum {ck}', flush=True)
print(f'{tag:8s} total {tot:.1f} us', flush=True)
# batched, as the models call it: PointNet++'s 8 geometry-plan maps (SA1-4 ball, FP1-3 + FP4 3-NN)
# in one call, DGCNN's 4 kNN maps in one call
batches = {'pnpp_plan8': [(32, 1024, 32, 4096), (32, 256, 32, 1024), (32, 64, 32, 256), (32, 16, 32, 64),
                          (32, 4096, 3, 1024), (32, 1024, 3, 256), (32, 256, 3, 64), (32, 64, 3, 16)],
           'dgcnn_knn4': [(32, 4096, 20, 4096)] * 4}
for name, shp in batches.items():
    tabs = [(torch.randint(0, T, (B, S, k), generator=g, device='cuda', dtype=torch.int32), T) for B, S, k, T in shp]
    for _ in range(3):
        res = ops.inverse_index_batch(tabs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        res = ops.inverse_index_batch(tabs)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    ck = sum(int((e.long() * torch.arange(1, e.numel() + 1, device='cuda') % 1000003).sum()) + int(o.long().sum())
             for o, e in res)
    print(f'{tag:8s} {name:10s} batched: {us:8.1f} us  checksum {ck}', flush=True)
