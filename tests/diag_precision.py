"""Print the three-way precision table (GPU fp32 / CPU fp32 / CPU fp64) per model."""
import sys
import os
sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)), os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '3d-semantic-segmentation-benchmark_amd')]
import torch
import pcseg
from oracle import ref_ops as R
from fp64_check import three_way, failures

cases = {
    'pointnetpp': (lambda: pcseg.PointNetpp(14), lambda: R.PointNetpp(14), 4, 4096, False),
    'pointnext': (lambda: pcseg.PointNeXt(14), lambda: R.PointNeXt(14), 2, 4096, False),
    'pointnet': (lambda: pcseg.PointNetSeg(part_classes=14), lambda: R.PointNetSeg(part_classes=14), 2, 1024, False),
    'dgcnn': (lambda: pcseg.DGCNNWithColor(14), lambda: R.DGCNNWithColor(14), 2, 1024, True),
}
for name in sys.argv[1:] or list(cases):
    p, r, B, N, ch = cases[name]
    rows = three_way(p, r, B, N, seed=11, chfirst=ch)
    worst = sorted(rows, key=lambda t: -(t[1] / max(t[3], 1e-30)))[:12]
    print(f'== {name}: {len(rows)} tensors; worst GPU rel-err vs fp64 (gpu_err, cpu32_err, norm):')
    for n, eg, ec, nn in worst:
        print(f'   {n:45s} gpu {eg/nn:9.2e}  cpu32 {ec/nn:9.2e}  ratio {eg/max(ec,1e-30):7.2f}')
    print('   failures(rtol=1e-3, factor=10):', len(failures(rows)))
    for f in failures(rows):
        print('   FAIL', f)
