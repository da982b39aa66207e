"""FlopCounterMode fwd+bwd GFLOP per sample of the oracle's PointNet++ MSG (SURVEY.md 8(d) asks for
it: the reference ships no MSG, so the count is taken on the oracle composition that the parity
tests pin).  Same method as SURVEY.md's counts for the other families: one training step (forward,
masked one-hot CE, backward) under torch.utils.flop_counter.FlopCounterMode, divided by the batch."""
import os
import sys

import torch
from torch.utils.flop_counter import FlopCounterMode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd')]
from oracle import ref_ops as R          # noqa: E402
from pcseg.synthetic import make_batch   # noqa: E402

torch.set_num_threads(8)
for name, ctor in [('PointNetpp', lambda: R.PointNetpp(14)), ('PointNetppMSG', lambda: R.PointNetppMSG(14))]:
    B, N = 2, 4096
    model = R.seeded_init_(ctor(), 0).train()
    pts, labels, lengths = make_batch(B, N, seed=1)
    with FlopCounterMode(display=False) as fc:
        loss = R.masked_onehot_cross_entropy(model(pts), labels, lengths)
        loss.backward()
    print(f'{name}: {fc.get_total_flops() / B / 1e9:.3f} GFLOP/sample fwd+bwd (N={N})')
