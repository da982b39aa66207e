"""pcseg.inference.predict_single_scene (batched windows + pcs_window_merge) against the
reference's sliding-window inference (models/dgcnn/utils.py:67-131, restated in the
oracle) on the same eval-mode DGCNN weights.  The oracle's per-window kNN graphs are
replayed into the batched forward (DGCNN's kNN is not index-reproducible across fp32
evaluation orders); predictions must agree on >= 99.9 % of points (fp32 near-ties of the
averaged logits may flip) and confidences within 1e-3 relative."""
import pytest
import torch

import pcseg
from pcseg.inference import predict_single_scene, _windows
from pcseg.synthetic import make_batch
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _models(seed):
    ref = R.seeded_init_(R.DGCNNWithColor(num_classes=13, k=20), seed)
    # non-trivial running statistics for eval-mode BatchNorm
    g = torch.Generator().manual_seed(seed + 1)
    for m in ref.modules():
        if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) + 0.5)
    prod = pcseg.DGCNNWithColor(num_classes=13, k=20)
    prod.load_state_dict(ref.state_dict())
    return ref.eval(), prod.to(DEV).eval()


@pytest.mark.parametrize('n,bs,ov', [(2500, 1024, 128), (700, 1024, 128), (3000, 512, 64)])
def test_sliding_window_matches_reference(n, bs, ov):
    pts, _, _ = make_batch(1, n, seed=n)
    scene = pts[0, :, :6].contiguous()
    ref, prod = _models(n + bs)
    rr = R.Replay()
    with R.replay(rr):
        p0, c0 = R.predict_single_scene(ref, scene, batch_size=bs, overlap=ov)
    # the oracle recorded 4 graphs per window; the product batches equal-size windows
    if n <= bs:
        sizes = [n]
    else:
        _, sizes = _windows(n, bs, bs - ov)
    per_win = [rr.rec_knn_idx[4 * w:4 * w + 4] for w in range(len(sizes))]
    replay, w = [], 0
    while w < len(sizes):
        e = w + 1
        while e < len(sizes) and sizes[e] == sizes[w] and e - w < 16:
            e += 1
        for layer in range(4):
            replay.append(torch.cat([per_win[v][layer] for v in range(w, e)]))
        w = e
    with pcseg.replay(pcseg.Replay(knn_idx=replay)):
        p1, c1 = predict_single_scene(prod, scene, device=DEV, batch_size=bs, overlap=ov)
    assert p1.dtype == torch.int64 and c1.dtype == torch.float32 and p1.shape == (n,)
    assert (p1 == p0).float().mean() >= 0.999
    assert torch.allclose(c1, c0, rtol=1e-3, atol=1e-6)
