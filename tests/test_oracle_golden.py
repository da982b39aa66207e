"""Pin the CPU oracle (oracle/ref_ops.py) against golden vectors captured from the reference.

The fixtures were produced by tests/golden/make_golden.py importing
/root/reference; these tests need neither the reference nor a GPU.
"""
import numpy as np
import pytest
import torch

from oracle import ref_ops as R


def T(a):
    return torch.from_numpy(np.array(a))


def test_fps_matches_reference(golden):
    z = golden('fps.npz')
    for sfx in ('', '_u', '_d'):
        coords = T(z['coords' + sfx])
        C = int(z['C' + sfx])
        idx = R.fps_indices(coords, C, T(z['starts' + sfx]))
        B = coords.shape[0]
        got = coords[torch.arange(B).view(B, 1), idx.long()]
        assert torch.equal(got, T(z['out' + sfx])), sfx


@pytest.mark.parametrize('case', ['sa1', 'sa2', 'sa3', 'sa4', 'irm1', 'irm4', 'uni', 'dup', 'big'])
def test_group_matches_reference(golden, case):
    z = golden('group.npz')
    B, N, C, K, norm = [int(v) for v in z[f'{case}/meta']]
    r = float(z[f'{case}/r'])
    coords, cent = T(z[f'{case}/coords']), T(z[f'{case}/cent'])
    feats = torch.arange(N, dtype=torch.float32).view(1, N, 1).expand(B, N, 1).contiguous()
    out = R.group(cent, coords, feats, r, K, bool(norm))
    ref = T(z[f'{case}/out'])
    # index sets are exact (gathered feature channel == point index)
    got_idx = out[..., 3].long().sort(-1).values
    ref_idx = ref[..., 3].long().sort(-1).values
    assert torch.equal(got_idx, ref_idx)
    assert torch.equal(out, ref)


@pytest.mark.parametrize('case', ['fp1', 'fp2', 'fp3', 'fp4'])
def test_interpolate_matches_reference(golden, case):
    z = golden('interp.npz')
    out = R.interpolate(T(z[f'{case}/f2']), T(z[f'{case}/c1']), T(z[f'{case}/c2']))
    assert torch.equal(out, T(z[f'{case}/out']))


def test_knn_and_graph_feature_match_reference(golden):
    z = golden('knn.npz')
    assert torch.equal(R.knn(T(z['x3']), 20).to(torch.int16), T(z['idx3']))
    assert torch.equal(R.knn(T(z['x64']), 20).to(torch.int16), T(z['idx64']))
    assert torch.equal(R.get_graph_feature(T(z['xs']), k=20), T(z['gf']))


def test_loss_matches_reference(golden):
    z = golden('loss.npz')
    logits, onehot, lengths = T(z['logits']), T(z['onehot']), T(z['lengths'])
    assert torch.equal(R.masked_onehot_cross_entropy(logits, onehot, lengths), T(z['loss']))
    assert float(R.masked_onehot_cross_entropy(logits, onehot, torch.zeros(3, dtype=torch.int64))) == 0.0
    lf = logits.clone().requires_grad_(True)
    R.masked_onehot_cross_entropy(lf, onehot.float(), lengths.to(torch.int32)).backward()
    assert torch.allclose(lf.grad, T(z['grad']), rtol=1e-6, atol=1e-9)


def _check_grads(model, z, rtol=2e-4):
    g = torch.Generator().manual_seed(7)
    # near-zero gradients (pre-BN conv biases, some BN betas) are rounding noise:
    # give every tensor an absolute floor of 1e-3 x the model's largest grad norm.
    gmax = max(float(z['g_l2/' + k]) for k, _ in model.named_parameters())
    for k, p in sorted(model.named_parameters()):
        gr = p.grad if p.grad is not None else torch.zeros_like(p)
        probe = torch.rand(gr.shape, generator=g) * 2 - 1
        flat = gr.reshape(-1).double()
        l2 = float(z['g_l2/' + k])
        scale = max(l2, 1e-3 * gmax)
        assert abs(float(flat.norm()) - l2) <= rtol * scale + 1e-9, k
        assert abs(float((flat * probe.reshape(-1).double()).sum()) - float(z['g_dot/' + k])) <= \
            rtol * scale * max(1.0, flat.numel() ** 0.5) + 1e-9, k


def _check_buffers(model, z):
    for k, v in model.state_dict().items():
        if 'running' in k:
            assert torch.allclose(v, T(z['buf/' + k]), rtol=1e-4, atol=1e-6), k


def _dropout_off(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()


@pytest.mark.parametrize('name,ctor,seed', [
    ('model_pointnetpp.npz', lambda: R.PointNetpp(14), 1234),
    ('model_pointnext.npz', lambda: R.PointNeXt(14), 4321),
])
def test_pointnet2_family_matches_reference(golden, name, ctor, seed):
    z = golden(name)
    m = R.seeded_init_(ctor(), seed)
    m.train()
    _dropout_off(m)
    starts = [T(z[k]) for k in sorted((k for k in z.files if k.startswith('fps_start')),
                                      key=lambda s: int(s[len('fps_start'):]))]
    with R.replay(R.Replay(fps_starts=starts)):
        logits = m(T(z['x']))
    assert torch.allclose(logits, T(z['logits']), rtol=1e-4, atol=1e-5)
    loss = R.masked_onehot_cross_entropy(logits, T(z['labels']), T(z['lengths']))
    assert abs(float(loss) - float(z['loss'])) < 1e-5
    loss.backward()
    _check_grads(m, z)
    _check_buffers(m, z)


def test_dgcnn_color_matches_reference(golden):
    z = golden('model_dgcnn_color.npz')
    m = R.seeded_init_(R.DGCNNWithColor(num_classes=14, k=20), 999)
    m.train()
    _dropout_off(m)
    x = T(z['x']).transpose(1, 2).contiguous().transpose(1, 2)  # non-contiguous (B,6,N) view
    knn = [T(z[f'knn{i}']).long() for i in range(4)]
    with R.replay(R.Replay(knn_idx=knn)):
        logits, x5, _ = m(x)
    assert torch.allclose(logits, T(z['logits']), rtol=1e-4, atol=1e-5)
    loss = R.masked_onehot_cross_entropy(logits, T(z['labels']).float(), T(z['lengths']).to(torch.int32))
    assert abs(float(loss) - float(z['loss'])) < 1e-5
    loss.backward()
    _check_grads(m, z)
    _check_buffers(m, z)


def test_dgcnn_rejects_wrong_channels():
    with pytest.raises(ValueError):
        R.DGCNNWithColor(num_classes=14)(torch.zeros(2, 9, 64))


def test_pointnet_matches_reference(golden):
    z = golden('model_pointnet.npz')
    m = R.seeded_init_(R.PointNetSeg(part_classes=14), 77)
    m.train()
    probs = m(T(z['x']))
    assert torch.allclose(probs, T(z['probs']), rtol=1e-4, atol=1e-6)
    loss = R.masked_onehot_cross_entropy(probs, T(z['labels']), T(z['lengths']))
    loss.backward()
    _check_grads(m, z)


def test_metrics_match_reference(golden):
    """Training/metrics.py restated (oracle) vs the reference's own outputs: argmax ties,
    padded / empty samples, an all-zero and a two-hot label row."""
    z = golden('metrics.npz')
    p, lab, n = T(z['probs']), T(z['labels']), T(z['lengths'])
    assert R.overall_accuracy(p, lab, n) == float(z['oa'])
    assert R.update_accuracy(p, lab, n) == (int(z['correct']), int(z['total']))
    assert torch.equal(R.confusion_matrix(p, lab, n), T(z['conf']))
    miou, ious = R.intersection_over_union(p, lab, n)
    assert miou == float(z['miou']) and torch.equal(ious, T(z['ious']))
    inter, union = R.update_intersection_over_union(p, lab, n)
    assert torch.equal(inter, T(z['inter'])) and torch.equal(union, T(z['union']))


def _preprocess_inputs(z):
    ns = [int(n) for n in z['ns']]
    x = [T(z[f'x{i}']) for i in range(len(ns))]
    flat = [str(v) for v in z['labels']]
    y, o = [], 0
    for n in ns:
        y.append(flat[o:o + n])
        o += n
    return x, y, [str(m) for m in z['mapping']]


PREPROCESS_CASES = [('plain', {}), ('cut', {'cut': 50}), ('samp', {'sampling': 0.5}),
                    ('both', {'cut': 40, 'sampling': 0.7})]


@pytest.mark.parametrize('tag,kw', PREPROCESS_CASES)
def test_preprocess_matches_reference(golden, tag, kw):
    z = golden('preprocess.npz')
    x, y, mapping = _preprocess_inputs(z)
    torch.manual_seed(int(z[f'{tag}_seed']))
    bi, lab, lengths, cont = R.preprocess_batch_to_train_format(x, y, mapping, **kw)
    assert torch.equal(bi.contiguous(), T(z[f'{tag}_x'])) and bi.shape[1] == x[0].shape[1]
    assert torch.equal(lab, T(z[f'{tag}_label']))
    assert torch.equal(lengths, T(z[f'{tag}_len'])) and lengths.dtype == torch.int32
    assert cont == bool(z[f'{tag}_cont'])


# ---------------------------------------------------------------- configs' real sizes
@pytest.mark.parametrize('name,ctor,seed', [
    ('model_pointnext_24576.npz', lambda: R.PointNeXt(14), 4322),          # BASELINE config 5 block size
])
def test_pointnext_24576_matches_reference(golden, name, ctor, seed):
    test_pointnet2_family_matches_reference(golden, name, ctor, seed)


def test_dgcnn_color_4096_matches_reference(golden):
    """BASELINE config 2's block size (N = 4096, k = 20), with the reference's kNN graphs."""
    z = golden('model_dgcnn_color_4096.npz')
    m = R.seeded_init_(R.DGCNNWithColor(num_classes=14, k=20), 999)
    m.train()
    _dropout_off(m)
    x = T(z['x']).transpose(1, 2).contiguous().transpose(1, 2)
    # the first graph (xyz) is recomputed, not replayed: the oracle's kNN must reproduce it
    assert torch.equal(R.knn(x[:, :3], 20).to(torch.int16), T(z['knn0']))
    with R.replay(R.Replay(knn_idx=[T(z[f'knn{i}']).long() for i in range(4)])):
        logits, x5, _ = m(x)
    assert torch.allclose(logits, T(z['logits']), rtol=1e-4, atol=1e-5)
    loss = R.masked_onehot_cross_entropy(logits, T(z['labels']).float(), T(z['lengths']).to(torch.int32))
    assert abs(float(loss) - float(z['loss'])) < 1e-5
    loss.backward()
    _check_grads(m, z)
    _check_buffers(m, z)


def test_pointnet_4096_matches_reference(golden):
    z = golden('model_pointnet_4096.npz')
    m = R.seeded_init_(R.PointNetSeg(part_classes=14), 78)
    m.train()
    probs = m(T(z['x']))
    assert torch.allclose(probs, T(z['probs']), rtol=1e-4, atol=1e-6)
    loss = R.masked_onehot_cross_entropy(probs, T(z['labels']), T(z['lengths']))
    loss.backward()
    _check_grads(m, z)
    _check_buffers(m, z)


# ---------------------------------------------------------------- section 8(f) row 4: sliding windows
@pytest.mark.parametrize('tag', ['a', 'b', 'c', 'd'])
def test_predict_single_scene_windows_match_reference(golden, tag):
    from scene_models import PerPointLinear
    z = golden('scene.npz')
    n, bs, ov = (int(v) for v in z[f'{tag}/meta'])
    lin = PerPointLinear(6, 13, seed=n)
    assert torch.equal(lin.weight.data, T(z[f'{tag}/lin_w']))
    p, c = R.predict_single_scene(lin, T(z[f'{tag}/scene']), batch_size=bs, overlap=ov)
    assert torch.equal(p, T(z[f'{tag}/lin_pred'])) and torch.equal(c, T(z[f'{tag}/lin_conf']))


def scene_dgcnn(z, cls=None):
    """The eval-mode DGCNNWithColor of golden_scene (seeded weights, randomised running stats)."""
    seed = int(z['dgcnn/init_seed'])
    m = R.seeded_init_((cls or R.DGCNNWithColor)(num_classes=13, k=20), seed)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            mod.running_mean.copy_(torch.randn(mod.running_mean.shape, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) + 0.5)
    return m


def test_predict_single_scene_dgcnn_matches_reference(golden):
    z = golden('scene.npz')
    m = scene_dgcnn(z)
    knn = [T(z[f'dgcnn/knn{i}']).long() for i in range(sum(k.startswith('dgcnn/knn') for k in z.files))]
    with R.replay(R.Replay(knn_idx=knn)):
        p, c = R.predict_single_scene(m, T(z['a/scene']), batch_size=1024, overlap=128)
    assert torch.equal(p, T(z['dgcnn/pred']))
    assert torch.allclose(c, T(z['dgcnn/conf']), rtol=1e-5, atol=1e-7)
