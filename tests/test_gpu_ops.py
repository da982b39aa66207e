"""GPU parity of every HIP primitive against the CPU oracle (oracle/ref_ops.py),
through the C ABI.  Index work must be bit-exact; float outputs exact where the
kernel replays the reference's arithmetic order, else within the stated tolerance.
"""
import numpy as np
import pytest
import torch

import pcseg
from pcseg import ops
from pcseg.synthetic import make_batch
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def T(a):
    return torch.from_numpy(np.array(a))


def cloud(B, N, seed, kind='surface'):
    if kind == 'dup':
        pts, _, _ = make_batch(B, max(8, N // 3), seed)
        g = torch.Generator().manual_seed(seed)
        return pts[:, torch.randint(0, pts.shape[1], (N,), generator=g), :3].contiguous()
    pts, _, _ = make_batch(B, N, seed, uniform=(kind == 'uniform'))
    return pts[:, :, :3].contiguous()


def sorted_rows(idx):
    return idx.long().sort(-1).values


# ----------------------------------------------------------------------------- FPS
@pytest.mark.parametrize('B,N,C,kind', [(2, 4096, 1024, 'surface'), (3, 1024, 256, 'surface'), (2, 256, 64, 'uniform'),
                                        (2, 64, 16, 'surface'), (2, 1000, 333, 'dup'), (1, 24576, 1024, 'surface'),
                                        (2, 5000, 1200, 'uniform'), (1, 37, 37, 'dup'), (4, 2048, 512, 'dup'),
                                        (2, 12000, 700, 'dup'), (1, 9000, 2000, 'uniform'), (1, 30000, 1024, 'surface')])
def test_fps_bit_exact(B, N, C, kind):
    xyz = cloud(B, N, seed=N + C, kind=kind)
    start = torch.randint(0, N, (B,), dtype=torch.int32, generator=torch.Generator().manual_seed(N))
    ref = R.fps_indices(xyz, C, start)
    idx, cent = ops.fps(xyz.to(DEV), C, start.to(DEV))
    assert torch.equal(idx.cpu(), ref)
    assert torch.equal(cent.cpu(), xyz[torch.arange(B).view(B, 1), ref.long()])


def test_fps_golden(golden):
    z = golden('fps.npz')
    for sfx in ('', '_u', '_d'):
        xyz = T(z['coords' + sfx])
        _, cent = ops.fps(xyz.to(DEV), int(z['C' + sfx]), T(z['starts' + sfx]).to(DEV))
        assert torch.equal(cent.cpu(), T(z['out' + sfx])), sfx


# ----------------------------------------------------------------------------- ball query
@pytest.mark.parametrize('case', ['sa1', 'sa2', 'sa3', 'sa4', 'irm1', 'irm4', 'uni', 'dup', 'big'])
def test_ball_query_golden(golden, case):
    z = golden('group.npz')
    B, N, C, K, norm = [int(v) for v in z[f'{case}/meta']]
    r = float(z[f'{case}/r'])
    coords, cent = T(z[f'{case}/coords']), T(z[f'{case}/cent'])
    idx = ops.ball_query(cent.to(DEV), coords.to(DEV), r, K)
    ref_idx = T(z[f'{case}/out'])[..., 3].long()
    assert torch.equal(sorted_rows(idx.cpu()), ref_idx.sort(-1).values)


@pytest.mark.parametrize('B,N,C,r,K,kind', [
    (4, 4096, 1024, 0.1, 32, 'surface'), (4, 1024, 256, 0.2, 32, 'surface'), (4, 256, 64, 0.4, 32, 'surface'),
    (4, 64, 16, 0.8, 32, 'surface'), (2, 1024, 1024, 0.1, 32, 'surface'), (2, 4096, 512, 0.1, 32, 'uniform'),
    (2, 2047, 300, 0.3, 32, 'dup'), (2, 2048, 300, 0.3, 32, 'dup'), (2, 16, 16, 0.8, 16, 'surface'),
    (2, 3000, 100, 0.05, 16, 'surface'), (1, 24576, 1024, 0.1, 32, 'surface'), (2, 100, 50, 2.0, 32, 'uniform'),
    (2, 8192, 512, 0.1, 32, 'surface'), (2, 4096, 256, 0.8, 32, 'surface'), (1, 24576, 512, 0.1, 32, 'dup'),
    (2, 12000, 700, 0.8, 32, 'surface'), (2, 9000, 400, 0.1, 16, 'uniform'),
    (2, 6000, 300, 0.1, 64, 'uniform')])
def test_ball_query_matches_oracle(B, N, C, r, K, kind):
    """Index sets equal to the reference's (topk over the radius-masked distances).  N > 8192 with
    k * 64 <= N runs the cell-grid heap path (grid_heap_select_kernel): underfull (uniform) and
    duplicate-heavy clouds, r = 0.8 (few cells), k = 16 and 32; smaller clouds the staged exhaustive
    heap kernel."""
    xyz = cloud(B, N, seed=7 * N + C, kind=kind)
    start = torch.zeros(B, dtype=torch.int32)
    cent = xyz[torch.arange(B).view(B, 1), R.fps_indices(xyz, C, start).long()]
    ref = R.ball_query(cent, xyz, r, K)
    got = ops.ball_query(cent.to(DEV), xyz.to(DEV), r, K).cpu()
    assert torch.equal(sorted_rows(got), sorted_rows(ref))


@pytest.mark.parametrize('N,r,K', [(12000, 0.2, 32), (24576, 0.1, 32), (9000, 0.05, 32)])
def test_ball_query_arbitrary_centroids(N, r, K):
    """Centroids that are not cloud points, some outside the cloud's box (clamped to its edge
    cells), some on cell boundaries: the grid path's candidate cells still hold every in-radius point."""
    B, C = 2, 300
    xyz = cloud(B, N, seed=N + 3)
    g = torch.Generator().manual_seed(N)
    cent = torch.rand(B, C, 3, generator=g) * torch.tensor([1.4, 1.4, 3.4]) - 0.2
    cent[:, :40] = xyz[:, :40] + r * (torch.rand(B, 40, 3, generator=g) - 0.5)
    cent[:, 40:60] = torch.round(cent[:, 40:60] / r) * r
    ref = R.ball_query(cent, xyz, r, K)
    got = ops.ball_query(cent.to(DEV), xyz.to(DEV), r, K).cpu()
    assert torch.equal(sorted_rows(got), sorted_rows(ref))


# ----------------------------------------------------------------------------- 3-NN
@pytest.mark.parametrize('case', ['fp1', 'fp2', 'fp3', 'fp4'])
def test_interpolate_golden_bit_exact(golden, case):
    z = golden('interp.npz')
    out = pcseg.interpolate(T(z[f'{case}/f2']).to(DEV), T(z[f'{case}/c1']).to(DEV), T(z[f'{case}/c2']).to(DEV))
    assert torch.equal(out.cpu(), T(z[f'{case}/out']))


@pytest.mark.parametrize('B,N,M,kind', [(4, 4096, 1024, 'surface'), (4, 1024, 256, 'surface'),
                                        (4, 256, 64, 'surface'), (4, 64, 16, 'surface'), (2, 24576, 1024, 'surface'),
                                        (2, 2000, 191, 'dup'), (2, 2000, 192, 'dup'), (2, 500, 3, 'uniform')])
def test_three_nn_matches_oracle(B, N, M, kind):
    c1 = cloud(B, N, seed=N + M, kind=kind)
    c2 = c1[torch.arange(B).view(B, 1), R.fps_indices(c1, M, torch.zeros(B, dtype=torch.int32)).long()]
    dref, iref = R.three_nn(c1, c2)
    idx, dist = ops.knn_select(c1.to(DEV), c2.to(DEV), 3)
    assert torch.equal(sorted_rows(idx.cpu()), sorted_rows(iref))
    assert torch.equal(dist.cpu().sort(-1).values, dref.sort(-1).values)


# ----------------------------------------------------------------------------- gathers
@pytest.mark.parametrize('normalize', [False, True])
def test_group_fwd_bwd(normalize):
    B, N, C, K, D, r = 3, 1024, 256, 32, 19, 0.2
    xyz = cloud(B, N, seed=5)
    g = torch.Generator().manual_seed(6)
    feats = torch.randn(B, N, D, generator=g)
    cent = xyz[:, :C].contiguous()
    ri = R.ball_query(cent, xyz, r, K)
    gi = ops.ball_query(cent.to(DEV), xyz.to(DEV), r, K).cpu().long()
    assert torch.equal(gi.sort(-1).values, ri.sort(-1).values)
    ref_in = feats.clone().requires_grad_(True)
    ref = R.group(cent, xyz, ref_in, r, K, normalize)
    fd = feats.to(DEV).requires_grad_(True)
    got = pcseg.group(cent.to(DEV), xyz.to(DEV), fd, r, K, normalize)
    # same neighbour set; canonical order may differ among ties -> align by index
    ps, pr = gi.argsort(-1), ri.argsort(-1)
    gs = got.detach().cpu().gather(2, ps.unsqueeze(-1).expand(B, C, K, 3 + D))
    rs = ref.detach().gather(2, pr.unsqueeze(-1).expand(B, C, K, 3 + D))
    assert torch.equal(gs, rs)

    def weights(idx):   # order-independent loss weights: a function of (b, c, point, channel)
        b = torch.arange(B).view(B, 1, 1, 1).double()
        c = torch.arange(C).view(1, C, 1, 1).double()
        ch = torch.arange(3 + D).view(1, 1, 1, 3 + D).double()
        return torch.sin(0.37 * idx.unsqueeze(-1).double() + 1.3 * ch + 0.11 * c + 2.9 * b).float()
    (ref * weights(ri)).sum().backward()
    (got * weights(gi).to(DEV)).sum().backward()
    assert torch.allclose(fd.grad.cpu(), ref_in.grad, rtol=1e-5, atol=1e-5)


def test_maxk_fwd_bwd():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 32, 48, generator=g)
    x[:, 5] = x[:, 2]                       # exact ties -> first index
    x = torch.relu(x)                        # many zero ties
    xr = x.clone().requires_grad_(True)
    ref = torch.max(xr, dim=1)[0]
    xd = x.to(DEV).reshape(64 * 32, 48).requires_grad_(True)
    got = ops.maxk(xd, 32)
    assert torch.equal(got.detach().cpu(), ref.detach())
    w = torch.randn(ref.shape, generator=g)
    (ref * w).sum().backward()
    (got * w.to(DEV)).sum().backward()
    assert torch.equal(xd.grad.cpu().view(64, 32, 48), xr.grad)


def test_interp_cat_fwd_bwd():
    B, N, M, D1, D2 = 2, 1024, 256, 7, 13
    c1 = cloud(B, N, seed=9)
    c2 = c1[:, :M]
    g = torch.Generator().manual_seed(9)
    f1, f2 = torch.randn(B, N, D1, generator=g), torch.randn(B, M, D2, generator=g)
    r1, r2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    ref = torch.cat([r1, R.interpolate(r2, c1, c2)], dim=-1)
    d1, d2 = f1.to(DEV).requires_grad_(True), f2.to(DEV).requires_grad_(True)
    idx, dist = ops.knn_select(c1.to(DEV), c2.to(DEV), 3)
    got = ops.interp_cat_rows(d1, d2, idx, dist).view(B, N, D1 + D2)
    assert torch.allclose(got.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-6)
    w = torch.randn(ref.shape, generator=g)
    (ref * w).sum().backward()
    (got * w.to(DEV)).sum().backward()
    assert torch.allclose(d1.grad.cpu(), r1.grad)
    assert torch.allclose(d2.grad.cpu(), r2.grad, rtol=1e-5, atol=1e-5)


def test_edge_fwd_bwd():
    B, N, D, k = 2, 512, 8, 20
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, D, N, generator=g)
    idx = R.knn(x, k)
    xr = x.clone().requires_grad_(True)
    ref = R.get_graph_feature(xr, k=k, idx=idx)            # (B, 2D, N, k)
    xd = x.transpose(1, 2).contiguous().to(DEV).requires_grad_(True)
    got = ops.edge_rows(xd, idx.to(torch.int32).to(DEV)).view(B, N, k, 2 * D).permute(0, 3, 1, 2)
    assert torch.equal(got.detach().cpu(), ref.detach())
    w = torch.randn(ref.shape, generator=g)
    (ref * w).sum().backward()
    (got * w.to(DEV)).sum().backward()
    assert torch.allclose(xd.grad.cpu().transpose(1, 2), xr.grad, rtol=1e-5, atol=1e-5)
    # fp64 truth of the same terms: each point's sum is accumulated in fp64 and rounded once
    w64 = w.double()
    ga, gb = w64[:, :D], w64[:, D:]                                  # (B, D, N, k)
    truth = (gb - ga).sum(-1)
    truth.scatter_add_(2, idx.reshape(B, 1, N * k).expand(-1, D, -1), ga.reshape(B, D, N * k))
    assert torch.equal(xd.grad.cpu().transpose(1, 2), truth.float())
    g1 = xd.grad.clone()
    xd.grad = None
    again = ops.edge_rows(xd, idx.to(torch.int32).to(DEV)).view(B, N, k, 2 * D).permute(0, 3, 1, 2)
    (again * w.to(DEV)).sum().backward()
    assert torch.equal(g1, xd.grad)


# ----------------------------------------------------------------------------- DGCNN kNN
@pytest.mark.parametrize('F_,seed,N', [(3, 1, 2048), (64, 2, 2048), (3, 3, 4096), (64, 4, 4096)])
def test_dgcnn_knn_agrees_with_oracle(F_, seed, N):
    """N = 4096 is BASELINE config 2's block: 4096 x 4096 distance tiles per cloud."""
    B, k = 2, 20
    if F_ == 3:
        x = cloud(B, N, seed).transpose(1, 2).contiguous()
    else:
        x = torch.randn(B, F_, N, generator=torch.Generator().manual_seed(seed))
    ref = R.knn(x, k)
    got = ops.knn(x.transpose(1, 2).contiguous().to(DEV), k).cpu().long()
    same = (got.sort(-1).values == ref.sort(-1).values).all(-1)
    assert same.float().mean() > 0.99
    # rows that differ may only swap near-ties: compare the k-th best distance
    xp = x.transpose(1, 2)
    d = torch.cdist(xp.double(), xp.double()) ** 2
    kth_ref = d.gather(2, ref).max(-1).values
    kth_got = d.gather(2, got).max(-1).values
    assert torch.allclose(kth_got, kth_ref, rtol=1e-4, atol=1e-5)
    assert (got[..., 0] == torch.arange(N)).float().mean() > 0.99   # self first


@pytest.mark.parametrize('F_,lo,hi,N', [(3, 0, 8, 2048), (64, -2, 3, 2048), (64, 0, 2, 1000), (3, 0, 4, 333),
                                        (3, 0, 16, 4096), (64, -1, 2, 4096)])
def test_dgcnn_knn_selection_exact_on_integer_grids(F_, lo, hi, N):
    """Integer features make every pd exact in fp32 (MFMA included), so the k best are
    fully determined: larger pd first, exact ties to the lower index.  Coarse grids put
    many exact ties on the k-th value (the running radix select's tie path, the final
    rank merge) and ragged N exercises the partial last tile."""
    B, k = 2, 20
    g = torch.Generator().manual_seed(F_ * 7 + N)
    x = torch.randint(lo, hi, (B, N, F_), generator=g).float()
    xd = x.double()
    d = torch.cdist(xd, xd) ** 2
    exp = torch.sort(d.round(), dim=-1, stable=True).indices[..., :k]
    got = ops.knn(x.contiguous().to(DEV), k).cpu().long()
    assert torch.equal(got, exp)
    # the pruned scan (Morton order of the first three features) through the same ties
    xd_ = x.contiguous().to(DEV)
    got_p = ops.knn(xd_, k, order=ops.knn_order(xd_)).cpu().long()
    assert torch.equal(got_p, exp)


@pytest.mark.parametrize('F_', [3, 64])
def test_dgcnn_knn_workspace_path_bitwise_equal(F_):
    """pcs_knn_ws (squared norms precomputed once per point, the path ops.knn takes) gives
    bitwise the same lists as pcs_knn (norms recomputed per streaming wave), B=4, N=4096."""
    from pcseg._lib import call, ptr, stream_ptr
    torch.manual_seed(F_)
    x = (torch.randn(4, 4096, F_) if F_ == 64 else make_batch(4, 4096, seed=9)[0][:, :, :3].contiguous()).to(DEV)
    a = torch.empty((4, 4096, 20), dtype=torch.int32, device=DEV)
    call('pcs_knn', ptr(x), 4, 4096, F_, 20, ptr(a), stream_ptr(x.device))
    b = ops.knn(x, 20)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize('k', [16, 20, 32])
def test_dgcnn_knn_seeded_bitwise_equal(k):
    """pcs_knn_seeded (rows start from the threshold of a previous neighbour list) gives
    bitwise the same lists as the unseeded search, whatever the seeds: the previous graph of a
    perturbed cloud (the DGCNN case), random seeds, seeds with repeats / out-of-range entries
    (those rows search unseeded), too few seeds, and exact ties on integer features."""
    g = torch.Generator().manual_seed(k)
    B, N = 2, 4096
    x = torch.randn(B, N, 64, generator=g).to(DEV)
    base = ops.knn(x, k)
    near = ops.knn((x + 0.3 * torch.randn(B, N, 64, generator=g).to(DEV)).contiguous(), k)
    rnd = torch.randint(0, N, (B, N, k), generator=g, dtype=torch.int32).to(DEV)
    bad = near.clone()
    bad[:, ::3, 1] = bad[:, ::3, 0]            # repeats
    bad[:, 1::3, 2] = N + 5                    # out of range
    bad[:, 2::7, 3] = -1
    for seeds in (near, rnd, bad, near[:, :, :k - 1].contiguous(), base):
        assert torch.equal(ops.knn(x, k, seeds=seeds), base)
    xi = torch.randint(-2, 3, (B, N, 64), generator=g).float().to(DEV)
    bi = ops.knn(xi, k)
    assert torch.equal(ops.knn(xi, k, seeds=ops.knn((xi + 0.5).contiguous(), k)), bi)
    assert torch.equal(ops.knn(xi, k, seeds=bi), bi)


def _knn_order_cases():
    # (name, x (B, N, F) on DEV, xyz the order is built from)
    g = torch.Generator().manual_seed(77)
    out = []
    for N in (4096, 2051, 333, 31, 8192):
        xyz = make_batch(2, N, seed=N)[0][:, :, :3].contiguous().to(DEV)
        out.append((f'xyz{N}', xyz, xyz))
    xyz = make_batch(2, 4096, seed=5)[0][:, :, :3].contiguous()
    W1, W2 = torch.randn(3, 32, generator=g), torch.randn(32, 64, generator=g)
    smooth = (torch.tanh(xyz @ W1 * 4.0) @ W2).contiguous()            # features of the geometry
    out.append(('smooth64', smooth.to(DEV), xyz.to(DEV)))
    out.append(('random64', torch.randn(2, 4096, 64, generator=g).to(DEV), xyz.to(DEV)))   # no locality
    dup = smooth.clone()
    dup[:, 1000:1600] = dup[:, 1000:1001]                                # 600 identical points
    out.append(('dup64', dup.contiguous().to(DEV), xyz.to(DEV)))
    grid = torch.randint(0, 3, (2, 4096, 64), generator=g).float()
    out.append(('grid64', grid.to(DEV), grid[:, :, :3].contiguous().to(DEV)))
    far = xyz.clone()
    far[:, :7] += 1e4                                                    # outliers: huge bounds / norms
    out.append(('outliers3', far.contiguous().to(DEV), far.contiguous().to(DEV)))
    return out


@pytest.mark.parametrize('k', [16, 20, 32])
def test_dgcnn_knn_pruned_bitwise_equal(k):
    """pcs_knn_pruned (candidate tiles scanned in a per-cloud Morton order, the provably farther
    ones skipped) gives bitwise the same lists as the full scan: clouds of 4096 / ragged / tiny /
    8192 points (the LDS sort's limit), 64-wide features that follow the geometry, random
    features (nothing to prune), 600 identical points, integer features (exact ties on the k-th
    value), far outliers; with and without seeds; k = 32 takes the unpruned kernel."""
    for name, x, xyz in _knn_order_cases():
        if x.shape[1] < k:
            continue
        od = ops.knn_order(xyz)
        base = ops.knn(x, k)
        got = ops.knn(x, k, order=od)
        assert torch.equal(got, base), name
        if x.shape[2] == 64:
            near = ops.knn((x + 0.1 * torch.randn_like(x)).contiguous(), k)
            assert torch.equal(ops.knn(x, k, seeds=near, order=od), base), name


def test_dgcnn_knn_order_is_a_permutation():
    """pcs_knn_order: per cloud a permutation of 0..N-1 (ragged and tiny clouds), consecutive
    points close in space (Morton locality); past 8192 points the identity; any permutation is
    a valid scan order (a random one gives the same lists)."""
    for N in (4096, 333, 5, 8192):
        xyz = make_batch(3, N, seed=N + 1)[0][:, :, :3].contiguous().to(DEV)
        od = ops.knn_order(xyz).long().cpu()
        assert torch.equal(od.sort(-1).values, torch.arange(N).expand(3, N))
        if N >= 4096:
            p = xyz.cpu().gather(1, od[..., None].expand(-1, -1, 3))
            step = (p[:, 1:] - p[:, :-1]).norm(dim=-1).median()
            rnd = (xyz.cpu()[:, 1:] - xyz.cpu()[:, :-1]).norm(dim=-1).median()
            assert step < 0.25 * rnd, (float(step), float(rnd))
    xyz = make_batch(2, 9000, seed=3)[0][:, :, :3].contiguous().to(DEV)
    assert torch.equal(ops.knn_order(xyz).long().cpu(), torch.arange(9000).expand(2, 9000))
    x = make_batch(2, 4096, seed=8)[0][:, :, :3].contiguous().to(DEV)
    perm = torch.stack([torch.randperm(4096) for _ in range(2)]).to(torch.int32).to(DEV)
    assert torch.equal(ops.knn(x, 20, order=perm), ops.knn(x, 20))


def test_dgcnn_knn_pruned_kernel_runs_in_model():
    """DGCNN's forward builds one Morton order; graphs 1-3 take the pruned kernel, graph 4 the
    seeded full scan (models.py, the note above DGCNN)."""
    from pcseg import _lib
    torch.manual_seed(0)
    m = pcseg.DGCNNWithColor(14).to(DEV).train()
    x = make_batch(2, 4096, seed=31)[0][:, :, :6].contiguous().transpose(1, 2).to(DEV)
    names = []
    orig = _lib.call

    def spy(name, *a):
        names.append(name)
        return orig(name, *a)
    pcseg.ops.call = spy
    try:
        with torch.no_grad():
            m(x)
    finally:
        pcseg.ops.call = orig
    assert names.count('pcs_knn_order') == 1 and names.count('pcs_knn_pruned') == 3, names
    assert names.count('pcs_knn_seeded') == 1, names


def test_dgcnn_model_seeded_graphs_equal_unseeded():
    """DGCNNWithColor's graphs 2-4 (seeded by the previous graph) equal the unseeded search on
    the same features (B=2, N=4096)."""
    torch.manual_seed(0)
    m = pcseg.DGCNNWithColor(14).to(DEV).train()
    pts, _, _ = make_batch(2, 4096, seed=31)
    x = pts[:, :, :6].contiguous().transpose(1, 2).to(DEV)
    feats, graphs = [], []
    orig = pcseg.models.EdgeConv.forward_graph

    def rec(self, xp, seeds=None, **kw):
        out, idx = orig(self, xp, seeds, **kw)
        feats.append(xp.detach().clone())
        graphs.append(idx)
        return out, idx
    pcseg.models.EdgeConv.forward_graph = rec
    try:
        with torch.no_grad():
            m(x)
    finally:
        pcseg.models.EdgeConv.forward_graph = orig
    assert len(graphs) == 4
    for f, gidx in zip(feats, graphs):               # graph 1: pruned, unseeded; 2-4: pruned + seeded
        assert torch.equal(gidx, ops.knn(f, 20))


def test_dgcnn_knn_vs_reference_graph_at_4096(golden):
    """The xyz graph the reference itself built for BASELINE config 2's block size
    (tests/golden/model_dgcnn_color_4096.npz, knn0: B=2, N=4096, k=20)."""
    z = golden('model_dgcnn_color_4096.npz')
    xyz = T(z['x'])[:, :3].transpose(1, 2).contiguous()
    ref = T(z['knn0']).long()
    got = ops.knn(xyz.to(DEV), 20).cpu().long()
    same = (got.sort(-1).values == ref.sort(-1).values).all(-1)
    assert same.float().mean() > 0.995, float(same.float().mean())


@pytest.mark.parametrize('dim9', [False, True])
def test_functional_get_graph_feature_and_knn(dim9):
    """pcseg.get_graph_feature / pcseg.knn: the reference's functional API (dgcnn.py:7-57)."""
    B, C, N, k = 2, 9 if dim9 else 3, 1024, 20
    g = torch.Generator().manual_seed(21)
    x = torch.randn(B, C, N, generator=g)
    src = x[:, 6:] if dim9 else x
    idx = R.knn(src, k)
    ref = R.get_graph_feature(x, k=k, idx=idx, dim9=dim9)
    got = pcseg.get_graph_feature(x.to(DEV), k=k, idx=idx.to(DEV), dim9=dim9)
    assert got.shape == ref.shape and got.is_contiguous()
    assert torch.equal(got.cpu(), ref)
    kn = pcseg.knn(src.to(DEV), k)
    assert kn.dtype == torch.int64 and kn.shape == (B, N, k)
    same = (kn.cpu().sort(-1).values == idx.sort(-1).values).all(-1)
    assert same.float().mean() > 0.99
    # without idx: our own graph, same shape
    assert pcseg.get_graph_feature(x.to(DEV), k=k, dim9=dim9).shape == ref.shape


def test_masked_ce_matches_reference_golden(golden):
    """Fused HIP cross entropy vs the reference's loss + gradient (tests/golden/loss.npz)."""
    z = golden('loss.npz')
    logits, onehot, lengths = (torch.from_numpy(np.array(z[k])) for k in ('logits', 'onehot', 'lengths'))
    got = pcseg.masked_onehot_cross_entropy(logits.to(DEV), onehot.to(DEV), lengths.to(DEV))
    assert torch.allclose(got.cpu(), torch.from_numpy(z['loss']), rtol=1e-6)
    zero = pcseg.masked_onehot_cross_entropy(logits.to(DEV), onehot.to(DEV), torch.zeros(3, dtype=torch.int64,
                                                                                         device=DEV))
    assert float(zero) == 0.0
    lf = logits.to(DEV).requires_grad_(True)
    pcseg.masked_onehot_cross_entropy(lf, onehot.float().to(DEV), lengths.to(torch.int32).to(DEV)).backward()
    assert torch.allclose(lf.grad.cpu(), torch.from_numpy(z['grad']), rtol=1e-5, atol=1e-8)
    # scaled upstream gradient
    lf.grad = None
    (3.0 * pcseg.masked_onehot_cross_entropy(lf, onehot.to(DEV), lengths.to(DEV))).backward()
    assert torch.allclose(lf.grad.cpu(), 3.0 * torch.from_numpy(z['grad']), rtol=1e-5, atol=1e-8)


# ----------------------------------------------------------------------------- inverse maps / CSR backward
@pytest.mark.parametrize('B,N,C,K,r', [(3, 1024, 256, 32, 0.2), (2, 4096, 1024, 32, 0.1), (2, 256, 256, 16, 0.4)])
def test_inverse_index_and_group_bwd_csr(B, N, C, K, r):
    xyz = cloud(B, N, seed=41).to(DEV)
    cent = xyz[:, :C].contiguous()
    idx = ops.ball_query(cent, xyz, r, K)
    off, ent = ops.inverse_index(idx, N)
    # the CSR lists exactly the slots reading each point, each list ascending: the
    # entries are the stable sort of the slots by target
    flat = idx.reshape(B, -1).long().cpu()
    key = (torch.arange(B).unsqueeze(1) * N + flat).reshape(-1)
    order = torch.sort(key, stable=True).indices
    counts = torch.bincount(key, minlength=B * N)
    offs = torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)])
    assert torch.equal(off.long().cpu(), offs)
    assert torch.equal(ent.long().cpu(), order)
    # backward with the forward's map == backward that builds the map itself, bitwise
    D = 19
    feats = torch.randn(B, N, D, device=DEV)
    fa = feats.clone().requires_grad_(True)
    fb = feats.clone().requires_grad_(True)
    ya = ops.group_rows(xyz, fa, cent, idx, r, False)
    yb = ops.group_rows(xyz, fb, cent, idx, r, False, (off, ent))
    assert torch.equal(ya, yb)
    w = torch.randn_like(ya)
    (ya * w).sum().backward()
    (yb * w).sum().backward()
    assert torch.equal(fa.grad, fb.grad)
    # against an fp64 scatter of the same terms (the GPU sums each list in fp64, rounds once)
    gw = w.double().cpu().view(B, C * K, -1)[:, :, 3:3 + D]
    ref = torch.zeros(B, N, D, dtype=torch.float64).scatter_add_(1, flat.unsqueeze(-1).expand(-1, -1, D), gw)
    assert torch.equal(fb.grad.cpu(), ref.float())
    # deterministic
    fb.grad = None
    (ops.group_rows(xyz, fb, cent, idx, r, False, (off, ent)) * w).sum().backward()
    g1 = fb.grad.clone()
    fb.grad = None
    (ops.group_rows(xyz, fb, cent, idx, r, False, (off, ent)) * w).sum().backward()
    assert torch.equal(g1, fb.grad)


@pytest.mark.parametrize('D2', [64, 128, 256])
def test_interp_bwd_csr_with_and_without_forward_map(D2):
    """D2 = 128 / 256 take the channel-vector kernel (one list pass, float2 / float4 lanes)."""
    B, N, M, D1 = 2, 4096, 1024, 8
    c1 = cloud(B, N, seed=42).to(DEV)
    c2 = c1[:, :M].contiguous()
    idx, dist = ops.knn_select(c1, c2, 3)
    inv = ops.inverse_index(idx, M)
    f1 = torch.randn(B, N, D1, device=DEV)
    f2a = torch.randn(B, M, D2, device=DEV).requires_grad_(True)
    f2b = f2a.detach().clone().requires_grad_(True)
    ya = ops.interp_cat_rows(f1, f2a, idx, dist)
    yb = ops.interp_cat_rows(f1, f2b, idx, dist, inv)
    assert torch.equal(ya, yb)
    w = torch.randn_like(ya)
    (ya * w).sum().backward()
    (yb * w).sum().backward()
    assert torch.equal(f2a.grad, f2b.grad)
    # against the fp64 sum of the fp32 terms (g / norm) * w_j, list (= slot) order, rounded once
    d = dist.double().cpu().float()
    wts = 1.0 / (d + 1e-9)
    nrm = (wts[..., 0] + wts[..., 1]) + wts[..., 2]
    g = w.cpu().view(B, N, D1 + D2)[:, :, D1:]
    terms = (g.unsqueeze(2) / nrm[..., None, None]) * wts[..., None]          # (B, N, 3, D2) fp32
    ref = torch.zeros(B, M, D2, dtype=torch.float64)
    ref.scatter_add_(1, idx.long().cpu().reshape(B, N * 3, 1).expand(-1, -1, D2), terms.reshape(B, N * 3, D2).double())
    assert torch.equal(f2b.grad.cpu(), ref.float())


@pytest.mark.parametrize('B,S,k,targets,kind', [(3, 500, 7, 1000, 'random'), (2, 1024, 32, 4096, 'same'),
                                                  (2, 3000, 3, 40000, 'random'), (1, 2048, 32, 50000, 'same'),
                                                  (2, 1, 1, 1, 'random'), (2, 1024, 32, 4096, 'skewed'),
                                                  (2, 4096, 20, 4096, 'skewed'), (2, 3000, 3, 6000, 'random'),
                                                  (3, 2048, 20, 8192, 'skewed'), (4, 100, 5, 333, 'same')])
def test_inverse_index_random_tables(B, S, k, targets, kind):
    """CSR of arbitrary tables: LDS-counter path (targets <= 32768) and global-counter path,
    including the degenerate table where every slot reads the same point, and skewed tables
    whose hub lists take the LDS bitonic (65..1024 entries) and run-merge (> 1024) sorts."""
    g = torch.Generator().manual_seed(7)
    if kind == 'same':
        idx = torch.full((B, S, k), targets // 3, dtype=torch.int32)
    elif kind == 'skewed':
        w = 1.0 / torch.arange(1, targets + 1, dtype=torch.float64) ** 1.1
        idx = torch.multinomial(w, B * S * k, replacement=True, generator=g).view(B, S, k).to(torch.int32)
    else:
        idx = torch.randint(0, targets, (B, S, k), generator=g, dtype=torch.int32)
    off, ent = ops.inverse_index(idx.to(DEV), targets)
    key = (torch.arange(B).unsqueeze(1) * targets + idx.reshape(B, -1).long()).reshape(-1)
    counts = torch.bincount(key, minlength=B * targets)
    assert torch.equal(off.long().cpu(), torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)]))
    assert torch.equal(ent.long().cpu(), torch.sort(key, stable=True).indices)      # ascending lists
    if kind == 'skewed':
        assert counts.max() > 1024 and ((counts > 64) & (counts <= 1024)).any()


def test_inverse_index_batch_matches_single_maps():
    """pcs_inverse_index_batch (one call, shared launches; blockIdx.z = map) == one
    pcs_inverse_index per table, bitwise: one-chunk and multi-chunk clouds, 4096- and
    8192-target rank widths, a > 8192-target table (legacy path after the batch), a skewed
    table 30 tables (two launch groups)."""
    g = torch.Generator().manual_seed(11)
    B = 3
    shapes = [(1024, 32, 4096), (256, 32, 1024), (64, 32, 256), (16, 32, 64), (4096, 3, 1024),
              (4096, 20, 4096), (3000, 3, 6000), (2048, 3, 20000), (100, 5, 333)]
    tabs = []
    for i in range(30):
        S, k, T = shapes[i % len(shapes)]
        if i % 4 == 1:
            w = 1.0 / torch.arange(1, T + 1, dtype=torch.float64) ** 1.1
            idx = torch.multinomial(w, B * S * k, replacement=True, generator=g).view(B, S, k).to(torch.int32)
        else:
            idx = torch.randint(0, T, (B, S, k), generator=g, dtype=torch.int32)
        tabs.append((idx.to(DEV), T))
    got = ops.inverse_index_batch(tabs)
    for (idx, T), (off, ent) in zip(tabs, got):
        o1, e1 = ops.inverse_index(idx, T)
        assert torch.equal(off, o1) and torch.equal(ent, e1), (idx.shape, T)


@pytest.mark.parametrize('D1,D2', [(0, 128), (64, 256), (12, 8)])
def test_interp_cat_fused_bit_exact(D1, D2):
    """pcs_interp_cat_fwd (float4, skip copy fused) == the scalar pcs_interp_fwd + copy, bitwise."""
    from pcseg._lib import call, ptr, stream_ptr
    B, N, M = 2, 2048, 512
    c1 = cloud(B, N, seed=43).to(DEV)
    c2 = c1[:, :M].contiguous()
    idx, dist = ops.knn_select(c1, c2, 3)
    f1 = torch.randn(B, N, D1, device=DEV) if D1 else None
    f2 = torch.randn(B, M, D2, device=DEV)
    W = D1 + D2
    fused = torch.full((B * N, W), float('nan'), device=DEV)
    call('pcs_interp_cat_fwd', ptr(f1), D1, ptr(f2), ptr(idx), ptr(dist), B, N, M, D2, ptr(fused), W,
         stream_ptr(f2.device))
    # scalar kernel: an odd row stride forces the per-element path
    ref = torch.zeros((B * N, W + 1), device=DEV)
    if f1 is not None:
        ref.view(B, N, W + 1)[:, :, :D1] = f1
    call('pcs_interp_fwd', ptr(f2), ptr(idx), ptr(dist), B, N, M, D2, ptr(ref), W + 1, D1, stream_ptr(f2.device))
    assert torch.equal(fused, ref[:, :W])


def test_fps_sqrt_tie_is_correctly_rounded():
    """Regression: two points whose running distances differ by 2 ulps in the square but share
    one correctly rounded sqrt (a tie the reference breaks on the lower index).  gfx950's
    v_sqrt_f32 is only faithful; FPS uses a correctly rounded sqrt (pcs_common.hpp sqrt_cr)."""
    pts, _, _ = make_batch(2, 4096, seed=102, uniform=True)
    xyz = pts[:, :, :3].contiguous()
    start = torch.tensor([3910, 920], dtype=torch.int32)
    ref = R.fps_indices(xyz, 1024, start)
    got, _ = ops.fps(xyz.to(DEV), 1024, start.to(DEV))
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize('D', [19, 64, 100, 128, 256, 300, 512, 700, 1024])
@pytest.mark.parametrize('kind', ['random', 'skewed'])
def test_csr_bwd_stream_all_widths_vs_fp64(D, kind):
    """The streaming CSR backward (round 5: one wave walks the lists of several consecutive
    targets as one entry range) against the fp64 sum of the same terms in list order, for every
    channel template (scalar lanes V = 1 / 2 / 4 / 8, float2 / float4 lanes) of both the group
    gather (rows [xyz, feats]) and the IDW interpolation, with hub lists, empty lists and more
    targets than waves (several targets per wave)."""
    from pcseg._lib import call, ptr, stream_ptr
    g = torch.Generator().manual_seed(D)
    B, targets, S, k = 2, 20000, 6000, 5
    if kind == 'skewed':
        w = 1.0 / torch.arange(1, targets + 1, dtype=torch.float64) ** 1.1
        idx = torch.multinomial(w, B * S * k, replacement=True, generator=g).view(B, S * k).to(torch.int32)
    else:
        idx = torch.randint(0, targets, (B, S * k), generator=g, dtype=torch.int32)
    off, ent = ops.inverse_index(idx.view(B, S, k).to(DEV), targets)
    slots = B * S * k
    key = (torch.arange(B).unsqueeze(1) * targets + idx.long()).reshape(-1)
    # group form: rows [xyz, D feats, pad], the gradient columns start at 3
    ld = (3 + D + 3) // 4 * 4
    gout = torch.randn(slots, ld, generator=g)
    gf = torch.full((B, targets, D), float('nan'), device=DEV)
    call('pcs_group_bwd_csr', ptr(gout.to(DEV)), ld, ptr(off), ptr(ent), B, targets, D, slots, ptr(gf),
         stream_ptr(torch.device(DEV)))
    ref = torch.zeros(B * targets, D, dtype=torch.float64).index_add_(0, key, gout[:, 3:3 + D].double())
    torch.cuda.synchronize()
    assert torch.equal(gf.cpu().view(-1, D), ref.float())
    # IDW form: fine rows (S*k/3 per cloud) of [D1 skip, D coarse] channels, slot s = 3 * row + j
    if (S * k) % 3:
        return
    rows = slots // 3
    D1 = 8
    W = D1 + D
    gi = torch.randn(rows, W, generator=g)
    dist = torch.rand(rows, 3, generator=g) * 0.01
    gp = torch.full((B, targets, D), float('nan'), device=DEV)
    call('pcs_interp_bwd_csr', ptr(gi.to(DEV)), W, D1, ptr(dist.to(DEV)), ptr(off), ptr(ent), B, targets, D, slots,
         ptr(gp), stream_ptr(torch.device(DEV)))
    wts = 1.0 / (dist + 1e-9)
    nrm = (wts[:, 0] + wts[:, 1]) + wts[:, 2]
    terms = (gi[:, D1:].unsqueeze(1) / nrm[:, None, None]) * wts[:, :, None]        # (rows, 3, D) fp32
    ref = torch.zeros(B * targets, D, dtype=torch.float64).index_add_(0, key, terms.reshape(slots, D).double())
    torch.cuda.synchronize()
    assert torch.equal(gp.cpu().view(-1, D), ref.float())
