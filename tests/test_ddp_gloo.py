"""Multi-process data-parallel path on the CPU (gloo, world size 2).

SURVEY.md section 8(e): blocks are independent, the one exchange is the gradient
all-reduce; BN statistics stay local per rank.  The check: after
`FlatGradAllReduce.synchronize()` every rank holds the mean over ranks of the
gradients each rank computes on its own shard with plain autograd (the
reference algorithm, oracle model, local BN), and `broadcast_model` makes
rank 1 start from rank 0's weights.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO  # noqa: F401  (sets sys.path)
from oracle import ref_ops as R
from pcseg.ddp import FlatGradAllReduce, broadcast_model
from pcseg.synthetic import make_batch


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _dropout_off(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()


def _step(model, x, lab, lengths, starts):
    with R.replay(R.Replay(fps_starts=starts)):
        loss = R.masked_onehot_cross_entropy(model(x), lab, lengths)
    loss.backward()


def _worker(rank, world, port, bucket_bytes, overlap, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        # rank-dependent init: broadcast_model must overwrite rank 1's weights
        model = R.seeded_init_(R.PointNetpp(14), 10 + rank)
        model.train()
        _dropout_off(model)
        broadcast_model(model)
        ref = R.seeded_init_(R.PointNetpp(14), 10)
        for (k, a), (_, b) in zip(model.state_dict().items(), ref.state_dict().items()):
            assert torch.equal(a, b), k
        pts, labels, lengths = make_batch(1, 1024, seed=500 + rank)
        starts = [torch.tensor([3 * rank + i], dtype=torch.int32) for i in range(4)]

        # local gradients with plain autograd on this rank's shard
        ref.train()
        _dropout_off(ref)
        _step(ref, pts, labels, lengths, starts)
        local = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
        gathered = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        expect = torch.stack(gathered).mean(0)

        # the data-parallel path: flat buffer, bucketed all-reduce from backward hooks
        grads = FlatGradAllReduce(model, bucket_bytes=bucket_bytes, overlap=overlap)
        for _ in range(2):                     # twice: zero_grad must reset the buckets
            grads.zero_grad()
            _step(model, pts, labels, lengths, starts)
            if grads.overlap:
                # every bucket launched exactly once from backward, and a repeated
                # announcement of a parameter is ignored
                assert grads._pending == [0] * len(grads.buckets) and all(grads._launched)
                n_handles = len(grads._handles)
                grads._hook(grads.params[0])
                assert len(grads._handles) == n_handles and grads._pending[-1] == 0
            grads.synchronize()
            got = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
            err = float((got - expect).abs().max())
            out[rank] = err
            assert err <= 1e-6 * float(expect.abs().max()) + 1e-9, err
            # the result is identical on both ranks
            other = [torch.empty_like(got) for _ in range(world)]
            dist.all_gather(other, got)
            assert torch.equal(other[0], other[1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('bucket_bytes,overlap', [(256 << 10, True), (64 << 20, True), (1 << 20, False)])
def test_flat_grad_allreduce_world2(bucket_bytes, overlap):
    world = 2
    ctx = mp.get_context('spawn')
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_bytes, overlap, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert len(out) == world


def test_bucket_layout_covers_every_parameter_once():
    model = R.PointNetpp(14)
    g = FlatGradAllReduce(model, bucket_bytes=128 << 10, overlap=False)
    seen = [p for _, _, ps in g.buckets for p in ps]
    assert len(seen) == len(g.params) and len({id(p) for p in seen}) == len(seen)
    # buckets tile the flat buffer contiguously, last layers first
    ends = [0] + [e for _, e, _ in g.buckets]
    assert [s for s, _, _ in g.buckets] == ends[:-1] and ends[-1] == g.flat.numel()
    assert g.buckets[0][2][0] is g.params[-1]
    for p in g.params:
        assert p.grad.data_ptr() >= g.flat.data_ptr()


def _gpu_worker(rank, world, port, out, overlap=True):
    """Product model on cuda:0 in both ranks, gloo over the GPU tensors: exercises the
    engine's in-place gradient writes + `_pcs_grad_ready` bucket hooks."""
    import pcseg
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        dev = torch.device('cuda', 0)
        sd = R.seeded_init_(R.PointNetpp(14), 10).state_dict()
        models = []
        for _ in range(2):
            m = pcseg.PointNetpp(14)
            m.load_state_dict(sd)
            m = m.to(dev).train()
            _dropout_off(m)
            models.append(m)
        ref, model = models
        pts, labels, lengths = make_batch(2, 4096, seed=700 + rank)
        x, lab, ln = pts.to(dev), labels.to(dev), lengths.to(dev)

        def step(m):
            torch.manual_seed(rank)
            loss = pcseg.masked_onehot_cross_entropy(m(x), lab, ln)
            loss.backward()
        step(ref)
        local = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
        gathered = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        expect = torch.stack(gathered).mean(0)
        grads = FlatGradAllReduce(model, bucket_bytes=256 << 10, overlap=overlap)
        calls = {}
        if grads.overlap:
            orig = grads._hook

            def counting_hook(p):
                calls[id(p)] = calls.get(id(p), 0) + 1
                orig(p)
            for p in grads.params:
                p._pcs_grad_ready = counting_hook
        grads.zero_grad()
        step(model)
        if grads.overlap:
            # every parameter's gradient is announced exactly once (engine or autograd hook)
            assert sorted(calls.values()) == [1] * len(calls)
            # after backward every bucket has been launched exactly once
            assert grads._pending == [0] * len(grads.buckets) and all(grads._launched)
        grads.synchronize()
        got = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
        rel = float((got - expect).norm() / expect.norm())
        out[rank] = rel
        if rel >= 1e-5 and rank == 0:
            off = 0
            for (name, p) in model.named_parameters():
                n = p.numel()
                e = float((got[off:off + n] - expect[off:off + n]).norm() / (expect[off:off + n].norm() + 1e-30))
                loc = float((local[off:off + n] - expect[off:off + n]).norm() / (expect[off:off + n].norm() + 1e-30))
                print(f'DDPDIAG {name} rel={e:.3e} local_vs_mean={loc:.3e}', flush=True)
                off += n
        assert rel < 1e-5, rel                 # the all-reduce sums in another order than the local mean
        assert all(h is not None for h in grads._handles) or not grads._handles
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize('overlap', [False, True])
def test_flat_grad_allreduce_world2_engine_on_gpu(overlap):
    world = 2
    ctx = mp.get_context('spawn')
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, out, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    print('DDPOUT', dict(out), flush=True)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _buffers_worker(rank, world, port, out, broadcast_buffers):
    """DDP broadcast_buffers: rank 0's BN running statistics reach every rank at the start of a
    training forward, then each rank updates them with its OWN batch statistics."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.BatchNorm1d(8)).train()
        broadcast_model(model)
        with torch.no_grad():                   # rank-dependent buffers after the initial broadcast
            model[1].running_mean.fill_(float(rank + 1))
            model[1].running_var.fill_(float(2 * rank + 1))
            model[1].num_batches_tracked.fill_(5 * rank)
        grads = FlatGradAllReduce(model, overlap=True, broadcast_buffers=broadcast_buffers)
        x = torch.randn(16, 4, generator=torch.Generator().manual_seed(rank))
        with torch.no_grad():
            z = model[0](x)
        bm, bv = z.mean(0), z.var(0, unbiased=True)
        grads.zero_grad()
        model(x).square().sum().backward()
        grads.synchronize()
        src = 0 if broadcast_buffers else rank
        exp_mean = 0.9 * float(src + 1) + 0.1 * bm
        exp_var = 0.9 * float(2 * src + 1) + 0.1 * bv
        assert torch.allclose(model[1].running_mean, exp_mean, atol=1e-6), (model[1].running_mean, exp_mean)
        assert torch.allclose(model[1].running_var, exp_var, atol=1e-6)
        assert int(model[1].num_batches_tracked) == 5 * src + 1
        # state_dict still names the rebound buffers and loads into them in place
        sd = model.state_dict()
        assert torch.equal(sd['1.running_mean'], model[1].running_mean)
        # an eval forward does not broadcast
        model.eval()
        with torch.no_grad():
            model(x)
        out[rank] = float(model[1].running_mean[0])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('broadcast_buffers', [True, False])
def test_broadcast_buffers_world2(broadcast_buffers):
    world = 2
    ctx = mp.get_context('spawn')
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_buffers_worker, args=(r, world, port, out, broadcast_buffers))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert len(out) == world
