"""Which part of the captured PointNet++ step makes hipGraphLaunch slow?  Captures pieces of
the step separately and prints the host wall per replay and the GPU wall per replay for each.

usage: python scripts/graph_pieces.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd')]

import torch  # noqa: E402

import pcseg  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402
from pcseg.common import side_stream  # noqa: E402

dev = torch.device('cuda', 0)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    return round(th / reps * 1e3, 3), round(tw / reps * 1e3, 3)


def capture(fn, warm=2):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def report(name, fn):
    eh, ew = timed(fn)
    g, _ = capture(fn)
    gh, gw = timed(g.replay)
    print(json.dumps({'piece': name, 'eager_host_ms': eh, 'eager_wall_ms': ew, 'graph_host_ms': gh,
                      'graph_wall_ms': gw}), flush=True)
    return g


torch.manual_seed(0)
model = pcseg.PointNetpp(14).to(dev).train()
for m in model.modules():
    if isinstance(m, torch.nn.Dropout):
        m.eval()
pts, labels, lengths = make_batch(32, 4096, seed=7)
x, lab, ln = pts.to(dev), labels.to(dev), lengths.to(dev)
c0 = x[:, :, :3].contiguous()

report('fps_only', lambda: pcseg.ops.fps(c0, 1024, torch.zeros(32, dtype=torch.int32, device=dev)))
cent = pcseg.ops.fps(c0, 1024, torch.zeros(32, dtype=torch.int32, device=dev))[1]
report('ball_query_only', lambda: pcseg.ops.ball_query(cent, c0, 0.1, 32))
idx = pcseg.ops.ball_query(cent, c0, 0.1, 32)
report('inverse_index_only', lambda: pcseg.ops.inverse_index(idx, 4096))
report('knn_select_only', lambda: pcseg.ops.knn_select(c0, cent, 3))


def plan_joined():
    p = model._plan_for(c0)
    torch.cuda.current_stream(dev).wait_stream(side_stream(dev))
    return p


report('geometry_plan', plan_joined)
rows = pcseg.ops.group_rows(c0, x[:, :, 3:].contiguous(), cent, idx, 0.1, False)
report('sa1_mlp_forward', lambda: model.sa1.point_net.forward_rows(rows, 9, pool_k=32))


def fwd_joined():
    out = model(x)
    torch.cuda.current_stream(dev).wait_stream(side_stream(dev))
    return out


with torch.no_grad():
    report('forward_no_grad', fwd_joined)


report('forward_train', fwd_joined)


def fwd_bwd():
    model.zero_grad(set_to_none=False)
    loss = pcseg.masked_onehot_cross_entropy(model(x), lab, ln)
    loss.backward()
    torch.cuda.current_stream(dev).wait_stream(side_stream(dev))
    return loss


for p in model.parameters():
    p.grad = torch.zeros_like(p)
report('forward_backward', fwd_bwd)
