"""RCCL (torch.distributed backend "nccl" on ROCm) on the one GPU of a lease: a world of one
process, FlatGradAllReduce with its bucket all-reduces forced on (collectives_at_world_1), so the
real RCCL launches run from the engine's post-accumulate notifications -- on the wgrad lane,
behind the deferred weight gradients (pcseg/ddp.py) -- and the step's gradients must be BITWISE
those of the same step without the data-parallel wrapper (an all-reduce over one rank is the
identity).  This is the stream-ordering half of SURVEY.md 8(e) that the gloo tests
(tests/test_ddp_gloo.py) cannot reach.  The child process initialises the process group before
it touches the GPU, as bench.py's rank processes do."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')

CHILD = r'''
import json, sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/3d-semantic-segmentation-benchmark_amd']
import torch
import torch.distributed as dist
dist.init_process_group('nccl', rank=0, world_size=1)
import pcseg
from pcseg.ddp import FlatGradAllReduce
from pcseg.synthetic import make_batch
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
model_name = sys.argv[2]

def build():
    torch.manual_seed(3)
    ctor = {'pointnetpp': lambda: pcseg.PointNetpp(14), 'pointnext': lambda: pcseg.PointNeXt(14)}[model_name]
    return ctor().to(dev).train()

pts, labels, lengths = make_batch(4, 2048 if model_name == 'pointnet' else 4096, seed=21)
x, lab, ln = pts.to(dev), labels.to(dev), lengths.to(dev)

def step(model, ddp):
    torch.manual_seed(77)                  # same FPS starts and dropout seeds in both runs
    if ddp is not None:
        ddp.zero_grad()
    else:
        model.zero_grad(set_to_none=True)
    loss = pcseg.masked_onehot_cross_entropy(model(x), lab, ln)
    loss.backward()
    launched = 0
    if ddp is not None:
        launched = sum(ddp._launched)      # buckets reduced from the backward's notifications
        ddp.synchronize()
    torch.cuda.synchronize()
    return float(loss), launched

plain = build()
l0, _ = step(plain, None)
l0b, _ = step(plain, None)
ref = {n: p.grad.detach().clone() for n, p in plain.named_parameters()}
wrapped = build()
ddp = FlatGradAllReduce(wrapped, bucket_bytes=1 << 20, collectives_at_world_1=True)
l1, launched = step(wrapped, ddp)
l1b, launched_b = step(wrapped, ddp)
launched = min(launched, launched_b)
diff = [n for n, p in wrapped.named_parameters() if not torch.equal(p.grad, ref[n])]
print(json.dumps({'backend': dist.get_backend(), 'world': dist.get_world_size(), 'buckets': len(ddp.buckets),
                  'launched': launched, 'loss': [l0, l0b, l1, l1b], 'diff': diff,
                  'nparams': len(ref)}))
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('model', ['pointnetpp', 'pointnext'])
def test_rccl_world1_bucket_allreduce_is_bitwise_identity(model):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()), RANK='0', WORLD_SIZE='1',
               LOCAL_RANK='0')
    p = subprocess.run([sys.executable, '-c', CHILD, ROOT, model], env=env, capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r['backend'] == 'nccl' and r['world'] == 1
    # every bucket's all-reduce was launched from the backward (post-accumulate notifications)
    assert r['launched'] == r['buckets'] >= 2, r
    assert r['loss'][0] == r['loss'][2] and r['loss'][1] == r['loss'][3], r['loss']
    assert r['diff'] == [], r['diff']
