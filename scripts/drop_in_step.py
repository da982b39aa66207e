"""The drop-in harness-A step alone (bench.run_drop_in: torch.optim.Adam, zero_grad, forward,
criterion, backward, step on the default stream), for a kernel trace of exactly that step.
usage: drop_in_step.py [model] [steps]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bench  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else 'pointnetpp'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
import torch  # noqa: E402

args = argparse.Namespace(warmup=3, steps=steps, no_roofline=True)
_, _, _, batch, npoints, _ = bench.WORKLOADS[key]
out = bench.run_drop_in(key, batch, npoints, args, torch.device('cuda', 0))
print(json.dumps({k: v for k, v in out.items() if k not in ('roofline', 'step_roofline')}))
