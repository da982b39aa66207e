"""HIP-graph replay cost on this ROCm: host wall per hipGraphLaunch and GPU time per replay
for graphs of N small kernels, single-stream vs forked/joined side streams (event nodes),
against the same launches issued eagerly.  Prints one JSON line per case.

usage: python scripts/graph_probe.py [n_kernels]
"""
import json
import os
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 240
dev = torch.device('cuda', 0)
x = torch.zeros(4096, device=dev)
side = torch.cuda.Stream(dev)


def body(fork_every):
    main = torch.cuda.current_stream(dev)
    for i in range(N):
        if fork_every and i % fork_every == 0:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                x.add_(1.0)
            main.wait_stream(side)
        else:
            x.add_(1.0)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    return th / reps * 1e3, tw / reps * 1e3


for fork in (0, 10, 3):
    host_e, wall_e = timed(lambda: body(fork))
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        body(fork)
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(fork)
    host_g, wall_g = timed(g.replay)
    print(json.dumps({'kernels': N, 'fork_every': fork, 'env_packet_capture': os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE'),
                      'eager_host_ms': round(host_e, 3), 'eager_wall_ms': round(wall_e, 3),
                      'graph_host_ms': round(host_g, 3), 'graph_wall_ms': round(wall_g, 3)}), flush=True)
