"""bench.py with DGCNN's round-4 head concatenation (A/B only): the EdgeConv outputs are not
written into the head buffer by their kernels, and _dgcnn_head copies every part (5 copy_cols
launches), as before round 5's second EdgeConv output.  usage: same flags as bench.py."""
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [root, os.path.join(root, '3d-semantic-segmentation-benchmark_amd')]
import pcseg.models as PM  # noqa: E402

_fg, _head = PM.EdgeConv.forward_graph, PM._dgcnn_head


def forward_graph(self, xp, seeds=None, inv_batch=None, also=None):
    return _fg(self, xp, seeds, inv_batch=inv_batch)


def head(self, parts, B, N, H=None):
    return _head(self, parts, B, N, None)


PM.EdgeConv.forward_graph = forward_graph
PM._dgcnn_head = head
sys.argv[0] = os.path.join(root, 'bench.py')
import bench  # noqa: E402
bench.main()
