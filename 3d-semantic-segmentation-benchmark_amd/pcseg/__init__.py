"""pcseg -- MI355X-native (gfx950) point-cloud segmentation training hot path.

Drop-in for the `models/` hot path of piotr-bledowski/3D-Semantic-Segmentation-
Benchmark: same module names, constructor/forward signatures, return
conventions and state_dict keys; the neighbour search, gathers, pooling and
interpolation run as hand-written HIP kernels (libpcseg.so, C ABI in
include/pcseg.h).
"""
from .common import (sample, group, reduce, interpolate, MiniPointNet, UnitPointNet, SetAbstraction,
                     FeaturePropagation, InvResMLP)
from .models import (PointNetpp, PointNetppMSG, PointNeXt, EdgeConv, DGCNN, DGCNNWithColor, get_model, get_loss,
                     TNet, PointNetEncoder, PointNetSeg, knn, get_graph_feature)
from .loss import masked_onehot_cross_entropy
from .replay import Replay, replay
from . import metrics, inference, graphs

__all__ = ['sample', 'group', 'reduce', 'interpolate', 'MiniPointNet', 'UnitPointNet', 'SetAbstraction',
           'FeaturePropagation', 'InvResMLP', 'PointNetpp', 'PointNetppMSG', 'PointNeXt', 'EdgeConv', 'DGCNN',
           'DGCNNWithColor', 'get_model', 'get_loss', 'TNet', 'PointNetEncoder', 'PointNetSeg',
           'masked_onehot_cross_entropy', 'Replay', 'replay', 'knn', 'get_graph_feature', 'metrics', 'inference']
