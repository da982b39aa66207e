"""Shared 1x1-conv MLP stacks on point-major rows.

A 1x1 Conv1d/Conv2d over (B, Cin, ...) is a GEMM over rows: Z = X W^T + b with
X (rows, Cin).  The modules keep the reference's nn.Conv*/nn.BatchNorm*
parameter holders (so state_dict keys and shapes are identical) and evaluate
them on row-major activations.

Training-mode BatchNorm follows nn.BatchNorm*'s own forward (batch statistics,
unbiased running_var update, num_batches_tracked increment).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def conv_rows(x: torch.Tensor, conv: nn.Module) -> torch.Tensor:
    """x (M, Cin) -> (M, Cout) for a 1x1 Conv1d/Conv2d (weight (Cout, Cin, 1[,1]))."""
    w = conv.weight.view(conv.weight.shape[0], -1)
    if conv.bias is not None:
        return torch.addmm(conv.bias, x, w.t())
    return x @ w.t()


def bn_rows(z: torch.Tensor, bn: nn.modules.batchnorm._BatchNorm) -> torch.Tensor:
    """nn.BatchNorm{1,2}d semantics on (M, C) rows."""
    if bn.momentum is None:
        eaf = 0.0
    else:
        eaf = bn.momentum
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        if bn.momentum is None:
            eaf = 1.0 / float(bn.num_batches_tracked)
    use_batch = bn.training or (bn.running_mean is None and bn.running_var is None)
    return F.batch_norm(z,
                        bn.running_mean if not bn.training or bn.track_running_stats else None,
                        bn.running_var if not bn.training or bn.track_running_stats else None,
                        bn.weight, bn.bias, use_batch, eaf, bn.eps)


def mlp_rows(x: torch.Tensor, convs, bns, act: str = 'relu', slope: float = 0.2) -> torch.Tensor:
    """Stack of conv -> BN -> act on rows (reference MiniPointNet/UnitPointNet.forward)."""
    for conv, bn in zip(convs, bns):
        z = bn_rows(conv_rows(x, conv), bn)
        x = F.relu(z) if act == 'relu' else F.leaky_relu(z, slope)
    return x
