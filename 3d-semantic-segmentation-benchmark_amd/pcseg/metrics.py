"""Segmentation metrics (reference Training/metrics.py:3-142) on the GPU.

Same functions, arguments and return types as the reference: predictions (B, N, C)
(softmax outputs), padded one-hot labels (B, N, C) (fp32 as harness B builds them, or
uint8 as the block loader stores them), mask = lengths (B).  One `pcs_seg_metrics`
pass (csrc/metrics.hip) counts the confusion matrix, correct points and per-class
intersections / unions; the reference loops over samples and classes with one host
sync per count.  Results come back to the host once, as the reference's Python
numbers / CPU tensors.
"""
from __future__ import annotations

import torch

from ._lib import call, check_cuda, ptr, stream_ptr


def _counts(predictions: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor):
    check_cuda(predictions, labels)
    if predictions.dim() != 3 or labels.shape != predictions.shape:
        raise ValueError(f'metrics: predictions {tuple(predictions.shape)} and labels {tuple(labels.shape)} '
                         'must both be (B, N, C)')
    B, N, C = labels.shape
    dev = predictions.device
    pred = predictions.detach().float().contiguous()
    if labels.dtype == torch.uint8:
        lab, u8 = labels.contiguous(), 1
    else:
        lab, u8 = labels.detach().float().contiguous(), 0
    lengths = mask.to(device=dev, dtype=torch.int32).contiguous()
    out = torch.zeros(C * C + 2 * C + 1, dtype=torch.int64, device=dev)
    call('pcs_seg_metrics', ptr(pred), ptr(lab), u8, ptr(lengths), B, N, C, ptr(out), ptr(out[C * C:]),
         ptr(out[C * C + C:]), ptr(out[C * C + 2 * C:]), stream_ptr(dev))
    out = out.cpu()
    return out[:C * C].view(C, C), out[C * C:C * C + C], out[C * C + C:C * C + 2 * C], int(out[-1])


def update_accuracy(predictions: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor) -> tuple[int, int]:
    """(correctly predicted points, mask.sum()) -- metrics.py:28-51."""
    _, _, _, correct = _counts(predictions, labels, mask)
    return correct, mask.sum().item()


def overall_accuracy(predictions: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor) -> float:
    """metrics.py:3-25."""
    correct, total = update_accuracy(predictions, labels, mask)
    return correct / total


def confusion_matrix(predictions: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """(C, C) int64 on the CPU, rows = label class, columns = predicted class -- metrics.py:53-79."""
    conf, _, _, _ = _counts(predictions, labels, mask)
    return conf.clone()


def update_intersection_over_union(predictions: torch.Tensor, labels: torch.Tensor,
                                   mask: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-class intersections and unions (float32, CPU) -- metrics.py:113-142."""
    _, inter, uni, _ = _counts(predictions, labels, mask)
    return inter.to(torch.float32), uni.to(torch.float32)


def intersection_over_union(predictions: torch.Tensor, labels: torch.Tensor,
                            mask: torch.Tensor) -> tuple[float, torch.Tensor]:
    """(mean IoU, per-class IoU float32 on the CPU), eps = 1e-6 -- metrics.py:82-110."""
    _, inter, uni, _ = _counts(predictions, labels, mask)
    eps = 1e-6
    ious = torch.zeros((inter.numel(),), dtype=torch.float32)
    for c in range(inter.numel()):
        ious[c] = (int(inter[c]) + eps) / (int(uni[c]) + eps)
    return ious.mean().item(), ious
