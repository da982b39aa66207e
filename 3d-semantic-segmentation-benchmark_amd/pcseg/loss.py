"""Masked one-hot cross entropy -- reference Training/train_model.py:15-57.

Same value as the reference: mean over un-padded positions of
-sum(onehot * log_softmax(logits)), computed by one HIP pass (csrc/loss.hip)
that also writes the gradient.  The reference's `.item()` zero check
(train_model.py:53) is replaced by a sync-free guard with the same result
(0.0 when every position is padding), so the training step never stalls the
GPU stream or blocks hipGraph capture.
"""
from __future__ import annotations

import torch

from ._lib import call, check_cuda, load, ptr, stream_ptr


class MaskedCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, lengths):
        B, L, C = logits.shape
        x = logits if logits.is_contiguous() else logits.contiguous()
        if targets.dtype in (torch.uint8, torch.bool):
            tgt, kind = targets.contiguous().view(torch.uint8), 0
        else:
            tgt, kind = targets.to(torch.float32).contiguous(), 1
        lens = lengths.to(device=x.device, dtype=torch.int32).contiguous()
        if lens.numel() != B:
            raise ValueError(f'lengths has {lens.numel()} entries for a batch of {B}')
        dev = x.device
        nb = load().pcs_masked_ce_blocks(B, L)
        part = torch.empty(nb, dtype=torch.float64, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        grad = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        call('pcs_masked_ce', ptr(x), C, ptr(tgt), kind, C, ptr(lens), B, L, C, ptr(part), ptr(loss), ptr(grad),
             stream_ptr(dev))
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        return grad * gout, None, None


def masked_onehot_cross_entropy(logits: torch.Tensor, targets_onehot: torch.Tensor, pad_starts: torch.Tensor,
                                eps: float = 1e-9) -> torch.Tensor:
    check_cuda(logits, targets_onehot)
    if logits.dtype != torch.float32:
        raise ValueError('pcseg masked_onehot_cross_entropy: fp32 logits expected')
    return MaskedCEFn.apply(logits, targets_onehot, pad_starts)
