"""Masked one-hot cross entropy -- reference Training/train_model.py:15-57.

Same value as the reference: mean over un-padded positions of
-sum(onehot * log_softmax(logits)).  The reference's `.item()` zero check
(train_model.py:53) is replaced by a sync-free guard with the same result
(0.0 when every position is padding), so the training step never stalls the
GPU stream or blocks hipGraph capture.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def masked_onehot_cross_entropy(logits: torch.Tensor, targets_onehot: torch.Tensor, pad_starts: torch.Tensor,
                                eps: float = 1e-9) -> torch.Tensor:
    B, L, C = logits.shape
    log_probs = F.log_softmax(logits, dim=-1)
    token_loss = -torch.sum(targets_onehot * log_probs, dim=-1)
    positions = torch.arange(L, device=logits.device).unsqueeze(0).expand(B, L)
    mask = (positions < pad_starts.to(logits.device).long().unsqueeze(1)).float()
    total = mask.sum()
    return (token_loss * mask).sum() / torch.clamp(total, min=1.0)
