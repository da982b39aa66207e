"""Injection / recording of the reference's random and rounding-sensitive choices.

The reference draws the FPS start index with `torch.randint` inside `sample`
(models/utils/common.py:22) and recomputes DGCNN kNN graphs whose near-ties
depend on MKL rounding (models/dgcnn/dgcnn.py:16-20).  Parity harnesses replay
the CPU oracle's choices into the GPU model through this context; training
never needs it.
"""
from __future__ import annotations

import contextlib

import torch


class Replay:
    def __init__(self, fps_starts=None, knn_idx=None):
        self.fps_starts = list(fps_starts) if fps_starts is not None else None
        self.knn_idx = list(knn_idx) if knn_idx is not None else None
        self.rec_fps_starts: list[torch.Tensor] = []
        self.rec_fps_idx: list[torch.Tensor] = []
        self.rec_group_idx: list[torch.Tensor] = []
        self.rec_interp_idx: list[torch.Tensor] = []
        self.rec_knn_idx: list[torch.Tensor] = []
        # max-pool argmax decisions (SA / InvResMLP / EdgeConv pools), forward order, (groups, channels)
        # uint8 -- the parity tests replay them into the fp64 oracle so a near-tie decided one way
        # here is evaluated the same way there
        self.rec_pool_arg: list[torch.Tensor] = []
        # sign decisions (y > 0) of every engine ReLU / LeakyReLU, (rows, channels) bool, forward order
        self.rec_act_mask: list[torch.Tensor] = []


_ACTIVE: list[Replay] = []


@contextlib.contextmanager
def replay(rp: Replay):
    _ACTIVE.append(rp)
    try:
        yield rp
    finally:
        _ACTIVE.pop()


def active() -> Replay | None:
    return _ACTIVE[-1] if _ACTIVE else None


def record_pool_arg(arg: torch.Tensor) -> None:
    rp = active()
    if rp is not None:
        rp.rec_pool_arg.append(arg.detach().cpu())


def recording() -> bool:
    return active() is not None


def record_act_mask(mask: torch.Tensor) -> None:
    rp = active()
    if rp is not None:
        rp.rec_act_mask.append(mask.detach().cpu())
