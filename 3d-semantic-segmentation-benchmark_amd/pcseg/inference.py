"""Sliding-window whole-scene inference (reference `predict_single_scene`,
models/dgcnn/utils.py:67-131).

The reference runs one B=1 forward per window of `batch_size` points (stride
`batch_size - overlap`), accumulating logits window by window.  In eval mode a window's
logits do not depend on the other windows (BatchNorm uses running statistics, the kNN
graph is per cloud), so here equal-size windows run as ONE batched forward (zero-copy
strided views of the scene, up to `max_windows` per launch), and the overlap average,
argmax and softmax confidence are one HIP pass (`pcs_window_merge`).  Same arguments
and returns: (predictions int64, confidences fp32), both on the CPU.
"""
from __future__ import annotations

import torch

from ._lib import call, ptr, stream_ptr


def _windows(n: int, win: int, step: int):
    starts = list(range(0, n, step))
    return starts, [min(win, n - s) for s in starts]


def predict_single_scene(model, points: torch.Tensor, device: str = 'cuda', batch_size: int = 4096,
                         overlap: int = 512, max_windows: int = 16):
    model.eval()
    dev = torch.device(device)
    if dev.type != 'cuda':
        raise RuntimeError('pcseg inference runs only on the GPU (no CPU fallback)')
    points = points.to(dev, dtype=torch.float32).contiguous()
    n, F = points.shape
    C = model.num_classes
    if n <= batch_size:
        starts, sizes, step = [0], [n], max(batch_size - overlap, 1)
    else:
        step = batch_size - overlap
        starts, sizes = _windows(n, batch_size, step)
    rows = [0]
    for s in sizes[:-1]:
        rows.append(rows[-1] + s)
    logits_all = torch.empty((sum(sizes), C), dtype=torch.float32, device=dev)
    with torch.no_grad():
        w = 0
        while w < len(starts):
            size = sizes[w]
            e = w + 1                       # a run of consecutive equal-size windows
            while e < len(starts) and sizes[e] == size and e - w < max_windows:
                e += 1
            nb = e - w
            # (nb, size, F) zero-copy strided view of the scene, as (nb, F, size) model input
            view = points.as_strided((nb, size, F), ((step if n > batch_size else 0) * F, F, 1),
                                     starts[w] * F)
            logits, _, _ = model(view.transpose(1, 2))
            logits_all[rows[w]:rows[w] + nb * size] = logits.reshape(nb * size, C)
            w = e
    wo = torch.tensor(rows, dtype=torch.int64, device=dev)
    pred = torch.empty(n, dtype=torch.int64, device=dev)
    conf = torch.empty(n, dtype=torch.float32, device=dev)
    call('pcs_window_merge', ptr(logits_all), ptr(wo), len(starts), n, C, step, max(batch_size, n) if n <= batch_size
         else batch_size, ptr(pred), ptr(conf), stream_ptr(dev))
    return pred.cpu(), conf.cpu()
