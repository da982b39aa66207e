"""Deterministic stand-in model for sliding-window inference fixtures (tests/golden/scene.npz)."""
import torch


class PerPointLinear(torch.nn.Module):
    """DGCNN's call contract ((B, F, n) -> (logits (B, n, C), _, _), `num_classes`) with a
    per-point linear map: pins the windowing / averaging / argmax of predict_single_scene
    (models/dgcnn/utils.py:67-131) independently of kNN rounding."""

    def __init__(self, F, C, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.num_classes = C
        self.weight = torch.nn.Parameter(torch.randn(C, F, generator=g) * 0.01)
        self.bias = torch.nn.Parameter(torch.randn(C, generator=g) * 0.1)

    def forward(self, x):
        return (x.transpose(1, 2) @ self.weight.t() + self.bias), None, None
