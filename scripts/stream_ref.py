"""Attainable streaming bandwidth for the thin-layer shapes (torch elementwise kernels):
the HBM rate a row GEMM over M rows could reach if it only streamed its operands."""
import torch

dev = 'cuda'
for M, C in [(1 << 20, 32), (1 << 20, 64), (1 << 18, 64), (1 << 17, 128)]:
    a = torch.randn(M, C, device=dev)
    b = torch.randn(M, C, device=dev)
    out = torch.empty(M, C, device=dev)
    for _ in range(3):
        torch.add(a, b, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.add(a, b, out=out)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f'M={M} C={C}: a+b -> out {us:7.1f} us  {3 * 4 * M * C / us / 1e3:6.0f} GB/s', flush=True)
