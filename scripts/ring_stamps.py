"""Per-phase s_memtime cycles of the ring kernel's waves (workgroup 0), diagnostic build only
(build_ab.sh stamps with -DBR_STAMPS, loaded by PCS_LIB): phases 0 loop top, 1 vmcnt wait,
2 dZ rebuild, 3 barrier, 4 refill issue, 5 MFMAs, 6 epilogue, 7 tail."""
import ctypes
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg import _lib  # noqa: E402
from pcseg.common import UnitPointNet  # noqa: E402
from pcseg.engine import lane_join  # noqa: E402

dev = torch.device('cuda')
lib = _lib.load()
torch.manual_seed(0)
M, kin = 131072, 128
mod = UnitPointNet(kin, [128, 128, 128]).to(dev).train()
x = torch.randn(M, kin, device=dev).requires_grad_(True)
for it in range(3):
    y = mod.forward_rows(x, kin)
    y.backward(torch.randn_like(y))
    lane_join(dev)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 64)()
lib.pcs_debug_ring_stamps(buf)
names = ['top', 'vmwait', 'rebuild', 'barrier', 'refill', 'mfma', 'epilogue', 'tail']
for w in range(8):
    row = [buf[w * 8 + k] for k in range(8)]
    tot = sum(row)
    print(f'wave {w} ({"dA" if w < 4 else "dW"}): total {tot:8d} cyc ({tot / 100:.1f} us at 100 MHz?) ' +
          ' '.join(f'{n}={c}' for n, c in zip(names, row)))
