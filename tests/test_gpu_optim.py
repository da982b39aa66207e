"""pcs_adam (pcseg.optim.FlatAdam) against torch.optim.Adam, the reference's optimizer
(Training/train_model.py:263), on the same parameters and gradients for several steps.

Tolerance: per element rtol 1e-5, atol 1e-8 -- the same fp32 update formula; torch's
foreach kernels are compiled with FMA contraction (ours keep the separate roundings),
a few ulps per step on values of order lr."""
import pytest
import torch

from pcseg.ddp import FlatGradAllReduce
from pcseg.optim import FlatAdam

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _model(seed):
    torch.manual_seed(seed)
    # odd sizes so the flat buffer has a non-multiple-of-4 tail
    return torch.nn.Sequential(torch.nn.Linear(13, 33), torch.nn.BatchNorm1d(33), torch.nn.Linear(33, 7)).to(DEV)


@pytest.mark.parametrize('wd', [0.0, 1e-4])
def test_flat_adam_matches_torch_adam(wd):
    ref = _model(0)
    ours = _model(0)
    ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=wd)
    grads = FlatGradAllReduce(ours)
    opt = FlatAdam(grads, lr=1e-3, weight_decay=wd)
    g = torch.Generator(device=DEV).manual_seed(5)
    for step in range(6):
        # identical gradients into both (a forward/backward per model would let step-k
        # parameter ulps change the gradients, which Adam amplifies where |g| is tiny)
        ref_opt.zero_grad(set_to_none=False)
        opt.zero_grad()
        for a, b in zip(ref.parameters(), ours.parameters()):
            gr = torch.randn(a.shape, device=DEV, generator=g) * (10.0 ** (step % 3 - 2))
            a.grad = gr.clone()
            b.grad.copy_(gr)
        grads.synchronize()
        ref_opt.step()
        opt.step()
        for (n, a), b in zip(ref.named_parameters(), ours.parameters()):
            assert torch.allclose(b.detach(), a.detach(), rtol=1e-5, atol=1e-8), \
                (step, n, float((a.detach() - b.detach()).abs().max()))
    # parameters stay views of the optimizer's flat buffer
    for p in ours.parameters():
        assert p.data.untyped_storage().data_ptr() == opt.flat.untyped_storage().data_ptr()


def test_flat_adam_empty_tail_and_alignment():
    lin = torch.nn.Linear(4, 4, bias=False).to(DEV)      # 16 params: no scalar tail
    grads = FlatGradAllReduce(lin)
    opt = FlatAdam(grads)
    lin.weight.grad.fill_(1.0)
    before = lin.weight.detach().clone()
    opt.step()
    torch.cuda.synchronize()
    # first Adam step moves every parameter by -lr * sign(g)
    assert torch.allclose(lin.weight.detach(), before - 1e-3, atol=1e-6)
