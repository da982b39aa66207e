"""pcseg.metrics (csrc/metrics.hip) against the reference's Training/metrics.py: the
golden fixture captured from the reference, and the oracle restatement on larger
random batches (fp32 and uint8 labels, argmax ties, padded lengths).  Counts are
integers: bit-exact."""
import numpy as np
import pytest
import torch

from pcseg import metrics as M
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def T(a):
    return torch.from_numpy(np.array(a))


def test_metrics_match_reference_golden(golden):
    z = golden('metrics.npz')
    p, lab, n = T(z['probs']), T(z['labels']), T(z['lengths'])
    pd, ld = p.to(DEV), lab.to(DEV)
    assert M.overall_accuracy(pd, ld, n) == float(z['oa'])
    assert M.update_accuracy(pd, ld, n) == (int(z['correct']), int(z['total']))
    assert torch.equal(M.confusion_matrix(pd, ld, n), T(z['conf']))
    miou, ious = M.intersection_over_union(pd, ld, n)
    assert miou == float(z['miou']) and torch.equal(ious, T(z['ious']))
    inter, union = M.update_intersection_over_union(pd, ld, n.to(DEV))
    assert torch.equal(inter, T(z['inter'])) and torch.equal(union, T(z['union']))


@pytest.mark.parametrize('u8', [False, True])
def test_metrics_match_oracle_random(u8):
    g = torch.Generator().manual_seed(17 + u8)
    B, N, C = 6, 4096, 14
    logits = torch.randn(B, N, C, generator=g)
    logits[:, ::5, 0] = logits[:, ::5, 9] = 7.0
    p = torch.softmax(logits, -1)
    lab = torch.nn.functional.one_hot(torch.randint(0, C, (B, N), generator=g), C)
    lab = lab.to(torch.uint8) if u8 else lab.float()
    n = torch.tensor([4096, 4000, 1, 0, 2048, 3333], dtype=torch.int32)
    pd, ld = p.to(DEV), lab.to(DEV)
    assert M.update_accuracy(pd, ld, n) == R.update_accuracy(p, lab, n)
    assert torch.equal(M.confusion_matrix(pd, ld, n), R.confusion_matrix(p, lab, n))
    m1, i1 = M.intersection_over_union(pd, ld, n)
    m0, i0 = R.intersection_over_union(p, lab, n)
    assert m1 == m0 and torch.equal(i1, i0)
    a1, b1 = M.update_intersection_over_union(pd, ld, n)
    a0, b0 = R.update_intersection_over_union(p, lab, n)
    assert torch.equal(a1, a0) and torch.equal(b1, b0)


def test_metrics_reject_cpu_and_bad_shapes():
    with pytest.raises(RuntimeError):
        M.overall_accuracy(torch.rand(1, 4, 3), torch.rand(1, 4, 3), torch.tensor([4]))
    with pytest.raises(ValueError):
        M.overall_accuracy(torch.rand(1, 4, 3, device=DEV), torch.rand(1, 4, 2, device=DEV), torch.tensor([4]))
