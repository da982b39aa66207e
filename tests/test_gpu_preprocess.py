"""pcseg.data.preprocess_batch_to_train_format (pcs_pad_onehot) against the reference's
harness-B batch builder (Training/train_model.py:89-171): golden fixtures captured from
the reference, same torch RNG seeding (the sampling perms are the reference's own
`torch.randperm` calls).  Integer/byte work: bit-exact."""
import pytest
import torch

from pcseg.data import preprocess_batch_to_train_format
from test_oracle_golden import PREPROCESS_CASES, T, _preprocess_inputs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('tag,kw', PREPROCESS_CASES)
def test_preprocess_matches_reference_golden(golden, tag, kw):
    z = golden('preprocess.npz')
    x, y, mapping = _preprocess_inputs(z)
    torch.manual_seed(int(z[f'{tag}_seed']))
    bi, lab, lengths, cont = preprocess_batch_to_train_format(x, y, mapping, **kw)
    assert bi.is_cuda and lab.is_cuda
    assert bi.shape == T(z[f'{tag}_x']).shape and bi.shape[1] == x[0].shape[1]     # (B, D, L) view
    assert torch.equal(bi.cpu().contiguous(), T(z[f'{tag}_x']))
    assert torch.equal(lab.cpu(), T(z[f'{tag}_label']))
    assert torch.equal(lengths, T(z[f'{tag}_len']))
    assert cont == bool(z[f'{tag}_cont'])


def test_preprocess_errors_like_reference():
    x = [torch.zeros(3, 2)]
    with pytest.raises(ValueError):
        preprocess_batch_to_train_format(x, [['a', 'b', 'zz']], ['a', 'b'])
    with pytest.raises(ValueError):
        preprocess_batch_to_train_format(x, [['a', 'b', 'a']], ['a', 'b'], sampling=1.5)
    # names beyond the cut are never looked up (the reference breaks out of its loop first)
    bi, lab, n, cont = preprocess_batch_to_train_format(x, [['a', 'b', 'zz']], ['a', 'b'], cut=2)
    assert lab.shape == (1, 2, 2) and int(n[0]) == 2 and cont is False
