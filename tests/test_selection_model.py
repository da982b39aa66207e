"""The kernel's selection algorithm (tests/selection_model.py) == CPU torch.topk index sets.

Validates, without a GPU, the emulation the HIP ball-query and 3-NN kernels
implement, including the wave-parallel closed form of
the Hoare partition.
"""
import random

import pytest
import torch

import selection_model as S


def _rows(n, count, seed, inf_frac, dup):
    g = torch.Generator().manual_seed(seed)
    rows = []
    for _ in range(count):
        v = torch.rand(n, generator=g)
        if dup:
            v = (v * 8).floor() / 8             # heavy ties
        v[torch.rand(n, generator=g) < inf_frac] = torch.inf
        rows.append(v)
    return rows


@pytest.mark.parametrize('n,k', [(64, 32), (256, 32), (1000, 32), (1024, 32), (2047, 32), (16, 16),
                                 (64, 3), (16, 3), (191, 3), (2048, 32), (4096, 32), (256, 3), (40, 20)])
@pytest.mark.parametrize('inf_frac,dup', [(0.0, False), (0.97, False), (0.999, False), (0.5, True), (1.0, False)])
def test_selection_matches_torch_topk(n, k, inf_frac, dup):
    count = 6 if n >= 1024 else 12
    for v in _rows(n, count, seed=n * 7 + k, inf_frac=inf_frac, dup=dup):
        ref = sorted(torch.topk(v, k, largest=False, sorted=True)[1].tolist())
        assert S.topk_smallest_set(v.tolist(), k) == ref
        if k * 64 > n:
            assert S.topk_smallest_set(v.tolist(), k, parallel=True) == ref


def test_parallel_partition_equals_serial():
    rnd = random.Random(5)
    for trial in range(300):
        n = rnd.randint(4, 200)
        vals = [rnd.choice([0.1, 0.2, 0.3, float('inf')]) if trial % 2 else rnd.random() for _ in range(n)]
        q = [(v, i) for i, v in enumerate(vals)]
        S.move_median_to_first(q, 0, 1, n // 2, n - 1)
        q2 = list(q)
        c1 = S.partition_serial(q, 1, n, 0)
        c2 = S.partition_parallel(q2, 1, n, q2[0][0])
        assert c1 == c2 and q == q2
