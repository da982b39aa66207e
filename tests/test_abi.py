"""CPU-side checks of the boundary: the C-ABI library loads and exports every symbol
include/pcseg.h declares; the product API mirrors the reference's (names,
signatures, state_dict keys); ops refuse CPU tensors (no silent fallback)."""
import ctypes
import inspect
import os
import re

import pytest
import torch

from conftest import REPO

import pcseg
from pcseg import _lib
from oracle import ref_ops as R

HEADER = os.path.join(REPO, 'include', 'pcseg.h')


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(pcs_[a-z0-9_]+)\s*\(', txt)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    # every typed binding corresponds to a header declaration and vice versa
    assert set(_lib.SIGNATURES) | {'pcs_last_error', 'pcs_abi_version'} == set(syms)
    assert lib.pcs_abi_version() == _lib.ABI_VERSION == 4
    assert lib.pcs_operand_size() == ctypes.sizeof(_lib.Operand)


def test_mlp_layer_record_layout():
    """The engine's packed pcs_mlp_layer records (pcseg.engine._REC) match the C struct."""
    from pcseg import engine
    assert engine._REC.size == 200
    assert _lib.load().pcs_mlp_layer_size() == engine._REC.size
    assert engine._STATIC.size + engine._DYN.size == engine._REC.size


def test_binding_arity_matches_header():
    txt = re.sub(r'/\*.*?\*/', '', open(HEADER).read(), flags=re.S)
    for name, params in re.findall(r'\b(pcs_[a-z0-9_]+)\s*\(([^)]*)\)\s*;', txt):
        params = params.strip()
        n = 0 if params in ('', 'void') else params.count(',') + 1
        if name in _lib.SIGNATURES:
            assert len(_lib.SIGNATURES[name]) == n, name


def test_nm_exports_are_c_abi():
    so = _lib.LIB_PATH
    out = os.popen(f'nm -D --defined-only {so}').read()
    for s in header_symbols():
        assert re.search(rf'\bT {s}$', out, flags=re.M), s


def test_error_path_without_gpu_compute():
    """A bad-size call returns an error code + message without touching the device."""
    lib = _lib.load()
    rc = lib.pcs_fps(None, 1, 0, 4, None, None, None, None)
    assert rc != 0
    assert b'pcs_fps' in lib.pcs_last_error()


def test_ops_refuse_cpu_tensors():
    x = torch.rand(1, 64, 3)
    with pytest.raises(RuntimeError, match='GPU'):
        pcseg.ops.fps(x, 8, torch.zeros(1, dtype=torch.int32))
    with pytest.raises(RuntimeError, match='GPU'):
        pcseg.ops.ball_query(x[:, :8], x, 0.1, 4)


@pytest.mark.parametrize('name', ['PointNetpp', 'PointNeXt', 'DGCNN', 'DGCNNWithColor', 'PointNetSeg',
                                  'SetAbstraction', 'FeaturePropagation', 'InvResMLP', 'MiniPointNet',
                                  'UnitPointNet', 'EdgeConv'])
def test_constructor_signatures_match_reference(name):
    a = inspect.signature(getattr(pcseg, name).__init__)
    b = inspect.signature(getattr(R, name).__init__)
    assert [(p.name, p.default) for p in a.parameters.values()] == \
        [(p.name, p.default) for p in b.parameters.values()]


@pytest.mark.parametrize('ctor', [lambda m: m.PointNetpp(14), lambda m: m.PointNeXt(14),
                                  lambda m: m.DGCNNWithColor(14), lambda m: m.DGCNN(13),
                                  lambda m: m.PointNetSeg(14), lambda m: m.PointNetppMSG(14)])
def test_state_dict_layout_matches_reference(ctor):
    a, b = ctor(pcseg).state_dict(), ctor(R).state_dict()
    assert list(a) == list(b)
    for k in a:
        assert a[k].shape == b[k].shape and a[k].dtype == b[k].dtype, k
    # checkpoints interchange
    ctor(pcseg).load_state_dict(b)


def test_loss_refuses_cpu_tensors():
    with pytest.raises(RuntimeError, match='GPU'):
        pcseg.masked_onehot_cross_entropy(torch.zeros(1, 4, 14), torch.zeros(1, 4, 14, dtype=torch.uint8),
                                          torch.ones(1, dtype=torch.int64))


def test_reduce_rejects_unknown_pooling():
    with pytest.raises(ValueError):
        pcseg.reduce(torch.zeros(1, 2, 3, 4), 'sum')


@pytest.mark.parametrize('name', ['sample', 'group', 'reduce', 'interpolate', 'knn', 'get_graph_feature',
                                  'masked_onehot_cross_entropy'])
def test_functional_signatures_match_reference(name):
    a = inspect.signature(getattr(pcseg, name))
    b = inspect.signature(getattr(R, name))
    assert [(p.name, p.default) for p in a.parameters.values()] == \
        [(p.name, p.default) for p in b.parameters.values()]


def test_engine_abi_argument_checks_without_gpu():
    """The C ABI validates operands before any launch (host-only paths)."""
    lib = _lib.load()
    fake = 0x1000                       # never dereferenced: every call below fails its checks first
    op = _lib.Operand(fake, 12, _lib.OP_PLAIN, None, None, 0, 0.0, None, 0, None, None, None, None, None, 0)
    # weight rows must hold K values, k-major rows N values (unpadded / unaligned rows are fine:
    # the loaders switch to scalar loads)
    assert lib.pcs_gemm_rows(op, 8, 9, fake, 8, None, fake, 32, 32, None, None, None, None) != 0
    assert b'ldw' in lib.pcs_last_error()
    assert lib.pcs_gemm_rows_kmajor(op, 8, 9, fake, 31, fake, 32, 32, None, None, None) != 0
    assert b'ldw' in lib.pcs_last_error()
    # transform modes need K % 4 == 0 and their coefficient vectors
    bad = _lib.Operand(fake, 12, _lib.OP_BNACT, None, None, 0, 0.0, None, 0, None, None, None, None, None, 0)
    assert lib.pcs_gemm_rows(bad, 8, 8, fake, 8, None, fake, 32, 32, None, None, None, None) != 0
    assert b'needs s/t' in lib.pcs_last_error()
    bad = _lib.Operand(fake, 12, 7, None, None, 0, 0.0, None, 0, None, None, None, None, None, 0)
    assert lib.pcs_gemm_rows(bad, 8, 8, fake, 8, None, fake, 32, 32, None, None, None, None) != 0
    assert b'mode' in lib.pcs_last_error()
    # pooled-backward operands need the argmax and 1 <= pool_k <= 256
    pb = _lib.Operand(fake, 32, _lib.OP_POOLBWD, fake, fake, 0, 0.0, fake, 32, fake, None, fake, fake, None, 0)
    assert lib.pcs_wgrad(pb, 32, op, 12, 64, fake, None, None, 0, None) != 0
    assert b'pool_k' in lib.pcs_last_error()
    # the wgrad Y operand cannot be a backward transform
    assert lib.pcs_wgrad(op, 32, pb, 32, 64, fake, None, None, 0, None) != 0
