"""ctypes binding of libpcseg.so, the gfx950 HIP library behind include/pcseg.h.

The library is built in-tree by `csrc/Makefile` (see `__graft_entry__.build`).
There is no CPU fallback: if the library is missing or a GPU op is called on a
CPU tensor, the call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCS_LIB: another build of the library (A/B scripts only)
LIB_PATH = os.environ.get('PCS_LIB') or os.path.join(_HERE, 'libpcseg.so')

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_longlong
F32 = ctypes.c_float
F64 = ctypes.c_double


QMAX = 4     # PCS_GEO_MAX_QUERIES


class GeoLevel(ctypes.Structure):
    """pcs_geo_level (include/pcseg.h): one level of a native geometry plan."""
    _fields_ = [('C', ctypes.c_int64), ('nq', ctypes.c_int64), ('r2', ctypes.c_double * QMAX),
                ('K', ctypes.c_int64 * QMAX), ('on_self', ctypes.c_int64 * QMAX),
                ('fps_idx', ctypes.c_void_p), ('cent', ctypes.c_void_p), ('ball', ctypes.c_void_p * QMAX),
                ('ball_off', ctypes.c_void_p * QMAX), ('ball_ent', ctypes.c_void_p * QMAX),
                ('nn_idx', ctypes.c_void_p), ('nn_dist', ctypes.c_void_p), ('nn_off', ctypes.c_void_p),
                ('nn_ent', ctypes.c_void_p), ('event', ctypes.c_void_p)]


class Operand(ctypes.Structure):
    """pcs_operand (include/pcseg.h): an engine GEMM operand and its on-load transform."""
    _fields_ = [('data', P), ('ld', ctypes.c_int), ('mode', ctypes.c_int),
                ('s', P), ('t', P), ('act', ctypes.c_int), ('slope', ctypes.c_float),
                ('z', P), ('ldz', ctypes.c_int),
                ('mean', P), ('inv', P), ('alpha', P), ('kb', P),
                ('arg', P), ('pool_k', ctypes.c_int)]


class InverseMap(ctypes.Structure):
    """pcs_inverse_map (include/pcseg.h): one neighbour table of a batched inverse-map call."""
    _fields_ = [('idx', P), ('per_batch', ctypes.c_int), ('targets', ctypes.c_int), ('offsets', P),
                ('entries', P)]


# the C ABI these bindings are written for (include/pcseg.h pcs_abi_version): 4 = round 6
# (pcs_knn_order / pcs_knn_pruned added; round 5: pcs_group_bwd_csr / pcs_interp_bwd_csr take n_slots)
ABI_VERSION = 4
OP_PLAIN, OP_BNACT, OP_BNBWD, OP_POOLBWD = 0, 1, 2, 3
OPP = ctypes.POINTER(Operand)

# name -> argtypes (all return int status), mirrors include/pcseg.h
SIGNATURES = {
    'pcs_fps': [P, I32, I32, I32, P, P, P, P],
    'pcs_ball_query': [P, P, I32, I32, I32, F32, I32, P, P],
    'pcs_knn_select': [P, P, I32, I32, I32, I32, P, P, P],
    'pcs_knn': [P, I32, I32, I32, I32, P, P],
    'pcs_knn_workspace': [I32, I32, P],
    'pcs_dropout_bwd': [P, I32, I32, I32, ctypes.c_double, I64, P, I32, P],
    'pcs_copy_cols': [P, I32, I32, I32, P, I32, P],
    'pcs_knn_ws': [P, I32, I32, I32, I32, P, P, ctypes.c_size_t, P],
    'pcs_knn_seeded': [P, I32, I32, I32, I32, P, I32, P, P, ctypes.c_size_t, P],
    'pcs_knn_order': [P, I32, I32, I32, P, P],
    'pcs_knn_pruned_workspace': [I32, I32, I32, P],
    'pcs_knn_pruned': [P, I32, I32, I32, I32, P, P, I32, P, P, ctypes.c_size_t, P],
    'pcs_group_fwd': [P, P, P, P, I32, I32, I32, I32, I32, F32, I32, P, I32, P],
    'pcs_maxk_fwd': [P, I64, I32, I32, P, P, P],
    'pcs_maxk_bwd': [P, P, I64, I32, I32, P, P],
    'pcs_interp_fwd': [P, P, P, I32, I32, I32, I32, P, I32, I32, P],
    'pcs_interp_cat_fwd': [P, I32, P, P, P, I32, I32, I32, I32, P, I32, P],
    'pcs_edge_fwd': [P, P, I32, I32, I32, I32, P, I32, P],
    'pcs_edge_bwd': [P, I32, P, P, I32, I32, I32, I32, P, P],
    # shared-MLP engine
    'pcs_gemm_row_blocks': [I32, I32],
    'pcs_gemm_row_blocks_dgrad': [I32, I32],
    'pcs_probe_begin': [],
    'pcs_probe_end': [],
    'pcs_probe_get': [I32, ctypes.c_char_p, I32, P, P, P],
    'pcs_probe_replay': [ctypes.c_char_p, I32, P, P],
    'pcs_probe_stream': [I32, P],
    'pcs_probe_times': [I32, P, P],
    'pcs_spin': [I32, P],
    'pcs_mlp_workspace': [I32, I32, I32, ctypes.c_char_p, I32, I32, I32, P],
    'pcs_mlp_forward': [P, I32, I32, I32, ctypes.c_char_p, I32, I32, P, I32, P, P, ctypes.c_size_t, P],
    'pcs_mlp_backward': [P, I32, I32, I32, ctypes.c_char_p, I32, I32, P, P, I32, P, I32, P, ctypes.c_size_t, P],
    'pcs_mlp_backward_deferred': [P, I32, I32, I32, ctypes.c_char_p, I32, I32, P, P, I32, P, I32, P,
                                  ctypes.c_size_t, P],
    'pcs_wgrad_lane': [P],
    'pcs_wgrad_lane_join': [P],
    'pcs_geometry_stream': [P],
    'pcs_operand_size': [],
    'pcs_mlp_layer_size': [],
    'pcs_gemm_rows': [OPP, I32, I32, P, I32, P, P, I32, I32, P, OPP, P, P],
    'pcs_gemm_rows_kmajor': [OPP, I32, I32, P, I32, P, I32, I32, OPP, P, P],
    'pcs_gemm_rows_kmajor_variant': [OPP, I32, I32, P, I32, P, I32, I32, OPP, P, I32, P],
    'pcs_gemm_rows_variant': [OPP, I32, I32, P, I32, P, P, I32, I32, P, I32, P],
    'pcs_set_kernel_variant': [I32],
    'pcs_gemm_nt': [P, I32, P, I32, I32, I32, I32, P, P, I32, P, P],
    'pcs_gemm_nt_row_tiles': [I32],
    'pcs_wgrad_workspace': [I32, I32, I32, P],
    'pcs_wgrad': [OPP, I32, OPP, I32, I32, P, P, P, ctypes.c_size_t, P],
    'pcs_bn_finalize': [P, I32, I32, I64, P, P, F32, F32, P, P, P, P, P, P, P],
    'pcs_bn_bwd_finalize': [P, I32, I32, I64, P, P, P, P, P, P, I32, P],
    'pcs_bn_bwd_reduce_blocks': [I32],
    'pcs_bn_bwd_reduce': [P, I32, P, I32, I32, I32, P, P, P, P, I32, F32, P, P],
    'pcs_pool_fwd': [P, I32, I64, I32, P, P, I32, F32, P, P, P],
    'pcs_pool_bwd_reduce_blocks': [I64],
    'pcs_pool_bwd_reduce': [P, P, P, I32, I64, I32, P, P, P, P, I32, F32, P, P],
    'pcs_bn_act': [P, I32, I32, I32, P, P, I32, F32, P, I32, P],
    # sliding-window inference
    'pcs_window_merge': [P, P, I32, I64, I32, I64, I64, P, P, P],
    # metrics
    'pcs_seg_metrics': [P, P, I32, P, I32, I32, I32, P, P, P, P, P],
    # fused EdgeConv
    'pcs_edgeconv_workspace': [I32, I32, I32, I32, I32, P],
    'pcs_edgeconv_fwd': [P, I32, I32, P, I32, I32, I32, P, I32, P, P, P, P, P, F32, F32, F32,
                         P, P, P, P, P, P, P, P, P, I32, P, ctypes.c_size_t, P],
    'pcs_edgeconv_bwd': [P, I32, I32, P, P, I32, I32, I32, P, I32, P, P, P, P, P, P, F32,
                         P, I32, P, I32, P, P, P, P, ctypes.c_size_t, P],
    # inverse neighbour maps
    'pcs_inverse_index_workspace': [I64, I64, P],
    'pcs_inverse_index': [P, I32, I32, I32, P, P, P, ctypes.c_size_t, P],
    'pcs_inverse_index_batch_workspace': [P, I32, I32, P],
    'pcs_inverse_index_batch': [P, I32, I32, P, ctypes.c_size_t, P],
    'pcs_group_bwd_csr': [P, I32, P, P, I32, I32, I32, I64, P, P],
    'pcs_interp_bwd_csr': [P, I32, I32, P, P, P, I32, I32, I32, I64, P, P],
    # block batches
    'pcs_gather_blocks': [P, P, P, I64, P, P, P],
    'pcs_pad_onehot': [P, I32, P, P, P, I32, I32, I32, P, P, P],
    # optimizer
    'pcs_adam': [P, P, P, P, I64, F32, F32, F32, F32, F32, F32, F32, P],
    'pcs_geometry_plan_workspace': [I32, I32, P, I32, I32, I32, P],
    'pcs_geometry_plan': [P, I32, I32, P, P, I32, I32, I32, P, P, ctypes.c_size_t, P],
    'pcs_adam_dev': [P, P, P, P, I64, F32, F32, F32, F64, F64, F64, F32, F32, P, P],
    # loss
    'pcs_masked_ce_blocks': [I32, I32],
    'pcs_masked_ce': [P, I32, P, I32, I32, P, I32, I32, I32, P, P, P, P],
}

_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and type the library; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f'pcseg: HIP library not built ({LIB_PATH} missing); '
                                   'run `python -c "import __graft_entry__ as g; g.build()"` or '
                                   '`make -C 3d-semantic-segmentation-benchmark_amd/csrc`')
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            lib.pcs_last_error.restype = ctypes.c_char_p
            lib.pcs_last_error.argtypes = []
            lib.pcs_abi_version.restype = ctypes.c_int
            if lib.pcs_abi_version() != ABI_VERSION:
                raise RuntimeError(f'pcseg: {LIB_PATH} has ABI {lib.pcs_abi_version()}, these bindings expect '
                                   f'{ABI_VERSION}; rebuild the library')
            for name, args in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = ctypes.c_int
            _lib = lib
    return _lib


_raw_stream = torch._C._cuda_getCurrentRawStream


def stream_ptr(device: torch.device | None = None) -> int:
    """hipStream_t of the current stream of `device` (a torch.device, an index or None = the
    current device), without building a torch.cuda.Stream object (host enqueue cost)."""
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = device.index if device.index is not None else torch.cuda.current_device()
    return _raw_stream(idx)


_fns: dict = {}


def call(name: str, *args) -> None:
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(load(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f'{name} failed ({rc}): {load().pcs_last_error().decode(errors="replace")}')


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def check_cuda(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError('pcseg ops run only on the GPU (no CPU fallback); got a CPU tensor')
