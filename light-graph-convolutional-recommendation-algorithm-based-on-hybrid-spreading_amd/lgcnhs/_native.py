"""ctypes binding of ``liblgcnhs.so`` (the C ABI declared in ``include/lgcnhs.h``).

The library is built in-tree (``lib/liblgcnhs.so``) by ``lgcnhs.build``. It is loaded
after ``torch`` so that its ``libamdhip64.so.7`` dependency binds to the HIP runtime
torch already mapped (same soname): device pointers and the ``hipStream_t`` of
``torch.cuda.current_stream()`` are then valid on both sides.

There is no CPU fallback anywhere in the product path: if the library is missing, fails
to load, or no GPU is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the library: shared HIP runtime)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "liblgcnhs.so")
# measurement builds (scripts/ab_*): another build of the same library
LIB_PATH = os.environ.get("LGCNHS_LIB_PATH") or LIB_PATH

LG_OK = 0
LG_ACC_NONE, LG_ACC_FIRST, LG_ACC_MID, LG_ACC_LAST, LG_ACC_ONLY = 0, 1, 2, 3, 4
LG_EXCL_DROP, LG_EXCL_NONE = 0, 1
ABI_VERSION = 15

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_sz = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/lgcnhs.h one to one
SIGNATURES = {
    "lg_abi_version": (ctypes.c_int, []),
    "lg_last_error": (ctypes.c_char_p, []),
    "lg_csr_rowptr_from_sorted": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp]),
    "lg_gcn_norm_f32": (ctypes.c_int, [_vp, _i64, _vp, _vp]),
    "lg_gcn_edge_weight_f32": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp, _vp]),
    "lg_spmm_layer_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _f32, _i64, _vp],
    ),
    "lg_spmm_layer_live_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _f32, _i64, _vp,
         _vp],
    ),
    "lg_spmm_long_rows_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32,
         _f32, _vp, _vp],
    ),
    "lg_spmm_layer_rows_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _i32, _f32, _i64, _vp,
         _vp],
    ),
    "lg_spmm_long_rows_masked_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32,
         _f32, _vp, _vp, _vp],
    ),
    "lg_mark_neighbors_u8": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "lg_score_topk_ws_bytes": (_sz, [_i64, _i64, _i32, _i32, _i32]),
    "lg_score_topk_screened_ws_bytes": (_sz, [_i64, _i64, _i32, _i32, _i32]),
    "lg_score_topk_f32": (
        ctypes.c_int,
        [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _f32, _i32, _i32, _vp, _vp, _vp, _sz, _vp],
    ),
    "lg_score_topk_screened_f32": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _f32, _i32, _i32, _vp, _vp, _vp,
         _sz, _vp],
    ),
    "lg_score_dense_f32": (
        ctypes.c_int,
        [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _f32, _vp, _i64, _vp],
    ),
    "lg_spread_general_f64": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp]),
    "lg_hybrid_weight_f64": (ctypes.c_int, [_vp, _vp, _i64, _f64, _i32, _vp, _vp]),
    "lg_spread_hybrid_ws_bytes": (_sz, [_i64, _i64]),
    "lg_spread_hybrid_f64": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _f64, _vp, _vp,
                                            _sz, _vp]),
    "lg_spread_resource_f64": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp]),
    "lg_rows_topk_f64": (
        ctypes.c_int,
        [_vp, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _vp],
    ),
    "lg_hybrid_recip_f64": (ctypes.c_int, [_vp, _i64, _f64, _vp, _vp, _vp]),
    "lg_inv_degree_f64": (ctypes.c_int, [_vp, _i64, _vp, _vp]),
    "lg_spread_group_cursor": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _vp,
                                              _vp, _vp, _vp, _vp]),
    "lg_spread_group_bound": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i32, _vp, _vp]),
    "lg_spread_group_units": (ctypes.c_int, [_vp, _i64, _i32, _i32, _i32, _i32, _i64, _vp, _vp]),
    "lg_spread_group_rows_ws_bytes": (_sz, [_i64, _i32]),
    "lg_spread_group_rows_f64": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _vp,
         _vp, _vp, _vp, _sz, _vp],
    ),
    "lg_spread_tile_seek": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "lg_topk_lists_merge_f64": (ctypes.c_int, [_vp, _vp, _i32, _i64, _i32, _vp, _vp, _vp]),
    "lg_spread_tile_resource_topk_lds_bytes": (_sz, [_i32, _i32, _i32]),
    "lg_spread_tile_resource_topk_f64": (
        ctypes.c_int,
        [_vp, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _vp,
         _i32, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _i64, _i64, _vp]),
    "lg_bound_prep_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "lg_score_chunk_bound": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _vp,
                                            _vp, _i32, _vp]),
    "lg_rec_hits": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _vp, _vp, _vp]),
    "lg_rec_pair_overlap": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _vp]),
    "lg_rec_intra_similarity_f64": (
        ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _i64, _vp, _vp]),
}

# the test-reference entry points (include/lgcnhs_ref.h), exported only by
# lib/liblgcnhs_ref.so: never bound to the product library
REF_LIB_PATH = os.path.join(PKG_DIR, "lib", "liblgcnhs_ref.so")
REF_SIGNATURES = {
    "lg_spread_tile_cursor": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "lg_spread_tile_bound": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "lg_spread_tile_rows_ws_bytes": (_sz, [_i64]),
    "lg_spread_tile_rows_f64": (
        ctypes.c_int,
        [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i32, _i32, _vp, _i64, _vp, _vp, _vp, _vp,
         _vp, _sz, _vp],
    ),
    "lg_spread_tile_resource_f64": (
        ctypes.c_int,
        [_vp, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _i64, _vp],
    ),
    "lg_tile_topk_f64": (
        ctypes.c_int,
        [_vp, _i64, _i64, _i32, _i32, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp],
    ),
}

_lib = None
_ref = None
_lock = threading.Lock()


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the native library; raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"lgcnhs native library not found at {path}; run "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
            )
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.lg_abi_version()
        if ver != ABI_VERSION:
            raise RuntimeError(f"liblgcnhs ABI {ver} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def lib() -> ctypes.CDLL:
    return _lib if _lib is not None else load_library()


def ref_lib() -> ctypes.CDLL:
    """The test-reference build (lib/liblgcnhs_ref.so: the product library plus the
    per-tile reference paths of include/lgcnhs_ref.h), for tests only; its entry points
    report errors through its own lg_last_error (use ref_check)."""
    global _ref
    with _lock:
        if _ref is None:
            if not os.path.exists(REF_LIB_PATH):
                raise RuntimeError(f"test-reference library not found at {REF_LIB_PATH}")
            r = ctypes.CDLL(REF_LIB_PATH)
            for name, (res, args) in {**SIGNATURES, **REF_SIGNATURES}.items():
                fn = getattr(r, name)
                fn.restype = res
                fn.argtypes = args
            if r.lg_abi_version() != ABI_VERSION:
                raise RuntimeError("liblgcnhs_ref ABI mismatch")
            _ref = r
        return _ref


def ref_check(status: int, what: str) -> None:
    if status != LG_OK:
        msg = ref_lib().lg_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def check(status: int, what: str) -> None:
    if status != LG_OK:
        msg = lib().lg_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def require_gpu(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(
            f"{name} must be a GPU tensor: the lgcnhs hot path has no CPU fallback"
        )


def ptr(t) -> ctypes.c_void_p:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
