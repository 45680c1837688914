"""The C-ABI library loads and exports exactly what include/lgcnhs.h declares; argument
validation rejects bad calls before any launch. CPU only (no kernel runs)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, REPO


def declared_functions(header="lgcnhs.h"):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lg_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from lgcnhs import _native as N
    assert declared_functions() == sorted(N.SIGNATURES)
    assert declared_functions("lgcnhs_ref.h") == sorted(N.REF_SIGNATURES)


def test_reference_paths_only_in_the_reference_build():
    """The per-tile reference paths (include/lgcnhs_ref.h) are exported by
    lib/liblgcnhs_ref.so for the tests and NOT by the product library."""
    from lgcnhs import _native as N
    prod = N.load_library()
    ref = N.ref_lib()
    for name in declared_functions("lgcnhs_ref.h"):
        assert not hasattr(prod, name), name
        assert hasattr(ref, name), name
    for name in declared_functions():
        assert hasattr(ref, name), name
    assert ref.lg_abi_version() == prod.lg_abi_version() == N.ABI_VERSION


def test_library_exports_every_symbol():
    from lgcnhs import _native as N
    lib = N.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.lg_abi_version() == N.ABI_VERSION


def test_integration_table_lists_every_product_export():
    """INTEGRATION.md §2 names every function of include/lgcnhs.h by its full name."""
    txt = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = txt[txt.index("## 2. The C ABI"):txt.index("## 3.")]
    named = set(re.findall(r"`(lg_[a-z0-9_]+)`", sec))
    missing = [f for f in declared_functions() if f not in named]
    assert not missing, missing


def test_argument_validation_without_gpu():
    from lgcnhs import _native as N
    lib = N.load_library()
    z = ctypes.c_void_p(0)
    one = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    st = lib.lg_spmm_layer_f32(one, one, one, z, one, z, z, z, z, 10, 0, 48, 0, 1.0, 0, z)
    assert st == 1 and b"dim" in lib.lg_last_error()
    st = lib.lg_score_topk_f32(one, one, 4, 4, 64, z, z, -1024.0, 0, 1, one, one, z, 0, z)
    assert st == 1 and b"k=0" in lib.lg_last_error()
    st = lib.lg_score_topk_f32(one, one, 4, 4, 64, one, z, -1024.0, 5, 1, one, one, z, 0, z)
    assert st == 1
    st = lib.lg_rows_topk_f64(one, 4, 4, 4, z, z, 0, z, z, 7, 3, one, one, z)
    assert st == 1 and b"excl_mode" in lib.lg_last_error()
    st = lib.lg_spmm_layer_f32(one, one, one, z, one, one, z, z, z, 5, 0, 64, 3, 4.0, 0, z)
    assert st == 1  # LAST needs acc/out
    st = lib.lg_spmm_layer_live_f32(one, one, one, z, one, z, z, z, z, 10, 0, 64, 0, 1.0, 0, z, z)
    assert st == 1 and b"live" in lib.lg_last_error()
    st = lib.lg_spmm_layer_live_f32(one, one, one, z, one, z, z, z, z, 10, 0, 48, 0, 1.0, 0, one, z)
    assert st == 1 and b"lg_spmm_layer_live_f32" in lib.lg_last_error()
    # the walk's 32-bit stream positions: the caller's bounds are checked before any launch
    args = [one, one, one, 10, one, one, 5, one, one, 0, 2048, 2048, z, z, 0, z, 0, z, 0,
            z, z, z, 20, 1, one, one]
    st = lib.lg_spread_tile_resource_topk_f64(*args, 2**31, 0, z)
    assert st == 1 and b"32-bit positions" in lib.lg_last_error()
    st = lib.lg_spread_tile_resource_topk_f64(*args, 1000, 2**33, z)
    assert st == 1 and b"32-bit positions" in lib.lg_last_error()
    # the chunk-bound kernel's per-chunk norm table holds 64 chunks: wider tiles are refused
    st = lib.lg_score_chunk_bound(one, one, 10, one, one, 64, 0, 4097, one, z, 0, z)
    assert st == 1 and b"width 4097 > 4096" in lib.lg_last_error()
    # the dense spreading entries dereference their column arrays: NULL is refused, not faulted
    st = lib.lg_spread_hybrid_f64(one, z, one, one, one, 4, 4, 0.5, one, one, 1 << 20, z)
    assert st == 1 and b"lg_spread_hybrid_f64" in lib.lg_last_error()
    st = lib.lg_spread_hybrid_f64(one, one, one, z, one, 4, 4, 0.5, one, one, 1 << 20, z)
    assert st == 1
    st = lib.lg_spread_general_f64(one, z, one, one, 4, 4, one, z)
    assert st == 1 and b"lg_spread_general_f64" in lib.lg_last_error()
    st = lib.lg_spread_resource_f64(one, z, one, 4, 4, one, 4, z)
    assert st == 1 and b"lg_spread_resource_f64" in lib.lg_last_error()
    assert lib.lg_score_topk_ws_bytes(100, 1000, 64, 10, 1) == 0
    assert lib.lg_score_topk_ws_bytes(100, 1000, 64, 10, 4) == 4 * 100 * 10 * 8
    # catalogs of more than 2^20 items: the screened kernel's splits (16-bit tile indices)
    assert lib.lg_score_topk_ws_bytes(100, (1 << 20) + 1, 64, 10, 1) == 2 * 100 * 10 * 8
    assert lib.lg_score_topk_ws_bytes(100, 1 << 20, 64, 10, 1) == 0
    # the screened call: k <= 32 keeps its lists in LDS; above, one slab per user and split
    assert lib.lg_score_topk_screened_ws_bytes(100, 1000, 64, 10, 1) == 0
    assert lib.lg_score_topk_screened_ws_bytes(100, 1000, 64, 64, 1) == 100 * 128 * 8
    assert lib.lg_score_topk_screened_ws_bytes(100, 1000, 64, 100, 3) == \
        3 * 100 * 100 * 8 + 3 * 100 * 256 * 8


def test_missing_library_fails_loudly(tmp_path):
    from lgcnhs import _native as N
    with pytest.raises(RuntimeError, match="not found"):
        N._lib_backup = N._lib
        try:
            N._lib = None
            N.load_library(str(tmp_path / "nope.so"))
        finally:
            N._lib = N._lib_backup


def test_product_never_imports_oracle():
    """The product package must not import, call or link anything under oracle/."""
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")) or f == "Makefile":
                txt = open(os.path.join(root, f), errors="ignore").read()
                hit = re.search(r"(import\s+oracle|from\s+oracle|lgcn_oracle|liboracle|"
                                r"oracle/build|score_chain\.(so|o)\b)", txt)
                assert not hit, (os.path.join(root, f), hit.group(0))
