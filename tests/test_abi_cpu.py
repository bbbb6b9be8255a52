"""CPU-only checks of the C-ABI boundary: the library loads, exports every entry point that
include/newsrec_hip.h declares, and the ctypes signatures cover exactly those entries.
(No compute calls: there is no GPU here.)"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "newsrec_hip.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(nr_\w+)\s*\(", txt, flags=re.M)))


def declared_arity():
    """name -> number of parameters, from the prototypes in the header."""
    txt = open(HEADER).read()
    out = {}
    for m in re.finditer(r"^(?:int|int64_t|const char\*)\s+(nr_\w+)\s*\(([^)]*)\)\s*;", txt, flags=re.M):
        params = [p for p in m.group(2).replace("\n", " ").split(",") if p.strip() and p.strip() != "void"]
        out[m.group(1)] = len(params)
    return out


def test_header_declares_entry_points():
    names = declared()
    assert "nr_gemm_f32" in names and "nr_mha_pool_fwd" in names and "nr_adam" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from newsrec_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in declared():
        assert hasattr(lib, n), "missing export %s" % n


def test_bindings_match_header():
    from newsrec_amd import _lib
    assert sorted(_lib.declared_symbols()) == declared()
    arity = declared_arity()
    assert sorted(arity) == declared()
    for name in declared():
        assert len(_lib._SIGS[name]) == arity[name], "%s: %d ctypes args vs %d in the header" % (
            name, len(_lib._SIGS[name]), arity[name])


def test_product_path_fails_loudly_without_gpu():
    import torch
    from newsrec_amd import _lib, kernels
    t = torch.zeros(4, 4)
    with pytest.raises(_lib.HipError):
        kernels.colsum(t, 4, 4, torch.zeros(4))


def test_library_built_from_this_tree():
    """Build provenance: the hash embedded in the library equals the hash of csrc/ + include/."""
    import importlib.util
    from newsrec_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    spec = importlib.util.spec_from_file_location("nr_build", os.path.join(ROOT, "news-recommendation-mind_amd",
                                                                           "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.nr_build_hash.restype = ctypes.c_char_p
    assert lib.nr_build_hash().decode() == b.source_hash()
