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


def test_bert_attn_bwd_workspace_sizes():
    """Host-side size query (no device call): D per (query, head) rounded to 16 B, plus for four-wave
    launches (L > 96) the padded dS tiles of the stored-dS backward (4 KB per (sequence, head, key
    tile, query tile))."""
    from newsrec_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.nr_bert_attn_bwd_workspace
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]

    def want(nseq, L, heads):
        d = (nseq * L * heads + 3) // 4 * 4
        nkb = (L + 31) // 32
        return 4 * (d + (nseq * heads * nkb * nkb * 1024 if L > 96 else 0))
    for nseq, L, heads in [(7, 30, 2), (5, 1, 1), (3, 96, 2), (3, 97, 2), (2, 140, 3), (32, 501, 12)]:
        assert f(nseq, L, heads) == want(nseq, L, heads), (nseq, L, heads)
    assert f(32, 501, 12) - 4 * 32 * 501 * 12 == 402_653_184   # the XFormer user sequence's dS tiles
    assert f(-1, 30, 2) == 0 and f(2, 0, 2) == 0 and f(2, 30, 0) == 0
