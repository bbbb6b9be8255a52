"""ctypes binding of libnewsrec_hip.so (C ABI: include/newsrec_hip.h).

This is the only place Python touches the native library.  There is NO fallback: if the
library is missing, or a call fails, the product path raises — a silent eager/CPU
fallback would void every parity claim.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# NR_LIB_PATH: load another build of the library (A/B timing of two builds in one session)
LIB_PATH = os.environ.get("NR_LIB_PATH") or os.path.join(_HERE, "lib", "libnewsrec_hip.so")

c_f32p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_u64 = ctypes.c_uint64
c_ptr = ctypes.c_void_p

# enum nr_rows_map / nr_layout / nr_epilogue / nr_mask_dtype
ROWS_PLAIN, ROWS_GATHER, ROWS_CONV3 = 0, 1, 2
KCONTIG, MNCONTIG = 0, 1
EPI_STORE, EPI_STORE_RELU, EPI_ATOMIC, EPI_SCATTER = 0, 1, 2, 3
MASK_U8, MASK_I64, MASK_F64, MASK_F32 = 0, 1, 2, 3
EPI_STORE_TANH, EPI_ACCUM_GATE, EPI_ACCUM, EPI_SCATTER_STORE = 4, 5, 6, 7
EPI_STORE_GELU, EPI_GELU_GRAD, EPI_SCATTER_ZEROED = 8, 9, 10
GEMM_F32, GEMM_BF16X6, GEMM_BF16 = 0, 1, 2
CELL_LSTM, CELL_GRU = 0, 1
SCORE_RAW, SCORE_LOG_SOFTMAX, SCORE_SIGMOID = 0, 1, 2


class nr_operand(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("ld", c_i64), ("rows", ctypes.c_void_p),
                ("map", c_i32), ("seq_len", c_i32), ("seg", c_i32), ("layout", c_i32)]


class nr_adam_tensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", c_i64), ("lr", c_f32), ("step", c_i64),
                ("step_dev", ctypes.c_void_p), ("lr_dev", ctypes.c_void_p),
                ("row_touched", ctypes.c_void_p), ("row_len", c_i64)]


# name -> argtypes (restype int32 unless listed in _RESTYPES)
_SIGS = {
    "nr_gemm_f32": [c_i64, c_i64, c_i64, ctypes.POINTER(nr_operand), ctypes.POINTER(nr_operand),
                    c_ptr, c_i64, c_ptr, c_i32, ctypes.POINTER(nr_operand), c_i64, c_i32, c_i32, c_ptr],
    "nr_gemm_f32_dyn": [c_i64, c_i64, c_i64, ctypes.POINTER(nr_operand), ctypes.POINTER(nr_operand),
                        c_ptr, c_i64, c_ptr, c_i32, ctypes.POINTER(nr_operand), c_i64, c_i32, c_ptr, c_ptr, c_i32,
                        c_ptr],
    "nr_gemm_f32_dyn_cus": [c_i64, c_i64, c_i64, ctypes.POINTER(nr_operand), ctypes.POINTER(nr_operand),
                            c_ptr, c_i64, c_ptr, c_i32, ctypes.POINTER(nr_operand), c_i64, c_i32, c_ptr, c_ptr, c_i32,
                            c_i32, c_ptr],
    "nr_gemm_f32_ws": [c_i64, c_i64, c_i64, ctypes.POINTER(nr_operand), ctypes.POINTER(nr_operand),
                       c_ptr, c_i64, c_ptr, c_i32, ctypes.POINTER(nr_operand), c_i64, c_i32, c_ptr, c_ptr, c_i32,
                       c_i32, c_ptr, c_i64, c_ptr, ctypes.POINTER(c_i32), c_ptr],
    "nr_gemm_splitk_workspace": [],
    "nr_score_nll_fwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_score_nll_workspace": [c_i64],
    "nr_score_nll_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_i32, c_i32, c_ptr, c_i64,
                         c_ptr, c_i64, c_ptr],
    "nr_unique_rows": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                       c_ptr],
    "nr_segment_rows_sum": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                            c_ptr],
    "nr_segment_rows_sum_multi": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                  c_ptr],
    "nr_unique_rows_zero_absent": [c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_ptr],
    "nr_segment_rows_sum_workspace": [c_i64, c_i64],
    "nr_unique_rows_workspace": [c_i64],
    "nr_segment_rows_sum_conv3": [c_ptr, c_i64, c_i64, c_i32, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr,
                                  c_i64, c_ptr],
    "nr_cnn_pack_weights": [c_ptr, c_ptr, c_ptr, c_i32, c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_cnn_unpack_grads": [c_ptr, c_ptr, c_ptr, c_i32, c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_cnn_keypool_fwd": [c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i32, c_ptr, c_i32, c_i64, c_i32, c_i32, c_f32, c_i32,
                           c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_ptr],
    "nr_cnn_keypool_workspace": [c_i64, c_i32],
    "nr_cnn_keypool_bwd": [c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i32, c_i64, c_i32, c_i32, c_i32, c_f32, c_i32,
                           c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i64,
                           c_ptr, c_i64, c_ptr],
    "nr_conv3_rows_fwd": [c_ptr, c_i64, c_i32, c_i32, c_ptr, c_i64, c_i32, c_ptr, c_i32, c_ptr, c_i64, c_ptr],
    "nr_mha_user_pool_fwd": [c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_ptr, c_ptr,
                             c_i64, c_i32, c_ptr],
    "nr_mha_attn_fwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32,
                        c_f32, c_ptr, c_i64, c_ptr],
    "nr_mha_attn_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32,
                        c_f32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr],
    "nr_attn_pool_fwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_ptr, c_ptr, c_f32, c_f32, c_u64,
                         c_u64, c_ptr, c_i64, c_i32, c_i32, c_f32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr],
    "nr_attn_pool_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_ptr, c_ptr, c_f32, c_u64, c_u64,
                         c_ptr, c_i64, c_i32, c_i32, c_f32, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64,
                         c_ptr, c_i64, c_i32, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_seq_pool_fwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i32, c_ptr, c_i32, c_i64, c_i32, c_i32, c_f32, c_ptr,
                        c_i64, c_ptr, c_ptr],
    "nr_seq_pool_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i32, c_ptr, c_i32, c_i64, c_i32, c_i32, c_f32, c_ptr,
                        c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_ptr, c_ptr],
    "nr_rnn_fwd": [c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_i32, c_i64, c_i32,
                   c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr],
    "nr_rnn_bwd": [c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i32, c_i32, c_i64, c_i32, c_i32, c_ptr, c_i64,
                   c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr],
    "nr_score_fwd": [c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i64, c_i32, c_i32, c_i32, c_ptr, c_ptr],
    "nr_score_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i32, c_i32, c_i32, c_ptr, c_i64, c_ptr,
                     c_i64, c_ptr],
    "nr_adam": [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_i64, c_ptr, c_f32, c_ptr],
    "nr_embedding_fwd": [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr, c_ptr],
    "nr_embedding_bwd": [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_ptr],
    "nr_rows_add_ordered": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    "nr_transpose_f32": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    "nr_xsoftmax_fwd": [c_ptr, c_ptr, c_i32, c_i64, c_i64, c_ptr, c_ptr],
    "nr_xsoftmax_bwd": [c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_ptr],
    "nr_gather_rows_f32": [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    "nr_colsum": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr],
    "nr_colsum_ws": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_colsum_workspace": [c_i64, c_i64],
    "nr_mha_pool_fwd": [c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_ptr, c_ptr, c_f32, c_f32,
                        c_u64, c_u64, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i32,
                        c_ptr],
    "nr_mha_pool_bwd": [c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_ptr, c_ptr, c_f32, c_u64,
                        c_u64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64,
                        c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i32, c_ptr, c_i64, c_i64, c_ptr,
                        c_i32, c_ptr],
    "nr_form_train_batch": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i64,
                            c_i32, c_i32, c_i32, c_i32, c_u64, c_u64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                            c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_rng_take": [c_ptr, c_ptr, c_u64, c_ptr],
    "nr_form_eval_batch": [c_i64, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_i32, c_i32,
                           c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_gather_news_rows": [c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i32, c_ptr, c_ptr, c_ptr, c_ptr],
    "nr_score_ragged": [c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i32, c_i32, c_ptr,
                        c_ptr, c_ptr],
    "nr_impression_metrics": [c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i32, c_ptr, c_ptr, c_ptr],
    "nr_bert_embed_fwd": [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i32, c_i32, c_ptr, c_ptr, c_f32,
                          c_f32, c_u64, c_u64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr],
    "nr_bert_embed_bwd": [c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_i32, c_i32, c_ptr, c_f32, c_u64, c_u64,
                          c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr],
    "nr_bert_add_ln_fwd": [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_f32, c_f32, c_u64, c_u64,
                           c_ptr, c_ptr, c_i64, c_ptr, c_ptr],
    "nr_bert_add_ln_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i32, c_ptr, c_f32, c_u64, c_u64, c_ptr, c_ptr,
                           c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr],
    "nr_bert_attn_fwd": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, c_i64, c_i32, c_i32, c_f32, c_u64, c_u64,
                         c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i32, c_ptr],
    "nr_bert_attn_keep_words": [c_i64, c_i32, c_i32],
    "nr_bert_attn_bwd_workspace": [c_i64, c_i32, c_i32],
    "nr_bert_attn_bwd": [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, c_i64, c_i32, c_i32, c_f32, c_u64, c_u64,
                         c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i32, c_ptr],
    "nr_tanh_bwd": [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i32, c_ptr, c_i64, c_ptr],
    "nr_adam_multi": [ctypes.POINTER(nr_adam_tensor), c_i32, c_f32, c_f32, c_f32, c_f32, c_f32, c_ptr],
    "nr_adam_multi_step": [ctypes.POINTER(nr_adam_tensor), c_i32, c_f32, c_f32, c_f32, c_f32, c_f32, c_ptr,
                           c_ptr],
    "nr_build_hash": [],
}

_RESTYPES = {"nr_segment_rows_sum_workspace": c_i64, "nr_bert_attn_keep_words": c_i64, "nr_unique_rows_workspace": c_i64, "nr_bert_attn_bwd_workspace": c_i64,
             "nr_colsum_workspace": c_i64, "nr_score_nll_workspace": c_i64,
             "nr_gemm_splitk_workspace": c_i64, "nr_cnn_keypool_workspace": c_i64,
             "nr_build_hash": ctypes.c_char_p}

# enum nr_batch_flags / nr_metric_flags
BATCH_REVERSE_HISTORY, BATCH_SHUFFLE_POS, BATCH_CURSOR = 1, 2, 4
METRIC_ONE_CLASS, METRIC_NONBINARY = 1, 2

_lib = None


class HipError(RuntimeError):
    pass


def _expected_hash():
    """Hash of the sources next to the package (build.py's source_hash), or None when the tree
    carries no sources (an installed library) or NR_LIB_PATH points at another build."""
    if os.environ.get("NR_LIB_PATH"):
        return None
    build_py = os.path.join(os.path.dirname(_HERE), "build.py")
    if not os.path.exists(build_py):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_newsrec_build", build_py)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_hash()


def load():
    """Load (once) and return the ctypes library.  Raises if it is missing or was built from
    other sources than the ones in this tree (build provenance, see build.py)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipError("libnewsrec_hip.so not built (%s): run __graft_entry__.build()" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        lib.nr_build_hash.restype = ctypes.c_char_p
        lib.nr_build_hash.argtypes = []
        built = lib.nr_build_hash().decode()
        want = _expected_hash()
        if want is not None and built != want:
            raise HipError("libnewsrec_hip.so was built from other sources (hash %s, tree %s): run "
                           "__graft_entry__.build()" % (built, want))
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, c_i32)
        _lib = lib
    return _lib


def declared_symbols():
    return list(_SIGS)


def register(name, argtypes):
    _SIGS[name] = argtypes
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.argtypes = argtypes
        fn.restype = c_i32


def check(rc, name):
    if rc != 0:
        if rc <= -1000:
            raise HipError("%s: invalid argument %d" % (name, -1000 - rc))
        raise HipError("%s failed: hipError %d" % (name, -rc))


def call(name, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)


def stream_ptr(t=None):
    dev = t.device if t is not None else torch.device("cuda", torch.cuda.current_device())
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def require_gpu(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise HipError("newsrec_amd kernels run on the GPU only (got a %s tensor)" % t.device)


def operand(t, ld=None, rows=None, mapping=ROWS_PLAIN, seq_len=1, seg=1, layout=KCONTIG):
    return nr_operand(t.data_ptr(), ld if ld is not None else t.stride(-2) if t.dim() >= 2 else t.shape[-1],
                      rows.data_ptr() if rows is not None else 0, mapping, seq_len, seg, layout)
