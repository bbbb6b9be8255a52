"""Thin tensor-level wrappers over the C ABI (one function per entry point).

Each wrapper validates shapes/dtypes on the host BEFORE launching (a wrong shape on the
device is a memory fault, not an exception), then calls the kernel on the current stream.
"""
import contextlib
import ctypes
import os
import threading

import torch

from . import _lib as L


def _f32(*ts):
    for t in ts:
        if t is not None and (t.dtype != torch.float32 or not t.is_cuda):
            raise L.HipError("expected a float32 CUDA tensor, got %s on %s" % (t.dtype, t.device))


def _check_rows(rows, limit, name):
    if rows is not None:
        if rows.dtype != torch.int64 or not rows.is_cuda or not rows.is_contiguous():
            raise L.HipError("%s: row table must be a contiguous int64 CUDA tensor" % name)


_PREC_NAMES = {"f32": L.GEMM_F32, "bf16x6": L.GEMM_BF16X6, "bf16": L.GEMM_BF16}
_prec_state = threading.local()


def _env_precision():
    e = os.environ.get("NR_GEMM_PREC", "bf16x6")
    if e not in _PREC_NAMES:
        raise L.HipError("NR_GEMM_PREC must be one of %s, got %r" % (sorted(_PREC_NAMES), e))
    return _PREC_NAMES[e]


def get_gemm_precision():
    """The calling thread's default GEMM arithmetic (L.GEMM_F32 / GEMM_BF16X6 / GEMM_BF16); the
    process default comes from NR_GEMM_PREC ("bf16x6").  The library itself is stateless: every
    nr_gemm_f32 call carries its arithmetic."""
    p = getattr(_prec_state, "mode", None)
    return _env_precision() if p is None else p


def set_gemm_precision(mode):
    """Set the calling thread's default GEMM arithmetic; returns the previous one."""
    if mode not in _PREC_NAMES.values():
        raise L.HipError("invalid GEMM precision %r" % (mode,))
    old = get_gemm_precision()
    _prec_state.mode = int(mode)
    return old


@contextlib.contextmanager
def gemm_precision(mode):
    """``with gemm_precision(L.GEMM_BF16): ...`` — the arithmetic of the GEMMs launched inside
    (autograd Functions record it at forward time, so their backward uses the same)."""
    old = set_gemm_precision(mode)
    try:
        yield
    finally:
        _prec_state.mode = old


def _prec(prec):
    return get_gemm_precision() if prec is None else int(prec)


def gemm(M, N, K, A, B, C, ldc=None, bias=None, epilogue=L.EPI_STORE, c_rows=None,
         pad_row=-1, split_k=1, prec=None, colsum=None):
    """C (op)= A(m,k) B(k,n); A, B, c_rows are nr_operand structs built by ``operand``; ``prec``:
    the GEMM arithmetic (None: the thread default, ``get_gemm_precision``).  ``colsum`` (split-K
    weight gradients with an MN-contiguous A): colsum[m] += Σ_k A[k][m] folded into the GEMM where
    the library can (nr_gemm_f32_ws); returns True then, False when the caller must reduce it."""
    _f32(C, bias, colsum)
    if bias is not None and bias.numel() < N:
        raise L.HipError("gemm: bias has %d < N=%d entries" % (bias.numel(), N))
    if colsum is not None and (colsum.numel() < M or not colsum.is_contiguous()):
        raise L.HipError("gemm: colsum must be a contiguous [M] float tensor")
    if epilogue == L.EPI_ATOMIC and split_k > 1 and colsum is not None:
        # the workspace path only where it carries the bias gradient: alone (plain partial stores +
        # one reduction) it measured slower than the atomic epilogue on the NRMS weight gradient
        # (292-301 vs 277 µs) and equal on the BERT ones; with the column sums folded in it saves
        # the two colsum launches (BERT FFN: 401 µs vs 409 + colsum)
        work = _splitk_work(C)
        folded = ctypes.c_int32(0)
        L.call("nr_gemm_f32_ws", M, N, K, A, B, L.ptr(C), ldc if ldc is not None else C.stride(0),
               L.ptr(bias), epilogue, c_rows, pad_row, split_k, None, None, _prec(prec), 0, L.ptr(work),
               work.numel(), L.ptr(colsum), ctypes.byref(folded) if colsum is not None else None,
               L.stream_ptr(C))
        return bool(folded.value)
    L.call("nr_gemm_f32", M, N, K, A, B, L.ptr(C), ldc if ldc is not None else C.stride(0),
           L.ptr(bias), epilogue, c_rows, pad_row, split_k, _prec(prec), L.stream_ptr(C))
    return False


def _splitk_work(like):
    """Workspace of a split-K weight-gradient GEMM with its bias gradient folded in (nr_gemm_f32_ws:
    partial tiles and column sums through plain stores and one reduction); from the caching
    allocator, so it is reused from call to call (and from the graph pool inside a capture)."""
    return torch.empty(int(L.load().nr_gemm_splitk_workspace()), device=like.device, dtype=torch.float32)


def gemm_dyn(M, N, K, A, B, C, m_dev=None, k_dev=None, ldc=None, bias=None, epilogue=L.EPI_STORE,
             c_rows=None, pad_row=-1, split_k=1, prec=None, max_cus=0, workspace=False):
    """``gemm`` with device-resident extents: M, K are upper bounds, the kernel reads the actual
    M / K from the int32 CUDA scalars ``m_dev`` / ``k_dev`` (e.g. ``UniqueRows.counts[1:2]``).
    ``max_cus`` > 0 limits the persistent grid to that many CUs (nr_gemm_f32_dyn_cus).
    ``workspace`` (split-K NR_EPI_ATOMIC, or the NR_EPI_SCATTER_ZEROED table dgrad's stream-K tail):
    partial tiles through plain stores into a workspace and one ordered reduction instead of fp32
    atomics (nr_gemm_f32_ws)."""
    _f32(C, bias)
    for t in (m_dev, k_dev):
        if t is not None and (t.dtype != torch.int32 or not t.is_cuda):
            raise L.HipError("gemm_dyn: device extents must be int32 CUDA tensors")
    if bias is not None and bias.numel() < N:
        raise L.HipError("gemm_dyn: bias has %d < N=%d entries" % (bias.numel(), N))
    if K % 32:
        raise L.HipError("gemm_dyn: K must be a multiple of 32")
    if workspace and ((epilogue == L.EPI_ATOMIC and split_k > 1) or epilogue == L.EPI_SCATTER_ZEROED):
        work = _splitk_work(C)
        L.call("nr_gemm_f32_ws", M, N, K, A, B, L.ptr(C), ldc if ldc is not None else C.stride(0),
               L.ptr(bias), epilogue, c_rows, pad_row, split_k, L.ptr(m_dev), L.ptr(k_dev), _prec(prec),
               int(max_cus), L.ptr(work), work.numel(), L.ptr(None), None, L.stream_ptr(C))
        return
    if max_cus:
        L.call("nr_gemm_f32_dyn_cus", M, N, K, A, B, L.ptr(C), ldc if ldc is not None else C.stride(0),
               L.ptr(bias), epilogue, c_rows, pad_row, split_k, L.ptr(m_dev), L.ptr(k_dev), _prec(prec),
               int(max_cus), L.stream_ptr(C))
        return
    L.call("nr_gemm_f32_dyn", M, N, K, A, B, L.ptr(C), ldc if ldc is not None else C.stride(0),
           L.ptr(bias), epilogue, c_rows, pad_row, split_k, L.ptr(m_dev), L.ptr(k_dev), _prec(prec),
           L.stream_ptr(C))


def _ceil32(n):
    return (n + 31) // 32 * 32


_SELF_CLEANING = {}
_RETIRED = []   # outgrown buffers stay allocated: a captured graph may still address them


_CLEAN_WORDS = {}   # (device, name) -> [(start, end)] word spans the kernels leave zero (the rest is scratch)


def self_cleaning_workspace(dev, name, n, clean=None):
    """A persistent zeroed int32 device buffer of at least ``n`` words per (device, name) for the
    kernels whose counters start at zero and that leave them zero again (nr_unique_rows,
    nr_score_nll_fwd): no zero-fill launch per call.  ``clean``: how many leading words are such
    counters (default all; nr_unique_rows' scan outputs and the NLL head's per-impression terms that
    follow are scratch), or a list of (start, end) word spans when the counters are not one prefix
    (nr_unique_rows' tile totals sit after its scratch arrays), for ``self_cleaning_check``.

    Created (or grown) by an eager call, never inside a graph capture: a buffer first zero-filled
    during a capture would only be zero once that graph had replayed.  Steps run one at a time on
    a device, so one buffer per (device, name) serves every stream."""
    key = (_dev_key(dev), name)
    ws = _SELF_CLEANING.get(key)
    if ws is None or ws.numel() < n:
        if torch.cuda.is_current_stream_capturing():
            raise L.HipError(f"{name} workspace must be created by an eager call before graph capture")
        if ws is not None:
            _RETIRED.append(ws)
        ws = _SELF_CLEANING[key] = torch.zeros(max(int(n), 4), device=dev, dtype=torch.int32)
    if clean is None:
        clean = [(0, int(n))]
    elif not isinstance(clean, (list, tuple)):
        clean = [(0, int(clean))]
    _CLEAN_WORDS[key] = [(int(a), int(b)) for a, b in clean]
    return ws


def _dev_key(dev):
    """torch.device with an explicit index ("cuda" -> the current device), as the workspaces are keyed."""
    d = torch.device(dev)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def self_cleaning_check(dev=None, reset=False):
    """Debug check of the self-cleaning workspaces: every kernel using one leaves its counters zero,
    so after a synchronize each buffer's counter words (``clean`` of self_cleaning_workspace) must
    read zero.  A launch that never completed, or two launches on one buffer from concurrent
    streams, leaves a counter set and silently corrupts later calls: -> the names of the buffers found
    non-zero; ``reset``: zero them again (after an error)."""
    torch.cuda.synchronize()
    bad = []
    for (d, name), ws in _SELF_CLEANING.items():
        if dev is not None and d != _dev_key(dev):
            continue
        spans = _CLEAN_WORDS.get((d, name), [(0, ws.numel())])
        if any(bool((ws[a:b] != 0).any().item()) for a, b in spans):
            bad.append(name)
            if reset:
                for a, b in spans:
                    ws[a:b].zero_()
    return bad


def score_nll_status(dev, clear=True):
    """The sticky label status of nr_score_nll_fwd on ``dev`` (True: some call since the last check
    saw a label outside [0, C) other than the ignored -100 and returned a NaN loss, where
    torch.nn.functional.nll_loss raises).  Reads the device (synchronises)."""
    ws = _SELF_CLEANING.get((_dev_key(dev), "nr_score_nll_fwd"))
    if ws is None:
        return False
    bad = bool(ws[1].item() != 0)
    if bad and clear:
        ws[1].zero_()
    return bad


_UR_GEN = {}   # (device, vocab) -> calls of nr_unique_rows on that workspace (UniqueRows.zero_absent_rows)


class UniqueRows:
    """Distinct ids of a token batch (``nr_unique_rows``), sizes left on the device.

    uids [cap] int64 (valid prefix counts[1], ascending, padded with fill_row), inv [T] int64,
    seg_off [cap + 1] / seg_tok [T] / seg_of [T] int32 CSR of the tokens with ``grad_mask`` set
    (all tokens if None), counts [4] int32 = (U, U_pad, bad, T_csr); cap = ceil32(min(T, V))
    is the host-side upper bound of U_pad."""

    def __init__(self, ids, vocab, fill_row=0, grad_mask=None):
        _check_rows(ids, None, "unique_rows")
        T = ids.numel()
        dev = ids.device
        self.T, self.vocab = T, vocab
        self.cap = max(32, _ceil32(min(T, vocab)))
        i32 = dict(device=dev, dtype=torch.int32)
        # ctrl[4] | cnt_all | cnt_csr | cursor | pos | tot (dedup.hip): ctrl, the two counter arrays and
        # the vocabulary tiles' totals are zero on entry and left zero; cursor and pos are scratch
        nwords = L.load().nr_unique_rows_workspace(vocab)
        v4 = (vocab + 3) // 4 * 4
        work = self_cleaning_workspace(dev, f"nr_unique_rows/{vocab}", nwords,
                                       clean=[(0, 4 + 2 * v4), (4 + 4 * v4, nwords)])
        # the workspace keeps this call's presence scan until the next call on it (zero_absent_rows)
        key = (torch.device(dev), vocab)
        _UR_GEN[key] = self._gen = _UR_GEN.get(key, 0) + 1
        self._key, self._work = key, work
        self.uids = torch.empty(self.cap, device=dev, dtype=torch.int64)
        self.inv = torch.empty(T, device=dev, dtype=torch.int64)
        self.seg_off = torch.empty(self.cap + 1, **i32)
        self.seg_tok = torch.empty(max(T, 1), **i32)
        self.seg_of = torch.empty(max(T, 1), **i32)
        self.counts = torch.empty(4, **i32)
        mp, mdt = mask_arg(grad_mask, T) if grad_mask is not None else (None, 0)
        self.all_tokens = grad_mask is None
        L.call("nr_unique_rows", L.ptr(ids), T, vocab, fill_row, mp, mdt, L.ptr(work), L.ptr(self.uids),
               L.ptr(self.inv), L.ptr(self.seg_off), L.ptr(self.seg_tok), L.ptr(self.seg_of), L.ptr(self.counts),
               L.stream_ptr(ids))
        self.n_rows = self.counts[0:1]  # device scalar: U
        self.u_pad = self.counts[1:2]   # device scalar: U_pad, the GEMM extent

    def segment_sum(self, src, dst):
        """dst[u] = Σ src[t] over the tokens t of distinct row u (zeros on pad rows)."""
        _f32(src, dst)
        _rows_ok(src, self.T, src.shape[1], "segment_sum src")
        _rows_ok(dst, self.cap, src.shape[1], "segment_sum dst")
        width = src.shape[1]
        nbytes = L.load().nr_segment_rows_sum_workspace(self.T, width)
        work = torch.empty(max(1, nbytes // 4), device=src.device, dtype=torch.float32)
        L.call("nr_segment_rows_sum", L.ptr(src), src.stride(0), width, self.T, L.ptr(self.seg_off),
               L.ptr(self.seg_tok), L.ptr(self.seg_of), L.ptr(self.counts), self.cap, L.ptr(work), L.ptr(dst),
               dst.stride(0), L.stream_ptr(src))


    def zero_absent_rows(self, dst, pad_row, flags=None):
        """Zero the rows of dst [vocab, W] whose id is absent from this batch, and the pad row (the
        present rows are left for the distinct-row scatter GEMM).  flags (uint8 [vocab], optional)
        receives 1 for a present row, 0 for a zeroed one.  Falls back to a full zero fill when
        another UniqueRows call on the same vocabulary has since replaced this one's presence scan;
        returns False then (flags not written), True otherwise."""
        _f32(dst)
        if dst.dim() != 2 or dst.shape[0] != self.vocab or dst.stride(1) != 1:
            raise L.HipError("zero_absent_rows: dst must be a row-major [vocab, W] matrix")
        if flags is not None and (flags.dtype != torch.uint8 or flags.numel() != self.vocab or
                                  not flags.is_contiguous() or flags.device != dst.device):
            raise L.HipError("zero_absent_rows: flags must be a contiguous uint8 [vocab] tensor on dst's device")
        if _UR_GEN.get(self._key) != self._gen:
            dst.zero_()
            return False
        L.call("nr_unique_rows_zero_absent", L.ptr(self._work), L.ptr(self.counts), self.vocab, int(pad_row),
               L.ptr(dst), dst.stride(0), dst.shape[1], L.ptr(flags) if flags is not None else None,
               L.stream_ptr(dst))
        return True

    def segment_sum_multi(self, src, dst):
        """segment_sum for the distinct rows of two or more CSR tokens; a one-token row of dst is left
        as it is (its producer wrote it: mha_pool_bwd with seg=)."""
        _f32(src, dst)
        _rows_ok(src, self.T, src.shape[1], "segment_sum src")
        _rows_ok(dst, self.cap, src.shape[1], "segment_sum dst")
        width = src.shape[1]
        nbytes = L.load().nr_segment_rows_sum_workspace(self.T, width)
        work = torch.empty(max(1, nbytes // 4), device=src.device, dtype=torch.float32)
        L.call("nr_segment_rows_sum_multi", L.ptr(src), src.stride(0), width, self.T, L.ptr(self.seg_off),
               L.ptr(self.seg_tok), L.ptr(self.seg_of), L.ptr(self.counts), self.cap, L.ptr(work), L.ptr(dst),
               dst.stride(0), L.stream_ptr(src))

    def segment_sum_conv3(self, src, dst, tap_width, seq_len):
        """dst[u][tap*tap_width + c] = Σ src[t + 1 - tap][c] over the tokens t of distinct row u (taps
        outside t's title skipped): the CNN encoder's per-distinct-row conv gradient input.  The CSR
        must hold every token (grad_mask None)."""
        _f32(src, dst)
        _rows_ok(src, self.T, tap_width, "segment_sum_conv3 src")
        _rows_ok(dst, self.cap, 3 * tap_width, "segment_sum_conv3 dst")
        if not self.all_tokens:
            raise L.HipError("segment_sum_conv3 needs the CSR of every token (grad_mask=None)")
        nbytes = L.load().nr_segment_rows_sum_workspace(self.T, 3 * tap_width)
        work = torch.empty(max(1, nbytes // 4), device=src.device, dtype=torch.float32)
        L.call("nr_segment_rows_sum_conv3", L.ptr(src), src.stride(0), tap_width, seq_len, self.T,
               L.ptr(self.seg_off), L.ptr(self.seg_tok), L.ptr(self.seg_of), L.ptr(self.counts), self.cap,
               L.ptr(work), L.ptr(dst), dst.stride(0), L.stream_ptr(src))


def conv3_rows_fwd(P, tap_width, H, inv, seq_len, bias, out, relu=True):
    """out[t][:H] = act(bias + Σ_tap P[inv[t + tap - 1]][tap block]) (taps inside the title), out[t][H:
    tap_width] = 0.  P [U, >= 3*tap_width], inv [T] int64, out [T, >= tap_width]."""
    _f32(P, bias, out)
    _check_rows(inv, None, "inv")
    T = inv.numel()
    _al(P, "conv3_rows P")
    _al(out, "conv3_rows out")
    _rows_ok(P, 1, 3 * tap_width, "conv3_rows P")
    _rows_ok(out, T, tap_width, "conv3_rows out")
    if bias is not None and bias.numel() < H:
        raise L.HipError("conv3_rows: bias has %d < %d entries" % (bias.numel(), H))
    L.call("nr_conv3_rows_fwd", L.ptr(P), P.stride(0), tap_width, H, L.ptr(inv), T, seq_len, L.ptr(bias),
           int(relu), L.ptr(out), out.stride(0), L.stream_ptr(P))


def cnn_keypool_supported(Hp, seq_len):
    return Hp % 32 == 0 and 32 <= Hp <= 160 and 1 <= seq_len <= 32


def _kp_key(kbuf, rows, Hp, name):
    if kbuf is None:
        return None, 0
    _f32(kbuf)
    if kbuf.dim() != 2 or kbuf.stride(1) != 1 or kbuf.shape[0] < rows or kbuf.shape[1] < Hp:
        raise L.HipError("%s: the key buffer must be [T, >= Hp] with unit column stride" % name)
    return L.ptr(kbuf), kbuf.stride(0)


def cnn_keypool_fwd(C, wq, bq, query, mask, nseq, seq_len, news, probs, qn, prec=None, kout=None):
    """nr_cnn_keypool_fwd: K = tanh(C wqᵀ + bq), p = XSoftmax(q·K / sqrt(qn), mask), news = Σ p C per
    title.  C [nseq*L, Hp] (zero past qn), wq [Hp, Hp], bq [Hp] padded, query [>= qn]; news [nseq, >= Hp].
    ``kout`` [T, >= Hp]: K kept for the backward (``cnn_keypool_bwd(kin=)``)."""
    _f32(C, wq, bq, query, news, probs)
    Hp = wq.shape[0]
    if not cnn_keypool_supported(Hp, seq_len):
        raise L.HipError("cnn_keypool: Hp %% 32 == 0, Hp <= 160, L <= 32 required (Hp=%d, L=%d)" % (Hp, seq_len))
    _al(C, "cnn_keypool C")
    _rows_ok(C, nseq * seq_len, Hp, "cnn_keypool C")
    if not wq.is_contiguous() or wq.shape != (Hp, Hp) or bq.numel() < Hp or query.numel() < qn:
        raise L.HipError("cnn_keypool: wq [Hp, Hp] contiguous, bq [Hp], query [qn] required")
    _rows_ok(news, nseq, Hp, "cnn_keypool news")
    if probs.numel() < nseq * seq_len:
        raise L.HipError("cnn_keypool: probs needs nseq*L floats")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    prec = get_gemm_precision() if prec is None else prec
    kp, ldk = _kp_key(kout, nseq * seq_len, Hp, "cnn_keypool_fwd")
    L.call("nr_cnn_keypool_fwd", L.ptr(C), C.stride(0), L.ptr(wq), L.ptr(bq), L.ptr(query), qn, mp, mdt, nseq, seq_len,
           Hp, 1.0 / float(qn) ** 0.5, prec, L.ptr(news), news.stride(0), L.ptr(probs), kp, ldk, L.stream_ptr(C))


def cnn_keypool_bwd(C, wq, bq, query, nseq, seq_len, H, probs, dnews, dc, dwq, dbq, dq, dconv_b, dz=None, prec=None,
                    kin=None):
    """Backward of cnn_keypool_fwd: dc [T, >= Hp] = ReLU'(C) (p dnews + dK wq + dz); dwq [Hp, Hp], dbq [Hp],
    dq [qn], dconv_b [H] are STORED.  dnews [nseq, >= qn] (row stride any), dz [T, >= H] optional; ``kin``
    the forward's ``kout`` (K read instead of recomputed)."""
    _f32(C, wq, bq, query, probs, dnews, dc, dwq, dbq, dq, dconv_b, dz)
    Hp = wq.shape[0]
    qn = dq.numel()
    if not cnn_keypool_supported(Hp, seq_len):
        raise L.HipError("cnn_keypool: Hp %% 32 == 0, Hp <= 160, L <= 32 required (Hp=%d, L=%d)" % (Hp, seq_len))
    _al(C, "cnn_keypool C")
    _rows_ok(C, nseq * seq_len, Hp, "cnn_keypool C")
    _rows_ok(dc, nseq * seq_len, Hp, "cnn_keypool dc")
    if not (dwq.is_contiguous() and dwq.numel() == Hp * Hp and dbq.numel() >= Hp and dconv_b.numel() >= H
            and query.numel() >= qn and wq.is_contiguous()):
        raise L.HipError("cnn_keypool_bwd: dwq [Hp, Hp] contiguous, dbq [Hp], dconv_b [H] required")
    if dnews.stride(-1) != 1 or dnews.shape[0] < nseq:
        raise L.HipError("cnn_keypool_bwd: dnews rows must be unit-stride")
    if dz is not None and (dz.stride(-1) != 1 or dz.shape[0] < nseq * seq_len or dz.shape[1] < H):
        raise L.HipError("cnn_keypool_bwd: dz [T, >= H] with unit column stride required")
    nws = int(L.load().nr_cnn_keypool_workspace(nseq, Hp))
    ws = torch.empty(max(nws, 1), device=C.device)
    prec = get_gemm_precision() if prec is None else prec
    L.call("nr_cnn_keypool_bwd", L.ptr(C), C.stride(0), L.ptr(wq), L.ptr(bq), L.ptr(query), qn, nseq, seq_len, Hp, H,
           1.0 / float(qn) ** 0.5, prec, L.ptr(probs), L.ptr(dnews), dnews.stride(0), L.ptr(dz),
           dz.stride(0) if dz is not None else 0, L.ptr(dc), dc.stride(0), L.ptr(dwq), L.ptr(dbq), L.ptr(dq),
           L.ptr(dconv_b), L.ptr(ws), ws.numel(), *_kp_key(kin, nseq * seq_len, Hp, "cnn_keypool_bwd"),
           L.stream_ptr(C))


def operand(t, layout, rows=None, mapping=L.ROWS_PLAIN, seq_len=1, seg=1, ld=None):
    """Describe a stored matrix ``t`` (2-D, row-major, ld % 4 == 0, 16-B aligned)."""
    _f32(t)
    if t.dim() != 2 or t.stride(1) != 1:
        raise L.HipError("operand must be a 2-D row-major tensor")
    ld = t.stride(0) if ld is None else ld
    if mapping != L.ROWS_PLAIN and (ld % 4 or t.data_ptr() % 16):
        raise L.HipError("gathered operand needs ld %% 4 == 0 and 16-B alignment (ld=%d)" % ld)
    _check_rows(rows, None, "operand")
    if mapping != L.ROWS_PLAIN and rows is None:
        raise L.HipError("gather/conv3 operand needs a row table")
    op = L.nr_operand(t.data_ptr(), ld, rows.data_ptr() if rows is not None else 0,
                      mapping, seq_len, seg, layout)
    op._keep = (t, rows)   # the struct holds raw pointers: keep the tensors alive with it
    return op


def rows_map(rows, mapping, seq_len=1, seg=1):
    """A row map for the SCATTER epilogue (no data)."""
    _check_rows(rows, None, "rows_map")
    op = L.nr_operand(0, 0, rows.data_ptr(), mapping, seq_len, seg, 0)
    op._keep = (rows,)
    return op


_MASK_DT = {torch.uint8: L.MASK_U8, torch.bool: L.MASK_U8, torch.int64: L.MASK_I64,
            torch.float64: L.MASK_F64, torch.float32: L.MASK_F32}


def mask_arg(mask, numel):
    """(pointer, dtype code) of a contiguous CUDA mask with ``numel`` elements."""
    if mask.dtype not in _MASK_DT or not mask.is_cuda or not mask.is_contiguous():
        raise L.HipError("mask must be a contiguous CUDA bool/u8/i64/f32/f64 tensor")
    if mask.numel() != numel:
        raise L.HipError("mask has %d elements, expected %d" % (mask.numel(), numel))
    return L.ptr(mask), _MASK_DT[mask.dtype]


def _cols(t, need, name):
    if t.dim() != 2 or t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
        raise L.HipError("%s: 2-D row-major, ld %% 4 == 0, 16-B aligned required" % name)
    if t.shape[1] < need:
        raise L.HipError("%s: needs %d columns, has %d" % (name, need, t.shape[1]))


def mha_attn_fwd(qk, v, mask, nseq, seq_len, heads, dk, dv, out, rows=None):
    """Tied-QK multi-head attention core (Attention.py:115-147).  qk: [nseq*L, >=heads*dk]
    (column views allowed), v: [nseq*L, >=heads*dv], mask: [nseq, L], out: [nseq*L, heads*dv].
    rows (int64 [nseq*L], optional): token t reads qk / v row rows[t] (values < qk.shape[0])."""
    _f32(qk, v, out)
    for t, need, n in ((qk, heads * dk, "qk"), (v, heads * dv, "v"), (out, heads * dv, "out")):
        _cols(t, need, n)
        if rows is None and t.shape[0] != nseq * seq_len:
            raise L.HipError("%s has %d rows, expected %d" % (n, t.shape[0], nseq * seq_len))
    if out.shape[0] != nseq * seq_len:
        raise L.HipError("out has %d rows, expected %d" % (out.shape[0], nseq * seq_len))
    if rows is not None:
        _check_rows(rows, None, "rows")
        if rows.numel() != nseq * seq_len or qk.shape[0] != v.shape[0]:
            raise L.HipError("rows must hold nseq*L entries over qk / v of equal height")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    L.call("nr_mha_attn_fwd", L.ptr(qk), qk.stride(0), L.ptr(v), v.stride(0), L.ptr(rows), mp, mdt, nseq,
           seq_len, heads, dk, dv, 1.0 / float(dk) ** 0.5, L.ptr(out), out.stride(0), L.stream_ptr(out))


MHA_USER_POOL_SHAPES = {(32, 32, 384), (64, 32, 384), (64, 64, 768)}
# gfx950: 160 KB of LDS per CU, the most one workgroup may allocate (mha_pool.hip NR_MAX_LDS)
MAX_LDS_BYTES = 160 * 1024


def mha_user_pool_smem(seq_len, H):
    """Dynamic LDS of mha_user_pool_fwd_kernel (mha_pool.hip user_pool_smem): row offsets, O [L][H+1],
    the pooling scores."""
    return (64 + seq_len * (H + 1) + 64) * 4


def mha_user_pool_supported(seq_len, heads, dk, dv):
    return (seq_len <= 64 and heads <= 12 and (dk, dv, heads * dv) in MHA_USER_POOL_SHAPES
            and mha_user_pool_smem(seq_len, heads * dv) <= MAX_LDS_BYTES)


def mha_user_pool_fwd(y, rows, mask, nseq, seq_len, heads, dk, dv, q, out, prec=None):
    """Eval MHA user encoder + pooling (MHA.py:58-75 with Pooling.py:12-25) in one launch
    (nr_mha_user_pool_fwd): y [R, >= heads*(dk+dv)] per-news [key | value] projections, rows int64
    [nseq*L] (history slot -> y row), mask [nseq, L], q [heads*dv] -> out [nseq, heads*dv]."""
    _f32(y, q, out)
    H = heads * dv
    _cols(y, heads * (dk + dv), "y")
    _cols(out, H, "out")
    if out.shape[0] != nseq or q.numel() != H or not q.is_contiguous():
        raise L.HipError("mha_user_pool_fwd: out [nseq, H] and a contiguous q [H] expected")
    _check_rows(rows, None, "rows")
    if rows.numel() != nseq * seq_len:
        raise L.HipError("mha_user_pool_fwd: rows must hold nseq*L entries")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    L.call("nr_mha_user_pool_fwd", L.ptr(y), y.stride(0), y.shape[0], L.ptr(rows), mp, mdt, nseq, seq_len, heads,
           dk, dv, L.ptr(q), L.ptr(out), out.stride(0), _prec(prec), L.stream_ptr(out))


def mha_attn_bwd(qk, v, mask, nseq, seq_len, heads, dk, dv, dout, dqk, dvv, dbias=None):
    """``dbias`` [heads*(dk+dv)] (optional): += the column sums of [dqk | dvv] (the projection bias
    gradient, accumulated atomically inside the kernel)."""
    _f32(qk, v, dout, dqk, dvv, dbias)
    if dbias is not None and (dbias.numel() < heads * (dk + dv) or not dbias.is_contiguous()):
        raise L.HipError("mha_attn_bwd: dbias needs heads*(dk+dv) contiguous floats")
    for t, need, n in ((qk, heads * dk, "qk"), (v, heads * dv, "v"), (dout, heads * dv, "dout"),
                       (dqk, heads * dk, "dqk"), (dvv, heads * dv, "dv")):
        _cols(t, need, n)
        if t.shape[0] != nseq * seq_len:
            raise L.HipError("%s has %d rows, expected %d" % (n, t.shape[0], nseq * seq_len))
    mp, mdt = mask_arg(mask, nseq * seq_len)
    L.call("nr_mha_attn_bwd", L.ptr(qk), qk.stride(0), L.ptr(v), v.stride(0), mp, mdt, nseq, seq_len,
           heads, dk, dv, 1.0 / float(dk) ** 0.5, L.ptr(dout), dout.stride(0), L.ptr(dqk), dqk.stride(0),
           L.ptr(dvv), dvv.stride(0), L.ptr(dbias[:heads * dk]) if dbias is not None else None,
           L.ptr(dbias[heads * dk:]) if dbias is not None else None, L.stream_ptr(dout))


def aux_operand(t):
    """The gate matrix of NR_EPI_ACCUM_GATE (passed through the c_rows slot)."""
    _f32(t)
    op = L.nr_operand(t.data_ptr(), t.stride(0), 0, L.ROWS_PLAIN, 1, 1, 0)
    op._keep = (t,)
    return op


def _rows_ok(t, rows, ncols, name):
    if t is None:
        return
    if t.dim() != 2 or t.stride(1) != 1 or t.shape[0] < rows or t.shape[1] < ncols:
        raise L.HipError("%s: expected a row-major [>=%d, >=%d] matrix, got %s stride %s"
                         % (name, rows, ncols, tuple(t.shape), t.stride()))


def _rng_ok(rng):
    if rng is not None and (rng.dtype != torch.int64 or not rng.is_cuda or rng.numel() < 2):
        raise L.HipError("rng must be an int64 CUDA tensor holding (seed, offset)")


def attn_pool_fwd(x, q, mask, nseq, seq_len, out, probs, key=None, gamma=None, beta=None, stats=None,
                  eps=1e-5, p_drop=0.0, seed=0, offset=0, scale=None, zout=None, rng=None):
    D = q.numel()
    _f32(x, q, out, probs, key, gamma, beta, stats, zout)
    _rows_ok(zout, nseq * seq_len, D, "zout")
    _rows_ok(x, nseq * seq_len, D, "x")
    _rows_ok(key, nseq * seq_len, D, "key")
    _rows_ok(out, nseq, D, "out")
    if probs.numel() < nseq * seq_len or (gamma is not None and stats.numel() < 2 * nseq * seq_len):
        raise L.HipError("attn_pool_fwd: probs/stats too small")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    scale = 1.0 / float(D) ** 0.5 if scale is None else scale
    L.call("nr_attn_pool_fwd", L.ptr(x), x.stride(0), L.ptr(key), key.stride(0) if key is not None else 0,
           L.ptr(q), mp, mdt, L.ptr(gamma), L.ptr(beta), eps, p_drop, seed, offset, L.ptr(rng), nseq, seq_len,
           D, scale, L.ptr(out), out.stride(0), L.ptr(zout), zout.stride(0) if zout is not None else 0,
           L.ptr(stats), L.ptr(probs), L.stream_ptr(x))


def attn_pool_bwd(x, q, mask, nseq, seq_len, probs, dout, dx, dq, key=None, dk=None, key_tanh=False,
                  gamma=None, beta=None, stats=None, dgamma=None, dbeta=None, p_drop=0.0, seed=0, offset=0,
                  scale=None, dz=None, rng=None):
    D = q.numel()
    _f32(x, q, probs, dout, dx, dq, key, dk, gamma, beta, stats, dgamma, dbeta, dz)
    _rows_ok(dz, nseq * seq_len, D, "dz")
    _rows_ok(x, nseq * seq_len, D, "x")
    _rows_ok(dx, nseq * seq_len, D, "dx")
    _rows_ok(key, nseq * seq_len, D, "key")
    _rows_ok(dk, nseq * seq_len, D, "dk")
    _rows_ok(dout, nseq, D, "dout")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    scale = 1.0 / float(D) ** 0.5 if scale is None else scale
    L.call("nr_attn_pool_bwd", L.ptr(x), x.stride(0), L.ptr(key), key.stride(0) if key is not None else 0,
           L.ptr(q), mp, mdt, L.ptr(gamma), L.ptr(beta), p_drop, seed, offset, L.ptr(rng), nseq, seq_len, D,
           scale, L.ptr(stats), L.ptr(probs), L.ptr(dout), dout.stride(0), L.ptr(dz),
           dz.stride(0) if dz is not None else 0, L.ptr(dx), dx.stride(0), L.ptr(dk),
           dk.stride(0) if dk is not None else 0, int(key_tanh), L.ptr(dq), L.ptr(dgamma), L.ptr(dbeta),
           L.stream_ptr(x))


def seq_pool_supported(D, L):
    return 1 <= D <= 1024 and 1 <= L <= 64


def _sp_rows(t, rows, D, name):
    if t is None:
        return
    _al(t, name)
    _rows_ok(t, rows, D, name)


def _vec_ok(v, n, name):
    if v.numel() < n or (v.dim() > 1 and v.stride(-1) != 1):
        raise L.HipError("%s: needs %d contiguous floats" % (name, n))


def seq_pool_fwd(x, q, mask, nseq, seq_len, D, out, probs, key=None, scale=None, qn=None):
    """nr_seq_pool_fwd: pooling of nseq sequences of seq_len rows of D features (row matrices 16-B
    aligned, ld % 4 == 0); q holds qn <= D valid floats (features past qn count as zero)."""
    _f32(x, q, out, probs, key)
    qn = D if qn is None else qn
    if not seq_pool_supported(D, seq_len):
        raise L.HipError("seq_pool: D <= 1024, L <= 64 required (D=%d, L=%d)" % (D, seq_len))
    _sp_rows(x, nseq * seq_len, D, "seq_pool x")
    _sp_rows(key, nseq * seq_len, D, "seq_pool key")
    _sp_rows(out, nseq, D, "seq_pool out")
    _vec_ok(q, qn, "seq_pool q")
    if probs.numel() < nseq * seq_len:
        raise L.HipError("seq_pool: probs needs nseq*L floats")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    scale = 1.0 / float(qn) ** 0.5 if scale is None else scale
    L.call("nr_seq_pool_fwd", L.ptr(x), x.stride(0), L.ptr(key), key.stride(0) if key is not None else 0, L.ptr(q),
           qn, mp, mdt, nseq, seq_len, D, scale, L.ptr(out), out.stride(0), L.ptr(probs), L.stream_ptr(x))


def seq_pool_bwd(x, q, mask, nseq, seq_len, D, probs, dout, dx, dq, key=None, dk=None, key_tanh=False, dz=None,
                 scale=None, qn=None):
    """dout [nseq, >= qn] (any alignment, row stride dout.stride(0)); dq accumulates qn floats."""
    _f32(x, q, probs, dout, dx, dq, key, dk, dz)
    qn = D if qn is None else qn
    if not seq_pool_supported(D, seq_len):
        raise L.HipError("seq_pool: D <= 1024, L <= 64 required (D=%d, L=%d)" % (D, seq_len))
    for t, r, n in ((x, nseq * seq_len, "x"), (key, nseq * seq_len, "key"), (dk, nseq * seq_len, "dk"),
                    (dx, nseq * seq_len, "dx"), (dz, nseq * seq_len, "dz")):
        _sp_rows(t, r, D, "seq_pool_bwd " + n)
    _rows_ok(dout, nseq, qn, "seq_pool_bwd dout")
    if key is not None and dk is None:
        raise L.HipError("seq_pool_bwd: a separate key needs dk")
    _vec_ok(q, qn, "seq_pool_bwd q")
    _vec_ok(dq, qn, "seq_pool_bwd dq")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    scale = 1.0 / float(qn) ** 0.5 if scale is None else scale
    L.call("nr_seq_pool_bwd", L.ptr(x), x.stride(0), L.ptr(key), key.stride(0) if key is not None else 0, L.ptr(q),
           qn, mp, mdt, nseq, seq_len, D, scale, L.ptr(probs), L.ptr(dout), dout.stride(0), L.ptr(dz),
           dz.stride(0) if dz is not None else 0, L.ptr(dx), dx.stride(0), L.ptr(dk),
           dk.stride(0) if dk is not None else 0, int(key_tanh), L.ptr(dq), L.stream_ptr(x))


def rnn_fwd(cell, gx, whh_t, bhh, B, N, H, gates, hprev, cprev, hout, h0=None, h0_idx=None, mask=None,
            reverse=False):
    G = 4 if cell == L.CELL_LSTM else 3
    _f32(gx, whh_t, bhh, gates, hprev, cprev, hout, h0)
    _rows_ok(gx, B * N, G * H, "gx")
    if tuple(whh_t.shape) != (H, G * H) or not whh_t.is_contiguous():
        raise L.HipError("rnn_fwd: whh_t must be contiguous [H, G*H]")
    _rows_ok(gates, B * N, 4 * H, "gates")
    _rows_ok(hprev, B * N, H, "hprev")
    _rows_ok(hout, B, H, "hout")
    if gates.stride(0) != 4 * H or hprev.stride(0) != H or (cprev is not None and cprev.stride(0) != H):
        raise L.HipError("rnn_fwd: gates/hprev/cprev must be dense")
    if h0_idx is not None:
        _check_rows(h0_idx, None, "h0_idx")
    mp, mdt = mask_arg(mask, B * N) if mask is not None else (L.ptr(None), 0)
    L.call("nr_rnn_fwd", cell, L.ptr(gx), gx.stride(0), L.ptr(whh_t), L.ptr(bhh), L.ptr(h0),
           h0.stride(0) if h0 is not None else 0, L.ptr(h0_idx), mp, mdt, int(reverse), B, N, H,
           L.ptr(gates), L.ptr(hprev), L.ptr(cprev), L.ptr(hout), hout.stride(0), L.stream_ptr(gx))


def rnn_bwd(cell, whh, gates, hprev, cprev, B, N, H, dhout, dgi, dgh=None, dh0=None, mask=None, reverse=False):
    G = 4 if cell == L.CELL_LSTM else 3
    _f32(whh, gates, hprev, cprev, dhout, dgi, dgh, dh0)
    if tuple(whh.shape) != (G * H, H) or not whh.is_contiguous():
        raise L.HipError("rnn_bwd: whh must be contiguous [G*H, H]")
    _rows_ok(dgi, B * N, G * H, "dgi")
    _rows_ok(dgh, B * N, G * H, "dgh")
    if dgh is not None and dgh.stride(0) != dgi.stride(0):
        raise L.HipError("rnn_bwd: dgi/dgh must share a leading dimension")
    _rows_ok(dhout, B, H, "dhout")
    mp, mdt = mask_arg(mask, B * N) if mask is not None else (L.ptr(None), 0)
    L.call("nr_rnn_bwd", cell, L.ptr(whh), L.ptr(gates), L.ptr(hprev), L.ptr(cprev), mp, mdt, int(reverse), B,
           N, H, L.ptr(dhout), dhout.stride(0), L.ptr(dgi), L.ptr(dgh), dgi.stride(0), L.ptr(dh0),
           dh0.stride(0) if dh0 is not None else 0, L.stream_ptr(dhout))


def score_fwd(cdd, user, B, C, H, mode, logits, cdd_idx=None):
    _f32(cdd, user, logits)
    _rows_ok(user, B, H, "user")
    if cdd_idx is None:
        _rows_ok(cdd, B * C, H, "cdd")
    else:
        _check_rows(cdd_idx, None, "cdd_idx")
        if cdd_idx.numel() != B * C:
            raise L.HipError("score_fwd: cdd_idx has %d entries, expected %d" % (cdd_idx.numel(), B * C))
        _rows_ok(cdd, 1, H, "cdd")
    if logits.numel() < B * C or not logits.is_contiguous():
        raise L.HipError("score_fwd: logits must be contiguous [B, C]")
    L.call("nr_score_fwd", L.ptr(cdd), cdd.stride(0), L.ptr(cdd_idx), L.ptr(user), user.stride(0), B, C, H,
           mode, L.ptr(logits), L.stream_ptr(user))


def score_bwd(cdd, user, logits, dlogits, B, C, H, mode, dcdd, duser):
    _f32(cdd, user, logits, dlogits, dcdd, duser)
    _rows_ok(cdd, B * C, H, "cdd")
    _rows_ok(dcdd, B * C, H, "dcdd")
    _rows_ok(user, B, H, "user")
    _rows_ok(duser, B, H, "duser")
    if not (logits.is_contiguous() and dlogits.is_contiguous()):
        raise L.HipError("score_bwd: logits/dlogits must be contiguous")
    L.call("nr_score_bwd", L.ptr(cdd), cdd.stride(0), L.ptr(user), user.stride(0), L.ptr(logits),
           L.ptr(dlogits), B, C, H, mode, L.ptr(dcdd), dcdd.stride(0), L.ptr(duser), duser.stride(0),
           L.stream_ptr(user))


def score_nll_fwd(cdd, user, label, B, C, H, logits, loss):
    """Training head + mean NLL in one launch (nr_score_nll_fwd)."""
    _f32(cdd, user, logits, loss)
    _rows_ok(cdd, B * C, H, "cdd")
    _rows_ok(user, B, H, "user")
    _check_rows(label, None, "label")
    if label.numel() != B or not logits.is_contiguous() or logits.numel() < B * C:
        raise L.HipError("score_nll_fwd: label [B] int64, logits contiguous [B, C]")
    # word 0: the ticket; word 1: the sticky label status (not a counter); then per-impression scratch
    work = self_cleaning_workspace(user.device, "nr_score_nll_fwd", L.load().nr_score_nll_workspace(B), clean=1)
    L.call("nr_score_nll_fwd", L.ptr(cdd), cdd.stride(0), L.ptr(user), user.stride(0), L.ptr(label), B, C, H,
           L.ptr(logits), L.ptr(loss), L.ptr(work), L.stream_ptr(user))


def score_nll_bwd(cdd, user, logits, label, dloss, dlogits, B, C, H, dcdd, duser):
    _f32(cdd, user, logits, dcdd, duser)
    _rows_ok(cdd, B * C, H, "cdd")
    _rows_ok(dcdd, B * C, H, "dcdd")
    _rows_ok(user, B, H, "user")
    _rows_ok(duser, B, H, "duser")
    if dlogits is not None and not dlogits.is_contiguous():
        raise L.HipError("score_nll_bwd: dlogits must be contiguous")
    L.call("nr_score_nll_bwd", L.ptr(cdd), cdd.stride(0), L.ptr(user), user.stride(0), L.ptr(logits), L.ptr(label),
           L.ptr(dloss), L.ptr(dlogits), B, C, H, L.ptr(dcdd), dcdd.stride(0), L.ptr(duser), duser.stride(0),
           L.stream_ptr(user))


def adam(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    """``step``: an int (host count) or an int64 CUDA scalar tensor (device count, graph replays)."""
    _f32(param, grad, exp_avg, exp_avg_sq)
    step_dev = None
    if torch.is_tensor(step):
        if step.dtype != torch.int64 or not step.is_cuda:
            raise L.HipError("adam: a device step count must be an int64 CUDA tensor")
        step_dev, step = step, 0
    n = param.numel()
    for t in (param, grad, exp_avg, exp_avg_sq):
        if not t.is_contiguous() or t.numel() != n:
            raise L.HipError("adam: tensors must be contiguous with equal numel")
    L.call("nr_adam", L.ptr(param), L.ptr(grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), n, lr, beta1, beta2, eps,
           weight_decay, step, L.ptr(step_dev), grad_scale, L.stream_ptr(param))


def adam_multi(entries, beta1, beta2, eps, weight_decay, grad_scale=1.0, advance_steps=False):
    """entries: [(param, grad, exp_avg, exp_avg_sq, lr, step)] with ``step`` an int or an int64 CUDA
    scalar and ``lr`` a float or a float32 CUDA scalar (read on the device); one nr_adam_multi call
    (a launch per <= 32 tensors).  ``advance_steps``: the device step counts hold the count BEFORE
    this step and the launch itself adds 1 to each (nr_adam_multi_step)."""
    if not entries:
        return
    arr = (L.nr_adam_tensor * len(entries))()
    for i, ent in enumerate(entries):
        p, g, m, v, lr, step = ent[:6]
        rt = ent[6] if len(ent) > 6 else None   # optional uint8 per-row "gradient non-zero" flags
        _f32(p, g, m, v)
        rlen = 0
        if rt is not None:
            if rt.dtype != torch.uint8 or not rt.is_cuda or rt.numel() < 1 or p.numel() % rt.numel():
                raise L.HipError("adam_multi: row flags must be a uint8 CUDA tensor dividing the parameter")
            rlen = p.numel() // rt.numel()
        n = p.numel()
        for t in (p, g, m, v):
            if not t.is_contiguous() or t.numel() != n:
                raise L.HipError("adam_multi: tensors must be contiguous with equal numel")
        sd, ld = 0, 0
        if torch.is_tensor(step):
            if step.dtype != torch.int64 or not step.is_cuda:
                raise L.HipError("adam_multi: a device step count must be an int64 CUDA tensor")
            sd, step = step.data_ptr(), 0
        if torch.is_tensor(lr):
            if lr.dtype != torch.float32 or not lr.is_cuda or lr.numel() != 1:
                raise L.HipError("adam_multi: a device learning rate must be a float32 CUDA scalar")
            ld, lr = lr.data_ptr(), 0.0
        arr[i] = L.nr_adam_tensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, float(lr), int(step), sd,
                                  ld, rt.data_ptr() if rt is not None else 0, rlen)
    if advance_steps:
        ticket = self_cleaning_workspace(entries[0][0].device, "nr_adam_multi_step", 4)
        L.call("nr_adam_multi_step", arr, len(entries), beta1, beta2, eps, weight_decay, grad_scale,
               L.ptr(ticket), L.stream_ptr(entries[0][0]))
        return
    L.call("nr_adam_multi", arr, len(entries), beta1, beta2, eps, weight_decay, grad_scale,
           L.stream_ptr(entries[0][0]))


def embedding_fwd(table, idx, out):
    _f32(table, out)
    _check_rows(idx, None, "idx")
    V, E = table.shape
    if not table.is_contiguous() or out.numel() != idx.numel() * E or not out.is_contiguous():
        raise L.HipError("embedding_fwd: shape mismatch")
    L.call("nr_embedding_fwd", L.ptr(table), V, E, L.ptr(idx), idx.numel(), L.ptr(out), L.stream_ptr(table))


def embedding_bwd(dout, idx, dtable, padding_idx=-1):
    _f32(dout, dtable)
    _check_rows(idx, None, "idx")
    V, E = dtable.shape
    if not dtable.is_contiguous() or not dout.is_contiguous() or dout.numel() != idx.numel() * E:
        raise L.HipError("embedding_bwd: shape mismatch")
    L.call("nr_embedding_bwd", L.ptr(dout), V, E, L.ptr(idx), idx.numel(),
           -1 if padding_idx is None else padding_idx, L.ptr(dtable), L.stream_ptr(dtable))


def xsoftmax_fwd(x, mask, out):
    """nr_xsoftmax_fwd over the last dimension of contiguous x / mask (mask: same shape, any mask dtype)."""
    _f32(x, out)
    if not x.is_contiguous() or not out.is_contiguous() or out.shape != x.shape:
        raise L.HipError("xsoftmax: contiguous x / out of one shape required")
    cols = x.shape[-1] if x.dim() else 1
    mp, mdt = mask_arg(mask, x.numel())
    L.call("nr_xsoftmax_fwd", L.ptr(x), mp, mdt, x.numel() // max(cols, 1), cols, L.ptr(out), L.stream_ptr(x))


def xsoftmax_bwd(y, dy, dx):
    _f32(y, dy, dx)
    for t in (y, dy, dx):
        if not t.is_contiguous() or t.shape != y.shape:
            raise L.HipError("xsoftmax_bwd: contiguous tensors of one shape required")
    cols = y.shape[-1] if y.dim() else 1
    L.call("nr_xsoftmax_bwd", L.ptr(y), L.ptr(dy), y.numel() // max(cols, 1), cols, L.ptr(dx), L.stream_ptr(y))


def gather_rows(src, idx, out=None):
    """out[i] = src[idx[i]] (nr_gather_rows_f32): src [V, cols] row-major, idx int64 [n]."""
    _f32(src, out)
    _check_rows(idx, None, "gather_rows")
    if src.dim() != 2 or src.stride(1) != 1:
        raise L.HipError("gather_rows: a row-major 2-D source required")
    n = idx.numel()
    if out is None:
        out = torch.empty(n, src.shape[1], device=src.device)
    elif out.dim() != 2 or out.shape != (n, src.shape[1]) or out.stride(1) != 1:
        raise L.HipError("gather_rows: out must be a row-major [n, cols] matrix")
    L.call("nr_gather_rows_f32", L.ptr(src), src.stride(0), src.shape[0], L.ptr(idx), n, src.shape[1], L.ptr(out),
           out.stride(0), L.stream_ptr(src))
    return out


def transpose(src, out=None):
    """src [rows, cols] (row-major, any leading dimension) -> out [cols, rows] contiguous
    (nr_transpose_f32)."""
    _f32(src, out)
    if src.dim() != 2 or src.stride(1) != 1:
        raise L.HipError("transpose: a row-major 2-D source required")
    rows, cols = src.shape
    if out is None:
        out = torch.empty(cols, rows, device=src.device)
    elif out.shape != (cols, rows) or out.stride(1) != 1:
        raise L.HipError("transpose: out must be a row-major [cols, rows] matrix")
    L.call("nr_transpose_f32", L.ptr(src), src.stride(0), rows, cols, L.ptr(out), out.stride(0), L.stream_ptr(src))
    return out


def rows_add_ordered(dout, idx, dtable, padding_idx=None):
    """dtable[idx[i]] += dout[i], each id's rows summed in ascending i by one wave (nr_rows_add_ordered:
    deterministic with duplicate ids, for row-sparse gradients of few rows).  dout [n, E] and dtable
    [V, E] row-major (any leading dimension), idx int64 [n]."""
    _f32(dout, dtable)
    _check_rows(idx, None, "idx")
    n = idx.numel()
    V, E = dtable.shape
    if dout.dim() != 2 or dout.shape != (n, E) or dout.stride(1) != 1 or dtable.stride(1) != 1:
        raise L.HipError("rows_add_ordered: dout [n, E] and dtable [V, E] must be row-major")
    L.call("nr_rows_add_ordered", L.ptr(dout), dout.stride(0), V, E, L.ptr(idx), n,
           -1 if padding_idx is None else padding_idx, L.ptr(dtable), dtable.stride(0), L.stream_ptr(dtable))


def colsum(x, rows, cols, out):
    _f32(x, out)
    _rows_ok(x, rows, cols, "x")
    if out.numel() < cols:
        raise L.HipError("colsum: out too small")
    nbytes = L.load().nr_colsum_workspace(rows, cols)
    work = torch.empty(max(1, nbytes // 4), device=x.device, dtype=torch.float32)
    tick = self_cleaning_workspace(x.device, "nr_colsum", (cols + 63) // 64)
    L.call("nr_colsum_ws", L.ptr(x), x.stride(0), rows, cols, L.ptr(out), L.ptr(work), L.ptr(tick), L.stream_ptr(x))


MHA_POOL_SHAPES = {(64, 32, 384), (64, 64, 768), (64, 32, 256), (32, 32, 384)}


def mha_pool_supported(seq_len, heads, dk, dv):
    return seq_len <= 32 and (dk, dv, heads * dv) in MHA_POOL_SHAPES


def _yrows_ok(y, yrows, T, ncols, name):
    if yrows is None:
        _rows_ok(y, T, ncols, name)
    else:
        _check_rows(yrows, None, name)
        if yrows.numel() < T:
            raise L.HipError("%s: yrows has %d < %d entries" % (name, yrows.numel(), T))
        _rows_ok(y, 1, ncols, name)


def mha_pool_fwd(y, mask, nseq, seq_len, heads, dk, dv, gamma, beta, q, news, stats, probs, eps=1e-5,
                 p_drop=0.0, seed=0, offset=0, zout=None, yrows=None, rng=None, oout=None, prec=None):
    """Fused tied-QK attention + LayerNorm + dropout + query pooling per title.  ``yrows``:
    token t reads projection row yrows[t] (distinct-row projections).  ``rng``: int64 CUDA
    (seed, offset base) read by the kernel (graph replays draw fresh masks).  ``prec``: the
    attention products' arithmetic (default: this thread's GEMM precision)."""
    _rng_ok(rng)
    H = heads * dv
    _f32(y, gamma, beta, q, news, stats, probs, zout)
    _yrows_ok(y, yrows, nseq * seq_len, heads * (dk + dv), "y")
    if y.stride(0) % 4 or y.data_ptr() % 16:
        raise L.HipError("mha_pool_fwd: y needs ld % 4 == 0 and 16-B alignment")
    _rows_ok(news, nseq, H, "news")
    _rows_ok(zout, nseq * seq_len, H, "zout")
    if stats.numel() < 2 * nseq * seq_len or probs.numel() < nseq * seq_len:
        raise L.HipError("mha_pool_fwd: stats/probs too small")
    mp, mdt = mask_arg(mask, nseq * seq_len)
    L.call("nr_mha_pool_fwd", L.ptr(y), y.stride(0), L.ptr(yrows), mp, mdt, nseq, seq_len, heads, dk, dv, L.ptr(gamma),
           L.ptr(beta), eps, p_drop, seed, offset, L.ptr(rng), L.ptr(q), L.ptr(news), news.stride(0), L.ptr(zout),
           zout.stride(0) if zout is not None else 0, L.ptr(oout), oout.stride(0) if oout is not None else 0,
           L.ptr(stats), L.ptr(probs), _prec(prec), L.stream_ptr(y))


def mha_pool_bwd(y, mask, nseq, seq_len, heads, dk, dv, gamma, beta, q, stats, probs, dnews, dy, dbias, dq,
                 dgamma, dbeta, p_drop=0.0, seed=0, offset=0, dz=None, yrows=None, rng=None, o=None, dob=None,
                 prec=None, ws=None, ws_copies=0, seg=None, dyu_row0=0):
    """``o`` (the forward's ``oout``) with ``dob`` [T, >= 8] (the LN pass's per-token row terms, from
    which the head pass rebuilds dO) selects the split backward, ``o`` without ``dob`` the fused
    backward on the saved O (dO kept in LDS); ``ws`` (forms
    with ``o``) a zeroed [ws_copies, >= 3*heads*dv + heads*(dk+dv)] buffer that spreads the
    parameter-gradient atomics (left zero).  ``seg`` (a UniqueRows built with the token mask, with
    ``yrows`` = its inv): tokens alone in their distinct row's segment write their gradient row to dy
    row ``dyu_row0`` + u of ``dy`` (the whole buffer) directly (then ``seg.segment_sum_multi``), masked
    tokens write nothing."""
    _rng_ok(rng)
    H = heads * dv
    _f32(y, gamma, beta, q, stats, probs, dnews, dy, dbias, dq, dgamma, dbeta, dz)
    _yrows_ok(y, yrows, nseq * seq_len, heads * (dk + dv), "y")
    _rows_ok(dy, nseq * seq_len, heads * (dk + dv), "dy")
    _rows_ok(dnews, nseq, H, "dnews")
    _rows_ok(dz, nseq * seq_len, H, "dz")
    if dbias.numel() < heads * (dk + dv):
        raise L.HipError("mha_pool_bwd: dbias too small")
    if ws is not None:
        _f32(ws)
        w = (3 * heads * dv + heads * (dk + dv) + 3) // 4 * 4
        if o is None or ws_copies < 1 or ws.numel() < ws_copies * w or not ws.is_contiguous():
            raise L.HipError("mha_pool_bwd: ws needs the saved O and ws_copies x %d contiguous floats" % w)
    dy_rows = dy.shape[0]
    dsto = None
    if seg is not None:
        if yrows is None or seg.all_tokens or seg.T != nseq * seq_len:
            raise L.HipError("mha_pool_bwd: seg needs yrows and the token-masked UniqueRows of these tokens")
        # dy: the whole buffer -- token rows [0, T), the distinct-row sums at rows [dyu_row0, + cap)
        if dyu_row0 < nseq * seq_len or dy.shape[0] < dyu_row0 + seg.cap:
            raise L.HipError("mha_pool_bwd: dy must hold the distinct-row rows [dyu_row0, dyu_row0 + cap)")
        dsto = torch.empty(nseq * seq_len, device=dy.device, dtype=torch.int32)
    mp, mdt = mask_arg(mask, nseq * seq_len)
    L.call("nr_mha_pool_bwd", L.ptr(y), y.stride(0), L.ptr(yrows), mp, mdt, nseq, seq_len, heads, dk, dv, L.ptr(gamma),
           L.ptr(beta), p_drop, seed, offset, L.ptr(rng), L.ptr(q), L.ptr(stats), L.ptr(probs), L.ptr(dnews), dnews.stride(0),
           L.ptr(dz), dz.stride(0) if dz is not None else 0, L.ptr(o), o.stride(0) if o is not None else 0,
           L.ptr(dob), dob.stride(0) if dob is not None else 0, L.ptr(dy), dy.stride(0), L.ptr(dbias), L.ptr(dq),
           L.ptr(dgamma), L.ptr(dbeta), L.ptr(ws), int(ws_copies), L.ptr(seg.seg_off) if seg is not None else None,
           int(dyu_row0), int(dy_rows), L.ptr(dsto), _prec(prec), L.stream_ptr(y))


# ---------------------------------------------------------------------- BERT towers

def _al(t, name):
    if t.dim() != 2 or t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
        raise L.HipError("%s: 2-D row-major, ld %% 4 == 0, 16-B aligned required" % name)


def _drop(p, seed, offset, rng):
    _rng_ok(rng)
    return float(p), int(seed), int(offset), L.ptr(rng)


def bert_embed_fwd(word, pos, type0, ids, nseq, seq_len, gamma, beta, eps, out, stats, p_drop=0.0, seed=0,
                   offset=0, rng=None, status=None):
    """BertEmbeddings: out = Dropout(LN(word[ids] + pos[l] + type0)), stats [T, 2]."""
    _f32(word, pos, type0, gamma, beta, out, stats)
    _check_rows(ids, None, "ids")
    V, H = word.shape
    T = nseq * seq_len
    if ids.numel() != T or pos.shape[1] != H or type0.numel() < H or not word.is_contiguous():
        raise L.HipError("bert_embed_fwd: shape mismatch")
    if pos.shape[0] < seq_len:
        raise L.HipError("bert_embed_fwd: %d positions < sequence length %d" % (pos.shape[0], seq_len))
    _al(out, "bert_embed_fwd out")
    _rows_ok(out, T, H, "out")
    if stats.numel() < 2 * T:
        raise L.HipError("bert_embed_fwd: stats too small")
    p, s, o, r = _drop(p_drop, seed, offset, rng)
    L.call("nr_bert_embed_fwd", L.ptr(word), V, L.ptr(pos), pos.shape[0], L.ptr(type0), L.ptr(ids), nseq,
           seq_len, H, L.ptr(gamma), L.ptr(beta), float(eps), p, s, o, r, L.ptr(out), out.stride(0), L.ptr(stats),
           L.ptr(status), L.stream_ptr(word))


def bert_embed_bwd(word, pos, type0, ids, nseq, seq_len, gamma, stats, dout, ds, dgamma, dbeta, p_drop=0.0,
                   seed=0, offset=0, rng=None):
    _f32(word, pos, type0, gamma, stats, dout, ds, dgamma, dbeta)
    _check_rows(ids, None, "ids")
    V, H = word.shape
    T = nseq * seq_len
    if ids.numel() != T:
        raise L.HipError("bert_embed_bwd: shape mismatch")
    _al(dout, "dout")
    _al(ds, "ds")
    _rows_ok(dout, T, H, "dout")
    _rows_ok(ds, T, H, "ds")
    p, s, o, r = _drop(p_drop, seed, offset, rng)
    L.call("nr_bert_embed_bwd", L.ptr(word), V, L.ptr(pos), L.ptr(type0), L.ptr(ids), nseq, seq_len, H,
           L.ptr(gamma), p, s, o, r, L.ptr(stats), L.ptr(dout), dout.stride(0), L.ptr(ds), ds.stride(0),
           L.ptr(dgamma), L.ptr(dbeta), L.stream_ptr(word))


def bert_add_ln_fwd(x, res, gamma, beta, eps, out, stats, p_drop=0.0, seed=0, offset=0, rng=None):
    """out = LayerNorm(Dropout(x) + res)."""
    _f32(x, res, gamma, beta, out, stats)
    T, H = x.shape
    for t, n in ((x, "x"), (res, "res"), (out, "out")):
        _al(t, n)
        _rows_ok(t, T, H, n)
    if stats.numel() < 2 * T or gamma.numel() < H:
        raise L.HipError("bert_add_ln_fwd: shape mismatch")
    p, s, o, r = _drop(p_drop, seed, offset, rng)
    L.call("nr_bert_add_ln_fwd", L.ptr(x), x.stride(0), L.ptr(res), res.stride(0), T, H, L.ptr(gamma), L.ptr(beta),
           float(eps), p, s, o, r, L.ptr(out), out.stride(0), L.ptr(stats), L.stream_ptr(x))


def bert_add_ln_bwd(x, res, gamma, stats, dout, dres, dx, dgamma, dbeta, p_drop=0.0, seed=0, offset=0, rng=None):
    _f32(x, res, gamma, stats, dout, dres, dx, dgamma, dbeta)
    T, H = x.shape
    for t, n in ((x, "x"), (res, "res"), (dout, "dout"), (dres, "dres"), (dx, "dx")):
        _al(t, n)
        _rows_ok(t, T, H, n)
    p, s, o, r = _drop(p_drop, seed, offset, rng)
    L.call("nr_bert_add_ln_bwd", L.ptr(x), x.stride(0), L.ptr(res), res.stride(0), T, H, L.ptr(gamma), p, s, o, r,
           L.ptr(stats), L.ptr(dout), dout.stride(0), L.ptr(dres), dres.stride(0), L.ptr(dx), dx.stride(0),
           L.ptr(dgamma), L.ptr(dbeta), L.stream_ptr(x))


def _attn_check(qkv, heads, koff, voff, mask, nseq, seq_len):
    _f32(qkv)
    _al(qkv, "qkv")
    T = nseq * seq_len
    _rows_ok(qkv, T, max(koff, voff) + heads * 64, "qkv")
    return mask_arg(mask, T)


def bert_attn_keep_buffer(nseq, seq_len, heads, device):
    """The dropout keep-bit words of one nr_bert_attn_fwd call (nr_bert_attn_keep_words int32)."""
    n = int(L.load().nr_bert_attn_keep_words(nseq, seq_len, heads))
    return torch.empty(max(n, 1), device=device, dtype=torch.int32)


def _keep_ok(keep, nseq, seq_len, heads, name):
    if keep is None:
        return
    if keep.dtype != torch.int32 or not keep.is_cuda or not keep.is_contiguous() or \
            keep.numel() < int(L.load().nr_bert_attn_keep_words(nseq, seq_len, heads)):
        raise L.HipError("%s: keep must be a contiguous int32 CUDA buffer of nr_bert_attn_keep_words words" % name)


def bert_attn_fwd(qkv, heads, mask, nseq, seq_len, ctx, ml, koff=None, voff=None, p_drop=0.0, seed=0, offset=0,
                  rng=None, prec=None, keep=None):
    """BertSelfAttention core on a fused [T, 3*heads*64] (Q | K | V) projection.  ``prec``: the
    attention products' arithmetic (default: this thread's GEMM precision).  ``keep``
    (bert_attn_keep_buffer; bf16-MFMA arithmetic with dropout): the dropout keep bits are stored
    there for the backward."""
    koff = heads * 64 if koff is None else koff
    voff = 2 * heads * 64 if voff is None else voff
    mp, mdt = _attn_check(qkv, heads, koff, voff, mask, nseq, seq_len)
    _f32(ctx, ml)
    _al(ctx, "ctx")
    T = nseq * seq_len
    _rows_ok(ctx, T, heads * 64, "ctx")
    if ml.numel() < 2 * T * heads:
        raise L.HipError("bert_attn_fwd: ml too small")
    _keep_ok(keep, nseq, seq_len, heads, "bert_attn_fwd")
    p, s, o, r = _drop(p_drop, seed, offset, rng)
    L.call("nr_bert_attn_fwd", L.ptr(qkv), qkv.stride(0), koff, voff, mp, mdt, nseq, seq_len, heads, p, s, o, r,
           L.ptr(ctx), ctx.stride(0), L.ptr(ml), L.ptr(keep), _prec(prec), L.stream_ptr(qkv))


def bert_attn_bwd(qkv, heads, mask, nseq, seq_len, ctx, ml, dctx, dqkv, koff=None, voff=None, p_drop=0.0, seed=0,
                  offset=0, rng=None, prec=None, keep=None):
    koff = heads * 64 if koff is None else koff
    voff = 2 * heads * 64 if voff is None else voff
    mp, mdt = _attn_check(qkv, heads, koff, voff, mask, nseq, seq_len)
    _f32(ctx, ml, dctx, dqkv)
    T = nseq * seq_len
    for t, n, w in ((ctx, "ctx", heads * 64), (dctx, "dctx", heads * 64), (dqkv, "dqkv", max(koff, voff) + heads * 64)):
        _al(t, n)
        _rows_ok(t, T, w, n)
    nbytes = L.load().nr_bert_attn_bwd_workspace(nseq, seq_len, heads)
    work = torch.empty(max(1, nbytes // 4), device=qkv.device, dtype=torch.float32)
    _keep_ok(keep, nseq, seq_len, heads, "bert_attn_bwd")
    p, s, o, r = _drop(p_drop, seed, offset, rng)
    L.call("nr_bert_attn_bwd", L.ptr(qkv), qkv.stride(0), koff, voff, mp, mdt, nseq, seq_len, heads, p, s, o, r,
           L.ptr(ctx), ctx.stride(0), L.ptr(ml), L.ptr(keep), L.ptr(dctx), dctx.stride(0), L.ptr(work), L.ptr(dqkv),
           dqkv.stride(0), _prec(prec), L.stream_ptr(qkv))


def tanh_bwd(y, dy, dx):
    _f32(y, dy, dx)
    rows, cols = y.shape
    _rows_ok(dy, rows, cols, "dy")
    _rows_ok(dx, rows, cols, "dx")
    L.call("nr_tanh_bwd", L.ptr(y), y.stride(0), L.ptr(dy), dy.stride(0), rows, cols, L.ptr(dx), dx.stride(0),
           L.stream_ptr(y))
