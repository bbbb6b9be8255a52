"""autograd.Functions over the HIP kernels — the fused hot path of the two towers.

Every forward/backward here launches only libnewsrec_hip.so kernels (plus torch allocations
and zero-fills); nothing computes on the CPU.  Token ids are int64 [T] (T = news * L), masks
are passed in their reference dtype (i64 token masks, f64 history masks).

News towers read the word-embedding table directly (the gather is fused into the first GEMM's
operand loader) and scatter the table gradient straight out of the dgrad GEMM, so the
[T, 768] embedding activations are never materialised.  A standalone ``encoderN(emb, mask)``
call uses the same functions with the embeddings as the "table" and identity row ids.
"""
import functools
import os
import threading
import weakref

import torch

from . import _lib as L
from . import kernels as K


def _gemm_backward(fn):
    """Run a Function's backward under the GEMM arithmetic its forward recorded in ``ctx.prec``
    (the autograd engine runs CUDA backwards on its own thread, which has its own default)."""
    @functools.wraps(fn)
    def wrapper(ctx, *grads):
        with K.gemm_precision(ctx.prec):
            return fn(ctx, *grads)
    return wrapper


def _ceil32(n):
    return (n + 31) // 32 * 32


def _pad4(n):
    return (n + 3) // 4 * 4


def _empty(rows, cols, like, ld=None):
    """[rows, cols] view of a row-major buffer with a float4-friendly leading dimension."""
    ld = _pad4(cols) if ld is None else ld
    buf = torch.empty(rows, ld, device=like.device, dtype=torch.float32)
    return buf[:, :cols]


GRAD_COPIES = 32
_GRAD_COPIES_WS = {}


def _grad_copies(dev, width):
    """A persistent zeroed [GRAD_COPIES, ceil4(width)] workspace per (device, width) for
    nr_mha_pool_bwd's spread parameter-gradient atomics (the kernel leaves it zero again).

    Created eagerly, never inside a graph capture: a buffer first allocated (and zero-filled) during
    a capture would only be zero once that graph had replayed, and a later graph reusing it would
    depend on that replay order.  Steps run one at a time on a device, so one workspace per
    (device, width) serves every stream."""
    key = (torch.device(dev), width)
    ws = _GRAD_COPIES_WS.get(key)
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            raise L.HipError("nr_mha_pool_bwd workspace must be created by an eager step before graph capture")
        ws = _GRAD_COPIES_WS[key] = torch.zeros(GRAD_COPIES, (width + 3) // 4 * 4, device=dev)
    return ws


def _zeros_views(dev, *shapes):
    """Views of ONE zero-filled buffer (one fill launch instead of one per gradient), each
    starting 16-B aligned."""
    sizes = [int(torch.Size(sh).numel()) for sh in shapes]
    offs, tot = [], 0
    for n in sizes:
        offs.append(tot)
        tot += _pad4(n)
    buf = torch.zeros(max(tot, 1), device=dev)
    return [buf[o:o + n].view(sh) for o, n, sh in zip(offs, sizes, shapes)]


class _ZeroArena:
    """One zero fill for the small zero-initialised gradients of a training step.

    A Function's forward reserves the shapes its backward will zero-fill (``reserve``, only when a
    backward can run); the first backward that takes its views (``take``) zero-fills every
    reservation made since the previous fill with ONE launch.  The NRMS step had three such fills
    (the news tower's five parameter gradients, the user encoder's two, the pooling query's), each a
    launch of its own in the graph.  A token is taken once: a second backward over the same graph
    (retain_graph) gets fresh zeros, as do reservations past LIMIT floats."""

    LIMIT = 8 << 20

    def __init__(self):
        self.cur = None

    def reserve(self, dev, *shapes):
        sizes = [int(torch.Size(sh).numel()) for sh in shapes]
        need = sum(_pad4(n) for n in sizes)
        a = self.cur
        if a is None or a["buf"] is not None or a["dev"] != dev or a["tot"] + need > self.LIMIT:
            a = self.cur = {"dev": dev, "tot": 0, "buf": None}
        offs = []
        for n in sizes:
            offs.append(a["tot"])
            a["tot"] += _pad4(n)
        return {"arena": a, "offs": offs, "sizes": sizes, "shapes": shapes, "taken": False}

    def take(self, tok, dev, *shapes):
        """The reserved views (zero), or ``_zeros_views(dev, *shapes)`` without a usable token."""
        if tok is None or tok["taken"] or tuple(tok["shapes"]) != tuple(shapes):
            return _zeros_views(dev, *shapes)
        tok["taken"] = True
        a = tok["arena"]
        if a["buf"] is None:
            a["buf"] = torch.zeros(max(a["tot"], 1), device=a["dev"])
            if self.cur is a:
                self.cur = None
        buf = a["buf"]
        return [buf[o:o + n].view(sh) for o, n, sh in zip(tok["offs"], tok["sizes"], shapes)]


ZERO_ARENA = _ZeroArena()


_CALLER_GRAD = threading.local()


class _GradAwareFn(torch.autograd.Function):
    """A Function whose forward may ask ``_backward_possible``: torch runs forward() with grad mode
    OFF whatever the caller's mode, so apply() records the caller's mode for it (per thread, restored
    on exit, so nested applies see their own caller's)."""

    @classmethod
    def apply(cls, *args, **kwargs):
        prev = getattr(_CALLER_GRAD, "on", None)
        _CALLER_GRAD.on = torch.is_grad_enabled()
        try:
            return super().apply(*args, **kwargs)
        finally:
            _CALLER_GRAD.on = prev


def _backward_possible(ctx):
    """A backward can follow this forward (of a _GradAwareFn): its caller had autograd recording (not
    torch.no_grad(), where needs_input_grad still reports the parameters' requires_grad) and some input
    wants a gradient."""
    on = getattr(_CALLER_GRAD, "on", None)
    if on is None:
        raise RuntimeError("_backward_possible needs a _GradAwareFn forward")
    return on and any(ctx.needs_input_grad)


def _reserve_zeros(ctx, dev, *shapes):
    """Forward side of ZERO_ARENA: reserve the backward's zero-initialised gradients (when one can run)."""
    ctx.zero_tok = ZERO_ARENA.reserve(dev, *shapes) if _backward_possible(ctx) else None


def _backward_zeros(ctx, dev, *shapes):
    return ZERO_ARENA.take(getattr(ctx, "zero_tok", None), dev, *shapes)


class _GradDest:
    """Where a consumer's backward may write the gradient of one of its inputs directly: SplitRowsFn
    offers the two halves of its joined gradient buffer for its two outputs; a consumer Function
    (scorer, user encoder) that takes the offer in its forward stores its input gradient there, and
    SplitRowsFn's backward then finds both halves in place and skips the join copy.  The written
    values are that consumer's true gradient either way, so a stale or unused offer costs nothing
    but the copy it fails to save."""

    def __init__(self):
        self.offers = {}

    @staticmethod
    def _key(t):
        return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.device)

    def offer(self, t, dest):
        self.offers[self._key(t)] = dest

    def clear(self):
        self.offers.clear()

    def take(self, t):
        if not self.offers:
            return None
        d = self.offers.pop(self._key(t), None)
        if d is None or d.shape != t.shape:
            return None
        return d


GRAD_DEST = _GradDest()


def _grad_out(dest, rows, cols, like):
    """The backward's output buffer for an input gradient: the offered destination or a new one."""
    if dest is not None:
        return dest
    return _empty(rows, cols, like)


class SplitRowsFn(torch.autograd.Function):
    """``torch.split(x, [n0, rows - n0])`` of a row-major [rows, H] activation (the joint news-encoder
    output -> candidates | history).  torch's backward joins the two gradients with a copy (a cat);
    here the joined gradient buffer is allocated in the forward and its halves offered (GRAD_DEST) to
    the Functions that consume the two outputs, so the join is free when both write in place."""

    stats = {"in_place": 0, "copied": 0}   # backward joins by path (tests)

    @staticmethod
    def forward(ctx, x, n0):
        rows, H = x.shape
        g = _empty(rows, H, x)
        a, b = x[:n0], x[n0:]
        GRAD_DEST.clear()
        GRAD_DEST.offer(a, g[:n0])
        GRAD_DEST.offer(b, g[n0:])
        ctx.g, ctx.n0 = g, n0
        return a, b

    @staticmethod
    def backward(ctx, da, db):
        g, n0 = ctx.g, ctx.n0
        ga, gb = g[:n0], g[n0:]
        if (da is not None and db is not None and da.data_ptr() == ga.data_ptr() and
                db.data_ptr() == gb.data_ptr() and da.stride() == ga.stride() and db.stride() == gb.stride()):
            SplitRowsFn.stats["in_place"] += 1
            return g, None
        SplitRowsFn.stats["copied"] += 1
        out = torch.empty_like(g)
        for d, o in ((da, out[:n0]), (db, out[n0:])):
            if d is None:
                o.zero_()
            else:
                o.copy_(d)
        return out, None


def _split_k(m, n, k, slots=512):
    """Split-K factor for a wgrad GEMM: fill the 256 CUs x 2 resident 128x128 blocks in ONE
    wave (a 1.16-wave grid runs as two), keeping >= 512 k per split."""
    tiles = max(1, ((m + 127) // 128) * ((n + 127) // 128))
    return int(max(1, min(64, slots // tiles, k // 512)))


def _proj_wgrad(dY, X_op, dW, db, M_rows):
    """dW[n_out, k_in] += dYᵀ X ; db += colsum(dY).  dY: [rows, n_out] view, X_op: operand of
    the layer input with MN-contiguous layout (rows = token index)."""
    n_out = dW.shape[0]
    k_in = dW.shape[1]
    # db folds into the GEMM on its split-K workspace path (the first column tile's units sum the dY
    # tiles they load); other routings leave it to the two-pass column sum
    folded = K.gemm(n_out, k_in, M_rows, K.operand(dY, L.MNCONTIG), X_op, dW, epilogue=L.EPI_ATOMIC,
                    split_k=_split_k(n_out, k_in, M_rows), colsum=db)
    if db is not None and not folded:
        K.colsum(dY, M_rows, n_out, db)


class _Probe:
    """Per-launch timing of the step's dominant kernels (the news tower's three projection GEMMs).

    While enabled, ``run(name, fn, out, ur)`` launches ``fn`` as usual and keeps the first launch of
    each name as a closure over its real operands.  ``time()`` then replays every kept closure
    ``reps`` times, each replay bracketed by HIP events on the launch stream and preceded by a 512 MB
    write that evicts the L2s and the Infinity Cache (in the step the operands arrive cold: Adam has
    just streamed 0.7 GB; back-to-back replays with warm operands ran ~8 % faster than the graphed
    step's launches), and restores the output it overwrote: the average per-launch duration of
    exactly the kernels the step runs, free of the eager step's host gaps.  A closure is the whole
    unit of work (the weight gradient = its split-K GEMM + the ordered reduction)."""

    def __init__(self):
        self.on = False
        self.launches = {}

    def enable(self):
        self.on, self.launches = True, {}

    def disable(self):
        self.on, self.launches = False, {}

    def run(self, name, fn, out, ur=None):
        """``fn()`` launches the kernel(s) writing ``out``; ``ur``: the launch's UniqueRows (its
        device-side row count, the GEMM's M or K, is read back at time() for the FLOP count)."""
        fn()
        if self.on and name not in self.launches:
            self.launches[name] = (fn, out, ur)

    def time(self, reps=20, warm=2):
        res = {}
        flush = None
        for name, (fn, out, ur) in self.launches.items():
            if flush is None:
                flush = torch.empty(128 << 20, device=out.device)
            saved = out.clone()
            for _ in range(warm):
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for s, e in ev:
                flush.zero_()
                s.record()
                fn()
                e.record()
            torch.cuda.synchronize()
            out.copy_(saved)
            res[name + "_ms"] = sum(s.elapsed_time(e) for s, e in ev) / reps
            if ur is not None:
                res[name + "_rows"] = int(ur.counts[1].item())
        return res


PROBE = _Probe()

# Distinct-row projection in the news towers (False projects every token row: the token-wise form
# the parity tests compare it with; module attributes, not environment switches).
DEDUP_ROWS = True
# Training forward saves the attention output; the backward runs split (False: the fused backward
# that recomputes the attention).
SPLIT_BWD = True
# With the saved attention output: one fused kernel per title (LN backward + every head's attention
# backward, dO kept in LDS) instead of the split pair (dO through HBM)
FUSED_SAVED_BWD = False
# Split-K factor of the MHA user encoder's input gradient (dx = dY [Wk; Wv], K = 1152); a split keeps
# >= 512 k per piece.  One-box A/B of the NRMS step, interleaved rounds: unsplit 1.4206-1.4275 ms,
# two pieces 1.4292 ms -- kept unsplit
USER_DGRAD_SPLIT = 1
# CNN conv weight gradient: split-K partials through a workspace + one ordered reduction instead of
# fp32 atomics (one-box A/B, graphed steps): configs[1] bf16 0.741 -> 0.700 ms; bf16x6 CNN + attention
# 0.899 -> 0.860 ms, CNN + GRU 1.171 -> 1.126 ms
WGRAD_WS_BF16 = True
WGRAD_WS_BF16X6 = True
# CNN table dgrad with the conv weights transposed to k-contiguous (one 1.5 MB copy per step):
# one-box A/B of the graphed legs, bf16 0.698 -> 0.657 ms, fp32-class 0.851 -> 0.842 ms
CNN_DGRAD_KC = True
# NRMS table dgrad with the joint projection weight transposed to k-contiguous (one 3.5 MB copy per step),
# so both operands take the K-contiguous loaders (and the interleaved split-stores) instead of the
# MN-contiguous weight loader
PROJ_DGRAD_KC = False
# the NRMS projection weight gradient on the same workspace path: one process, interleaved rounds,
# 1.459 -> 1.446 ms per NRMS step (round 2 measured it slower, before the bf16x6 units lost SLP)
PROJ_WGRAD_WS = True
# the table dgrad's stream-K tail through the GEMM workspace + an ordered reduction (no fp32 atomics)
PROJ_DGRAD_TAIL_WS = True
# the MHA news backward writes the gradient row of a token alone in its distinct row's segment
# straight into the per-distinct-row sums (the segment sum then covers the rows of 2+ tokens)
SINGLE_ROWS_DIRECT = True
# the word-table gradient: only the rows absent from the batch (and the pad row) zero-filled
ABSENT_ROWS_ZERO = True
# ... and those rows flagged for Adam, which then skips reading them (optim.FusedAdam, row_touched)
WORD_ROW_FLAGS = True
# CNN word attention (tanh key projection + learned-query pooling) fused per title, forward and
# backward (nr_cnn_keypool_*; False: the key GEMM + pooling kernels the parity tests compare with).
FUSED_KEYPOOL = True
# The fused key-pool forward stores K = tanh(C Wqᵀ + bq) ([T, Hp], 34 MB at B = 32) and its backward
# reads it instead of recomputing the key products per title (False: recomputed, K stays on chip)
KEYPOOL_SAVE_K = True





class _TableGradHook:
    """Optional callback ``hook(table_param, dtable) -> bool`` run inside a news-tower backward
    as soon as the dense word-table gradient exists (before the weight-gradient GEMMs).  When it
    returns True it has taken ownership (e.g. started an async all-reduce and will install the
    gradient itself) and the Function returns None for the table."""

    def __init__(self):
        self.fn = None

    def set(self, fn):
        self.fn = fn

    def __call__(self, table, dtable):
        # only a leaf parameter's gradient may be taken over: a non-leaf "table" (an activation,
        # e.g. encoderN(embedding(tokens)) on the unfused path) must flow back through autograd
        if self.fn is None or not _is_param_leaf(table):
            return False
        return bool(self.fn(table, dtable))


def _is_param_leaf(t):
    return t is not None and t.is_leaf and t.requires_grad


TABLE_GRAD_HOOK = _TableGradHook()


def table_grad_buffer(table, V, E, device, zero):
    """The dense [V, E] gradient of a word table.  A table whose rows are sharded across ranks for
    its optimizer step (dist.GradSync(shard_tables=True) sets ``_nr_grad_rows`` = world x slab rows)
    gets a view of a buffer padded to that many rows, so the reduce-scatter runs on the gradient in
    place (no 94 MB copy into a padded send buffer); every other table a plain [V, E] tensor."""
    rows = int(getattr(table, "_nr_grad_rows", 0) or 0) if table is not None else 0
    alloc = torch.zeros if zero else torch.empty
    if rows > V:
        return alloc(rows, E, device=device)[:V]
    return alloc(V, E, device=device)


class _SparseGradHook:
    """Optional callback ``hook(table_param, rows [n] int64, grads [n, E]) -> bool`` for tables whose
    step gradient touches only a few rows (LSTUR's user table: B rows of 876,957).  Returning True
    means the callback owns the gradient (e.g. an exact row-sparse exchange across ranks) and the
    Function returns None for the table instead of a dense [V, E] gradient."""

    def __init__(self):
        self.fn = None

    def set(self, fn):
        self.fn = fn

    def __call__(self, table, rows, grads):
        if self.fn is None or not _is_param_leaf(table):
            return False
        return bool(self.fn(table, rows, grads))


SPARSE_GRAD_HOOK = _SparseGradHook()


class _LocalRowGrad:
    """Single-process gradient of a row-sparse table (LSTUR's user table: B rows of 876,957 per step)
    when no SPARSE_GRAD_HOOK owns it: a dense buffer zeroed ONCE and installed as ``table.grad``; each
    step re-zeroes only the rows the previous step wrote, then scatter-adds this step's rows (instead
    of a 526 MB zero fill per step).  Used only when ``table.grad`` is None at backward time
    (zero_grad(set_to_none=True), as Manager._train and bench do), so gradient accumulation across
    backward passes keeps torch's dense semantics."""

    def __init__(self):
        self.buf, self.prev, self.flags = {}, {}, {}

    def __call__(self, table, rows, grads):
        if not _is_param_leaf(table):
            return False
        if _multi_rank():
            # several ranks and no SPARSE_GRAD_HOOK owning the table (e.g. GradSync(sparse_tables=False)
            # or a DDP-style dense all-reduce): the gradient is reduced densely in place, so other ranks'
            # rows land in it -- this rank's flags and re-zeroing would miss them.  Dense semantics.
            table._nr_row_touched = None
            return False
        key = id(table)
        buf = self.buf.get(key)
        if table.grad is not None:
            # torch's dense accumulation into the existing gradient; if that is our buffer, it now
            # holds rows this class does not track: zero it whole before its next use
            if buf is not None and table.grad.data_ptr() == buf.data_ptr():
                self.prev[key] = None
            table._nr_row_touched = None
            return False
        flags = self.flags.get(key)
        if buf is None or buf.shape != table.shape or buf.device != table.device:
            buf = self.buf[key] = torch.zeros_like(table)
            # per-row "may be non-zero" flags for Adam (it skips reading the rows flagged zero)
            flags = self.flags[key] = torch.zeros(table.shape[0], dtype=torch.uint8, device=table.device)
            self.prev.pop(key, None)
        elif key in self.prev and self.prev[key] is None:
            buf.zero_()
            flags.zero_()
            del self.prev[key]
        prev = self.prev.get(key)
        if prev is not None:
            buf.index_fill_(0, prev, 0.0)
            flags.index_fill_(0, prev, 0)
        # fixed summation order for duplicate ids (no atomics): the same bits every run
        K.rows_add_ordered(grads.reshape(rows.numel(), -1), rows.reshape(-1), buf)
        flags.index_fill_(0, rows.reshape(-1), 1)
        if prev is not None and prev.numel() == rows.numel():
            prev.copy_(rows.reshape(-1))      # in place: a captured step replays the same buffer
        else:
            self.prev[key] = rows.reshape(-1).clone()
        table.grad = buf
        table._nr_row_touched = (buf, flags, buf._version)   # (optim: valid while buf is unmodified)
        return True

    def clear(self):
        self.buf.clear()
        self.prev.clear()
        self.flags.clear()


def _zero_absent_word_rows(table, dtable, ur, pad_row):
    """Zero dtable's rows of ids absent from the batch (and the pad row).  Returns Adam's per-row
    flags (1 = the dgrad stores the row) when the gradient will become ``table.grad`` as it is: a leaf
    table whose ``.grad`` is None (no accumulation into an older gradient) in a single process (a
    dense all-reduce would add other ranks' rows).  None otherwise."""
    track = WORD_ROW_FLAGS and _is_param_leaf(table) and table.grad is None and not _multi_rank()
    flags = torch.empty(dtable.shape[0], dtype=torch.uint8, device=dtable.device) if track else None
    return flags if ur.zero_absent_rows(dtable, pad_row, flags) else None


def _word_row_flags(table, dtable, flags):
    """Publish (or clear) the word table's row flags for optim.FusedAdam.  The backward only leaves
    them pending, keyed by the gradient buffer's address and version counter; the table's
    post-accumulate-grad hook (_row_flag_hook) turns them into flags bound to the very ``.grad``
    tensor autograd installed (a weak reference to it), and only if that is the buffer, unmodified
    (autograd installs a lone returned gradient as it is; a copy changes the address, an in-place
    accumulation -- another use of the table in the graph, a second backward -- the version).  So the
    flags die with that gradient: after zero_grad(set_to_none) a new gradient the caching allocator
    places at the same address is a different tensor and never picks them up."""
    if _is_param_leaf(table):
        table._nr_row_touched = None
        table._nr_row_pending = ((dtable.data_ptr(), flags, dtable._version)
                                 if dtable is not None and flags is not None else None)
        if getattr(table, "_nr_row_hook", None) is None:
            table._nr_row_hook = table.register_post_accumulate_grad_hook(_row_flag_hook)


def _row_flag_hook(p):
    """Post-accumulate-grad hook of a table with published row flags (see _word_row_flags)."""
    pend = getattr(p, "_nr_row_pending", None)
    p._nr_row_pending = None
    g = p.grad
    if pend is not None and g is not None and g.data_ptr() == pend[0] and g._version == pend[2]:
        p._nr_row_touched = (weakref.ref(g), pend[1], g._version)
    elif isinstance(getattr(p, "_nr_row_touched", None), tuple) and isinstance(p._nr_row_touched[0], weakref.ref):
        p._nr_row_touched = None


def _multi_rank():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


LOCAL_ROW_GRAD = _LocalRowGrad()


class _WgradDeferHook:
    """Optional callback ``hook(run, out) -> bool`` for the news tower's projection weight-gradient
    GEMM (the longest kernel of the backward, issued after the word-table gradient).  ``run(max_cus)``
    launches the GEMM into ``out`` (the zero-filled weight gradient already handed to autograd);
    returning True means the callback launches it later itself -- GradSync's graphed data-parallel
    step runs it in its own graph, beside the word-table all-reduce (twotower.py:49-50's DDP
    overlap of the bucket reduction with the rest of the backward).

    ``max_cus``: CUs the weight-gradient GEMM may occupy while a collective is in flight
    (0 = all), so that RCCL's kernels are not locked out by the GEMM's one-workgroup-per-CU grid."""

    def __init__(self):
        self.fn = None
        self.max_cus = 0

    def set(self, fn, max_cus=0):
        self.fn = fn
        self.max_cus = int(max_cus)

    def __call__(self, run, out):
        if self.fn is None:
            return False
        return bool(self.fn(run, out))


WGRAD_DEFER_HOOK = _WgradDeferHook()


# ---------------------------------------------------------------------- MHA news encoder

class MHANewsFn(_GradAwareFn):
    """MHA_Encoder.forward (models/Encoders/MHA.py:21-39) on gathered token rows:
    Y = X [Wk; Wv]ᵀ + b  (one GEMM, gather fused)  ->  tied-QK 12-head attention
    -> LayerNorm -> Dropout -> learned-query pooling.   Returns (news [n, H], tok [T, H] or None)."""

    @staticmethod
    def forward(ctx, table, ids, mask, w_cat, b_cat, gamma, beta, query, heads, dk, dv, seq_len,
                pad_row, p_drop, seed, offset, want_tokens, rng=None):
        ctx.prec = K.get_gemm_precision()
        T = ids.numel()
        n = T // seq_len
        V, E = table.shape
        H = heads * dv
        NQ = heads * dk
        NY = NQ + H
        fused = K.mha_pool_supported(seq_len, heads, dk, dv)
        ur = None
        if fused and DEDUP_ROWS:
            # project each distinct word-table row once (Y rows = distinct ids, read through inv);
            # the backward sums dY per distinct row over the unmasked tokens only — the fused
            # tail gives masked tokens an exactly-zero dY (their P rows and columns are zero)
            ur = K.UniqueRows(ids, V, fill_row=pad_row if 0 <= pad_row < V else 0, grad_mask=mask)
            Y = _empty(ur.cap, NY, table)
            PROBE.run("proj_fwd", lambda: K.gemm_dyn(
                ur.cap, NY, E, K.operand(table, L.KCONTIG, rows=ur.uids, mapping=L.ROWS_GATHER),
                K.operand(w_cat, L.KCONTIG), Y, m_dev=ur.u_pad, bias=b_cat), Y, ur)
        else:
            Y = _empty(T, NY, table)
            PROBE.run("proj_fwd", lambda: K.gemm(
                T, NY, E, K.operand(table, L.KCONTIG, rows=ids, mapping=L.ROWS_GATHER),
                K.operand(w_cat, L.KCONTIG), Y, bias=b_cat), Y)
        news = _empty(n, H, table)
        probs = torch.empty(T, device=table.device)
        stats = torch.empty(T, 2, device=table.device)
        tok = _empty(T, H, table) if want_tokens else None
        if fused:
            # attention + LN + dropout + pooling in one kernel per title; when a backward will
            # run, the attention output O is saved too (the backward then skips recomputing it)
            O = _empty(T, H, table) if SPLIT_BWD and _backward_possible(ctx) else None
            # rng (device (seed, offset) snapshot) supersedes the host pair: kernel offset 0
            K.mha_pool_fwd(Y, mask, n, seq_len, heads, dk, dv, gamma, beta, query, news, stats, probs,
                           p_drop=p_drop, seed=seed, offset=0 if rng is not None else offset, zout=tok,
                           yrows=ur.inv if ur else None, rng=rng, oout=O)
        else:
            O = _empty(T, H, table)
            K.mha_attn_fwd(Y[:, :NQ], Y[:, NQ:NY], mask, n, seq_len, heads, dk, dv, O)
            K.attn_pool_fwd(O, query, mask, n, seq_len, news, probs, gamma=gamma, beta=beta, stats=stats,
                            p_drop=p_drop, seed=seed, offset=0 if rng is not None else offset, zout=tok, rng=rng)
        ctx.save_for_backward(table, ids, mask, w_cat, gamma, beta, query, Y, O, probs, stats)
        _reserve_zeros(ctx, table.device, (H,), (H,), (H,), (NY,), (NY, E))
        ctx.cfg = (heads, dk, dv, seq_len, pad_row, p_drop, seed, offset, fused)
        ctx.table_ref = table
        ctx.ur = ur
        ctx.rng = rng
        return news, tok

    @staticmethod
    @_gemm_backward
    def backward(ctx, dnews, dtok):
        table, ids, mask, w_cat, gamma, beta, query, Y, O, probs, stats = ctx.saved_tensors
        _word_row_flags(ctx.table_ref, None, None)
        rflags = None
        heads, dk, dv, seq_len, pad_row, p_drop, seed, offset, fused = ctx.cfg
        T = ids.numel()
        n = T // seq_len
        V, E = table.shape
        H = heads * dv
        NQ = heads * dk
        NY = NQ + H
        dnews = dnews.contiguous()
        dq, dgamma, dbeta, db, dw = _backward_zeros(ctx, table.device, (H,), (H,), (H,), (NY,), (NY, E))
        dz = dtok.contiguous() if dtok is not None else None
        ur = ctx.ur
        # one buffer: per-token gradient rows [0, T), then the per-distinct-row sums [T, T + cap); with
        # SINGLE_ROWS_DIRECT a token alone in its row's segment writes its row straight to the sums
        direct = fused and ur is not None and SINGLE_ROWS_DIRECT
        dYall = _empty(T + (ur.cap if ur is not None else 0), NY, table)
        dY = dYall[:T]
        if fused:
            # split form: the LN pass's per-token row terms (the head pass rebuilds dO from O with them)
            dob = torch.empty(T, 8, device=table.device) if O is not None and not FUSED_SAVED_BWD else None
            ws = _grad_copies(table.device, 3 * H + NY) if O is not None else None
            K.mha_pool_bwd(Y, mask, n, seq_len, heads, dk, dv, gamma, beta, query, stats, probs, dnews,
                           dYall if direct else dY, db, dq,
                           dgamma, dbeta, p_drop=p_drop, seed=seed, offset=0 if ctx.rng is not None else offset,
                           dz=dz, yrows=ur.inv if ur else None, rng=ctx.rng, o=O, dob=dob, ws=ws,
                           ws_copies=GRAD_COPIES if ws is not None else 0, seg=ur if direct else None, dyu_row0=T)
        else:
            dO = _empty(T, H, table)
            K.attn_pool_bwd(O, query, mask, n, seq_len, probs, dnews, dO, dq, gamma=gamma, beta=beta, stats=stats,
                            dgamma=dgamma, dbeta=dbeta, p_drop=p_drop, seed=seed,
                            offset=0 if ctx.rng is not None else offset, dz=dz, rng=ctx.rng)
            K.mha_attn_bwd(Y[:, :NQ], Y[:, NQ:NY], mask, n, seq_len, heads, dk, dv, dO, dY[:, :NQ], dY[:, NQ:NY],
                           dbias=db)
        dtable = None
        if ur is not None:
            # per-distinct-row gradient, then the two GEMMs over U rows instead of T tokens
            dYu = dYall[T:]
            if direct:
                ur.segment_sum_multi(dY, dYu)
            else:
                ur.segment_sum(dY, dYu)
            inflight = False
            if ctx.needs_input_grad[0]:
                if PROJ_DGRAD_TAIL_WS and ABSENT_ROWS_ZERO and ctx.prec == L.GEMM_BF16X6 and 0 <= pad_row < V:
                    # every present row is stored by the dgrad (its tail through the workspace, no
                    # atomics): zero only the absent rows and the pad row instead of the whole table
                    dtable = table_grad_buffer(ctx.table_ref, V, E, table.device, zero=False)
                    rflags = _zero_absent_word_rows(ctx.table_ref, dtable, ur, pad_row)
                else:
                    dtable = table_grad_buffer(ctx.table_ref, V, E, table.device, zero=True)
                # distinct rows (M = U, not U_pad: no duplicate pad ids): plain row stores
                wt = K.transpose(w_cat) if PROJ_DGRAD_KC else None   # kept alive by the closure

                def dgrad(dtable=dtable):   # bound now: the hook below may take the name's buffer
                    w_b = K.operand(wt, L.KCONTIG) if wt is not None else K.operand(w_cat, L.MNCONTIG)
                    K.gemm_dyn(ur.cap, E, NY, K.operand(dYu, L.KCONTIG), w_b, dtable,
                               m_dev=ur.n_rows, epilogue=L.EPI_SCATTER_ZEROED,
                               c_rows=K.rows_map(ur.uids, L.ROWS_GATHER), pad_row=pad_row,
                               workspace=PROJ_DGRAD_TAIL_WS)
                PROBE.run("proj_dgrad", dgrad, dtable, ur)
                if TABLE_GRAD_HOOK(ctx.table_ref, dtable):
                    dtable = None
                    inflight = True   # the table's all-reduce runs beside the weight gradient
                _word_row_flags(ctx.table_ref, dtable, rflags)
            prec = ctx.prec

            def wgrad(max_cus=0):
                K.gemm_dyn(NY, E, ur.cap, K.operand(dYu, L.MNCONTIG),
                           K.operand(table, L.MNCONTIG, rows=ur.uids, mapping=L.ROWS_GATHER), dw, k_dev=ur.u_pad,
                           epilogue=L.EPI_ATOMIC, split_k=_split_k(NY, E, ur.cap), prec=prec, max_cus=max_cus,
                           workspace=PROJ_WGRAD_WS)
            if not WGRAD_DEFER_HOOK(wgrad, dw):
                cus = WGRAD_DEFER_HOOK.max_cus if inflight else 0
                PROBE.run("proj_wgrad", lambda: wgrad(cus), dw, ur)
        else:
            if ctx.needs_input_grad[0]:
                dtable = table_grad_buffer(ctx.table_ref, V, E, table.device, zero=True)
                K.gemm(T, E, NY, K.operand(dY, L.KCONTIG), K.operand(w_cat, L.MNCONTIG), dtable,
                       epilogue=L.EPI_SCATTER, c_rows=K.rows_map(ids, L.ROWS_GATHER), pad_row=pad_row)
                if TABLE_GRAD_HOOK(ctx.table_ref, dtable):
                    dtable = None
            _proj_wgrad(dY, K.operand(table, L.MNCONTIG, rows=ids, mapping=L.ROWS_GATHER), dw, None, T)
        return (dtable, None, None, dw, db, dgamma, dbeta, dq.view_as(query), None, None, None, None, None,
                None, None, None, None, None)


# ---------------------------------------------------------------------- CNN news encoder

class CNNNewsFn(torch.autograd.Function):
    """CNN_Encoder.forward (models/Encoders/CNN.py:30-50): Conv1d(E->H, k=3, pad=1) as a
    K = 3E GEMM over CONV3 rows of the table (gather fused) with bias+ReLU epilogue; key =
    tanh(C Wqᵀ + bq) (GEMM, tanh epilogue); learned-query pooling with the token mask.
    ``w3`` is the conv weight as [H][tap*E + e].  Returns (news [n, H], C [T, H])."""

    @staticmethod
    def forward(ctx, table, ids, mask, w3, conv_b, wq, bq, query, seq_len, pad_row):
        # the token output C is rarely consumed: an unused one must not cost a zero-filled gradient
        ctx.set_materialize_grads(False)
        ctx.prec = K.get_gemm_precision()
        T = ids.numel()
        n = T // seq_len
        E = table.shape[1]
        H = w3.shape[0]
        C = _empty(T, H, table)
        K.gemm(T, H, 3 * E, K.operand(table, L.KCONTIG, rows=ids, mapping=L.ROWS_CONV3, seq_len=seq_len, seg=E),
               K.operand(w3, L.KCONTIG), C, bias=conv_b, epilogue=L.EPI_STORE_RELU)
        Kq = _empty(T, H, table)
        K.gemm(T, H, H, K.operand(C, L.KCONTIG), K.operand(wq, L.KCONTIG), Kq, bias=bq, epilogue=L.EPI_STORE_TANH)
        news = _empty(n, H, table)
        probs = torch.empty(T, device=table.device)
        K.attn_pool_fwd(C, query, mask, n, seq_len, news, probs, key=Kq)
        ctx.save_for_backward(table, ids, mask, w3, wq, query, C, Kq, probs)
        ctx.cfg = (seq_len, pad_row)
        ctx.table_ref = table
        return news, C

    @staticmethod
    @_gemm_backward
    def backward(ctx, dnews, dC_out):
        table, ids, mask, w3, wq, query, C, Kq, probs = ctx.saved_tensors
        _word_row_flags(ctx.table_ref, None, None)
        seq_len, pad_row = ctx.cfg
        T = ids.numel()
        n = T // seq_len
        V, E = table.shape
        H = w3.shape[0]
        if dnews is None:   # (grads not materialised) the pooled output unused
            dnews = torch.zeros(n, H, device=table.device)
        dev = table.device
        dnews = dnews.contiguous()
        # dC with its columns padded to a multiple of 32 (zeros): the table dgrad below contracts
        # over H and takes the fast GEMM path only for K % 32 == 0
        Hp = (H + 31) // 32 * 32
        dC_full = torch.zeros(T, Hp, device=dev)
        dC = dC_full[:, :H]
        dKq = _empty(T, H, table)
        dq = torch.zeros(H, device=dev)
        K.attn_pool_bwd(C, query, mask, n, seq_len, probs, dnews, dC, dq, key=Kq, dk=dKq, key_tanh=True,
                        dz=dC_out.contiguous() if dC_out is not None else None)
        # key projection: dWq = dKqᵀ C, dbq = colsum(dKq); dC += dKq Wq, then ReLU'(C)
        dwq, dbq, dconv_b, dw3 = _zeros_views(dev, (H, H), (H,), (H,), (H, 3 * E))
        _proj_wgrad(dKq, K.operand(C, L.MNCONTIG), dwq, dbq, T)
        K.gemm(T, H, H, K.operand(dKq, L.KCONTIG), K.operand(wq, L.MNCONTIG), dC, epilogue=L.EPI_ACCUM_GATE,
               c_rows=K.aux_operand(C))
        _proj_wgrad(dC, K.operand(table, L.MNCONTIG, rows=ids, mapping=L.ROWS_CONV3, seq_len=seq_len, seg=E),
                    dw3, dconv_b, T)
        dtable = None
        if ctx.needs_input_grad[0]:
            dtable = table_grad_buffer(ctx.table_ref, V, E, dev, zero=True)
            w3p = w3 if Hp == H else torch.cat([w3, w3.new_zeros(Hp - H, 3 * E)], 0)
            K.gemm(T, 3 * E, Hp, K.operand(dC_full, L.KCONTIG), K.operand(w3p, L.MNCONTIG), dtable,
                   epilogue=L.EPI_SCATTER, c_rows=K.rows_map(ids, L.ROWS_CONV3, seq_len=seq_len, seg=E),
                   pad_row=pad_row)
            if TABLE_GRAD_HOOK(ctx.table_ref, dtable):
                dtable = None
        return dtable, None, None, dw3, dconv_b, dwq, dbq, dq.view_as(query), None, None


class CNNWeightsFn(torch.autograd.Function):
    """The distinct-row CNN encoder's weight operands (nr_cnn_pack_weights): the Conv1d weight
    [H, E, 3] as w3t [3*Hp, E] (row tap*Hp + h), its transpose w3tt [E, 3*Hp] (the table dgrad's
    K-contiguous weight, CNN_DGRAD_KC; None otherwise) and the key projection zero-padded to
    [Hp, Hp] / [Hp], in one launch; the backward maps the three gradients back in one launch."""

    @staticmethod
    def forward(ctx, conv_w, wq, bq, Hp):
        H, E = conv_w.shape[0], conv_w.shape[1]
        dev = conv_w.device
        w3t = torch.empty(3 * Hp, E, device=dev)
        w3tt = torch.empty(E, 3 * Hp, device=dev) if CNN_DGRAD_KC else None
        wqp = torch.empty(Hp, Hp, device=dev)
        bqp = torch.empty(Hp, device=dev)
        for t in (conv_w, wq, bq):
            if not t.is_contiguous():
                raise L.HipError("cnn weights must be contiguous")
        L.call("nr_cnn_pack_weights", L.ptr(conv_w), L.ptr(wq), L.ptr(bq), H, E, Hp, L.ptr(w3t), L.ptr(wqp),
               L.ptr(bqp), L.ptr(w3tt), L.stream_ptr(conv_w))
        ctx.cfg = (H, E, Hp)
        if w3tt is not None:
            ctx.mark_non_differentiable(w3tt)
        return w3t, wqp, bqp, w3tt

    @staticmethod
    def backward(ctx, dw3t, dwqp, dbqp, _dw3tt):
        H, E, Hp = ctx.cfg
        dev = (dw3t if dw3t is not None else dwqp).device
        dw3t = dw3t.contiguous() if dw3t is not None else torch.zeros(3 * Hp, E, device=dev)
        dwqp = dwqp.contiguous() if dwqp is not None else torch.zeros(Hp, Hp, device=dev)
        dbqp = dbqp.contiguous() if dbqp is not None else torch.zeros(Hp, device=dev)
        dcw = torch.empty(H, E, 3, device=dev)
        dwq = torch.empty(H, H, device=dev)
        dbq = torch.empty(H, device=dev)
        L.call("nr_cnn_unpack_grads", L.ptr(dw3t), L.ptr(dwqp), L.ptr(dbqp), H, E, Hp, L.ptr(dcw), L.ptr(dwq),
               L.ptr(dbq), L.stream_ptr(dw3t))
        return dcw, dwq, dbq, None


class CNNNewsRowsFn(_GradAwareFn):
    """CNN_Encoder.forward (models/Encoders/CNN.py:30-50) over DISTINCT word rows.

    The k = 3 Conv1d is linear per tap and the embedding lookup (BERT.py:39) is a row gather, so
    they commute: P = table[uids] · [W_0 | W_1 | W_2]ᵀ is ONE GEMM over the U distinct ids of the
    batch (U ≈ 24.6 k of T = 52.8 k tokens on uniform ids), and C[t] = ReLU(b + Σ_j P[inv[t+j-1]][j])
    is a three-row gather-add (nr_conv3_rows_fwd).  The backward sums the shifted dC rows per
    distinct id once (S = nr_segment_rows_sum_conv3), after which the table gradient
    (S · W3 -> plain stores into the distinct rows, no atomics) and the conv weight gradient
    (Sᵀ · table[uids]) are GEMMs over U rows instead of T tokens.

    w3t: [3*Hp, E] with row tap*Hp + h = Conv1d.weight[h, :, tap] (rows h >= H zero); wq, bq: the
    key projection zero-padded to [Hp, Hp] / [Hp] so every contraction has K % 32 == 0; query: the
    pooling query [1, H] (the pooling runs over the padded width, nr_seq_pool_*, with features past
    H of the query and of dnews taken as zero).
    Returns (news [n, H] view, C [T, H] view)."""

    @staticmethod
    def forward(ctx, table, ids, mask, w3t, conv_b, wq, bq, query, seq_len, pad_row, H, w3tt=None):
        # the token output C is rarely consumed: an unused one must not cost a zero-filled gradient
        # (and a padded copy of it) per step
        ctx.set_materialize_grads(False)
        ctx.prec = K.get_gemm_precision()
        T = ids.numel()
        n = T // seq_len
        V, E = table.shape
        Hp = w3t.shape[0] // 3
        ur = K.UniqueRows(ids, V, fill_row=pad_row if 0 <= pad_row < V else 0)
        P = _empty(ur.cap, 3 * Hp, table)
        K.gemm_dyn(ur.cap, 3 * Hp, E, K.operand(table, L.KCONTIG, rows=ur.uids, mapping=L.ROWS_GATHER),
                   K.operand(w3t, L.KCONTIG), P, m_dev=ur.u_pad)
        C = _empty(T, Hp, table)
        K.conv3_rows_fwd(P, Hp, H, ur.inv, seq_len, conv_b, C, relu=True)
        news = _empty(n, Hp, table)
        probs = torch.empty(T, device=table.device)
        fused = FUSED_KEYPOOL and K.cnn_keypool_supported(Hp, seq_len)
        if fused:
            # key projection + tanh + pooling per title; with a backward to come K is kept (the backward
            # reads it instead of recomputing the key products, KEYPOOL_SAVE_K)
            Kq = _empty(T, Hp, table) if KEYPOOL_SAVE_K and _backward_possible(ctx) else None
            K.cnn_keypool_fwd(C, wq, bq, query, mask, n, seq_len, news, probs, qn=H, prec=ctx.prec, kout=Kq)
        else:
            Kq = _empty(T, Hp, table)
            K.gemm(T, Hp, Hp, K.operand(C, L.KCONTIG), K.operand(wq, L.KCONTIG), Kq, bias=bq,
                   epilogue=L.EPI_STORE_TANH)
            # pooling over the padded width: C and Kq are exactly zero past H, and so is the padded query
            K.seq_pool_fwd(C, query, mask, n, seq_len, Hp, news, probs, key=Kq, qn=H)
        ctx.save_for_backward(table, ids, mask, w3t, wq, bq, query, C, Kq, probs, w3tt)
        ctx.cfg = (seq_len, pad_row, H, fused)
        _reserve_zeros(ctx, table.device, (Hp, Hp), (Hp,), (H,), (3 * Hp, E), (H,))
        ctx.table_ref = table
        ctx.ur = ur
        return news[:, :H], C[:, :H]

    @staticmethod
    @_gemm_backward
    def backward(ctx, dnews, dC_out):
        table, ids, mask, w3t, wq, bq, query, C, Kq, probs, w3tt = ctx.saved_tensors
        _word_row_flags(ctx.table_ref, None, None)
        rflags = None
        seq_len, pad_row, H, fused = ctx.cfg
        ur = ctx.ur
        T = ids.numel()
        n = T // seq_len
        if dnews is None:   # (grads not materialised) the pooled output unused
            dnews = torch.zeros(n, H, device=table.device)
        V, E = table.shape
        Hp = w3t.shape[0] // 3
        dev = table.device
        dC = _empty(T, Hp, table)
        dwq, dbq, dconv_b, dw3t, dq = _backward_zeros(ctx, dev, (Hp, Hp), (Hp,), (H,), (3 * Hp, E), (H,))
        if dnews.stride(-1) != 1:
            dnews = dnews.contiguous()
        if fused:
            # one pass per title: key recomputed, pooling / tanh / key-projection backward, ReLU gate,
            # dWq / dbq / dq / dconv_b summed over per-workgroup partials
            dz = dC_out if dC_out is None or dC_out.stride(-1) == 1 else dC_out.contiguous()
            K.cnn_keypool_bwd(C, wq, bq, query, n, seq_len, H, probs, dnews, dC, dwq, dbq, dq, dconv_b, dz=dz,
                              prec=ctx.prec, kin=Kq)
        else:
            dKq = _empty(T, Hp, table)
            # dC = p dnews (+ dC_out), dKq = ds q (1 - Kq²) over the padded width: exactly zero past H
            # (dnews and the query count as zero there)
            dz = torch.nn.functional.pad(dC_out, (0, Hp - H)) if dC_out is not None else None
            K.seq_pool_bwd(C, query, mask, n, seq_len, Hp, probs, dnews, dC, dq, key=Kq, dk=dKq, key_tanh=True,
                           dz=dz, qn=H)
            # key projection: dWq = dKqᵀ C, dbq = colsum(dKq); dC = ReLU'(C) ⊙ (dC + dKq Wq) (padded
            # columns of C are zero, so the gate also zeroes dC's padding)
            _proj_wgrad(dKq, K.operand(C, L.MNCONTIG), dwq, dbq, T)
            K.gemm(T, Hp, Hp, K.operand(dKq, L.KCONTIG), K.operand(wq, L.MNCONTIG), dC, epilogue=L.EPI_ACCUM_GATE,
                   c_rows=K.aux_operand(C))
            K.colsum(dC, T, H, dconv_b)
        S = _empty(ur.cap, 3 * Hp, table)
        ur.segment_sum_conv3(dC, S, Hp, seq_len)
        dtable = None
        inflight = False
        if ctx.needs_input_grad[0]:
            # the dgrad stores every present row -- bf16x6: its stream-K tail through the workspace;
            # bf16: as plain scatter stores (NR_EPI_SCATTER_STORE: no atomic tail, which would need
            # zeroed rows) -- so only the absent rows and the pad row are zeroed
            epi = L.EPI_SCATTER_ZEROED
            if ABSENT_ROWS_ZERO and 0 <= pad_row < V and ((PROJ_DGRAD_TAIL_WS and ctx.prec == L.GEMM_BF16X6) or
                                                          ctx.prec == L.GEMM_BF16):
                if ctx.prec == L.GEMM_BF16:
                    epi = L.EPI_SCATTER_STORE
                dtable = table_grad_buffer(ctx.table_ref, V, E, dev, zero=False)
                rflags = _zero_absent_word_rows(ctx.table_ref, dtable, ur, pad_row)
            else:
                dtable = table_grad_buffer(ctx.table_ref, V, E, dev, zero=True)
            if CNN_DGRAD_KC:   # the weights transposed (1.5 MB, by the pack launch) so both operands are k-contiguous
                w_b = K.operand(w3tt if w3tt is not None else w3t.t().contiguous(), L.KCONTIG)
            else:
                w_b = K.operand(w3t, L.MNCONTIG)
            K.gemm_dyn(ur.cap, E, 3 * Hp, K.operand(S, L.KCONTIG), w_b, dtable,
                       m_dev=ur.n_rows, epilogue=epi, c_rows=K.rows_map(ur.uids, L.ROWS_GATHER),
                       pad_row=pad_row, workspace=PROJ_DGRAD_TAIL_WS)
            if TABLE_GRAD_HOOK(ctx.table_ref, dtable):
                dtable = None
                inflight = True
            _word_row_flags(ctx.table_ref, dtable, rflags)
        K.gemm_dyn(3 * Hp, E, ur.cap, K.operand(S, L.MNCONTIG),
                   K.operand(table, L.MNCONTIG, rows=ur.uids, mapping=L.ROWS_GATHER), dw3t, k_dev=ur.u_pad,
                   epilogue=L.EPI_ATOMIC, split_k=_split_k(3 * Hp, E, ur.cap),
                   max_cus=WGRAD_DEFER_HOOK.max_cus if inflight else 0,
                   workspace=(WGRAD_WS_BF16 and ctx.prec == L.GEMM_BF16) or
                   (WGRAD_WS_BF16X6 and ctx.prec == L.GEMM_BF16X6))
        return (dtable, None, None, dw3t, dconv_b, dwq, dbq, dq.view_as(query), None, None, None, None)


# ---------------------------------------------------------------------- pooling user encoder

class AttnPoolFn(_GradAwareFn):
    """Attention_Pooling.forward (models/Encoders/Pooling.py:12-25): learned-query pooling of
    the history with the history mask.  x: [B*N, H] rows view; returns [B, H]."""

    @staticmethod
    def forward(ctx, x, query, mask, B, N):
        H = query.numel()
        probs = torch.empty(B * N, device=x.device)
        # one wave per sequence (nr_seq_pool_*) when the rows are float4-addressable
        sp = K.seq_pool_supported(H, N) and x.stride(-1) == 1 and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0
        out = _empty(B, H, x)
        if sp:
            K.seq_pool_fwd(x, query, mask, B, N, H, out, probs)
        else:
            K.attn_pool_fwd(x, query, mask, B, N, out, probs)
        ctx.save_for_backward(x, query, mask, probs)
        ctx.cfg = (B, N, H, sp)
        ctx.dx_dest = GRAD_DEST.take(x)
        _reserve_zeros(ctx, x.device, (H,))
        return out

    @staticmethod
    def backward(ctx, dout):
        x, query, mask, probs = ctx.saved_tensors
        B, N, H, sp = ctx.cfg
        dx = _grad_out(ctx.dx_dest, B * N, H, x)
        dq, = _backward_zeros(ctx, x.device, (H,))
        if sp:
            K.seq_pool_bwd(x, query, mask, B, N, H, probs, dout if dout.stride(-1) == 1 else dout.contiguous(), dx, dq)
            return dx, dq.view_as(query), None, None, None
        K.attn_pool_bwd(x, query, mask, B, N, probs, dout.contiguous(), dx, dq)
        return dx, dq.view_as(query), None, None, None


# ---------------------------------------------------------------------- MHA over rows

class MHAFn(_GradAwareFn):
    """MultiheadAttention.forward (models/Modules/Attention.py:115-147) on plain rows:
    Y = x [Wk; Wv]ᵀ + b (GEMM) -> tied-QK attention core (pairwise token mask).
    x: [nseq*L, D] -> [nseq*L, heads*dv].  Used by MHA_User_Encoder (MHA.py:58-75) and the
    standalone MultiheadAttention module."""

    @staticmethod
    def forward(ctx, x, mask, w_cat, b_cat, nseq, seq_len, heads, dk, dv):
        ctx.prec = K.get_gemm_precision()
        D = x.shape[1]
        NQ = heads * dk
        NY = w_cat.shape[0]
        rows = nseq * seq_len
        Y = _empty(rows, NY, x)
        K.gemm(rows, NY, D, K.operand(x, L.KCONTIG), K.operand(w_cat, L.KCONTIG), Y, bias=b_cat)
        O = _empty(rows, heads * dv, x)
        K.mha_attn_fwd(Y[:, :NQ], Y[:, NQ:NY], mask, nseq, seq_len, heads, dk, dv, O)
        ctx.save_for_backward(x, mask, w_cat, Y)
        ctx.cfg = (nseq, seq_len, heads, dk, dv)
        ctx.dx_dest = GRAD_DEST.take(x)
        _reserve_zeros(ctx, x.device, (NY, D), (NY,))
        return O

    @staticmethod
    @_gemm_backward
    def backward(ctx, dO):
        x, mask, w_cat, Y = ctx.saved_tensors
        nseq, seq_len, heads, dk, dv = ctx.cfg
        D = x.shape[1]
        NQ = heads * dk
        NY = w_cat.shape[0]
        rows = nseq * seq_len
        dev = x.device
        if dO.stride(-1) != 1 or dO.stride(0) % 4 or dO.data_ptr() % 16:
            dO = dO.contiguous()
        dY = _empty(rows, NY, x)
        dw, db = _backward_zeros(ctx, dev, (NY, D), (NY,))
        # the projection bias gradient (column sums of dY) accumulates inside the attention backward
        K.mha_attn_bwd(Y[:, :NQ], Y[:, NQ:NY], mask, nseq, seq_len, heads, dk, dv, dO, dY[:, :NQ], dY[:, NQ:NY],
                       dbias=db)
        split = USER_DGRAD_SPLIT if NY >= 512 * USER_DGRAD_SPLIT else 1
        if split > 1:
            # few output tiles (1600 x 384 for the NRMS user encoder) over a long contraction (1152): split
            # K and add the pieces atomically into a zeroed dx
            dx = torch.zeros(rows, D, device=dev)
            K.gemm(rows, D, NY, K.operand(dY, L.KCONTIG), K.operand(w_cat, L.MNCONTIG), dx, epilogue=L.EPI_ATOMIC,
                   split_k=split)
        else:
            dx = _grad_out(ctx.dx_dest, rows, D, x)
            K.gemm(rows, D, NY, K.operand(dY, L.KCONTIG), K.operand(w_cat, L.MNCONTIG), dx)
        _proj_wgrad(dY, K.operand(x, L.MNCONTIG), dw, None, rows)
        return dx, None, dw, db, None, None, None, None, None


# ---------------------------------------------------------------------- recurrent user encoders

class RNNUserFn(_GradAwareFn):
    """RNN_User_Encoder (RNN.py:50-73) and LSTUR_User_Encoder (RNN.py:88-104):
    gx = x W_ihᵀ + b_ih for all steps (GEMM) -> sequential cell kernel -> h at step len-1.
    LSTUR: reverse=True, mask=None (all N steps), h0 = user_table[h0_idx]."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, user_table, cell, mask, B, N, reverse, h0_idx):
        ctx.prec = K.get_gemm_precision()
        H = x.shape[1]
        G = 4 if cell == L.CELL_LSTM else 3
        dev = x.device
        ctx.dx_dest = GRAD_DEST.take(x)   # (before x is padded below)
        gx = _empty(B * N, G * H, x)
        # the input projection contracts over H: padded to a multiple of 32 with zero columns (a 1 MB
        # copy of x, 0.4 MB of w_ih) it runs on the fast GEMM path instead of the generic one
        Hp = _ceil32(H)
        if Hp != H:
            x = torch.nn.functional.pad(x, (0, Hp - H))
            w_k = torch.nn.functional.pad(w_ih.detach(), (0, Hp - H))
        else:
            w_k = w_ih
        K.gemm(B * N, G * H, Hp, K.operand(x, L.KCONTIG), K.operand(w_k, L.KCONTIG), gx, bias=b_ih)
        gates = torch.empty(B * N, 4 * H, device=dev)
        hprev = torch.empty(B * N, H, device=dev)
        cprev = torch.empty(B * N, H, device=dev) if cell == L.CELL_LSTM else None
        hout = _empty(B, H, x)
        whh_t = w_hh.detach().t().contiguous()
        K.rnn_fwd(cell, gx, whh_t, b_hh, B, N, H, gates, hprev, cprev, hout,
                  h0=user_table if user_table is not None else None, h0_idx=h0_idx, mask=mask, reverse=reverse)
        ctx.save_for_backward(x, w_ih, w_hh, gates, hprev, cprev, mask, h0_idx, user_table)
        ctx.cfg = (cell, B, N, reverse)
        _reserve_zeros(ctx, dev, (G * H, H), (G * H,), (G * H, H), (G * H,))
        ctx.table_ref = user_table
        return hout

    @staticmethod
    @_gemm_backward
    def backward(ctx, dh):
        x, w_ih, w_hh, gates, hprev, cprev, mask, h0_idx, user_table = ctx.saved_tensors
        cell, B, N, reverse = ctx.cfg
        H = w_ih.shape[1]
        Hp = x.shape[1]            # x saved zero-padded to a multiple of 32 columns (forward)
        G = 4 if cell == L.CELL_LSTM else 3
        GH = G * H
        GHp = _ceil32(GH) if Hp != H else GH
        dev = x.device
        # the gate gradients with zero columns up to GHp (the dx GEMM contracts over them) and the
        # padded operands below keep the three GEMMs on the fast path (K % 32 == 0, float4 rows)
        dgi_b = torch.empty(B * N, GHp, device=dev)
        dgh_b = torch.empty(B * N, GHp, device=dev) if cell == L.CELL_GRU else None
        for t in (dgi_b, dgh_b):
            if t is not None and GHp != GH:
                t[:, GH:].zero_()
        dgi = dgi_b[:, :GH]
        dgh = dgh_b[:, :GH] if dgh_b is not None else None
        dh0 = torch.empty(B, H, device=dev) if user_table is not None else None
        K.rnn_bwd(cell, w_hh.contiguous(), gates, hprev, cprev, B, N, H, dh.contiguous(), dgi, dgh=dgh, dh0=dh0,
                  mask=mask, reverse=reverse)
        dgh_ = dgi if dgh is None else dgh
        dx = _grad_out(ctx.dx_dest, B * N, H, x)
        if Hp != H:
            w_k = torch.nn.functional.pad(w_ih.detach(), (0, Hp - H, 0, GHp - GH))
            K.gemm(B * N, H, GHp, K.operand(dgi_b, L.KCONTIG), K.operand(w_k, L.MNCONTIG), dx)
            h_k = torch.nn.functional.pad(hprev, (0, Hp - H))
        else:
            K.gemm(B * N, H, GH, K.operand(dgi, L.KCONTIG), K.operand(w_ih, L.MNCONTIG), dx)
            h_k = hprev
        dw_ih, db_ih, dw_hh, db_hh = _backward_zeros(ctx, dev, (GH, H), (GH,), (GH, H), (GH,))
        _proj_wgrad(dgi, K.operand(x, L.MNCONTIG), dw_ih, db_ih, B * N)
        _proj_wgrad(dgh_, K.operand(h_k, L.MNCONTIG), dw_hh, db_hh, B * N)
        dtab = None
        if user_table is not None and ctx.needs_input_grad[5]:
            if not SPARSE_GRAD_HOOK(ctx.table_ref, h0_idx, dh0) and not LOCAL_ROW_GRAD(ctx.table_ref, h0_idx, dh0):
                dtab = torch.zeros_like(user_table)
                K.embedding_bwd(dh0, h0_idx, dtab, padding_idx=None)
        return dx, dw_ih, dw_hh, db_ih, db_hh, dtab, None, None, None, None, None, None


# ---------------------------------------------------------------------- scorer

class ScoreFn(torch.autograd.Function):
    """compute_score + log_softmax (training) / sigmoid (eval)
    (models/TwoTowerBaseModel.py:51-75).  cdd [B*C, H] rows view, user [B, H] -> [B, C]."""

    @staticmethod
    def forward(ctx, cdd, user, B, C, mode):
        H = user.shape[1]
        logits = torch.empty(B, C, device=user.device)
        K.score_fwd(cdd, user, B, C, H, mode, logits)
        ctx.save_for_backward(cdd, user, logits)
        ctx.cfg = (B, C, mode)
        ctx.dcdd_dest = GRAD_DEST.take(cdd)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        cdd, user, logits = ctx.saved_tensors
        B, C, mode = ctx.cfg
        H = user.shape[1]
        dcdd = _grad_out(ctx.dcdd_dest, B * C, H, user)
        duser = _empty(B, H, user)
        K.score_bwd(cdd, user, logits, dlogits.contiguous(), B, C, H, mode, dcdd, duser)
        return dcdd, duser, None, None, None


class ScoreNLLFn(torch.autograd.Function):
    """compute_score + log_softmax (models/TwoTowerBaseModel.py:51-75) and Manager._train's
    NLLLoss (utils/Manager.py:382,641; reduction 'mean') in one kernel each way.
    -> (logits [B, C], loss []); the backward takes either gradient or both."""

    @staticmethod
    def forward(ctx, cdd, user, B, C, label):
        H = user.shape[1]
        logits = torch.empty(B, C, device=user.device)
        loss = torch.empty((), device=user.device)
        label = label.to(user.device).reshape(-1)
        label = label if label.is_contiguous() else label.contiguous()
        K.score_nll_fwd(cdd, user, label, B, C, H, logits, loss)
        ctx.save_for_backward(cdd, user, logits, label)
        ctx.cfg = (B, C)
        ctx.dcdd_dest = GRAD_DEST.take(cdd)
        ctx.set_materialize_grads(False)
        return logits, loss

    @staticmethod
    def backward(ctx, dlogits, dloss):
        cdd, user, logits, label = ctx.saved_tensors
        B, C = ctx.cfg
        H = user.shape[1]
        dcdd = _grad_out(ctx.dcdd_dest, B * C, H, user)
        duser = _empty(B, H, user)
        if dlogits is not None and not dlogits.is_contiguous():
            dlogits = dlogits.contiguous()
        K.score_nll_bwd(cdd, user, logits, label, dloss, dlogits, B, C, H, dcdd, duser)
        return dcdd, duser, None, None, None


class EmbeddingFn(torch.autograd.Function):
    """BERT_Embedding.forward (models/Embeddings/BERT.py:24-40): row gather; the backward is
    a padding_idx-aware scatter-add into a dense table gradient (embedding_dense_backward)."""

    @staticmethod
    def forward(ctx, table, ids, padding_idx):
        out = torch.empty(ids.numel(), table.shape[1], device=table.device)
        K.embedding_fwd(table, ids, out)
        ctx.save_for_backward(ids)
        ctx.cfg = (tuple(table.shape), padding_idx)
        return out

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        shape, pad = ctx.cfg
        dtable = torch.zeros(shape, device=dout.device)
        K.embedding_bwd(dout.contiguous(), ids, dtable, padding_idx=pad)
        return dtable, None, None
