"""bf16x6 GEMM arithmetic (nr_gemm_set_precision(NR_GEMM_BF16X6)): every operand-mode combination
of the split kernel against an fp64 reference, held to the same error bound as the exact-f32 MFMA
path (the dropped split terms are O(2^-24) of each product)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import _lib as L
from newsrec_amd import kernels as K


@pytest.fixture
def bf16x6():
    old = K.set_gemm_precision(L.GEMM_BF16X6)
    yield
    K.set_gemm_precision(old)


def _tol(a, b, k):
    return 1e-5 * a.abs().max().item() * b.abs().max().item() * k ** 0.5 + 1e-6


def _run_both(fn):
    """-> (f32 result, bf16x6 result)"""
    old = K.set_gemm_precision(L.GEMM_F32)
    try:
        r32 = fn()
        K.set_gemm_precision(L.GEMM_BF16X6)
        r6 = fn()
    finally:
        K.set_gemm_precision(old)
    torch.cuda.synchronize()
    return r32, r6


def _check(r32, r6, want, tol):
    e32 = (r32.double().cpu() - want).abs().max().item()
    e6 = (r6.double().cpu() - want).abs().max().item()
    assert e6 <= tol, (e6, tol)
    assert e6 <= 4 * e32 + 1e-6, (e6, e32)   # fp32-class: within a small factor of the f32 MFMA
    assert not torch.equal(r32, r6) or e32 == 0.0   # the split kernel really ran (results differ in rounding)


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1)])
def test_split_plain_layouts(la, lb):
    g = torch.Generator().manual_seed(11 + la + 2 * lb)
    M, N, Kd = 1000, 520, 768
    a = torch.randn(M, Kd, generator=g)
    b = torch.randn(Kd, N, generator=g)
    bias = torch.randn(N, generator=g)
    As = (a if la == 0 else a.t().contiguous()).cuda()
    Bs = (b.t().contiguous() if lb == 0 else b).cuda()
    bd = bias.cuda()
    want = a.double() @ b.double()
    if la == 1:   # wgrad form: atomic epilogue, no bias
        def fn():
            C = torch.zeros(M, N, device="cuda")
            K.gemm_dyn(M, N, Kd, K.operand(As, la), K.operand(Bs, lb), C, epilogue=L.EPI_ATOMIC, split_k=3)
            return C
    else:
        want = want + bias.double()
        def fn():
            C = torch.empty(M, N, device="cuda")
            K.gemm_dyn(M, N, Kd, K.operand(As, la), K.operand(Bs, lb), C, bias=bd)
            return C
    r32, r6 = _run_both(fn)
    _check(r32, r6, want, _tol(a, b, Kd))


def test_split_gather_scatter_and_wgrad():
    g = torch.Generator().manual_seed(5)
    V, E, T, N = 3000, 768, 2016, 1152
    table = torch.randn(V, E, generator=g) * 0.5
    tok = torch.randint(1, V, (T,), generator=g)
    tok[:7] = 0
    W = torch.randn(N, E, generator=g) / 16
    tc, tokc, Wc = table.cuda(), tok.cuda(), W.cuda()
    want = table[tok].double() @ W.double().t()

    def fwd():
        Y = torch.empty(T, N, device="cuda")
        K.gemm_dyn(T, N, E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_GATHER), K.operand(Wc, L.KCONTIG), Y)
        return Y
    r32, r6 = _run_both(fwd)
    _check(r32, r6, want, _tol(table, W, E))

    dY = torch.randn(T, N, generator=g)
    dYc = dY.cuda()
    want_t = torch.zeros(V, E, dtype=torch.float64).index_add_(0, tok, dY.double() @ W.double())
    want_t[0] = 0

    def dgrad():
        dt = torch.zeros(V, E, device="cuda")
        K.gemm_dyn(T, E, N, K.operand(dYc, L.KCONTIG), K.operand(Wc, L.MNCONTIG), dt, epilogue=L.EPI_SCATTER,
                   c_rows=K.rows_map(tokc, L.ROWS_GATHER), pad_row=0)
        return dt
    r32, r6 = _run_both(dgrad)
    _check(r32, r6, want_t, 8 * _tol(dY, W, N))

    want_w = dY.double().t() @ table[tok].double()

    def wgrad():
        dw = torch.zeros(N, E, device="cuda")
        K.gemm_dyn(N, E, T, K.operand(dYc, L.MNCONTIG), K.operand(tc, L.MNCONTIG, rows=tokc, mapping=L.ROWS_GATHER),
                   dw, epilogue=L.EPI_ATOMIC, split_k=2)
        return dw
    r32, r6 = _run_both(wgrad)
    _check(r32, r6, want_w, _tol(dY, table, T))


def test_split_gelu_and_conv3():
    g = torch.Generator().manual_seed(9)
    M, N, Kd = 700, 3072, 768
    a = torch.randn(M, Kd, generator=g)
    w = torch.randn(N, Kd, generator=g) / 28
    b = torch.randn(N, generator=g) * 0.1
    ac, wc, bc = a.cuda(), w.cuda(), b.cuda()
    pre = a.double() @ w.double().t() + b.double()

    def fn():
        U = torch.empty(M, N, device="cuda")
        G = torch.empty(M, N, device="cuda")
        K.gemm_dyn(M, N, Kd, K.operand(ac, L.KCONTIG), K.operand(wc, L.KCONTIG), G, bias=bc,
                   epilogue=L.EPI_STORE_GELU, c_rows=K.operand(U, L.KCONTIG))
        return torch.cat([U, G], 1)
    r32, r6 = _run_both(fn)
    want = torch.cat([pre, torch.nn.functional.gelu(pre)], 1)
    _check(r32, r6, want, _tol(a, w, Kd))

    # conv3 (k = 3 taps x E) over gathered token rows, as CNN_Encoder's Conv1d
    V, E, n, Lq, H = 500, 256, 60, 30, 160
    table = torch.randn(V, E, generator=g)
    tok = torch.randint(0, V, (n * Lq,), generator=g)
    W3 = torch.randn(H, 3 * E, generator=g) / 20
    tcu, tokc, W3c = table.cuda(), tok.cuda(), W3.cuda()
    x = table[tok].view(n, Lq, E).double()
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1))
    cols = torch.cat([xp[:, 0:Lq], xp[:, 1:Lq + 1], xp[:, 2:Lq + 2]], -1).reshape(n * Lq, 3 * E)
    wantc = cols @ W3.double().t()

    def conv():
        Y = torch.empty(n * Lq, H, device="cuda")
        K.gemm_dyn(n * Lq, H, 3 * E, K.operand(tcu, L.KCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Lq, seg=E),
                   K.operand(W3c, L.KCONTIG), Y)
        return Y
    r32, r6 = _run_both(conv)
    _check(r32, r6, wantc, _tol(table, W3, 3 * E))


def test_split_conv3_wgrad():
    """dW3 = dCᵀ conv3(table[tok]) (MN_CONV3 B operand, split-K atomics): CNN_Encoder's conv wgrad."""
    from newsrec_amd import functions as F
    g = torch.Generator().manual_seed(4)
    V, E, n, Lq, H = 400, 256, 64, 30, 150
    table = torch.randn(V, E, generator=g)
    tok = torch.randint(0, V, (n * Lq,), generator=g)
    dC = torch.randn(n * Lq, H, generator=g)
    x = table[tok].view(n, Lq, E).double()
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1))
    cols = torch.cat([xp[:, 0:Lq], xp[:, 1:Lq + 1], xp[:, 2:Lq + 2]], -1).reshape(n * Lq, 3 * E)
    want = dC.double().t() @ cols
    tc, tokc = table.cuda(), tok.cuda()
    dCc = torch.zeros(n * Lq, 152, device="cuda")
    dCc[:, :H] = dC.cuda()

    def fn():
        dw = torch.zeros(H, 3 * E, device="cuda")
        K.gemm_dyn(H, 3 * E, n * Lq, K.operand(dCc[:, :H], L.MNCONTIG),
                   K.operand(tc, L.MNCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Lq, seg=E), dw,
                   epilogue=L.EPI_ATOMIC, split_k=F._split_k(H, 3 * E, n * Lq))
        return dw
    r32, r6 = _run_both(fn)
    _check(r32, r6, want, _tol(dC, table, n * Lq))


# ---------------------------------------------------------------- bf16 arithmetic (NR_GEMM_BF16)

def _bf(x):
    """fp32 -> bf16 (RNE) -> fp64: the operand values the bf16 kernel multiplies."""
    return x.bfloat16().double()


def _bf16_tol(a, b, k):
    # products of bf16 values are exact in fp32; only the fp32 accumulation over k rounds
    return 4e-7 * a.abs().max().item() * b.abs().max().item() * k + 1e-6


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 1)])
def test_bf16_plain_layouts(la, lb):
    """Every plain layout in bf16 arithmetic equals the fp64 product of the bf16-rounded operands
    to fp32 accumulation error (and so really ran on the one-product kernel: the f32 path's
    result is further from that reference than the bound)."""
    g = torch.Generator().manual_seed(21 + la + 2 * lb)
    M, N, Kd = 1000, 520, 768
    a = torch.randn(M, Kd, generator=g)
    b = torch.randn(Kd, N, generator=g)
    As = (a if la == 0 else a.t().contiguous()).cuda()
    Bs = (b.t().contiguous() if lb == 0 else b).cuda()
    C = torch.zeros(M, N, device="cuda")
    epi = L.EPI_ATOMIC if la == 1 else L.EPI_STORE
    K.gemm(M, N, Kd, K.operand(As, la), K.operand(Bs, lb), C, epilogue=epi, split_k=3 if la == 1 else 1,
           prec=L.GEMM_BF16)
    C32 = torch.zeros(M, N, device="cuda")
    K.gemm(M, N, Kd, K.operand(As, la), K.operand(Bs, lb), C32, epilogue=epi, split_k=3 if la == 1 else 1,
           prec=L.GEMM_F32)
    want = _bf(a) @ _bf(b)
    tol = _bf16_tol(a, b, Kd)
    e = (C.double().cpu() - want).abs().max().item()
    e32 = (C32.double().cpu() - want).abs().max().item()
    assert e <= tol, (e, tol)
    assert e32 > 10 * tol, (e32, tol)


def test_bf16_gather_conv3_scatter_wgrad():
    """Gathered rows, conv3 rows, the scatter-store dgrad and the gathered wgrad in bf16."""
    g = torch.Generator().manual_seed(31)
    V, E, T, N, Ls = 3000, 768, 2040, 480, 30
    table = torch.randn(V, E, generator=g) * 0.5
    tok = torch.randint(1, V, (T,), generator=g)
    W = torch.randn(N, E, generator=g) / 16
    tc, tokc, Wc = table.cuda(), tok.cuda(), W.cuda()
    Y = torch.empty(T, N, device="cuda")
    K.gemm(T, N, E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_GATHER), K.operand(Wc, L.KCONTIG), Y,
           prec=L.GEMM_BF16)
    want = _bf(table[tok]) @ _bf(W).t()
    assert (Y.double().cpu() - want).abs().max().item() <= _bf16_tol(table, W, E)

    # conv3 rows (k = 3E): tap j of token t reads token t + j - 1 of its title (zero outside)
    W3 = torch.randn(N, 3 * E, generator=g) / 32
    W3c = W3.cuda()
    Yc = torch.empty(T, N, device="cuda")
    K.gemm(T, N, 3 * E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Ls, seg=E),
           K.operand(W3c, L.KCONTIG), Yc, prec=L.GEMM_BF16)
    x = table[tok].view(T // Ls, Ls, E)
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1))
    x3 = torch.cat([xp[:, j:j + Ls] for j in range(3)], -1).reshape(T, 3 * E)
    want = _bf(x3) @ _bf(W3).t()
    assert (Yc.double().cpu() - want).abs().max().item() <= _bf16_tol(table, W3, 3 * E)

    # wgrad over gathered rows: dW = dYᵀ table[tok] (K = 2016 tokens: the fast path needs K % 32 == 0)
    Tw = 2016
    dY = torch.randn(Tw, N, generator=g)
    dw = torch.zeros(N, E, device="cuda")
    K.gemm(N, E, Tw, K.operand(dY.cuda(), L.MNCONTIG),
           K.operand(tc, L.MNCONTIG, rows=tokc[:Tw].contiguous(), mapping=L.ROWS_GATHER),
           dw, epilogue=L.EPI_ATOMIC, split_k=2, prec=L.GEMM_BF16)
    want = _bf(dY).t() @ _bf(table[tok[:Tw]])
    assert (dw.double().cpu() - want).abs().max().item() <= _bf16_tol(dY, table, Tw)

    # distinct-row dgrad scattered by plain stores (unique destination rows, pad row skipped)
    rows = torch.randperm(V - 1, generator=g)[:1024] + 1
    rows[5] = 0
    S = torch.randn(1024, N, generator=g)
    dt = torch.zeros(V, E, device="cuda")
    K.gemm(1024, E, N, K.operand(S.cuda(), L.KCONTIG), K.operand(Wc, L.MNCONTIG), dt,
           epilogue=L.EPI_SCATTER_STORE, c_rows=K.rows_map(rows.cuda(), L.ROWS_GATHER), pad_row=0, prec=L.GEMM_BF16)
    want = torch.zeros(V, E, dtype=torch.float64)
    want[rows] = _bf(S) @ _bf(W)
    want[0] = 0
    assert (dt.double().cpu() - want).abs().max().item() <= _bf16_tol(S, W, N)


def test_precision_is_per_call():
    """The library holds no precision state: alternating calls with different arithmetics on one
    stream give each call its own arithmetic's result."""
    g = torch.Generator().manual_seed(41)
    a = torch.randn(512, 256, generator=g).cuda()
    b = torch.randn(384, 256, generator=g).cuda()
    outs = {}
    for prec in (L.GEMM_BF16, L.GEMM_F32, L.GEMM_BF16X6, L.GEMM_BF16):
        C = torch.empty(512, 384, device="cuda")
        K.gemm(512, 384, 256, K.operand(a, L.KCONTIG), K.operand(b, L.KCONTIG), C, prec=prec)
        outs.setdefault(prec, []).append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[L.GEMM_BF16][0], outs[L.GEMM_BF16][1])
    want = _bf(a.cpu()) @ _bf(b.cpu()).t()
    assert (outs[L.GEMM_BF16][0].double().cpu() - want).abs().max().item() <= _bf16_tol(a, b, 256)
    exact = a.cpu().double() @ b.cpu().double().t()
    assert (outs[L.GEMM_F32][0].double().cpu() - exact).abs().max().item() < 1e-3
