"""The large-tile bf16 GEMM kernel (gemm_big_impl.h: 256 x BN tiles, 8 waves, double-buffered LDS),
which nr_gemm_f32 picks for big contractions under NR_GEMM_BF16X6 / NR_GEMM_BF16: every operand-mode
combination it instantiates, ragged M / N (tiles cut by the extents), device-resident M and K, both
tile widths (BN = 256 for N % 256 == 0 or N >= 1024, else 128), against fp64 references:
bf16x6 to the fp32-class bound of tests/test_gemm_split_gpu.py, bf16 to fp32 accumulation error of
the bf16-rounded operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import _lib as L
from newsrec_amd import kernels as K

PRECS = [L.GEMM_BF16X6, L.GEMM_BF16]


def _ref(a, b, prec):
    if prec == L.GEMM_BF16:
        return a.bfloat16().double() @ b.bfloat16().double()
    return a.double() @ b.double()


def _tol(a, b, k, prec):
    s = a.abs().max().item() * b.abs().max().item()
    if prec == L.GEMM_BF16:
        return 4e-7 * s * k + 1e-6
    return 1e-5 * s * k ** 0.5 + 1e-6


def _err(C, want):
    return (C.double().cpu() - want).abs().max().item()


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("N", [1152, 520, 768])
def test_big_gather_projection(prec, N):
    """Y = table[ids] Wᵀ + b (KC_GATHER x KC_PLAIN), M = 3000 rows (ragged last 256-row tile),
    device-resident M smaller than the host bound."""
    g = torch.Generator().manual_seed(N)
    V, E, M = 5000, 768, 3000
    table = torch.randn(V, E, generator=g)
    ids = torch.randint(0, V, (M,), generator=g)
    W = torch.randn(N, E, generator=g) / 16
    bias = torch.randn(N, generator=g)
    Y = torch.full((M, N), float("nan"), device="cuda")
    m_dev = torch.tensor([2900], dtype=torch.int32, device="cuda")
    K.gemm_dyn(M, N, E, K.operand(table.cuda(), L.KCONTIG, rows=ids.cuda(), mapping=L.ROWS_GATHER),
               K.operand(W.cuda(), L.KCONTIG), Y, m_dev=m_dev, bias=bias.cuda(), prec=prec)
    want = _ref(table[ids], W.t(), prec) + bias.double()
    assert _err(Y[:2900], want[:2900]) <= _tol(table, W, E, prec)
    assert torch.isnan(Y[2900:]).all()   # rows past the device M untouched


@pytest.mark.parametrize("Kd", [544, 800, 1312, 768])
def test_big_bf16_odd_k_tile_counts(Kd):
    """bf16 K-contiguous pairs run 32-deep k-tiles: 17 / 25 / 41 tiles take the peeled odd form of the
    two-tile k-loop (tile 0 alone, then pairs), 24 the even form; the bf16x6 run of the same shape
    (16-deep tiles, always an even count) alongside."""
    g = torch.Generator().manual_seed(Kd)
    V, M, N = 4000, 3000, 1152
    table = torch.randn(V, Kd, generator=g)
    ids = torch.randint(0, V, (M,), generator=g)
    W = torch.randn(N, Kd, generator=g) / 16
    for prec in PRECS:
        Y = torch.full((M, N), float("nan"), device="cuda")
        K.gemm(M, N, Kd, K.operand(table.cuda(), L.KCONTIG, rows=ids.cuda(), mapping=L.ROWS_GATHER),
               K.operand(W.cuda(), L.KCONTIG), Y, prec=prec)
        assert _err(Y, _ref(table[ids], W.t(), prec)) <= _tol(table, W, Kd, prec), prec


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("epi", [L.EPI_STORE_TANH, L.EPI_STORE_GELU])
def test_big_plain_epilogues(prec, epi):
    g = torch.Generator().manual_seed(7)
    M, N, Kd = 2600, 3072, 768
    a = torch.randn(M, Kd, generator=g)
    w = torch.randn(N, Kd, generator=g) / 28
    b = torch.randn(N, generator=g) * 0.1
    C = torch.empty(M, N, device="cuda")
    aux = torch.empty(M, N, device="cuda") if epi == L.EPI_STORE_GELU else None
    K.gemm(M, N, Kd, K.operand(a.cuda(), L.KCONTIG), K.operand(w.cuda(), L.KCONTIG), C, bias=b.cuda(), epilogue=epi,
           c_rows=K.operand(aux, L.KCONTIG) if aux is not None else None, prec=prec)
    pre = _ref(a, w.t(), prec) + b.double()
    if epi == L.EPI_STORE_TANH:
        want = torch.tanh(pre)
        assert _err(C, want) <= _tol(a, w, Kd, prec)
    else:
        assert _err(aux, pre) <= _tol(a, w, Kd, prec)
        want = 0.5 * pre * (1 + torch.erf(pre / 2 ** 0.5))
        assert _err(C, want) <= 2 * _tol(a, w, Kd, prec)


@pytest.mark.parametrize("prec", PRECS)
def test_big_dgrad_store_and_scatter_store(prec):
    """dX = dY W (KC_PLAIN x MN_PLAIN), plain store and the distinct-row scatter-store into a table."""
    g = torch.Generator().manual_seed(3)
    U, N, E, V = 2800, 1152, 768, 40000
    dY = torch.randn(U, N, generator=g)
    W = torch.randn(N, E, generator=g) / 30
    dX = torch.empty(U, E, device="cuda")
    K.gemm(U, E, N, K.operand(dY.cuda(), L.KCONTIG), K.operand(W.cuda(), L.MNCONTIG), dX, prec=prec)
    want = _ref(dY, W, prec)
    tol = _tol(dY, W, N, prec)
    assert _err(dX, want) <= tol
    rows = torch.randperm(V - 1, generator=g)[:U] + 1
    rows[17] = 0
    dt = torch.zeros(V, E, device="cuda")
    K.gemm(U, E, N, K.operand(dY.cuda(), L.KCONTIG), K.operand(W.cuda(), L.MNCONTIG), dt,
           epilogue=L.EPI_SCATTER_STORE, c_rows=K.rows_map(rows.cuda(), L.ROWS_GATHER), pad_row=0, prec=prec)
    full = torch.zeros(V, E, dtype=torch.float64)
    full[rows] = want
    full[0] = 0
    assert _err(dt, full) <= tol


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("gather,N", [(False, 1152), (True, 1152), (True, 1100), (True, 1200)])
def test_big_wgrad_split_k(prec, gather, N):
    """dW = dYᵀ X over K = rows (MN_PLAIN x MN_PLAIN / MN_GATHER), split-K atomics, device-resident K.  N = 1152 / 1100: the last row of 256-row
    tiles holds <= 128 live rows (its waves 4-7 skip their MFMAs); N = 1200: every tile row full."""
    g = torch.Generator().manual_seed(5 + gather)
    R, E, V = 24576, 768, 30000
    dY = torch.randn(R, N, generator=g)
    table = torch.randn(V, E, generator=g) * 0.5
    ids = torch.randint(0, V, (R,), generator=g)
    X = table[ids]
    dW = torch.zeros(N, E, device="cuda")
    k_dev = torch.tensor([R - 4096], dtype=torch.int32, device="cuda")
    Bop = (K.operand(table.cuda(), L.MNCONTIG, rows=ids.cuda(), mapping=L.ROWS_GATHER) if gather
           else K.operand(X.cuda(), L.MNCONTIG))
    K.gemm_dyn(N, E, R, K.operand(dY.cuda(), L.MNCONTIG), Bop, dW, k_dev=k_dev, epilogue=L.EPI_ATOMIC, split_k=9,
               prec=prec)
    Kr = R - 4096
    want = _ref(dY[:Kr].t(), X[:Kr], prec)
    assert _err(dW, want) <= _tol(dY, X, Kr, prec)


@pytest.mark.parametrize("kd", [24576, 20000, 992, 0])
def test_big_wgrad_split_k_workspace_accumulates(kd):
    """nr_gemm_f32_ws' workspace path: the split-K reduction ADDS into C (the atomic epilogue's
    contract), skips the splits whose k range starts past the device K (k_dev = 992: 16 of 17 splits
    hold rows; a device K is a multiple of 32), sums the splits in a fixed order (two runs bitwise
    equal), and matches the atomic path (no workspace) to rounding."""
    g = torch.Generator().manual_seed(11)
    R, N, E = 24576, 1152, 768
    dY = torch.randn(R, N, generator=g)
    X = torch.randn(R, E, generator=g)
    C0 = torch.randn(N, E, generator=g)
    k_dev = torch.tensor([kd], dtype=torch.int32, device="cuda")
    A, B = K.operand(dY.cuda(), L.MNCONTIG), K.operand(X.cuda(), L.MNCONTIG)
    outs = []
    for _ in range(2):   # the C ABI's workspace form (K.gemm_dyn itself keeps the atomic epilogue here)
        dW = C0.cuda()
        work = K._splitk_work(dW)
        L.call("nr_gemm_f32_ws", N, E, R, A, B, L.ptr(dW), dW.stride(0), None, L.EPI_ATOMIC, None, -1, 9, None,
               L.ptr(k_dev), L.GEMM_BF16X6, 0, L.ptr(work), work.numel(), None, None, L.stream_ptr(dW))
        outs.append(dW)
    want = C0.double() + _ref(dY[:kd].t(), X[:kd], L.GEMM_BF16X6)
    assert _err(outs[0], want) <= _tol(dY, X, max(kd, 1), L.GEMM_BF16X6)
    assert torch.equal(outs[0], outs[1])
    at = C0.cuda()   # the atomic epilogue (the C ABI without a workspace)
    L.call("nr_gemm_f32_dyn", N, E, R, A, B, L.ptr(at), at.stride(0), None, L.EPI_ATOMIC, None, -1, 9, None,
           L.ptr(k_dev), L.GEMM_BF16X6, L.stream_ptr(at))
    assert _err(at, want) <= _tol(dY, X, max(kd, 1), L.GEMM_BF16X6)


@pytest.mark.parametrize("prec", PRECS)
def test_big_wgrad_split_k_static(prec):
    """A BERT-shaped weight gradient through the static entry (K.gemm -> nr_gemm_f32_ws)."""
    g = torch.Generator().manual_seed(12)
    R, N, E = 8192, 3072, 768
    G = torch.randn(R, N, generator=g)
    X = torch.randn(R, E, generator=g)
    dW = torch.zeros(N, E, device="cuda")
    K.gemm(N, E, R, K.operand(G.cuda(), L.MNCONTIG), K.operand(X.cuda(), L.MNCONTIG), dW, epilogue=L.EPI_ATOMIC,
           split_k=8, prec=prec)
    assert _err(dW, _ref(G.t(), X, prec)) <= _tol(G, X, R, prec)


@pytest.mark.parametrize("ws", [False, True])
@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("U,u_dev", [(2800, None), (30000, 24600), (24576, None), (256, None)])
def test_big_dgrad_scatter_zeroed_tail(prec, U, u_dev, ws):
    """NR_EPI_SCATTER_ZEROED (the table dgrad into a zero-filled gradient): the tiles of the persistent
    grid's last partial round are split along K and their pieces added atomically (a stream-K tail),
    or -- with the workspace (bf16x6) -- stored as partial tiles and summed in piece order by one
    reduction launch, bitwise reproducible.  U = 2800: every tile split (33 tiles); device M 24,600:
    291 tiles = one full round + 35 split tiles; 24,576: 288 tiles; 256: three tiles."""
    g = torch.Generator().manual_seed(U)
    N, E, V = 1152, 768, 60000
    dY = torch.randn(U, N, generator=g)
    W = torch.randn(N, E, generator=g) / 30
    rows = torch.randperm(V - 1, generator=g)[:U] + 1
    rows[5] = 0   # the padding row is skipped
    m = u_dev or U
    dt = torch.zeros(V, E, device="cuda")
    m_dev = torch.tensor([m], dtype=torch.int32, device="cuda")
    args = (U, E, N, K.operand(dY.cuda(), L.KCONTIG), K.operand(W.cuda(), L.MNCONTIG))
    kw = dict(m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(rows.cuda(), L.ROWS_GATHER), pad_row=0,
              prec=prec, workspace=ws)
    K.gemm_dyn(*args, dt, **kw)
    want = _ref(dY[:m], W, prec)
    full = torch.zeros(V, E, dtype=torch.float64)
    full[rows[:m]] = want
    full[0] = 0
    assert _err(dt, full) <= _tol(dY, W, N, prec)
    if ws and prec == L.GEMM_BF16X6:   # no atomics left: a second run is bitwise equal
        dt2 = torch.zeros(V, E, device="cuda")
        K.gemm_dyn(*args, dt2, **kw)
        assert torch.equal(dt, dt2)


@pytest.mark.parametrize("kd", [None, 20000])
def test_big_wgrad_folds_bias_colsum(kd):
    """K.gemm(..., colsum=db): on the split-K workspace path the weight gradient's bias gradient
    db += Σ_k dY[k] is summed from the dY tiles the first column tile's units load (fp32, per split,
    then the reduction) -> True; device-resident K honoured.  A shape that stays off that path
    returns False and leaves db alone."""
    g = torch.Generator().manual_seed(13)
    R, N, E = 20832, 3072, 768
    dY = torch.randn(R, N, generator=g)
    X = torch.randn(R, E, generator=g)
    db0 = torch.randn(N, generator=g)
    dW = torch.zeros(N, E, device="cuda")
    db = db0.cuda()
    A, B = K.operand(dY.cuda(), L.MNCONTIG), K.operand(X.cuda(), L.MNCONTIG)
    if kd is None:
        folded = K.gemm(N, E, R, A, B, dW, epilogue=L.EPI_ATOMIC, split_k=8, colsum=db)
        kr = R
    else:
        K.gemm_dyn(N, E, R, A, B, dW, k_dev=torch.tensor([kd], dtype=torch.int32, device="cuda"),
                   epilogue=L.EPI_ATOMIC, split_k=8)   # (gemm_dyn takes no colsum: the weights only)
        folded = K.gemm(N, E, kd, A, B, torch.zeros(N, E, device="cuda"), epilogue=L.EPI_ATOMIC, split_k=8,
                        colsum=db)
        kr = kd
    assert folded
    want = db0.double() + dY[:kr].double().sum(0)
    assert _err(db, want) <= 1e-5 * kr ** 0.5 * dY.abs().max().item() + 1e-5
    assert _err(dW, _ref(dY[:kr].t(), X[:kr], L.GEMM_BF16X6)) <= _tol(dY, X, kr, L.GEMM_BF16X6)
    # a small contraction runs on the 64 x 64 kernel: not folded, db untouched
    small = db0.cuda()
    f2 = K.gemm(64, 64, 256, K.operand(dY[:256, :64].contiguous().cuda(), L.MNCONTIG),
                K.operand(X[:256, :64].contiguous().cuda(), L.MNCONTIG), torch.zeros(64, 64, device="cuda"),
                epilogue=L.EPI_ATOMIC, split_k=2, colsum=small[:64])
    assert not f2 and torch.equal(small.cpu(), db0)

