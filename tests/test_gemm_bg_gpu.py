"""The B-from-global large-tile GEMM (csrc/gemm_bg.hip): B pre-split by nr_split_b into bf16 planes in
MFMA fragment order (layout NR_BSPLIT), A (plain or gathered rows) staged through LDS.  The news
tower's projection runs on it (forward: gathered table rows x [Wk; Wv]ᵀ; table dgrad: dY x [Wk; Wv]
scattered into the distinct table rows of a zero-filled gradient).  Every shape class of the step:
ragged M / N (N = 1152 = 4.5 x 256: waves past N skip their MFMAs), device-resident M, the stream-K
tail of the zeroed scatter epilogue, both arithmetics, against fp64 references (the bounds of
tests/test_gemm_big_gpu.py), plus nr_split_b's layout itself."""
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
@pytest.mark.parametrize("layout", [L.KCONTIG, L.MNCONTIG])
def test_split_b_layout(prec, layout):
    """out[((p NB + n/32) KB + k/16) 512 + (n%32) 16 + k%16] = plane p of b(n, k), zero past N."""
    g = torch.Generator().manual_seed(1)
    N, Kd = 70, 96
    b = torch.randn(N, Kd, generator=g)
    src = b if layout == L.KCONTIG else b.t().contiguous()
    planes, _ = K.split_b(src.cuda(), layout, N, Kd, prec)
    NB, KB = (N + 31) // 32, Kd // 16
    np_ = 3 if prec == L.GEMM_BF16X6 else 1
    got = planes.cpu().view(np_, NB, KB, 32, 16).permute(0, 1, 3, 2, 4).reshape(np_, NB * 32, Kd)
    got = (got.to(torch.int32) << 16).view(torch.float32)   # bf16 bits -> fp32 values
    assert (got[:, N:] == 0).all()
    if np_ == 1:
        torch.testing.assert_close(got[0, :N], b.bfloat16().float(), rtol=0, atol=0)
    else:
        h, m, l = got[0, :N].double(), got[1, :N].double(), got[2, :N].double()
        assert ((h + m + l) - b.double()).abs().max().item() <= 2 ** -23 * b.abs().max().item()
        torch.testing.assert_close(got[0, :N], b.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("N", [1152, 520, 768])
def test_bg_gather_projection(prec, N):
    """Y = table[ids] Wᵀ + b, M = 3000 rows (ragged last tile), device-resident M < host bound."""
    g = torch.Generator().manual_seed(N)
    V, E, M = 5000, 768, 3000
    table = torch.randn(V, E, generator=g)
    ids = torch.randint(0, V, (M,), generator=g)
    W = torch.randn(N, E, generator=g) / 16
    bias = torch.randn(N, generator=g)
    Y = torch.full((M, N), float("nan"), device="cuda")
    m_dev = torch.tensor([2900], dtype=torch.int32, device="cuda")
    _, wop = K.split_b(W.cuda(), L.KCONTIG, N, E, prec)
    K.gemm_dyn(M, N, E, K.operand(table.cuda(), L.KCONTIG, rows=ids.cuda(), mapping=L.ROWS_GATHER), wop, Y,
               m_dev=m_dev, bias=bias.cuda(), prec=prec)
    want = _ref(table[ids], W.t(), prec) + bias.double()
    assert _err(Y[:2900], want[:2900]) <= _tol(table, W, E, prec)
    assert torch.isnan(Y[2900:]).all()   # rows past the device M untouched


@pytest.mark.parametrize("prec", PRECS)
def test_bg_plain_large(prec):
    """The step's projection shape on plain rows (24,576 x 1152 x 768): the bf16x6 result equals the
    both-operands-in-LDS kernel's to fp32 rounding."""
    g = torch.Generator().manual_seed(5)
    M, N, Kd = 24576, 1152, 768
    a = torch.randn(M, Kd, generator=g).cuda()
    W = (torch.randn(N, Kd, generator=g) / 16).cuda()
    C1 = torch.empty(M, N, device="cuda")
    C2 = torch.empty(M, N, device="cuda")
    _, wop = K.split_b(W, L.KCONTIG, N, Kd, prec)
    K.gemm(M, N, Kd, K.operand(a, L.KCONTIG), wop, C1, prec=prec)
    K.gemm(M, N, Kd, K.operand(a, L.KCONTIG), K.operand(W, L.KCONTIG), C2, prec=prec)
    rows = torch.randint(0, M, (512,), generator=g)
    want = _ref(a[rows].cpu(), W.t().cpu(), prec)
    assert _err(C1[rows], want) <= _tol(a, W, Kd, prec)
    scale = C2.abs().max().item()
    assert (C1 - C2).abs().max().item() <= (1e-5 if prec == L.GEMM_BF16X6 else 1e-3) * scale


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("M", [2000, 24600])
def test_bg_dgrad_scatter_zeroed(prec, M):
    """dT[uids] = dY [Wk; Wv] (B = W as MN-contiguous [K = 1152][N = 768], pre-split transposed),
    NR_EPI_SCATTER_ZEROED into a zero-filled table gradient: plain row stores plus the stream-K tail's
    atomic pieces; the padding row is skipped, untouched rows stay zero."""
    g = torch.Generator().manual_seed(M)
    V, E, NY = 30522, 768, 1152
    uids = torch.randperm(V - 1, generator=g)[:M] + 1
    uids[3] = 0   # the padding row: skipped
    dY = torch.randn(M, NY, generator=g)
    W = torch.randn(NY, E, generator=g) / 30
    dT = torch.zeros(V, E, device="cuda")
    n_dev = torch.tensor([M], dtype=torch.int32, device="cuda")
    _, wtop = K.split_b(W.cuda(), L.MNCONTIG, E, NY, prec)
    K.gemm_dyn(M, E, NY, K.operand(dY.cuda(), L.KCONTIG), wtop, dT, m_dev=n_dev, epilogue=L.EPI_SCATTER_ZEROED,
               c_rows=K.rows_map(uids.cuda(), L.ROWS_GATHER), pad_row=0, prec=prec)
    got = dT.cpu()
    sel = torch.randint(0, M, (600,), generator=g)
    sel = sel[uids[sel] != 0]
    want = _ref(dY[sel], W, prec)
    assert (got[uids[sel]].double() - want).abs().max().item() <= _tol(dY, W, NY, prec)
    assert (got[0] == 0).all()
    touched = torch.zeros(V, dtype=torch.bool)
    touched[uids] = True
    assert (got[~touched] == 0).all()
