"""nr_gemm_f32 against an fp64 CPU reference: every layout / row map / epilogue the
towers use, with ragged M, N, K."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import _lib as L
from newsrec_amd import kernels as K


def _ref_tol(a, b):
    # fp32 accumulation: error ~ eps * K * max|a||b|
    return 1e-5 * a.abs().max().item() * b.abs().max().item() * a.shape[1] ** 0.5 + 1e-6


@pytest.mark.parametrize("M,N,Kd", [(256, 128, 64), (200, 150, 100), (1, 7, 3), (513, 1152, 768), (70, 64, 2)])
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_layouts(M, N, Kd, la, lb):
    g = torch.Generator().manual_seed(M * 7 + N + Kd)
    a = torch.randn(M, Kd, generator=g)
    b = torch.randn(Kd, N, generator=g)
    bias = torch.randn(N, generator=g)
    want = (a.double() @ b.double() + bias.double()).float()
    Kp = (Kd + 3) // 4 * 4
    Mp = (M + 3) // 4 * 4
    Np = (N + 3) // 4 * 4
    if la == 0:   # [M][K]
        As = torch.zeros(M, Kp); As[:, :Kd] = a
    else:         # [K][M]
        As = torch.zeros(Kd, Mp); As[:, :M] = a.t()
    if lb == 0:   # [N][K]
        Bs = torch.zeros(N, Kp); Bs[:, :Kd] = b.t()
    else:
        Bs = torch.zeros(Kd, Np); Bs[:, :N] = b
    As, Bs, bias_d = As.cuda(), Bs.cuda(), bias.cuda()
    C = torch.full((M, N + 5), 7.0, device="cuda")
    K.gemm(M, N, Kd, K.operand(As, la), K.operand(Bs, lb), C, bias=bias_d)
    torch.cuda.synchronize()
    torch.testing.assert_close(C[:, :N].cpu(), want, rtol=0, atol=_ref_tol(a, b))
    assert torch.all(C[:, N:] == 7.0)


def test_gemm_gather_scatter_splitk():
    g = torch.Generator().manual_seed(3)
    V, E, T, N = 300, 96, 333, 136
    table = torch.randn(V, E, generator=g)
    tok = torch.randint(0, V, (T,), generator=g)
    tok[:10] = 0
    W = torch.randn(N, E, generator=g)
    X = table[tok]
    want = X.double() @ W.double().t()
    tc, tokc, Wc = table.cuda(), tok.cuda(), W.cuda()
    Y = torch.empty(T, N, device="cuda")
    K.gemm(T, N, E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_GATHER), K.operand(Wc, L.KCONTIG), Y)
    torch.testing.assert_close(Y.cpu().double(), want, rtol=0, atol=1e-3)
    # dgrad with fused scatter into a dense table gradient, padding row 0 skipped
    dY = torch.randn(T, N, generator=g)
    dX = dY.double() @ W.double()
    dtab = torch.zeros(V, E, dtype=torch.float64).index_add_(0, tok, dX)
    dtab[0] = 0
    dtc = torch.zeros(V, E, device="cuda")
    K.gemm(T, E, N, K.operand(dY.cuda(), L.KCONTIG), K.operand(Wc, L.MNCONTIG), dtc,
           epilogue=L.EPI_SCATTER, c_rows=K.rows_map(tokc, L.ROWS_GATHER), pad_row=0)
    torch.testing.assert_close(dtc.cpu().double(), dtab, rtol=0, atol=2e-3)
    # wgrad dW = dY^T X with split-K atomics and a gathered B
    dW = (dY.double().t() @ X.double())
    dWc = torch.zeros(N, E, device="cuda")
    K.gemm(N, E, T, K.operand(dY.cuda(), L.MNCONTIG), K.operand(tc, L.MNCONTIG, rows=tokc, mapping=L.ROWS_GATHER),
           dWc, epilogue=L.EPI_ATOMIC, split_k=5)
    torch.testing.assert_close(dWc.cpu().double(), dW, rtol=0, atol=5e-3)


def test_gemm_conv3():
    """k=3, pad=1 Conv1d over gathered tokens as a K=3E GEMM (CNN.py:12-17,41)."""
    g = torch.Generator().manual_seed(5)
    V, E, Lq, nn_, H = 100, 64, 7, 9, 40
    table = torch.randn(V, E, generator=g)
    tok = torch.randint(0, V, (nn_, Lq), generator=g)
    w = torch.randn(H, E, 3, generator=g)
    b = torch.randn(H, generator=g)
    x = table[tok].transpose(1, 2)                     # [n, E, L]
    want = torch.relu(torch.nn.functional.conv1d(x.double(), w.double(), b.double(), padding=1)).transpose(1, 2).reshape(-1, H)
    wr = w.permute(0, 2, 1).reshape(H, 3 * E).contiguous()   # [H][j*E + e]
    tc, tokc = table.cuda(), tok.reshape(-1).cuda()
    Y = torch.empty(nn_ * Lq, H, device="cuda")
    K.gemm(nn_ * Lq, H, 3 * E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Lq, seg=E),
           K.operand(wr.cuda(), L.KCONTIG), Y, bias=b.cuda(), epilogue=L.EPI_STORE_RELU)
    torch.testing.assert_close(Y.cpu().double(), want, rtol=0, atol=1e-3)
    # dgrad scatter through the conv taps and wgrad with a CONV3 B operand
    dC = torch.randn(nn_ * Lq, H, generator=g)
    xg = x.double().requires_grad_(True)
    wd = w.double().requires_grad_(True)
    out = torch.nn.functional.conv1d(xg, wd, None, padding=1).transpose(1, 2).reshape(-1, H)
    out.backward(dC.double())
    dtab = torch.zeros(V, E, dtype=torch.float64).index_add_(0, tok.reshape(-1), xg.grad.transpose(1, 2).reshape(-1, E))
    dtab[0] = 0
    Hp = (H + 3) // 4 * 4
    dCp = torch.zeros(nn_ * Lq, Hp); dCp[:, :H] = dC
    dtc = torch.zeros(V, E, device="cuda")
    K.gemm(nn_ * Lq, 3 * E, H, K.operand(dCp.cuda(), L.KCONTIG), K.operand(wr.cuda(), L.MNCONTIG), dtc,
           epilogue=L.EPI_SCATTER, c_rows=K.rows_map(tokc, L.ROWS_CONV3, seq_len=Lq, seg=E), pad_row=0)
    torch.testing.assert_close(dtc.cpu().double(), dtab, rtol=0, atol=2e-3)
    dwr = torch.zeros(H, 3 * E, device="cuda")
    K.gemm(H, 3 * E, nn_ * Lq, K.operand(dCp.cuda(), L.MNCONTIG),
           K.operand(tc, L.MNCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Lq, seg=E),
           dwr, epilogue=L.EPI_ATOMIC, split_k=3)
    want_dw = wd.grad.permute(0, 2, 1).reshape(H, 3 * E)
    torch.testing.assert_close(dwr.cpu().double(), want_dw, rtol=0, atol=2e-3)
