"""nr_cnn_keypool_fwd / nr_cnn_keypool_bwd (csrc/cnn_keypool.hip): CNN_Encoder's word attention fused
per title (models/Encoders/CNN.py:41-46 with scaled_dp_attention, Modules/Attention.py:5-30) against a
float64 autograd restatement:

    K = tanh(C Wqᵀ + bq), p = XSoftmax(q·K / sqrt(H), mask), news = Σ_l p_l C_l,

with C = ReLU(pre) (the conv output), so the backward's dc is the gradient of the conv PRE-activation
(the ReLU gate included) and dconv_b its column sums.  Ragged titles, holes, a fully masked title, the
optional token-output gradient dz, zero padding past H, and the three GEMM arithmetics (f32 MFMA and
bf16x6 at the fp32 bar, bf16 at a stated bf16 bar).  Then the CNN news encoder end to end: fused vs the
unfused key GEMM + pooling kernels (functions.FUSED_KEYPOOL = False) on every gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import _lib as L
from newsrec_amd import functions as F
from newsrec_amd import kernels as K


def _case(nseq, L_, H, Hp, seed, with_dz):
    g = torch.Generator().manual_seed(seed)
    pre = torch.randn(nseq, L_, H, generator=g, dtype=torch.float64)
    wq = torch.randn(H, H, generator=g, dtype=torch.float64) * (2.0 / H) ** 0.5
    bq = torch.randn(H, generator=g, dtype=torch.float64) * 0.1
    q = torch.randn(H, generator=g, dtype=torch.float64)
    lens = torch.randint(1, L_ + 1, (nseq,), generator=g)
    mask = (torch.arange(L_)[None] < lens[:, None]).long()
    mask[0] = 0                # fully masked title
    mask[1, ::4] = 0           # holes
    dnews = torch.randn(nseq, H, generator=g, dtype=torch.float64)
    dz = torch.randn(nseq, L_, H, generator=g, dtype=torch.float64) if with_dz else None
    return pre, wq, bq, q, mask, dnews, dz


def _ref(pre, wq, bq, q, mask, dnews, dz):
    pre = pre.clone().requires_grad_(True)
    wq = wq.clone().requires_grad_(True)
    bq = bq.clone().requires_grad_(True)
    q = q.clone().requires_grad_(True)
    C = torch.relu(pre)
    Kk = torch.tanh(C @ wq.t() + bq)
    s = (Kk @ q) / q.numel() ** 0.5
    keep = mask.bool()
    p = torch.nan_to_num(torch.softmax(s.masked_fill(~keep, float("-inf")), -1).masked_fill(~keep, 0.0), nan=0.0)
    news = (p.unsqueeze(-1) * C).sum(1)
    loss = (news * dnews).sum()
    if dz is not None:
        loss = loss + (C * dz).sum()
    loss.backward()
    return C.detach(), news.detach(), p.detach(), pre.grad, wq.grad, bq.grad, q.grad


@pytest.mark.parametrize("prec,tol", [(L.GEMM_F32, 5e-5), (L.GEMM_BF16X6, 5e-5), (L.GEMM_BF16, 3e-2)])
# 1000 titles: more than the forward's resident workgroups (three per CU), so its persistent loop
# runs several titles per workgroup, as the full-size step does
@pytest.mark.parametrize("nseq,L_,H,with_dz", [(700, 30, 150, False), (1000, 30, 150, True), (37, 32, 150, True),
                                               (300, 17, 64, True), (5, 30, 20, False)])
@pytest.mark.parametrize("save_k", [False, True])
def test_cnn_keypool_matches_float64(prec, tol, nseq, L_, H, with_dz, save_k):
    """save_k: the forward stores K = tanh(C wqᵀ + bq) (checked here too) and the backward reads it
    instead of recomputing the key products (functions.KEYPOOL_SAVE_K)."""
    Hp = (H + 31) // 32 * 32
    dev = "cuda"
    pre, wq, bq, q, mask, dnews, dz = _case(nseq, L_, H, Hp, nseq + H + L_, with_dz)
    C, news_r, p_r, dpre_r, dwq_r, dbq_r, dq_r = _ref(pre, wq, bq, q, mask, dnews, dz)
    dcb_r = dpre_r.sum((0, 1))

    T = nseq * L_
    Cd = torch.zeros(T, Hp, device=dev)
    Cd[:, :H] = C.reshape(T, H).float().to(dev)
    wqp = torch.zeros(Hp, Hp, device=dev)
    wqp[:H, :H] = wq.float().to(dev)
    bqp = torch.zeros(Hp, device=dev)
    bqp[:H] = bq.float().to(dev)
    qd = q.float().to(dev)
    M = mask.to(dev).reshape(-1)
    news = torch.empty(nseq, Hp, device=dev)
    probs = torch.empty(T, device=dev)
    # K rows live in [T, Hp] of a NaN-filled [T + 32, Hp + 4] block: the forward's stores must stay
    # inside the title's L rows (a title's slots past L are dropped, not written into the next
    # title's rows or past the last one) and inside the Hp columns
    kfull = torch.full((T + 32, Hp + 4), float("nan"), device=dev) if save_k else None
    kbuf = kfull[:T, :Hp] if save_k else None
    K.cnn_keypool_fwd(Cd, wqp, bqp, qd, M, nseq, L_, news, probs, qn=H, prec=prec, kout=kbuf)
    dc = torch.full((T, Hp), float("nan"), device=dev)
    dwq = torch.full((Hp, Hp), float("nan"), device=dev)
    dbq = torch.full((Hp,), float("nan"), device=dev)
    dq = torch.full((H,), float("nan"), device=dev)
    dcb = torch.full((H,), float("nan"), device=dev)
    dzd = dz.reshape(T, H).float().to(dev) if dz is not None else None
    K.cnn_keypool_bwd(Cd, wqp, bqp, qd, nseq, L_, H, probs, dnews.float().to(dev), dc, dwq, dbq, dq, dcb, dz=dzd,
                      prec=prec, kin=kbuf)
    torch.cuda.synchronize()

    def close(got, want, name, t=tol):
        got = got.double().cpu()
        assert torch.isfinite(got).all(), name
        err = (got - want).abs().max().item()
        assert err <= t * max(1.0, want.abs().max().item()), (name, err)

    if save_k:
        k_r = torch.tanh(C.reshape(T, H) @ wq.T + bq)
        close(kbuf[:, :H], k_r, "K")
        if Hp > H:
            assert kbuf[:, H:].abs().max().item() < 1e-6   # tanh(0 + 0) past H
        assert torch.isnan(kfull[T:]).all() and torch.isnan(kfull[:, Hp:]).all(), "K store outside [T, Hp]"
    close(news[:, :H], news_r, "news")
    assert news[:, H:].abs().sum().item() == 0.0 and news[0].abs().max().item() == 0.0
    close(probs.view(nseq, L_), p_r, "probs")
    close(dc[:, :H].view(nseq, L_, H), dpre_r, "dc")
    assert dc[:, H:].abs().sum().item() == 0.0
    close(dwq[:H, :H], dwq_r, "dwq")
    assert dwq[H:].abs().sum().item() == 0.0 and dwq[:, H:].abs().sum().item() == 0.0
    close(dbq[:H], dbq_r, "dbq")
    close(dq, dq_r, "dq")
    close(dcb, dcb_r, "dconv_b")


@pytest.mark.parametrize("prec", [L.GEMM_BF16X6, L.GEMM_BF16])
def test_cnn_encoder_fused_keypool_matches_unfused(prec):
    """The distinct-row CNN encoder with the fused word attention against the same encoder on the key
    GEMM + pooling kernels: news vectors and every parameter / table gradient."""
    from newsrec_amd.encoders import CNN_Encoder

    class M:
        hidden_dim = 150
        bert_dim = 768

    torch.manual_seed(0)
    dev = "cuda"
    enc = CNN_Encoder(M()).to(dev)
    table = torch.nn.Parameter(torch.randn(3000, 768, device=dev) * 0.3)
    ids = torch.randint(1, 3000, (64, 30), device=dev)
    ids[:, 25:] = 0
    mask = (ids != 0).long()
    mask[3] = 0
    dnews = torch.randn(64, 150, device=dev)

    def run(fused):
        F.FUSED_KEYPOOL = fused
        try:
            for p in list(enc.parameters()) + [table]:
                p.grad = None
            with K.gemm_precision(prec):
                _, news = enc.encode_tokens(table, ids, mask)
                (news * dnews).sum().backward()
            torch.cuda.synchronize()
            return news.detach().clone(), {n: p.grad.clone() for n, p in enc.named_parameters()}, table.grad.clone()
        finally:
            F.FUSED_KEYPOOL = True

    n1, g1, t1 = run(True)
    n0, g0, t0 = run(False)
    tol = 1e-4 if prec == L.GEMM_BF16X6 else 3e-2
    assert (n1 - n0).abs().max().item() <= tol * max(1.0, n0.abs().max().item())
    for name in g0:
        err = (g1[name] - g0[name]).abs().max().item()
        assert err <= tol * max(1e-6, g0[name].abs().max().item()), (name, err)
    err = (t1 - t0).abs().max().item()
    assert err <= tol * t0.abs().max().item(), ("table", err)
