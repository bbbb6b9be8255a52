"""The fused MHA news encoder (gather-GEMM + nr_mha_pool_fwd/bwd) against the oracle's
MHA_Encoder restatement in fp64, including ragged / empty titles and dropout."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import kernels as K
from newsrec_amd.functions import MHANewsFn
from oracle import restatement as R


def _params(g, E=768, H=384, dk=64):
    P = {
        "encoderN.mha.keyProject.weight": torch.randn(12 * dk, E, generator=g, dtype=torch.float64) / E ** 0.5,
        "encoderN.mha.keyProject.bias": torch.randn(12 * dk, generator=g, dtype=torch.float64) * 0.1,
        "encoderN.mha.valueProject.weight": torch.randn(H, E, generator=g, dtype=torch.float64) / E ** 0.5,
        "encoderN.mha.valueProject.bias": torch.randn(H, generator=g, dtype=torch.float64) * 0.1,
        "encoderN.layerNorm.weight": 1 + 0.1 * torch.randn(H, generator=g, dtype=torch.float64),
        "encoderN.layerNorm.bias": 0.1 * torch.randn(H, generator=g, dtype=torch.float64),
        "encoderN.query_words": torch.randn(1, H, generator=g, dtype=torch.float64),
    }
    return {k: v.requires_grad_(True) for k, v in P.items()}


@pytest.mark.parametrize("prec", ["f32", "bf16x6"])
@pytest.mark.parametrize("p_drop", [0.0, 0.2])
def test_fused_mha_news_encoder(p_drop, prec):
    """Under both fp32-class arithmetics of the projection GEMM and the attention products
    (nr_mha_pool_* prec: exact f32 MFMA / six-product bf16)."""
    from newsrec_amd import _lib as L
    with K.gemm_precision(L.GEMM_F32 if prec == "f32" else L.GEMM_BF16X6):
        _fused_mha_news_encoder(p_drop)


def _fused_mha_news_encoder(p_drop):
    g = torch.Generator().manual_seed(11)
    V, E, H, n, Lq = 500, 768, 384, 37, 30
    table = torch.randn(V, E, generator=g, dtype=torch.float64).requires_grad_(True)
    tok = torch.randint(0, V, (n, Lq), generator=g)
    lens = torch.randint(1, Lq + 1, (n,), generator=g)
    lens[0], lens[1], lens[2] = 0, Lq, 1
    mask = (torch.arange(Lq)[None] < lens[:, None]).long()
    P = _params(g)

    dev = "cuda"
    td = table.detach().float().to(dev).requires_grad_(True)
    Pd = {k: v.detach().float().to(dev).requires_grad_(True) for k, v in P.items()}
    w = torch.cat([Pd["encoderN.mha.keyProject.weight"], Pd["encoderN.mha.valueProject.weight"]], 0)
    b = torch.cat([Pd["encoderN.mha.keyProject.bias"], Pd["encoderN.mha.valueProject.bias"]], 0)
    assert K.mha_pool_supported(Lq, 12, 64, 32)
    news, tok_out = MHANewsFn.apply(td, tok.reshape(-1).to(dev), mask.reshape(-1).to(dev), w, b,
                                    Pd["encoderN.layerNorm.weight"], Pd["encoderN.layerNorm.bias"],
                                    Pd["encoderN.query_words"], 12, 64, 32, Lq, 0, p_drop, 1234, 77, True)
    keep = None
    if p_drop > 0:
        # recover the kernel's keep mask from its token output: Z = LN(O) * keep / (1 - p)
        with torch.no_grad():
            emb = R.word_embedding(table, tok)
            m = mask
            o = R.multihead_attention(emb, P["encoderN.mha.keyProject.weight"], P["encoderN.mha.keyProject.bias"],
                                      P["encoderN.mha.valueProject.weight"], P["encoderN.mha.valueProject.bias"],
                                      12, R.pairwise_mask(m))
            ln = R.layer_norm(o, P["encoderN.layerNorm.weight"], P["encoderN.layerNorm.bias"])
        keep = tok_out.detach().cpu().double().view(n, Lq, H).abs() > 1e-6
        frac = keep.double().mean().item()
        assert 0.75 < frac < 0.85, frac            # keep probability 0.8
        scaled = (ln / (1 - p_drop))[keep]
        torch.testing.assert_close(tok_out.detach().cpu().double().view(n, Lq, H)[keep], scaled, rtol=1e-4, atol=1e-4)
    emb = R.word_embedding(table, tok)
    _, want = R.mha_news(emb.unsqueeze(0), mask.unsqueeze(0), P, dropout_keep=keep.unsqueeze(0) if keep is not None else None,
                         p_drop=p_drop)
    want = want.squeeze(0)
    torch.testing.assert_close(news.detach().cpu().double(), want.detach(), rtol=1e-4, atol=2e-5)
    assert torch.all(news[0] == 0)                 # fully masked title pools to zero

    dn = torch.randn(n, H, generator=g, dtype=torch.float64)
    want.backward(dn)
    news.backward(dn.float().to(dev))
    torch.testing.assert_close(td.grad.cpu().double(), table.grad, rtol=0, atol=2e-4 * table.grad.abs().max().item())
    assert torch.all(td.grad[0] == 0) or not (tok == 0).any()   # padding row gets no gradient
    for k in P:
        ref = P[k].grad
        got = {"encoderN.layerNorm.weight": Pd[k].grad, "encoderN.layerNorm.bias": Pd[k].grad,
               "encoderN.query_words": Pd[k].grad}.get(k, Pd[k].grad)
        torch.testing.assert_close(got.cpu().double(), ref, rtol=0, atol=3e-4 * max(ref.abs().max().item(), 1e-3),
                                   msg=k)


@pytest.mark.parametrize("with_dz", [False, True])
@pytest.mark.parametrize("mode", ["split", "fused_saved", "fused_saved_ws"])
@pytest.mark.parametrize("p_drop", [0.0, 0.2])
def test_mha_pool_split_backward_matches_fused(p_drop, mode, with_dz):
    """The backward forms with the saved attention output O -- split (pooling/LN pass writing each
    token's row terms, per-head attention pass rebuilding its slice of dO from O) and fused on the saved
    O (dO kept in LDS; with and without the parameter-gradient copies) -- against the fused one that
    recomputes the attention; with_dz: a gradient of the token outputs Z too (MHANewsFn's dtok)."""
    from newsrec_amd import kernels as K
    torch.manual_seed(11)
    n, Lq, heads, dk, dv = 97, 30, 12, 64, 32
    T, NY, H = n * Lq, heads * (dk + dv), heads * dv
    y = torch.randn(T, NY, device="cuda") * 0.3
    mask = (torch.rand(n, Lq, device="cuda") < 0.8).long()
    mask[:, 0] = 1
    mask[5] = 0   # a fully masked title
    gamma = 1 + 0.1 * torch.randn(H, device="cuda")
    beta = 0.1 * torch.randn(H, device="cuda")
    q = torch.randn(H, device="cuda")
    dnews = torch.randn(n, H, device="cuda")
    dz = torch.randn(T, H, device="cuda") if with_dz else None
    outs = []
    for form in ("recompute", mode):
        saved = form != "recompute"
        news = torch.empty(n, H, device="cuda")
        stats = torch.empty(T, 2, device="cuda")
        probs = torch.empty(T, device="cuda")
        O = torch.empty(T, H, device="cuda") if saved else None
        K.mha_pool_fwd(y, mask, n, Lq, heads, dk, dv, gamma, beta, q, news, stats, probs, p_drop=p_drop, seed=9,
                       offset=3, oout=O)
        dy = torch.zeros(T, NY, device="cuda")
        db, dq, dg, dbt = (torch.zeros(NY, device="cuda"), torch.zeros(H, device="cuda"),
                           torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda"))
        dob = torch.empty(T, 8, device="cuda") if form == "split" else None
        ws = torch.zeros(32, (3 * H + NY + 3) // 4 * 4, device="cuda") if form == "fused_saved_ws" else None
        K.mha_pool_bwd(y, mask, n, Lq, heads, dk, dv, gamma, beta, q, stats, probs, dnews, dy, db, dq, dg, dbt,
                       p_drop=p_drop, seed=9, offset=3, dz=dz, o=O, dob=dob, ws=ws,
                       ws_copies=32 if ws is not None else 0)
        if ws is not None:
            torch.cuda.synchronize()
            assert not bool(ws.any().item())   # the copies are left zero
        outs.append((news, dy, db, dq, dg, dbt))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1:], outs[1][1:]):
        # dbias / dq / dgamma / dbeta are sums over the ~3k tokens in atomic order: the bar scales with
        # their magnitude (a random token-output gradient dz makes them O(10))
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-4 * max(1.0, a.abs().max().item()))
