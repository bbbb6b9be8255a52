"""HIP BERT tower (XFormer / PLM): kernel parity against fp64 torch references, and the
models against goldens the reference's own XFormer / PLM classes produced
(tests/golden/make_bert_golden.py) and against the CPU oracle at BERT-base width."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from golden_util import Golden, BERT_CONFIGS
from model_util import build_bert_model
from oracle import restatement as R

LOGIT_ATOL = 1e-4   # north_star: 1e-3


def _attn_ref(qkv, mask, nseq, L, heads):
    """fp64 BertSelfAttention core (eager additive mask)."""
    H = heads * 64
    x = qkv.double().view(nseq, L, 3, heads, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = q @ k.transpose(-1, -2) / 8.0 + R.bert_mask_add(mask.view(nseq, L)).double()[:, None, None, :]
    p = torch.softmax(s, -1)
    return (p @ v).transpose(1, 2).reshape(nseq * L, H)


# attention products' arithmetic -> (forward atol, backward atol relative to max |grad|): f32 and
# bf16x6 (fp32-class, 2^-24 per product) share the fp32 bars; plain bf16 rounds every operand to
# 8 bits (2^-9 relative), scaled by the O(1) scores / values here
ATTN_PRECS = {"f32": (2e-5, 1e-4), "bf16x6": (2e-5, 1e-4), "bf16": (3e-2, 3e-2)}


@pytest.mark.parametrize("prec", list(ATTN_PRECS))
@pytest.mark.parametrize("nseq,L,heads", [(7, 30, 2), (3, 77, 12), (2, 501, 12), (5, 1, 1), (4, 33, 2), (2, 140, 3), (3, 97, 2)])
def test_attention_fwd_bwd(nseq, L, heads, prec):
    from newsrec_amd import _lib as Lb, kernels as K
    mode = {"f32": Lb.GEMM_F32, "bf16x6": Lb.GEMM_BF16X6, "bf16": Lb.GEMM_BF16}[prec]
    fa, ba = ATTN_PRECS[prec]
    torch.manual_seed(L)
    H = heads * 64
    T = nseq * L
    qkv = torch.randn(T, 3 * H, device="cuda")
    lens = torch.randint(1, L + 1, (nseq,))
    mask = (torch.arange(L)[None] < lens[:, None]).long()
    if nseq > 2:
        mask[1] = 0                                   # a fully masked sequence: uniform rows
    mask = mask.reshape(-1).cuda()
    ctx = torch.empty(T, H, device="cuda")
    ml = torch.empty(T * heads * 2, device="cuda")
    K.bert_attn_fwd(qkv, heads, mask, nseq, L, ctx, ml, prec=mode)
    q64 = qkv.detach().cpu().double().requires_grad_()
    want = _attn_ref(q64, mask.cpu(), nseq, L, heads)
    np.testing.assert_allclose(ctx.cpu().numpy(), want.detach().numpy(), rtol=0, atol=fa)
    d = torch.randn(T, H, device="cuda")
    dqkv = torch.full((T, 3 * H), float("nan"), device="cuda")
    K.bert_attn_bwd(qkv, heads, mask, nseq, L, ctx, ml, d, dqkv, prec=mode)
    want.backward(d.cpu().double())
    g = q64.grad.numpy()
    np.testing.assert_allclose(dqkv.cpu().numpy(), g, rtol=0, atol=ba * max(1.0, np.abs(g).max()))


@pytest.mark.parametrize("L", [45, 140])   # 140: four-wave launches (the dS-tile backward), two chunks
@pytest.mark.parametrize("prec", ["f32", "bf16x6"])
def test_attention_dropout_consistent(prec, L, request):
    """Dropout on the probabilities: the backward regenerates the forward's mask (directional
    derivative of <ctx, d> matches finite differences under the same seed); about p of the
    mass is dropped."""
    from newsrec_amd import _lib as Lb, kernels as K
    torch.manual_seed(3)
    old = K.set_gemm_precision(Lb.GEMM_F32 if prec == "f32" else Lb.GEMM_BF16X6)
    request.addfinalizer(lambda: K.set_gemm_precision(old))
    nseq, heads, p = 3, 2, 0.3
    H, T = heads * 64, nseq * L
    qkv = torch.randn(T, 3 * H, device="cuda")
    mask = torch.ones(T, dtype=torch.long, device="cuda")
    ml = torch.empty(T * heads * 2, device="cuda")
    d = torch.randn(T, H, device="cuda")

    def f(z):
        c = torch.empty(T, H, device="cuda")
        K.bert_attn_fwd(z, heads, mask, nseq, L, c, ml, p_drop=p, seed=11, offset=5)
        return c
    ctx = f(qkv)
    dqkv = torch.empty(T, 3 * H, device="cuda")
    K.bert_attn_bwd(qkv, heads, mask, nseq, L, ctx, ml, d, dqkv, p_drop=p, seed=11, offset=5)
    u = torch.randn_like(qkv)
    eps = 1e-2
    fd = ((f(qkv + eps * u) * d).double().sum() - (f(qkv - eps * u) * d).double().sum()) / (2 * eps)
    an = (dqkv.double() * u.double()).sum()
    assert abs(fd.item() - an.item()) < 2e-2 * max(1.0, abs(an.item())), (fd.item(), an.item())
    # no dropout reference: E[ctx_drop] = ctx
    c0 = torch.empty(T, H, device="cuda")
    K.bert_attn_fwd(qkv, heads, mask, nseq, L, c0, ml)
    assert not torch.allclose(c0, ctx)
    rel = ((ctx - c0).norm() / c0.norm()).item()
    assert 0.05 < rel < 2.0


@pytest.mark.parametrize("prec", ["bf16x6", "bf16"])
@pytest.mark.parametrize("nseq,L,heads", [(3, 45, 2), (2, 501, 12), (4, 30, 12), (2, 33, 1), (3, 97, 2)])
def test_attention_dropout_keep_bits(nseq, L, heads, prec):
    """The bf16-MFMA forward's stored keep bits (nr_bert_attn_keep_words): the backward reading them
    is BITWISE the backward that re-hashes every probability's counter (the same masks, the same
    arithmetic), for the title shape, the 501-token user sequence, ragged key tiles and graph RNG
    pairs; about p of the bits are clear; a keep buffer with the f32 forward is refused."""
    from newsrec_amd import _lib as Lb, kernels as K
    mode = Lb.GEMM_BF16X6 if prec == "bf16x6" else Lb.GEMM_BF16
    torch.manual_seed(L + heads)
    p = 0.1
    H, T = heads * 64, nseq * L
    qkv = torch.randn(T, 3 * H, device="cuda")
    lens = torch.randint(1, L + 1, (nseq,))
    mask = (torch.arange(L)[None] < lens[:, None]).long().reshape(-1).cuda()
    rng = torch.tensor([123456789, 4242], dtype=torch.int64, device="cuda")
    ml = torch.empty(T * heads * 2, device="cuda")
    ctx0, ctx1 = torch.empty(T, H, device="cuda"), torch.empty(T, H, device="cuda")
    keep = K.bert_attn_keep_buffer(nseq, L, heads, "cuda")
    keep.fill_(-1)
    K.bert_attn_fwd(qkv, heads, mask, nseq, L, ctx0, ml, p_drop=p, rng=rng, prec=mode)
    K.bert_attn_fwd(qkv, heads, mask, nseq, L, ctx1, ml, p_drop=p, rng=rng, prec=mode, keep=keep)
    assert torch.equal(ctx0, ctx1)
    nkb = (L + 31) // 32
    words = keep[:nseq * heads * L * nkb].view(nseq * heads, L, nkb).cpu().numpy().view(np.uint32)
    valid = np.zeros((L, nkb, 32), bool)          # bit b of (q, kb) is a key < L
    for kb in range(nkb):
        for b in range(32):
            r, h = b % 16, b // 16
            valid[:, kb, b] = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h < L
    bits = (words[..., None] >> np.arange(32, dtype=np.uint32)) & 1
    frac = bits[:, valid].mean()
    assert abs((1 - frac) - p) < 0.02, frac
    d = torch.randn(T, H, device="cuda")
    g0 = torch.empty(T, 3 * H, device="cuda")
    g1 = torch.empty(T, 3 * H, device="cuda")
    K.bert_attn_bwd(qkv, heads, mask, nseq, L, ctx0, ml, d, g0, p_drop=p, rng=rng, prec=mode)
    K.bert_attn_bwd(qkv, heads, mask, nseq, L, ctx0, ml, d, g1, p_drop=p, rng=rng, prec=mode, keep=keep)
    assert torch.equal(g0, g1)
    with pytest.raises(Lb.HipError):
        K.bert_attn_fwd(qkv, heads, mask, nseq, L, ctx1, ml, p_drop=p, rng=rng, prec=Lb.GEMM_F32, keep=keep)


def test_add_ln_and_embed():
    from newsrec_amd import kernels as K
    torch.manual_seed(0)
    T, H = 97, 768
    x = torch.randn(T, H, device="cuda")
    res = torch.randn(T, H, device="cuda")
    gm = 1 + 0.1 * torch.randn(H, device="cuda")
    bt = 0.1 * torch.randn(H, device="cuda")
    out = torch.empty(T, H, device="cuda")
    st = torch.empty(T, 2, device="cuda")
    K.bert_add_ln_fwd(x, res, gm, bt, 1e-12, out, st)
    xs, rs, gs, bs = (t.cpu().double().requires_grad_() for t in (x, res, gm, bt))
    want = F.layer_norm(xs + rs, (H,), gs, bs, 1e-12)
    np.testing.assert_allclose(out.cpu().numpy(), want.detach().numpy(), rtol=0, atol=2e-5)
    d = torch.randn(T, H, device="cuda")
    dres, dx = torch.empty_like(x), torch.empty_like(x)
    dg, db = torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda")
    K.bert_add_ln_bwd(x, res, gm, st, d, dres, dx, dg, db)
    want.backward(d.cpu().double())
    np.testing.assert_allclose(dx.cpu().numpy(), xs.grad.numpy(), rtol=0, atol=1e-4)
    np.testing.assert_allclose(dres.cpu().numpy(), rs.grad.numpy(), rtol=0, atol=1e-4)
    np.testing.assert_allclose(dg.cpu().numpy(), gs.grad.numpy(), rtol=0, atol=1e-3)
    np.testing.assert_allclose(db.cpu().numpy(), bs.grad.numpy(), rtol=0, atol=1e-3)

    V, P, nseq, L = 300, 40, 5, 31
    word, pos, typ = (0.5 * torch.randn(n, H, device="cuda") for n in (V, P, 2))
    ids = torch.randint(0, V, (nseq * L,), device="cuda")
    out = torch.empty(nseq * L, H, device="cuda")
    st = torch.empty(nseq * L, 2, device="cuda")
    K.bert_embed_fwd(word, pos, typ[0], ids, nseq, L, gm, bt, 1e-12, out, st)
    P64 = {"bert.embeddings.word_embeddings.weight": word.cpu().double().requires_grad_(),
           "bert.embeddings.position_embeddings.weight": pos.cpu().double().requires_grad_(),
           "bert.embeddings.token_type_embeddings.weight": typ.cpu().double().requires_grad_(),
           "bert.embeddings.LayerNorm.weight": gm.cpu().double(), "bert.embeddings.LayerNorm.bias": bt.cpu().double()}
    want = R.bert_embeddings(P64, ids.cpu().view(nseq, L)).reshape(nseq * L, H)
    np.testing.assert_allclose(out.cpu().numpy(), want.detach().numpy(), rtol=0, atol=2e-5)


def test_gelu_epilogues():
    from newsrec_amd import _lib as Lb, kernels as K
    torch.manual_seed(1)
    M, N, Kd = 200, 384, 96
    a = torch.randn(M, Kd, device="cuda")
    w = torch.randn(N, Kd, device="cuda") / 8
    b = torch.randn(N, device="cuda")
    U = torch.empty(M, N, device="cuda")
    G = torch.empty(M, N, device="cuda")
    K.gemm(M, N, Kd, K.operand(a, Lb.KCONTIG), K.operand(w, Lb.KCONTIG), G, bias=b, epilogue=Lb.EPI_STORE_GELU,
           c_rows=K.operand(U, Lb.KCONTIG))
    pre = a.double().cpu() @ w.double().cpu().T + b.double().cpu()
    np.testing.assert_allclose(U.cpu().numpy(), pre.numpy(), rtol=0, atol=1e-4)
    np.testing.assert_allclose(G.cpu().numpy(), F.gelu(pre).numpy(), rtol=0, atol=1e-4)
    dy = torch.randn(M, Kd, device="cuda")
    wt = torch.randn(Kd, N, device="cuda").contiguous()   # B(k, n) stored [k][n]
    dU = torch.empty(M, N, device="cuda")
    K.gemm(M, N, Kd, K.operand(dy, Lb.KCONTIG), K.operand(wt, Lb.MNCONTIG), dU, epilogue=Lb.EPI_GELU_GRAD,
           c_rows=K.operand(U, Lb.KCONTIG))
    x = pre.clone().requires_grad_()
    F.gelu(x).backward(dy.double().cpu() @ wt.double().cpu())
    np.testing.assert_allclose(dU.cpu().numpy(), x.grad.numpy(), rtol=0, atol=1e-3)


def _oracle_fwd(g, P, x, training):
    if g.encU == "xformer":
        return R.xformer_forward(P, x, training, g.heads)
    return R.plm_forward(P, x, g.encU, training, g.heads)


@pytest.fixture(params=["bf16x6", "f32"])
def gemm_prec(request):
    from newsrec_amd import _lib as Lb, kernels as Kn
    old = Kn.set_gemm_precision(Lb.GEMM_BF16X6 if request.param == "bf16x6" else Lb.GEMM_F32)
    yield request.param
    Kn.set_gemm_precision(old)


@pytest.mark.parametrize("cfg", list(BERT_CONFIGS))
def test_bert_models_forward_parity(cfg, gemm_prec):
    g = Golden(cfg)
    model = build_bert_model(g)
    x = g.inputs("cuda")
    model.eval()
    with torch.no_grad():
        ev, _ = model(x)
        cdd = model.encode_news(x)
        user, _ = model.encode_user(x)
    model.train()
    with torch.no_grad():
        tr, _ = model(x)
    np.testing.assert_allclose(ev.cpu().numpy(), g["out.eval_logits"], rtol=0, atol=LOGIT_ATOL)
    np.testing.assert_allclose(tr.cpu().numpy(), g["out.train_logits"], rtol=0, atol=LOGIT_ATOL)
    np.testing.assert_allclose(cdd.cpu().numpy(), g["out.cdd_repr"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(user.cpu().numpy(), g["out.user_repr"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cfg", list(BERT_CONFIGS))
def test_bert_models_grad_parity(cfg, gemm_prec):
    g = Golden(cfg)
    model = build_bert_model(g)
    x = g.inputs("cuda")
    model.train()
    logits, _ = model(x)
    loss = F.nll_loss(logits, x["label"])
    loss.backward()
    assert abs(loss.item() - float(g["out.loss"])) < 1e-4
    ps = dict(model.named_parameters())
    for n in g.names:
        want = g["grad." + n]
        p = ps[n]
        got = p.grad.cpu().numpy() if p.grad is not None else np.zeros_like(want)
        scale = max(float(np.abs(want).max()), 1e-6)
        np.testing.assert_allclose(got, want, rtol=0, atol=max(1e-3 * scale, 2e-6), err_msg=n)


def test_xformer_bert_base_width_vs_oracle(gemm_prec):
    """BERT-base width (768, 12 heads, 3072) with 2 layers on the full 501-token user sequence
    and 30-token titles, against the fp32 CPU oracle (logits and a few gradients)."""
    from newsrec_amd.bert import BertConfig
    from newsrec_amd.manager import ManagerConfig
    from newsrec_amd.xformer import XFormer
    torch.manual_seed(7)
    B, C, N, Lt, V = 2, 5, 50, 30, 30522
    bc = BertConfig(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = ManagerConfig("bert", "xformer", 768, bert_dim=768)
    model = XFormer(m, bert_config=bc).cuda()
    with torch.no_grad():   # spread the scores (reference init gives a near-constant pooler)
        for n, p in model.named_parameters():
            if p.dim() == 2 and "embeddings" not in n:
                p.normal_(0, 1.5 / math.sqrt(p.shape[1]))
    gen = torch.Generator().manual_seed(0)
    def titles(n):
        t = torch.randint(1000, V, (n, Lt), generator=gen)
        lens = torch.randint(3, Lt + 1, (n,), generator=gen)
        msk = (torch.arange(Lt)[None] < lens[:, None]).long()
        t = t * msk
        t[:, 0] = 101
        return t, msk
    ct, cm = titles(B * C)
    ht, hm = titles(B * N)
    x = {"cdd_encoded_index": ct.view(B, C, Lt), "cdd_attn_mask": cm.view(B, C, Lt),
         "his_encoded_index": ht.view(B, N, Lt), "his_attn_mask": hm.view(B, N, Lt),
         "label": torch.zeros(B, dtype=torch.long)}
    xg = {k: v.cuda() for k, v in x.items()}
    model.train()
    logits, _ = model(xg)
    F.nll_loss(logits, xg["label"]).backward()
    P = {n: p.detach().cpu().clone().requires_grad_() for n, p in model.named_parameters()}
    want = R.xformer_forward(P, x, True, 12)
    np.testing.assert_allclose(logits.detach().cpu().numpy(), want.detach().numpy(), rtol=0, atol=1e-3)
    R.nll_loss(want, x["label"]).backward()
    ps = dict(model.named_parameters())
    for n in ["bert.embeddings.word_embeddings.weight", "bert.encoder.layer.0.attention.self.query.weight",
              "bert.encoder.layer.1.intermediate.dense.weight", "bert.pooler.dense.weight", "userBias"]:
        w = P[n].grad.numpy()
        scale = max(float(np.abs(w).max()), 1e-6)
        np.testing.assert_allclose(ps[n].grad.cpu().numpy(), w, rtol=0, atol=5e-3 * scale, err_msg=n)
