"""The BERT-tower oracle (oracle/restatement.py: bert_model, xformer_forward, plm_forward)
against goldens the reference's own XFormer / PLM classes produced around a locally built
transformers BertModel (tests/golden/make_bert_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from golden_util import Golden, BERT_CONFIGS
from oracle import restatement as R


def oracle_forward(g, P, x, training):
    if g.encU == "xformer":
        return R.xformer_forward(P, x, training, g.heads)
    return R.plm_forward(P, x, g.encU, training, g.heads)


@pytest.mark.parametrize("cfg", list(BERT_CONFIGS))
def test_bert_oracle_forward(cfg):
    g = Golden(cfg)
    P = g.torch_params()
    x = g.inputs()
    with torch.no_grad():
        ev = oracle_forward(g, P, x, False)
        tr = oracle_forward(g, P, x, True)
        B, C, L = x["cdd_encoded_index"].shape
        cdd = R.bert_model(P, x["cdd_encoded_index"].view(-1, L), x["cdd_attn_mask"].view(-1, L), g.heads)[1]
    np.testing.assert_allclose(cdd.view(B, C, -1).numpy(), g["out.cdd_repr"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(tr.numpy(), g["out.train_logits"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(ev.numpy(), g["out.eval_logits"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("cfg", list(BERT_CONFIGS))
def test_bert_oracle_grads(cfg):
    g = Golden(cfg)
    P = g.torch_params(requires_grad=True)
    x = g.inputs()
    loss = R.nll_loss(oracle_forward(g, P, x, True), x["label"])
    loss.backward()
    assert abs(loss.item() - float(g["out.loss"])) < 2e-5
    for n in g.names:
        want = g["grad." + n]
        got = P[n].grad.numpy() if P[n].grad is not None else np.zeros_like(want)
        scale = max(np.abs(want).max(), 1e-6)
        # key.bias has an exactly-zero true gradient (softmax is shift-invariant per row): the
        # golden holds rounding noise there, hence the absolute floor
        np.testing.assert_allclose(got, want, rtol=0, atol=max(2e-4 * scale, 1e-6), err_msg=n)


def test_xformer_user_sequence_shape():
    """XFormer.py:83-89: [CLS] + 50 x 10 tokens -> 501 positions."""
    g = Golden("xformer")
    x = g.inputs()
    t, m = R.xformer_user_tokens(x["his_encoded_index"], x["his_attn_mask"])
    assert t.shape == (x["his_encoded_index"].shape[0], 501) and m.shape == t.shape
    assert (t[:, 0] == x["his_encoded_index"][:, 0, 0]).all()
    assert (t[:, 1:11] == x["his_encoded_index"][:, 0, 1:11]).all()


def _scalar_keep(seed, offset, elem, p, mix=None):
    """One element of the device dropout, restated in plain Python integers (csrc/common.h
    nr_dropout_key / nr_hash32 / nr_dropout_keep; ``mix``: the attention kernels' per-(sequence, head)
    key, nr_hash32(k ^ uint32(mix * 0x85EBCA6B)), csrc/bert.hip attn_key)."""
    M64, M32 = (1 << 64) - 1, (1 << 32) - 1
    z = (seed * 0x9E3779B97F4A7C15 + offset * 0xD1B54A32D192ED03 + 0x632BE59BD9B4E019) & M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    key = z >> 32

    def h32(x):
        x ^= x >> 16
        x = (x * 0x7FEB352D) & M32
        x ^= x >> 15
        x = (x * 0x846CA68B) & M32
        return x ^ (x >> 16)
    if mix is not None:
        key = h32(key ^ ((mix * 0x85EBCA6B) & M32))
    return h32((key + elem * 0x9E3779B1) & M32) >= int(float(np.float32(p)) * 4294967296.0)


def test_bert_dropout_restatement():
    """R.BertDropout (the XFormer step's 37 device dropout sites) against a scalar restatement of
    the kernels' hash at sampled elements of every site kind; every site keeps ~1 - p and draws its
    own mask; and at p = 0 the dropout-replaying oracle is the reference's golden forward."""
    seed, off, T, H, layers, heads, p = 12345, 777, 2 * 5 * 30 + 2 * 501, 768, 12, 12, 0.1
    d = R.BertDropout(seed, off, T, H, layers, heads, p, p)
    r0 = 2 * 5 * 30
    rng = np.random.default_rng(0)
    emb = d.embed(r0, 2 * 501).numpy()                 # the user segment's embeddings
    for t, c in zip(rng.integers(0, 2 * 501, 50), rng.integers(0, H, 50)):
        assert emb[t, c] == _scalar_keep(seed, d.site[0] + r0 * H, int(t) * H + int(c), p)
    for li, which in ((0, 0), (11, 1), (5, 0)):
        den = d.dense(li, which, r0, 2 * 501).numpy()  # global rows r0 ...
        for t, c in zip(rng.integers(0, 2 * 501, 30), rng.integers(0, H, 30)):
            assert den[t, c] == _scalar_keep(seed, d.site[2 + 3 * li + which], (r0 + int(t)) * H + int(c), p)
        att = d.attn(li, r0, 2, 501).numpy()
        for s, h, q, k in zip(rng.integers(0, 2, 30), rng.integers(0, heads, 30), rng.integers(0, 501, 30),
                              rng.integers(0, 501, 30)):
            assert att[s, h, q, k] == _scalar_keep(seed, d.site[1 + 3 * li] + r0, int(q) * 501 + int(k), p,
                                                   mix=int(s) * heads + int(h))
        assert abs(att.mean() - (1 - p)) < 0.01 and abs(den.mean() - (1 - p)) < 0.01
    assert abs(emb.mean() - (1 - p)) < 0.01
    assert (d.dense(0, 0, 0, 100) != d.dense(0, 1, 0, 100)).any()   # sites draw their own masks
    g = Golden("xformer")
    P = g.torch_params()
    x = g.inputs()
    B, C, L = x["cdd_encoded_index"].shape
    d0 = R.BertDropout(seed, off, B * C * L + B * 501, P["bert.embeddings.word_embeddings.weight"].shape[1],
                       R.bert_layers(P), g.heads, 0.0, 0.0)
    with torch.no_grad():
        tr = R.xformer_forward(P, x, True, g.heads, drop=d0)
    np.testing.assert_allclose(tr.numpy(), g["out.train_logits"], rtol=0, atol=2e-5)
