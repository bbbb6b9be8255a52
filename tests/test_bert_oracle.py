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
