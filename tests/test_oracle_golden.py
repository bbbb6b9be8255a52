"""The CPU oracle (oracle/restatement.py) against goldens produced by the reference's
own modules (tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from golden_util import Golden, GOLDEN, CONFIG_ENCODERS
from oracle import restatement as R

CONFIGS = list(CONFIG_ENCODERS)


def _keep(g):
    return torch.from_numpy(g["in.lstur_keep"]) if "in.lstur_keep" in g.z else None


@pytest.mark.parametrize("cfg", CONFIGS)
def test_oracle_forward_matches_reference(cfg):
    g = Golden(cfg)
    P = g.torch_params()
    x = g.inputs()
    with torch.no_grad():
        ev = R.forward(P, x, g.encN, g.encU, False, _keep(g))
        tr = R.forward(P, x, g.encN, g.encU, True, _keep(g))
        cdd = R.encode_news(P, x["cdd_encoded_index"], x["cdd_attn_mask"], g.encN)
        user = R.encode_user(P, x, g.encN, g.encU, _keep(g))
    np.testing.assert_allclose(cdd.numpy(), g["out.cdd_repr"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(user.numpy(), g["out.user_repr"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(tr.numpy(), g["out.train_logits"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(ev.numpy(), g["out.eval_logits"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_oracle_grads_match_reference(cfg):
    g = Golden(cfg)
    P = g.torch_params(requires_grad=True)
    x = g.inputs()
    logits = R.forward(P, x, g.encN, g.encU, True, _keep(g))
    loss = R.nll_loss(logits, x["label"])
    loss.backward()
    assert abs(loss.item() - float(g["out.loss"])) < 1e-5
    for n in g.names:
        want = g["grad." + n]
        got = P[n].grad.numpy() if P[n].grad is not None else np.zeros_like(want)
        scale = max(np.abs(want).max(), 1e-6)
        np.testing.assert_allclose(got, want, rtol=0, atol=2e-4 * scale, err_msg=n)


def test_oracle_adam_matches_reference():
    g = Golden("cnn_attn")
    P = g.torch_params(requires_grad=True)
    x = g.inputs()
    base, bert = R.adam_groups(P)
    opt = torch.optim.Adam([{"params": [P[k] for k in base], "lr": 1e-4},
                            {"params": [P[k] for k in bert], "lr": 6e-6}])
    logits = R.forward(P, x, g.encN, g.encU, True)
    R.nll_loss(logits, x["label"]).backward()
    opt.step()
    opt.step()
    for n in g.names:
        np.testing.assert_allclose(P[n].detach().numpy(), g["adam2." + n], rtol=0, atol=1e-6, err_msg=n)


def test_oracle_cal_metric_known_answers():
    rows = json.load(open(os.path.join(GOLDEN, "cal_metric.json")))
    for r in rows:
        got = R.cal_metric(r["labels"], r["preds"], ["auc", "mean_mrr", "ndcg@5;10"])
        for k, v in got.items():
            assert abs(v - r["res"][k]) < 1e-4, (k, v, r["res"][k])


def test_bf16_restatement_structure_matches_reference(monkeypatch):
    """R.forward_cnn_bf16 (configs[1]'s bf16 GEMM arithmetic) with its rounding switched off is the
    reference's CNN + attention step: logits, loss and every gradient against the reference golden
    (the per-tap products, the per-distinct-id gradient sums and the joint candidate | history pass
    are a refactoring of CNN.py:30-50, not another algorithm).  With the rounding on, the step moves
    by the bf16 error only (logits ~1e-2, gradients a few 1e-2 of their norm)."""
    g = Golden("cnn_attn")
    x = g.inputs()

    def step(P):
        logits = R.forward_cnn_bf16(P, x, g.encU, True)
        loss = R.nll_loss(logits, x["label"])
        loss.backward()
        return logits.detach(), loss.item()

    monkeypatch.setattr(R, "bf16_round", lambda t: t)
    P = g.torch_params(requires_grad=True)
    logits, loss = step(P)
    np.testing.assert_allclose(logits.numpy(), g["out.train_logits"], rtol=0, atol=1e-5)
    assert abs(loss - float(g["out.loss"])) < 1e-5
    for n in g.names:
        want = g["grad." + n]
        scale = max(np.abs(want).max(), 1e-6)
        np.testing.assert_allclose(P[n].grad.numpy(), want, rtol=0, atol=2e-4 * scale, err_msg=n)
    monkeypatch.undo()
    P = g.torch_params(requires_grad=True)
    logits, loss = step(P)
    assert 1e-5 < np.abs(logits.numpy() - g["out.train_logits"]).max() < 2e-2
    for n in g.names:
        want = g["grad." + n]
        rel = np.linalg.norm(P[n].grad.numpy() - want) / max(np.linalg.norm(want), 1e-12)
        assert rel < 5e-2, (n, rel)
