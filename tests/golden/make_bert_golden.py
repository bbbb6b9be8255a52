"""Golden vectors for the BERT towers (XFormer, PLM) from the REFERENCE's own model classes.

Runs in the build container only (imports /root/reference read-only; the GPU box never sees it).
``XFormer.__init__`` / ``PLM.__init__`` call ``AutoModel.from_pretrained("bert-base-uncased")``
(models/XFormer.py:45-48, models/PLM.py:80-86), a remote fetch that is unavailable offline, so
both are built with ``__new__`` + ``TwoTowerBaseModel.__init__`` and handed a locally
constructed ``transformers.BertModel`` (SURVEY.md §8(c) recipe step 5):

  * a reduced BertConfig (hidden 128, 2 heads of 64, 2 layers, intermediate 512, vocab 256,
    512 positions) so the fixture stays small; the HIP kernels are the same code at BERT-base
    sizes, which the GPU tests check against the oracle directly;
  * attn_implementation="eager": the additive-mask softmax of the transformers releases the
    reference was written against (transformers is unpinned);
  * dropout probabilities 0 so the train-mode goldens are deterministic;
  * parameters from the seeded stream of tests/golden/params.py (O(1) score spread).

Writes xformer.npz (XFormer, debias userBias) and plm.npz (PLM bert branch + Attention_Pooling
user encoder + userBias): inputs, logits (train log-softmax, eval sigmoid), loss, every gradient.

Usage:  python tests/golden/make_bert_golden.py [--out tests/golden]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (news table + batch builders, Cfg)
from params import regen_params  # noqa: E402

REF = MG.REF
BERT_CFG = dict(vocab_size=MG.V, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                intermediate_size=512, max_position_embeddings=512, hidden_dropout_prob=0.0,
                attention_probs_dropout_prob=0.0)


def _bert():
    from transformers import BertConfig, BertModel
    cfg = BertConfig(**BERT_CFG, attn_implementation="eager")
    return BertModel(cfg)


def _base_cfg():
    m = MG.Cfg("bert", "attn", BERT_CFG["hidden_size"])
    m.bert_dim = BERT_CFG["hidden_size"]
    m.bert = "bert"
    m.debias = True
    return m


def build(kind, seed):
    sys.path.insert(0, REF)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    import models.Modules.Attention as A   # XSoftmax.backward, torch>=1.13 signature (same math)
    A._softmax_backward_data = lambda g, y, d, _o: torch._softmax_backward_data(g, y, d, y.dtype)
    from models.TwoTowerBaseModel import TwoTowerBaseModel
    torch.manual_seed(seed)
    m = _base_cfg()
    if kind == "xformer":
        from models.XFormer import XFormer
        model = XFormer.__new__(XFormer)
        TwoTowerBaseModel.__init__(model, m)
        model.bert_name = "bert"
        model.max_length, model.max_length_per_history = 512, 10   # Manager.py:1019 "bert"
        model.bert = _bert()
        model.userBias = nn.Parameter(torch.randn(1, m.bert_dim))
        model.name = "xformer__bert"
    else:
        from models.PLM import PLM
        from models.Encoders.Pooling import Attention_Pooling
        model = PLM.__new__(PLM)
        TwoTowerBaseModel.__init__(model, m)
        model.encoderU = Attention_Pooling(m)
        model.userBias = nn.Parameter(torch.randn(1, m.bert_dim))
        model.bert = _bert()
        model.name = "plm__bert__attn"
    vals = regen_params([(n, tuple(p.shape)) for n, p in model.named_parameters()], seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.copy_(torch.from_numpy(vals[name]))
    return model


def run(kind, seed, out_dir):
    rng = np.random.default_rng(seed)
    tok, msk = MG.make_news_table(rng)
    batch = MG.make_batch(rng, tok, msk, 40)
    model = build(kind, seed)
    x = {k: torch.from_numpy(v) for k, v in batch.items()}
    names = [n for n, _ in model.named_parameters()]
    params0 = {n: p.detach().clone() for n, p in model.named_parameters()}

    model.eval()
    with torch.no_grad():
        eval_logits, _ = model(x)
        cdd_repr = model.encode_news(x)
        user_repr, _ = model.encode_user(x)
    model.train()
    logits, _ = model(x)
    loss = nn.NLLLoss()(logits, x["label"])
    loss.backward()

    out = {"in." + k: v for k, v in batch.items()}
    for n in names:
        p0 = params0[n].numpy().astype(np.float64)
        out["pcheck." + n] = np.asarray([p0.sum(), np.abs(p0).sum()])
        g = model.get_parameter(n).grad
        out["grad." + n] = (g if g is not None else torch.zeros_like(params0[n])).numpy()
    out["out.cdd_repr"] = cdd_repr.numpy()
    out["out.user_repr"] = user_repr.numpy()
    out["out.train_logits"] = logits.detach().numpy()
    out["out.loss"] = np.asarray(loss.item(), np.float32)
    out["out.eval_logits"] = eval_logits.numpy()
    out["meta.hidden_dim"] = np.asarray(BERT_CFG["hidden_size"])
    out["meta.heads"] = np.asarray(BERT_CFG["num_attention_heads"])
    out["meta.vocab"] = np.asarray(MG.V)
    out["meta.seed"] = np.asarray(seed)
    out["meta.bert_cfg"] = np.asarray(sorted(BERT_CFG.items()), dtype=object).astype(str)
    path = os.path.join(out_dir, kind + ".npz")
    np.savez_compressed(path, **out)
    spread = float((logits.detach().max(1).values - logits.min(1).values).mean())
    print(f"{kind}: loss={loss.item():.5f} logit spread={spread:.3f} -> {path} "
          f"({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    a = ap.parse_args()
    run("xformer", 2000, a.out)
    run("plm", 2001, a.out)
