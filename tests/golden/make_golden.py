"""Generate golden vectors by running the REFERENCE's own PyTorch modules on CPU.

This script is the only place that touches /root/reference, and it only runs in the
build container (the GPU box never sees the reference).  It imports the reference
read-only (PYTHONDONTWRITEBYTECODE=1), applies the compatibility patches listed in
SURVEY.md §8(c), and writes one small ``<config>.npz`` per model configuration:

  inputs     tokens / masks / ids exactly as ``MIND.__getitem__`` returns them
             (utils/MIND.py:311-365), batched by the default collate
  params     every named parameter (reference init, then scaled, see ``SCALE``)
  outputs    encode_news, encode_user, train log-softmax logits, NLL loss,
             eval sigmoid logits                     (models/TwoTowerBaseModel.py:51-75)
  grads      d loss / d param for every parameter    (Manager.py:641-644)
  adam       params after one Adam step, two groups  (Manager.py:389-413, 647)

Patches (none modifies a reference file):
  1. the BERT word table is an ``nn.Embedding(V, 768, padding_idx=0)`` with seeded weights
     (same module type as ``bert.embeddings.word_embeddings``; pretrained weights are
     not available offline) -- models/Embeddings/BERT.py:16-21
  2. ``XSoftmax.backward`` calls ``_softmax_backward_data`` with the torch>=1.13
     signature (same math) -- models/Modules/Attention.py:79
  3. NRMS: ``MHA_User_Encoder`` pools with the history mask transposed to [B,1,N]
     as ``Attention_Pooling`` does (Pooling.py:23); the unpatched reference returns
     [B,N,H] (MHA.py:71)
  4. LSTUR: ``user_id`` is forwarded as ``user_index`` (TwoTower.py:47 vs RNN.py:88) and
     the Bernoulli id-drop mask is injected (RNN.py:100-101)
  5. dropout p = 0 for the MHA configs so the train goldens are deterministic

Usage:  python tests/golden/make_golden.py [--out tests/golden]
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch.nn as nn

REF = "/root/reference"
V = 256          # reduced vocabulary (row 0 = [PAD] is a real, non-zero vector)
E = 768
B = 4
C = 5
NH = 50
L = 30
N_NEWS = 96      # synthetic news table rows (row 0 = the reference's padded "" news)


def make_news_table(rng):
    """Token table shaped like the reference's news.pkl cache (MIND.py:124-151), already
    truncated to L columns with the last column forced to [SEP] when it is not [PAD]
    (MIND.py:103-108).  Row 0 is tokenizer("") = [CLS, SEP, PAD...]."""
    tok = np.zeros((N_NEWS, L), np.int64)
    msk = np.zeros((N_NEWS, L), np.int64)
    tok[0, 0], tok[0, 1] = 101, 102
    msk[0, :2] = 1
    for n in range(1, N_NEWS):
        ln = int(rng.integers(5, L + 8))          # some titles are longer than L
        ln_eff = min(ln, L)
        tok[n, :ln_eff] = rng.integers(103, V, ln_eff)
        tok[n, 0] = 101
        if ln <= L:
            tok[n, ln - 1] = 102
        msk[n, :ln_eff] = 1
    sep_pos = tok[:, -1] != 0
    tok[:, -1] = np.where(sep_pos, 102, tok[:, -1])
    return tok, msk


def make_batch(rng, tok, msk, user_num):
    """One collated train batch, following MIND.__getitem__ (MIND.py:311-365) and
    newsample (utils.py:83-98): [pos] + npratio negatives, zero-padded when too few."""
    his_len = [0, 50, 7, 23][:B]
    neg_len = [4, 2, 9, 0][:B]
    cdd_id = np.zeros((B, C), np.int64)
    his_id = np.zeros((B, NH), np.int64)
    his_mask = np.zeros((B, NH, 1), np.float64)
    for b in range(B):
        pos = int(rng.integers(1, N_NEWS))
        negs = list(rng.choice(np.arange(1, N_NEWS), neg_len[b], replace=False))
        if len(negs) < C - 1:
            negs = negs + [0] * (C - 1 - len(negs))
        else:
            negs = list(rng.choice(negs, C - 1, replace=False))
        cdd_id[b] = [pos] + negs
        h = list(rng.integers(1, N_NEWS, his_len[b]))
        if len(h) == 0:
            his_mask[b, 0] = 1
        else:
            his_mask[b, :len(h)] = 1
        his_id[b] = h + [0] * (NH - len(h))
    user_id = rng.integers(1, user_num + 1, B).astype(np.int64)
    return {
        "cdd_id": cdd_id, "his_id": his_id,
        "cdd_encoded_index": tok[cdd_id], "cdd_attn_mask": msk[cdd_id],
        "his_encoded_index": tok[his_id], "his_attn_mask": msk[his_id],
        "his_mask": his_mask, "user_id": user_id,
        "label": np.zeros(B, np.int64),
    }


class Cfg:
    """Stand-in for ``Manager`` (utils/Manager.py:38-147): only the attributes the model
    constructors read."""
    def __init__(self, encN, encU, hidden):
        self.scale = "demo"; self.mode = "train"; self.cdd_size = C
        self.impr_size = 2000; self.batch_size_news = 500
        self.his_size = NH; self.signal_length = L; self.device = "cpu"
        self.bert_dim = E; self.embedding_dim = E; self.hidden_dim = hidden
        self.head_num = 12; self.dropout_p = 0.0; self.descend_history = False
        self.encoderN = encN; self.encoderU = encU
        self.user_num = 40

    def get_user_num(self):
        return self.user_num


CONFIGS = {
    # name: (encoderN, encoderU, hidden_dim)
    "cnn_attn": ("cnn", "attn", 150),
    "cnn_avg": ("cnn", "avg", 150),
    "cnn_lstm": ("cnn", "lstm", 150),
    "cnn_gru": ("cnn", "gru", 150),
    "cnn_lstur": ("cnn", "lstur", 150),
    "nrms": ("mha", "mha", 384),
}

# Parameters are NOT the reference's random init: reference init gives score spreads of
# ~1e-4 (SURVEY §7 "Hard parts"), which would make a 1e-3 logit check vacuous.  Every
# parameter is overwritten from a seeded numpy stream (tests/golden/params.py) whose scale
# spreads candidate scores by O(1); the tests regenerate the same values from the seed, so
# the fixtures carry only inputs, outputs and gradients.


def build(cfg_name, seed):
    sys.path.insert(0, REF)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    import models.Modules.Attention as A
    A._softmax_backward_data = lambda g, y, d, _o: torch._softmax_backward_data(g, y, d, y.dtype)
    from models.TwoTower import TwoTower
    from models.Embeddings.BERT import BERT_Embedding

    encN, encU, hidden = CONFIGS[cfg_name]
    m = Cfg(encN, encU, hidden)
    torch.manual_seed(seed)

    emb = BERT_Embedding.__new__(BERT_Embedding)
    nn.Module.__init__(emb)
    emb.hidden_dim = E
    emb.bert_word_embedding = nn.Embedding(V, E, padding_idx=0)

    if encN == "cnn":
        from models.Encoders.CNN import CNN_Encoder
        en = CNN_Encoder(m)
    else:
        from models.Encoders.MHA import MHA_Encoder
        en = MHA_Encoder(m)

    if encU in ("lstm", "gru"):
        from models.Encoders.RNN import RNN_User_Encoder
        eu = RNN_User_Encoder(m)
    elif encU == "attn":
        from models.Encoders.Pooling import Attention_Pooling
        eu = Attention_Pooling(m)
    elif encU == "avg":
        from models.Encoders.Pooling import Average_Pooling
        eu = Average_Pooling(m)
    elif encU == "lstur":
        from models.Encoders.RNN import LSTUR_User_Encoder
        eu = LSTUR_User_Encoder(m)
        orig = eu.forward

        def fwd(news_repr, his_mask=None, user_id=None, **kw):
            drop = eu._inject_mask
            saved = torch.Tensor.bernoulli_
            torch.Tensor.bernoulli_ = lambda self, *a, **k: self.copy_(drop)
            try:
                return orig(news_repr, his_mask=his_mask, user_index=user_id)
            finally:
                torch.Tensor.bernoulli_ = saved
        eu.forward = fwd
    else:
        from models.Encoders.MHA import MHA_User_Encoder
        from models.Modules.Attention import get_attn_mask, scaled_dp_attention
        eu = MHA_User_Encoder(m)

        def fwd(news_repr, his_mask=None, **kw):
            ext = get_attn_mask(his_mask.squeeze(-1))
            h = eu.mha(news_repr, ext)
            return scaled_dp_attention(eu.query_news, h, h, his_mask.transpose(-1, -2))
        eu.forward = fwd

    model = TwoTower(m, emb, en, eu)
    from params import regen_params
    vals = regen_params([(n, tuple(p.shape)) for n, p in model.named_parameters()], seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.copy_(torch.from_numpy(vals[name]))
    return model


def run(cfg_name, seed, out_dir):
    rng = np.random.default_rng(seed)
    tok, msk = make_news_table(rng)
    batch = make_batch(rng, tok, msk, 40)
    model = build(cfg_name, seed)
    if CONFIGS[cfg_name][1] == "lstur":
        drop = torch.tensor([1, 0, 1, 1][:B], dtype=torch.long)
        model.encoderU._inject_mask = drop
        batch["lstur_keep"] = drop.numpy()
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
    grads = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
             for n, p in model.named_parameters()}

    base = [p for n, p in model.named_parameters() if "bert" not in n]
    bert = [p for n, p in model.named_parameters() if "bert" in n]
    opt = torch.optim.Adam([{"params": base, "lr": 1e-4}, {"params": bert, "lr": 6e-6}])
    opt.step()
    # second step with the same grads: exercises the bias correction at t=2
    opt.step()
    adam2 = {n: p.detach().clone() for n, p in model.named_parameters()}

    out = {}
    for k, v in batch.items():
        out["in." + k] = v
    out["news.tok"] = tok
    out["news.msk"] = msk
    for n in names:
        p0 = params0[n].numpy().astype(np.float64)
        out["pcheck." + n] = np.asarray([p0.sum(), np.abs(p0).sum()])
        out["grad." + n] = grads[n].numpy()
        if cfg_name == "cnn_attn":
            out["adam2." + n] = adam2[n].numpy()
    out["out.cdd_repr"] = cdd_repr.numpy()
    out["out.user_repr"] = user_repr.numpy()
    out["out.train_logits"] = logits.detach().numpy()
    out["out.loss"] = np.asarray(loss.item(), np.float32)
    out["out.eval_logits"] = eval_logits.numpy()
    out["meta.hidden_dim"] = np.asarray(CONFIGS[cfg_name][2])
    out["meta.vocab"] = np.asarray(V)
    out["meta.seed"] = np.asarray(seed)
    path = os.path.join(out_dir, cfg_name + ".npz")
    np.savez_compressed(path, **out)
    spread = float((logits.detach().max(1).values - logits.min(1).values).mean())
    print(f"{cfg_name}: loss={loss.item():.5f} logit spread={spread:.3f} -> {path} "
          f"({os.path.getsize(path) / 1e6:.2f} MB)")


def metric_goldens(out_dir):
    """Known answers of the reference's ``cal_metric`` (utils/Manager.py:1276-1345)."""
    sys.path.insert(0, REF)
    from utils.Manager import cal_metric
    cases = [
        ([[1, 0, 0, 1], [0, 1, 0]], [[.9, .2, .5, .4], [.1, .3, .2]]),
        ([[0, 0, 1, 0, 0, 1, 0], [1, 0], [0, 0, 0, 1, 0]],
         [[.1, .7, .3, .2, .9, .8, .05], [.4, .6], [.5, .1, .9, .3, .2]]),
    ]
    rows = []
    # hit@k is left out: the reference's hit_score compares a list to 1 and fails under
    # numpy 2 (Manager.py:1250), so it has no answer to pin.
    metrics = ["auc", "mean_mrr", "ndcg@5;10", "acc", "f1", "logloss"]
    for labels, preds in cases:
        res = {}
        for mname in metrics:
            flat = mname in ("acc", "f1", "logloss")
            lab = [x for l in labels for x in l] if flat else labels
            prd = [x for p in preds for x in p] if flat else preds
            res.update(cal_metric(lab, prd, [mname]))
        rows.append({"labels": labels, "preds": preds,
                     "res": {k: float(v) for k, v in res.items()}})
    import json
    with open(os.path.join(out_dir, "cal_metric.json"), "w") as f:
        json.dump(rows, f, indent=1)
    print("cal_metric:", [r["res"] for r in rows])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--configs", default=",".join(CONFIGS))
    a = ap.parse_args()
    for i, c in enumerate(a.configs.split(",")):
        run(c, 1000 + i, a.out)
    metric_goldens(a.out)
