"""End-to-end parity at the BENCHMARKED configuration (BASELINE configs[2], bench.py's headline):
one NRMS train step at B = 32 impressions, V = 30522, H = 384, 12 heads, 5 candidates, 50-click
history, 30-token titles — the bench's exact kernels (the 256x256 persistent bf16x6 GEMMs over the
distinct-row projection, the fused attention kernels, the split backward, Adam) — against the fp32 CPU oracle
(oracle/restatement.py, which tests/test_oracle_golden.py pins to the reference's goldens):

* logits within the north star's 1e-3 (models/TwoTowerBaseModel.py:65-75), the loss — through the
  head bench.py times (``TwoTowerBaseModel.forward_loss``: scorer + log-softmax + NLLLoss fused,
  nr_score_nll_*), on a host-fed ragged batch AND on a batch formed on the device by
  bench.DeviceFeed (nr_form_train_batch, the timed step's own input path);
* the word-table, projection and every other gradient within 1e-3 of each one's max magnitude;
* every parameter after one Adam step (Manager.py:404-413,647);
* the same step replayed as a HIP graph (bench.GraphedStep) against eager steps;
* XFormer at BERT-base width with enough rows (B = 16, 2 layers: 10,416 token rows, QKV = 1,476
  tiles of 128x128) that its GEMMs run the bf16x6 kernel, against the oracle.
The NRMS step runs at dropout 0 and at the bench's 0.2: the oracle restates the device RNG's keep
masks (R.dropout_keep) and applies them where nn.Dropout would."""
import copy
import math
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

from oracle import restatement as R

B, C, NH, L, V, H = 32, 5, 50, 30, 30522, 384


def _nrms(dev, p_drop=0.0):
    from newsrec_amd.manager import build_model
    torch.manual_seed(42)
    m = build_model("mha", "mha", H, vocab=V, device=dev, user_num=876956, dropout_p=p_drop)
    with torch.no_grad():   # spread the candidate scores (reference init gives near-equal logits)
        m.embedding.bert_word_embedding.weight.normal_(0, 0.5)
        m.encoderN.query_words.normal_(0, 1.0)
        m.encoderU.query_news.normal_(0, 1.0)
    return m


def _batch(seed):
    """bench.synth_batch with ragged titles (lengths U[5, 30]) and ragged / empty histories (the
    reference forces his_mask[0] = 1 for an empty history, MIND.py:330-337)."""
    import bench
    gen = torch.Generator().manual_seed(seed)
    x = bench.synth_batch(gen, "cpu", full=False)
    lens = torch.randint(0, NH + 1, (B,), generator=gen)
    lens[:4] = 0
    his = (torch.arange(NH)[None] < lens[:, None]).double()
    his[:, 0] = 1.0
    x["his_mask"] = his.unsqueeze(-1)
    return x


def _device_batch(dev):
    """One batch formed on the device exactly as the timed steps form theirs (bench.DeviceFeed:
    nr_form_train_batch over a resident MIND-shaped train split, negatives from the device RNG);
    -> (device batch, host copy for the oracle)."""
    import bench
    feed = bench.DeviceFeed(dev, 1, 0, n_impr=4096)
    x = {k: v.clone() for k, v in feed.form().items()}
    feed.store.check_status()
    return x, {k: v.cpu() for k, v in x.items()}


def _oracle_params(model):
    return {n: p.detach().cpu().clone().requires_grad_(True) for n, p in model.named_parameters()}


def _close_grads(model, P, names=None, rel=1e-3):
    ps = dict(model.named_parameters())
    for n in (names or list(P)):
        want = P[n].grad
        assert want is not None, n
        got = ps[n].grad
        assert got is not None, n
        scale = max(want.abs().max().item(), 1e-8)
        err = (got.detach().cpu() - want).abs().max().item()
        assert err <= rel * scale, (n, err, scale)


def _news_dropout_kw(model, p, B_, C_, N_, L_):
    """The keep masks of the step's news-encoder dropout (MHA.py:37) restated by the oracle
    (R.dropout_keep) from the encoder's device RNG pair as the forward is about to take it: one joint
    token batch, the candidates' B*C*L rows first, then the history's."""
    if p <= 0:
        return None, None
    rng = model.encoderN._rng
    seed, off = rng.seed, rng.offset
    T = B_ * (C_ + N_) * L_
    keep = R.dropout_keep(seed, off, T, H, p)
    nc = B_ * C_ * L_
    return {"dropout_keep": keep[:nc], "p_drop": p}, {"dropout_keep": keep[nc:], "p_drop": p}


@pytest.mark.parametrize("p_drop", [0.0, 0.2])
@pytest.mark.parametrize("feed", ["host", "device"])
def test_nrms_fullsize_step_vs_oracle(feed, p_drop):
    """bench.forward_backward's path: forward_loss (fused scorer + log-softmax + NLL) and backward;
    p_drop = 0.2 is the bench's own step (MHA.py:19,37's Dropout(0.2) on the device RNG), the oracle
    applying the same keep masks (R.dropout_keep)."""
    import bench
    from newsrec_amd.manager import get_optim
    dev = torch.device("cuda", 0)
    model = _nrms(dev, p_drop)
    model.train()
    if feed == "host":
        x = _batch(1)
        xg = {k: v.to(dev) for k, v in x.items()}
    else:
        xg, x = _device_batch(dev)
    P = _oracle_params(model)
    opt = get_optim(model)
    cdd_kw, his_kw = _news_dropout_kw(model, p_drop, B, C, NH, L)
    # bench.forward_backward, keeping the logits
    opt.zero_grad(set_to_none=True)
    logits, loss = model.forward_loss(xg)
    loss.backward(bench._one(loss))
    opt.step()
    torch.cuda.synchronize()
    want_loss, want_logits, _ = R.train_step(P, x, "mha", "mha", cdd_kw=cdd_kw, his_kw=his_kw)
    assert want_logits.std().item() > 0.05   # the comparison is not between constants
    err = (logits.detach().cpu() - want_logits).abs().max().item()
    print("NRMS full size: max |logit err| %.3e, loss %.6f vs %.6f" % (err, loss.item(), want_loss.item()))
    assert err <= 1e-3
    assert abs(loss.item() - want_loss.item()) <= 1e-4
    _close_grads(model, P)
    # parameters after Adam: torch.optim.Adam on the oracle's gradients vs nr_adam_multi on ours.
    # Adam's first step moves every element by lr * g / |g|, so an element whose gradient is at the
    # rounding level may flip sign (a 2 lr difference): every element within 2 lr, all but
    # max(2, 1e-3 of) the elements that received a gradient within 1e-3 lr.
    worst = 0.0
    for n, p in model.named_parameters():
        d = (p.detach().cpu() - P[n].detach()).abs()
        lr = 6e-6 if "bert" in n else 1e-4
        assert d.max().item() <= 2 * lr + 1e-7, n
        moved = P[n].grad != 0
        off = int((d[moved] > 1e-3 * lr).sum().item())
        worst = max(worst, off / max(1, int(moved.sum().item())))
        assert off <= max(2, 1e-3 * int(moved.sum().item())), (n, off)
    print("NRMS full size: worst fraction of updated elements off by > 1e-3 lr: %.2e" % worst)


def test_nrms_fullsize_graph_replay_matches_eager():
    """bench.GraphedStep at the benchmark's size: 2 eager warm-up steps + 2 replays vs 4 eager steps."""
    import bench
    from newsrec_amd.manager import get_optim
    dev = torch.device("cuda", 0)
    m_eager = _nrms(dev)
    m_graph = copy.deepcopy(m_eager)
    batches = [{k: v.to(dev) for k, v in _batch(10 + i).items()} for i in range(4)]
    o_eager = get_optim(m_eager)
    o_graph = get_optim(m_graph, capturable=True)
    m_eager.train()
    m_graph.train()
    for i in range(2):
        bench.train_step(m_eager, o_eager, batches[i], None)
    g = bench.GraphedStep(m_graph, o_graph, bench.ResidentFeed(batches), None, 2)
    for i in range(2, 4):
        bench.train_step(m_eager, o_eager, batches[i], None)
        g(i)
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(m_eager.named_parameters(), m_graph.named_parameters()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=2e-5, msg=n)


def test_xformer_bf16x6_gemms_vs_oracle():
    """XFormer at BERT-base width, B = 16, 2 layers: 16*5*30 + 16*501 = 10,416 token rows, so the
    dense layers take the 128x128 bf16x6 kernel (>= 400 tiles), against the fp32 oracle."""
    from newsrec_amd import _lib as Lb, kernels as Kn
    from newsrec_amd.bert import BertConfig
    from newsrec_amd.manager import ManagerConfig
    from newsrec_amd.xformer import XFormer
    assert Kn.get_gemm_precision() == Lb.GEMM_BF16X6
    torch.manual_seed(7)
    Bx, Cx, N, Lt = 16, 5, 50, 30
    bc = BertConfig(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = ManagerConfig("bert", "xformer", 768, bert_dim=768)
    model = XFormer(m, bert_config=bc).cuda()
    with torch.no_grad():
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
    ct, cm = titles(Bx * Cx)
    ht, hm = titles(Bx * N)
    x = {"cdd_encoded_index": ct.view(Bx, Cx, Lt), "cdd_attn_mask": cm.view(Bx, Cx, Lt),
         "his_encoded_index": ht.view(Bx, N, Lt), "his_attn_mask": hm.view(Bx, N, Lt),
         "label": torch.zeros(Bx, dtype=torch.long)}
    xg = {k: v.cuda() for k, v in x.items()}
    model.train()
    logits, _ = model(xg)
    F.nll_loss(logits, xg["label"]).backward()
    P = {n: p.detach().cpu().clone().requires_grad_() for n, p in model.named_parameters()}
    want = R.xformer_forward(P, x, True, 12)
    err = (logits.detach().cpu() - want.detach()).abs().max().item()
    print("XFormer B=16 bf16x6: max |logit err| %.3e" % err)
    assert want.detach().std().item() > 0.05
    assert err <= 1e-3
    R.nll_loss(want, x["label"]).backward()
    _close_grads(model, P, ["bert.embeddings.word_embeddings.weight",
                            "bert.encoder.layer.0.attention.self.query.weight",
                            "bert.encoder.layer.0.attention.output.dense.weight",
                            "bert.encoder.layer.1.intermediate.dense.weight",
                            "bert.encoder.layer.1.output.dense.weight", "bert.pooler.dense.weight", "userBias"],
                 rel=5e-3)


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_xformer_12_layers_step_vs_oracle(p_drop):
    """configs[4] at full BERT-base depth: XFormer (12 layers, 768 wide, 12 heads, 3072 FFN, V = 30522)
    over B = 2 impressions -- 5 candidate titles each and the 501-token user sequence (CLS + 10
    word-pieces of each of 50 history titles, XFormer.py:80-89) -- one train step through the bench's
    path (forward_loss, backward, FusedAdam with the two parameter groups) against the fp32 oracle:
    logits within 1e-3, EVERY gradient within 1e-3 of its max magnitude, every parameter after Adam
    within 2 lr (all but a rounding-level handful within 1e-3 lr).  Gradients are checked against the
    oracle run in float64 (see below).  At p = 0.1 -- the dropout the bench times (bench.py xformer
    leg: BERT's own hidden / attention-probability dropout) -- the oracle replays the step's device
    masks at all 37 sites (R.BertDropout: embeddings, and per layer the attention probabilities and
    both dense outputs), from the forward's single counter snapshot.  The key biases' gradient is zero
    in exact arithmetic (softmax cancels q . b_k), so it is held to its attention block's gradient
    scale."""
    import bench
    from newsrec_amd import _lib as Lb, kernels as Kn
    from newsrec_amd.bert import BertConfig
    from newsrec_amd.manager import ManagerConfig, get_optim
    from newsrec_amd.xformer import XFormer
    assert Kn.get_gemm_precision() == Lb.GEMM_BF16X6
    torch.manual_seed(5)
    Bx, Cx, N, Lt = 2, 5, 50, 30
    bc = BertConfig(hidden_dropout_prob=p_drop, attention_probs_dropout_prob=p_drop)
    # built and initialised on the host (CPU generator: the draw -- and so the conditioning of every
    # gradient against the float64 oracle, fp32 error <= 2e-5 of max -- is the same on every box)
    model = XFormer(ManagerConfig("bert", "xformer", 768, bert_dim=768), bert_config=bc)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() == 2 and "embeddings" not in n:
                # 0.8 / sqrt(fan_in) (~0.029, BERT's own init is 0.02): at 1.5 / sqrt(fan_in) the deep
                # layers' attention saturates and their query / key gradients fall to 1e-8..1e-10 of
                # the value path's -- rounding noise in every arithmetic, fp32 included
                p.normal_(0, 0.8 / math.sqrt(p.shape[1]))
    model = model.cuda()
    gen = torch.Generator().manual_seed(1)

    def titles(n):
        t = torch.randint(1000, V, (n, Lt), generator=gen)
        lens = torch.randint(12, Lt + 1, (n,), generator=gen)
        msk = (torch.arange(Lt)[None] < lens[:, None]).long()
        t = t * msk
        t[:, 0] = 101
        return t, msk
    ct, cm = titles(Bx * Cx)
    ht, hm = titles(Bx * N)
    x = {"cdd_encoded_index": ct.view(Bx, Cx, Lt), "cdd_attn_mask": cm.view(Bx, Cx, Lt),
         "his_encoded_index": ht.view(Bx, N, Lt), "his_attn_mask": hm.view(Bx, N, Lt),
         "label": torch.tensor([0, 3])}
    xg = {k: v.cuda() for k, v in x.items()}
    P = _oracle_params(model)
    # float64 copies of the SAME starting point (ropt.step() below moves P in place)
    P64 = {n: p.detach().double().requires_grad_(True) for n, p in P.items()}
    model.train()
    opt = get_optim(model)
    opt.zero_grad(set_to_none=True)
    rng = model.bert._rng
    seed, off0 = rng.seed, rng.offset       # the forward's dropout counter range starts here
    logits, loss = model.forward_loss(xg)
    loss.backward(bench._one(loss))
    opt.step()
    torch.cuda.synchronize()
    T = Bx * Cx * Lt + Bx * 501
    drop = R.BertDropout(seed, off0, T, 768, 12, 12, p_drop, p_drop) if p_drop > 0 else None
    if drop is not None:
        assert rng.offset == off0 + T * 768 + 12 * T * (64 + 2 * 768)   # one range, all 37 sites
        kd = drop.attn(0, Bx * Cx * Lt, Bx, 501).float().mean().item()
        assert abs(kd - (1 - p_drop)) < 0.01
    base, bert = R.adam_groups(P)
    ropt = torch.optim.Adam([{"params": [P[k] for k in base], "lr": 1e-4},
                             {"params": [P[k] for k in bert], "lr": 6e-6}])
    want = R.xformer_forward(P, x, True, 12, drop=drop)
    want_loss = R.nll_loss(want, x["label"])
    want_loss.backward()
    ropt.step()
    err = (logits.detach().cpu() - want.detach()).abs().max().item()
    print("XFormer 12 layers B=2 p=%.1f: logit std %.3f, max |logit err| %.3e, loss %.6f vs %.6f"
          % (p_drop, want.detach().std().item(), err, loss.item(), want_loss.item()))
    assert want.detach().std().item() > 0.05
    assert err <= 1e-3
    assert abs(loss.item() - want_loss.item()) <= 1e-3
    # gradients against the oracle in float64 (the exact values to ~1e-15): every one within 1e-3 of its
    # max magnitude (the fp32 oracle's own error is <= 2e-5 of it at this init)
    R.nll_loss(R.xformer_forward(P64, x, True, 12, drop=drop), x["label"]).backward()
    ps = dict(model.named_parameters())
    worst, worst32 = 0.0, 0.0
    for n in P:
        want_g, got, g32 = P64[n].grad, ps[n].grad, P[n].grad
        assert got is not None and g32 is not None, n
        scale = max(want_g.abs().max().item(), 1e-12)
        if n.endswith("attention.self.key.bias"):
            # exact value 0 (softmax cancels q . b_k): rounding noise of the dK column sums, held to
            # 1e-3 of the attention block's gradient scale (its query / key / value weight gradients)
            blk = n.rsplit(".", 2)[0]
            scale = max(P64[blk + "." + w + ".weight"].grad.abs().max().item() for w in ("query", "key", "value"))
        gerr = (got.detach().cpu().double() - want_g).abs().max().item()
        e32 = (g32.double() - want_g).abs().max().item()
        worst, worst32 = max(worst, gerr / scale), max(worst32, e32 / scale)
        assert gerr <= 1e-3 * scale, (n, gerr, e32, scale)
    print("XFormer 12 layers p=%.1f: worst gradient error / max %.3e over %d tensors (fp32 oracle %.3e)"
          % (p_drop, worst, len(P), worst32))
    # parameters after Adam: within 2 lr of the oracle's step (Adam's first update is lr * g / (|g| + eps),
    # about lr * sign(g): an element whose exact gradient is within the rounding error of zero may step
    # either way, so elementwise agreement with the oracle's step is not the test), and the GPU step
    # equal to torch.optim.Adam's first step applied to the GPU's own gradients from the same start
    ps = dict(model.named_parameters())
    names = list(P)
    base_n = [n for n in names if n in base]
    bert_n = [n for n in names if n in bert]
    Q = {n: P64[n].detach().float().clone().requires_grad_(True) for n in names}
    for n in names:
        Q[n].grad = ps[n].grad.detach().cpu().clone()
    qopt = torch.optim.Adam([{"params": [Q[k] for k in base_n], "lr": 1e-4},
                             {"params": [Q[k] for k in bert_n], "lr": 6e-6}])
    qopt.step()
    for n, p in model.named_parameters():
        got = p.detach().cpu()
        lr = 6e-6 if "bert" in n else 1e-4
        assert (got - P[n].detach()).abs().max().item() <= 2 * lr + 1e-7, n
        dq = (got - Q[n].detach()).abs().max().item()
        assert dq <= 1e-3 * lr + 2 * torch.finfo(torch.float32).eps * got.abs().max().item(), (n, dq)
