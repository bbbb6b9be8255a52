"""Oracle parity of the CNN-family legs at the size bench.py times them (BASELINE configs[1] and
[3], plus the GRU user encoder): one train step at B = 32 impressions, V = 30522 trainable word
table, H = 150, 5 candidates, 50-click history, 30-token titles — with the bench's kernels and
routing (the distinct-row CNN encoder: tap projection over the batch's distinct word rows on the
128 x 128 bf16x6 GEMM kernels, the three-row gather-add, the per-distinct-row shifted sums and the
table-gradient / conv weight-gradient GEMMs over those rows; the additive-attention word pooling;
the user encoders; Adam) — against the fp32 CPU oracle (oracle/restatement.py, pinned to the
reference's goldens by tests/test_oracle_golden.py):

* configs[1]: CNN news encoder + additive-attention user encoder
  (models/Encoders/CNN.py:30-50, models/Encoders/Pooling.py:12-25);
* configs[3]: CNN + LSTUR with the MIND-large user table (876,957 rows) and an injected
  Bernoulli id-drop draw (models/Encoders/RNN.py:76-104);
* CNN + GRU over the packed history (models/Encoders/RNN.py:50-73).

Bars as for NRMS (tests/test_fullsize_gpu.py): logits within the north star's 1e-3, every
gradient within 1e-3 of its max magnitude, every parameter after one Adam step within 2 lr (all
but a rounding-level handful within 1e-3 lr).  The LSTUR step is also replayed as a HIP graph
(bench.GraphedStep) against eager steps."""
import copy
import os
import sys

import pytest
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

from oracle import restatement as R

B, C, NH, L, V, H, USERS = 32, 5, 50, 30, 30522, 150, 876956
LEGS = {"cnn_attn": "attn", "cnn_lstur": "lstur", "cnn_gru": "gru"}


def _model(encU, dev):
    """Reference init, then every parameter redrawn at the golden generator's scales
    (tests/golden/params.py: candidate scores spread by O(1); reference init spreads them ~1e-4)."""
    from newsrec_amd.manager import build_model
    from params import param_std
    torch.manual_seed(42)
    m = build_model("cnn", encU, H, vocab=V, device=dev, user_num=USERS)
    with torch.no_grad():
        for n, p in m.named_parameters():
            # x4 on the conv: 1,760 titles of random words give news vectors with a large common
            # part, and the user vector (a pooled mean of 50 of them) mostly scores that part
            p.normal_(0, float(param_std(n, tuple(p.shape))) * (4.0 if n == "encoderN.cnn.weight" else 1.0))
        if hasattr(m.encoderU, "userEmbedding"):
            m.encoderU.userEmbedding.weight[0].zero_()   # RNN.py:82
    return m


def _batch(seed):
    """bench.synth_batch with ragged titles and ragged / empty histories (his_mask[0] = 1 for an
    empty history, MIND.py:330-337); a repeated user id so the LSTUR table gradient adds rows."""
    import bench
    gen = torch.Generator().manual_seed(seed)
    x = bench.synth_batch(gen, "cpu", full=False)
    lens = torch.randint(0, NH + 1, (B,), generator=gen)
    lens[:4] = 0
    his = (torch.arange(NH)[None] < lens[:, None]).double()
    his[:, 0] = 1.0
    x["his_mask"] = his.unsqueeze(-1)
    x["user_id"][1] = x["user_id"][5]
    return x


def _keep(seed):
    return torch.zeros(B, dtype=torch.long).bernoulli_(0.5, generator=torch.Generator().manual_seed(seed))


@pytest.mark.parametrize("leg", list(LEGS))
def test_cnn_leg_fullsize_step_vs_oracle(leg):
    from newsrec_amd.manager import get_optim
    dev = torch.device("cuda", 0)
    encU = LEGS[leg]
    model = _model(encU, dev)
    model.train()
    x = _batch(3)
    keep = _keep(4) if encU == "lstur" else None
    if keep is not None:
        model.encoderU.keep_override = keep
    xg = {k: v.to(dev) for k, v in x.items()}
    P = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in model.named_parameters()}
    opt = get_optim(model)
    opt.zero_grad(set_to_none=True)
    logits, _ = model(xg)
    loss = F.nll_loss(logits, xg["label"])
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    want_loss, want_logits, _ = R.train_step(P, x, "cnn", encU, lstur_keep=keep)
    err = (logits.detach().cpu() - want_logits).abs().max().item()
    print("%s full size: logit std %.3f, max |logit err| %.3e, loss %.6f vs %.6f"
          % (leg, want_logits.std().item(), err, loss.item(), want_loss.item()))
    assert want_logits.std().item() > 0.05   # the comparison is not between constants
    assert err <= 1e-3
    assert abs(loss.item() - want_loss.item()) <= 1e-4
    ps = dict(model.named_parameters())
    for n in P:
        want, got = P[n].grad, ps[n].grad
        assert want is not None and got is not None, n
        scale = max(want.abs().max().item(), 1e-8)
        gerr = (got.detach().cpu() - want).abs().max().item()
        assert gerr <= 1e-3 * scale, (n, gerr, scale)
    worst = 0.0
    for n, p in model.named_parameters():
        d = (p.detach().cpu() - P[n].detach()).abs()
        lr = 6e-6 if "bert" in n else 1e-4
        assert d.max().item() <= 2 * lr + 1e-7, n
        moved = P[n].grad != 0
        off = int((d[moved] > 1e-3 * lr).sum().item())
        worst = max(worst, off / max(1, int(moved.sum().item())))
        assert off <= max(2, 1e-3 * int(moved.sum().item())), (n, off)
    print("%s full size: worst fraction of updated elements off by > 1e-3 lr: %.2e" % (leg, worst))


def test_lstur_fullsize_graph_replay_matches_eager():
    """bench.GraphedStep on the LSTUR leg (876,957-row user table): 2 eager warm-up steps + 2
    replays vs 4 eager steps, one fixed id-drop draw."""
    import bench
    from newsrec_amd.manager import get_optim
    dev = torch.device("cuda", 0)
    m_eager = _model("lstur", dev)
    m_graph = copy.deepcopy(m_eager)
    keep = _keep(9).to(dev)   # device-resident: read inside the captured graph
    m_eager.encoderU.keep_override = keep
    m_graph.encoderU.keep_override = keep
    batches = [{k: v.to(dev) for k, v in _batch(20 + i).items()} for i in range(4)]
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
