"""Graph-replayed train step (bench.py's launch mode): two replays of a captured NRMS step must
reproduce two eager steps from the same state — same dropout draws (device RNG pair), same
Adam bias corrections (device step counts), same parameters within fp32 atomic-order noise."""
import copy
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _small_model(dev):
    from newsrec_amd.manager import build_model
    torch.manual_seed(7)
    return build_model("mha", "mha", 384, vocab=2000, device=dev, user_num=50, dropout_p=0.2)


def _batch(gen, dev, b=4, c=5, nh=10, l=30, vocab=2000):
    def titles(n):
        tok = torch.randint(1000, vocab, (n, l), generator=gen)
        lens = torch.randint(5, l + 1, (n,), generator=gen)
        mask = (torch.arange(l)[None] < lens[:, None]).long()
        tok = tok * mask
        tok[:, 0] = 101
        return tok, mask
    ct, cm = titles(b * c)
    ht, hm = titles(b * nh)
    x = {"cdd_encoded_index": ct.view(b, c, l), "cdd_attn_mask": cm.view(b, c, l),
         "his_encoded_index": ht.view(b, nh, l), "his_attn_mask": hm.view(b, nh, l),
         "his_mask": torch.ones(b, nh, 1, dtype=torch.float64), "user_id": torch.randint(1, 50, (b,), generator=gen),
         "label": torch.zeros(b, dtype=torch.long)}
    return {k: v.to(dev) for k, v in x.items()}


def test_graph_replay_matches_eager():
    import bench
    from newsrec_amd.manager import get_optim
    dev = torch.device("cuda", 0)
    gen = torch.Generator().manual_seed(3)
    batches = [_batch(gen, dev) for _ in range(4)]
    m_eager = _small_model(dev)
    m_graph = copy.deepcopy(m_eager)
    o_eager = get_optim(m_eager, capturable=False)
    o_graph = get_optim(m_graph, capturable=True)
    # GraphedStep runs max(2, warmup) eager warm-up steps on batches 0, 1 before capturing
    for i in range(2):
        bench.train_step(m_eager, o_eager, batches[i], None)
    g = bench.GraphedStep(m_graph, o_graph, bench.ResidentFeed(batches), None, 2)
    for i in range(2, 4):
        bench.train_step(m_eager, o_eager, batches[i], None)
        g(i)
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(m_eager.named_parameters(), m_graph.named_parameters()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=2e-5, msg=n)
    # the replays really trained: parameters moved away from the post-warm-up state
    assert m_graph.encoderN.query_words.abs().sum() > 0


def test_graph_replay_follows_lr_schedule():
    """A captured step replays with the CURRENT group["lr"] (device learning rates, synced before each
    replay), as the reference's linear-warmup scheduler changes it (Manager.py:415-420)."""
    import bench
    from newsrec_amd.manager import get_optim
    dev = torch.device("cuda", 0)
    gen = torch.Generator().manual_seed(5)
    batches = [_batch(gen, dev) for _ in range(5)]
    m_eager = _small_model(dev)
    m_graph = copy.deepcopy(m_eager)
    o_eager = get_optim(m_eager, capturable=False)
    o_graph = get_optim(m_graph, capturable=True)
    for i in range(2):
        bench.train_step(m_eager, o_eager, batches[i], None)
    g = bench.GraphedStep(m_graph, o_graph, bench.ResidentFeed(batches), None, 2)
    for i, scale in zip(range(2, 5), (0.25, 3.0, 0.5)):
        for o in (o_eager, o_graph):
            for grp, base in zip(o.param_groups, (1e-4, 6e-6)):
                grp["lr"] = base * scale
        bench.train_step(m_eager, o_eager, batches[i], None)
        g(i)
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(m_eager.named_parameters(), m_graph.named_parameters()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=2e-5, msg=n)
