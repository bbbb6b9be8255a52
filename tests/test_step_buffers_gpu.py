"""The step's gradient buffers: the candidates | history split joins its two gradients in place
(SplitRowsFn: the scorer and the user encoder write straight into the joined buffer, no cat), and
the small zero-initialised parameter gradients of a step come from one fill (functions.ZERO_ARENA)
-- against the reference goldens, and under a retained graph's second backward (dense accumulation)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from golden_util import Golden
from model_util import build_model, load_golden_params


def _setup(cfg):
    g = Golden(cfg)
    model = build_model(g.encN, g.encU, g.hidden, vocab=int(g["meta.vocab"]))
    load_golden_params(model, g)
    if g.encU == "lstur":
        model.encoderU.keep_override = torch.from_numpy(g["in.lstur_keep"])
    return g, model, g.inputs("cuda")


def _check(g, model, mult=1.0):
    grads = dict(model.named_parameters())
    for n in g.names:
        want = mult * g["grad." + n]
        p = grads.get(n)
        got = p.grad.cpu().numpy() if (p is not None and p.grad is not None) else np.zeros_like(want)
        scale = max(float(np.abs(want).max()), 1e-6)
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-3 * scale, err_msg=n)


@pytest.mark.parametrize("cfg", ["nrms", "cnn_attn", "cnn_lstur"])
@pytest.mark.parametrize("head", ["forward", "forward_loss"])
def test_split_join_in_place(cfg, head):
    from newsrec_amd.functions import SplitRowsFn
    g, model, x = _setup(cfg)
    model.train()
    SplitRowsFn.stats.update(in_place=0, copied=0)
    if head == "forward":
        logits, _ = model(x)
        loss = torch.nn.functional.nll_loss(logits, x["label"])
    else:
        _, loss = model.forward_loss(x)
    loss.backward()
    assert abs(loss.item() - float(g["out.loss"])) < 1e-4
    assert SplitRowsFn.stats == {"in_place": 1, "copied": 0}, SplitRowsFn.stats
    _check(g, model)


@pytest.mark.parametrize("cfg", ["nrms", "cnn_attn"])
def test_retained_graph_second_backward(cfg):
    """Two backward passes over one retained graph accumulate (torch's dense semantics): every
    gradient is twice the golden one -- the second pass must not reuse the first one's zero arena
    views or write into the gradient buffers the first pass returned."""
    g, model, x = _setup(cfg)
    model.train()
    logits, _ = model(x)
    loss = torch.nn.functional.nll_loss(logits, x["label"])
    loss.backward(retain_graph=True)
    loss.backward()
    _check(g, model, mult=2.0)


def test_nrms_training_forward_saves_for_the_split_backward(monkeypatch):
    """A training forward (autograd recording) saves the attention output O and the arena reservations,
    so the backward runs the split MHA backward (nr_mha_pool_bwd with o and dob) and one zero fill; under
    torch.no_grad() nothing backward-only is saved.  (torch runs Function.forward with grad mode off:
    the gate must look at the CALLER's mode, functions._GradAwareFn.)"""
    from newsrec_amd import functions as F, kernels as Kn
    calls = []
    fwd, bwd = Kn.mha_pool_fwd, Kn.mha_pool_bwd

    def rec_fwd(*a, **kw):
        calls.append(("fwd", kw.get("oout") is not None))
        return fwd(*a, **kw)

    def rec_bwd(*a, **kw):
        calls.append(("bwd", kw.get("o") is not None and kw.get("dob") is not None))
        return bwd(*a, **kw)
    monkeypatch.setattr(Kn, "mha_pool_fwd", rec_fwd)
    monkeypatch.setattr(Kn, "mha_pool_bwd", rec_bwd)
    g, model, x = _setup("nrms")
    model.train()
    _, loss = model.forward_loss(x)
    loss.backward()
    assert calls and all(ok for _, ok in calls) and ("bwd", True) in calls, calls
    calls.clear()
    with torch.no_grad():
        model.forward_loss(x)
    assert calls and not any(ok for _, ok in calls), calls
    _check(g, model)


def test_probe_replays_with_a_hook_owned_table_gradient():
    """functions.PROBE (bench.py's per-launch GEMM timing) keeps each projection GEMM as a closure over
    the operands it launched with: when TABLE_GRAD_HOOK takes the word-table gradient (a data-parallel
    all-reduce owns it), the dgrad closure still holds that buffer -- the replays run, and the buffer
    is restored bitwise afterwards (the closure had looked the name up late and replayed
    into None)."""
    from newsrec_amd import functions as F
    g, model, x = _setup("nrms")
    model.train()
    taken = {}

    def hook(table, dtable):
        taken["g"] = dtable
        return True

    F.TABLE_GRAD_HOOK.set(hook)
    F.PROBE.enable()
    try:
        _, loss = model.forward_loss(x)
        loss.backward()
        torch.cuda.synchronize()
        assert "g" in taken
        before = taken["g"].clone()
        res = F.PROBE.time(reps=2, warm=1)
        torch.cuda.synchronize()
    finally:
        F.PROBE.disable()
        F.TABLE_GRAD_HOOK.set(None)
    assert {"proj_fwd_ms", "proj_dgrad_ms", "proj_wgrad_ms"} <= set(res), res
    assert all(res[k] > 0 for k in ("proj_fwd_ms", "proj_dgrad_ms", "proj_wgrad_ms"))
    assert torch.equal(taken["g"], before)

