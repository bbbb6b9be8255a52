"""End-to-end parity of the HIP two-tower path with goldens produced by the reference's
own modules (tests/golden/make_golden.py): forward logits (train log-softmax and eval
sigmoid), news / user representations, loss, every parameter gradient, and Adam."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from golden_util import Golden, CONFIG_ENCODERS
from model_util import build_model, load_golden_params

CONFIGS = list(CONFIG_ENCODERS)
# north_star: forward logits within 1e-3 of the reference (fp32).  We hold 1e-4.
LOGIT_ATOL = 1e-4


def _setup(cfg):
    g = Golden(cfg)
    model = build_model(g.encN, g.encU, g.hidden, vocab=int(g["meta.vocab"]))
    load_golden_params(model, g)
    if g.encU == "lstur":
        model.encoderU.keep_override = torch.from_numpy(g["in.lstur_keep"])
    return g, model, g.inputs("cuda")


@pytest.fixture(params=["bf16x6", "f32"])
def gemm_prec(request):
    """Both GEMM arithmetics (nr_gemm_set_precision) are held to the same parity bars."""
    from newsrec_amd import _lib as Lb, kernels as Kn
    old = Kn.set_gemm_precision(Lb.GEMM_BF16X6 if request.param == "bf16x6" else Lb.GEMM_F32)
    yield request.param
    Kn.set_gemm_precision(old)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_forward_parity(cfg, gemm_prec):
    g, model, x = _setup(cfg)
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


@pytest.mark.parametrize("cfg", CONFIGS)
def test_grad_parity(cfg, gemm_prec):
    g, model, x = _setup(cfg)
    model.train()
    logits, _ = model(x)
    loss = torch.nn.functional.nll_loss(logits, x["label"])
    loss.backward()
    assert abs(loss.item() - float(g["out.loss"])) < 1e-4
    grads = dict(model.named_parameters())
    for n in g.names:
        want = g["grad." + n]
        p = grads.get(n)
        got = p.grad.cpu().numpy() if (p is not None and p.grad is not None) else np.zeros_like(want)
        scale = max(float(np.abs(want).max()), 1e-6)
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-3 * scale, err_msg=n)


def test_fused_adam_parity():
    from newsrec_amd.optim import FusedAdam
    g, model, x = _setup("cnn_attn")
    base = [p for n, p in model.named_parameters() if "bert" not in n]
    bert = [p for n, p in model.named_parameters() if "bert" in n]
    opt = FusedAdam([{"params": base, "lr": 1e-4}, {"params": bert, "lr": 6e-6}])
    model.train()
    logits, _ = model(x)
    torch.nn.functional.nll_loss(logits, x["label"]).backward()
    opt.step()
    opt.step()
    named = dict(model.named_parameters())
    for n in g.names:
        got, want = named[n].detach().cpu().numpy(), g["adam2." + n]
        # Adam normalises each gradient by its own RMS, so an element whose gradient is ~0
        # can move by up to lr per step on fp32 noise; bound those by 2 steps x lr and hold
        # everything else to 2e-6.
        d = np.abs(got - want)
        assert d.max() <= 2 * 1e-4 + 1e-7, n
        assert (d > 2e-6).mean() < 1e-4, n


def test_fused_adam_kernel_matches_torch_adam():
    """nr_adam against torch.optim.Adam on identical gradients (no model noise)."""
    from newsrec_amd.optim import FusedAdam
    g = torch.Generator().manual_seed(0)
    shapes = [(1000, 77), (3,), (4097,)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    gs = [[torch.randn(s, generator=g) * 10 ** -k for s in shapes] for k in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [p.clone().cuda().requires_grad_(True) for p in ps]
    o1 = torch.optim.Adam(ref, lr=1e-3, weight_decay=0.01)
    o2 = FusedAdam(mine, lr=1e-3, weight_decay=0.01)
    for step in range(3):
        for p, q, gg in zip(ref, mine, gs[step]):
            p.grad = gg.clone()
            q.grad = gg.clone().cuda()
        o1.step()
        o2.step()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach().cpu(), p.detach(), rtol=0, atol=1e-6)


@pytest.mark.parametrize("capturable", [False, True])
def test_adam_multi_many_tensors(capturable):
    """nr_adam_multi over 90 tensors (three launches of <= 40), ragged sizes, two param groups,
    host and device step counts, against torch.optim.Adam."""
    from newsrec_amd.optim import FusedAdam
    g = torch.Generator().manual_seed(1)
    shapes = [(int(n),) for n in torch.randint(1, 9000, (88,), generator=g)] + [(4096,), (30522 * 3,)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [p.clone().cuda().requires_grad_(True) for p in ps]
    o1 = torch.optim.Adam([{"params": ref[:50], "lr": 1e-3}, {"params": ref[50:], "lr": 6e-6}])
    o2 = FusedAdam([{"params": mine[:50], "lr": 1e-3}, {"params": mine[50:], "lr": 6e-6}], capturable=capturable)
    for step in range(3):
        for p, q in zip(ref, mine):
            gg = torch.randn(p.shape, generator=g)
            p.grad = gg.clone()
            q.grad = gg.cuda()
        o1.step()
        o2.step()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach().cpu(), p.detach(), rtol=0, atol=1e-6)


def test_unfused_composition_matches_fused():
    """encoderN(embedding(tokens), mask) (the reference composition) == the fused path."""
    g, model, x = _setup("nrms")
    model.eval()
    with torch.no_grad():
        fused = model.encode_news(x)
        emb = model.embedding(x["cdd_encoded_index"])
        _, unfused = model.encoderN(emb, x["cdd_attn_mask"])
    torch.testing.assert_close(unfused, fused, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cfg", ["cnn_attn", "nrms", "cnn_lstur"])
def test_forward_loss_fused_head(cfg):
    """TwoTowerBaseModel.forward_loss (scorer + log-softmax + NLLLoss in one kernel, one kernel back)
    against forward(x) followed by torch's nll_loss (Manager.py:641): logits, loss and every
    gradient; also the reference golden loss."""
    g, model, x = _setup(cfg)
    model.train()
    logits_f, loss_f = model.forward_loss(x)
    loss_f.backward()
    grads_f = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    logits, _ = model(x)
    loss = torch.nn.functional.nll_loss(logits, x["label"])
    loss.backward()
    torch.testing.assert_close(logits_f, logits, rtol=0, atol=1e-6)
    assert abs(loss_f.item() - loss.item()) <= 1e-6
    assert abs(loss_f.item() - float(g["out.loss"])) < 1e-4
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        scale = max(p.grad.abs().max().item(), 1e-6)
        torch.testing.assert_close(grads_f[n], p.grad, rtol=0, atol=1e-5 * scale, msg=n)
    # both gradients at once: d(loss + sum(logits * w)) through the fused head
    model.zero_grad(set_to_none=True)
    w = torch.randn_like(logits_f)
    lf, lo = model.forward_loss(x)
    (lo + (lf * w).sum()).backward()
    gf = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    lr_, _ = model(x)
    (torch.nn.functional.nll_loss(lr_, x["label"]) + (lr_ * w).sum()).backward()
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        scale = max(p.grad.abs().max().item(), 1e-6)
        torch.testing.assert_close(gf[n], p.grad, rtol=0, atol=1e-5 * scale, msg=n)


@pytest.mark.parametrize("B,C,H", [(1, 5, 150), (32, 5, 150), (300, 5, 150), (64, 20, 400), (7, 1, 3)])
def test_score_nll_kernel_vs_torch(B, C, H):
    """nr_score_nll_fwd / _bwd against torch (scores, log_softmax, nll_loss mean): one workgroup per
    impression, the last arrival sums the loss terms; run three times on the one self-cleaning
    ticket (a stale ticket would leave the loss unwritten)."""
    from newsrec_amd import kernels as K
    g = torch.Generator().manual_seed(B * 31 + C)
    cdd = torch.randn(B * C, H, generator=g).cuda()
    user = torch.randn(B, H, generator=g).cuda()
    label = torch.randint(0, C, (B,), generator=g).cuda()
    cr, ur = cdd.clone().requires_grad_(), user.clone().requires_grad_()
    lg = torch.log_softmax((cr.view(B, C, H) * ur[:, None]).sum(-1) / H ** 0.5, -1)
    lref = torch.nn.functional.nll_loss(lg, label)
    lref.backward()
    for _ in range(3):
        logits = torch.full((B, C), float("nan"), device="cuda")
        loss = torch.full((1,), float("nan"), device="cuda")
        K.score_nll_fwd(cdd, user, label, B, C, H, logits, loss)
        dcdd, duser = torch.empty_like(cdd), torch.empty_like(user)
        K.score_nll_bwd(cdd, user, logits, label, torch.ones(1, device="cuda"), None, B, C, H, dcdd, duser)
        torch.cuda.synchronize()
        torch.testing.assert_close(logits, lg.detach(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(loss[0], lref.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dcdd, cr.grad, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(duser, ur.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("rows,cols,ld", [(1600, 1152, 1152), (52800, 150, 152), (7, 3, 4), (20832, 3072, 3072),
                                          (4000, 700, 768)])
def test_colsum_one_launch(rows, cols, ld):
    """K.colsum (nr_colsum_ws: the last workgroup per 64-column chunk sums the partial rows) against
    fp64 and against the two-launch nr_colsum; out is accumulated into (+=); three calls in a row on
    the one self-cleaning counter array."""
    from newsrec_amd import _lib as L
    from newsrec_amd import kernels as K
    g = torch.Generator().manual_seed(rows + cols)
    x = torch.randn(rows, ld, generator=g)[:, :cols].cuda()
    base = torch.randn(cols, generator=g)
    want = base.double() + x.cpu().double().sum(0)
    for _ in range(3):
        out = base.cuda()
        K.colsum(x, rows, cols, out)
        torch.cuda.synchronize()
        assert (out.cpu().double() - want).abs().max().item() <= 1e-5 * rows ** 0.5 + 1e-5
    two = base.cuda()
    work = torch.empty(max(1, L.load().nr_colsum_workspace(rows, cols) // 4), device="cuda")
    L.call("nr_colsum", L.ptr(x), x.stride(0), rows, cols, L.ptr(two), L.ptr(work), L.stream_ptr(x))
    # both orders of the fp32 sums within the same bound of fp64
    assert (two.cpu().double() - want).abs().max().item() <= 1e-5 * rows ** 0.5 + 1e-5
