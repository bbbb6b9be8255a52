"""functions.LOCAL_ROW_GRAD: the single-process row-sparse gradient of LSTUR's user table
(models/Encoders/RNN.py:88-104, nn.Embedding of the user ids) -- a persistent dense buffer that
re-zeroes only the previous step's rows.  Checked against a fresh dense gradient each step: new
rows, repeated rows in a batch, rows of the previous step cleared, and torch's accumulation
semantics when .grad is kept between backward passes."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import functions as F


def _dense(V, E, rows, grads):
    want = torch.zeros(V, E, device="cuda")
    want.index_add_(0, rows, grads)
    return want


def test_local_row_grad_steps():
    torch.manual_seed(0)
    V, E = 5000, 150
    table = torch.nn.Parameter(torch.randn(V, E, device="cuda"))
    h = F._LocalRowGrad()
    for step in range(4):
        rows = torch.randint(0, V, (32,), device="cuda")
        rows[3] = rows[7]                       # a user twice in one batch
        grads = torch.randn(32, E, device="cuda")
        table.grad = None                       # zero_grad(set_to_none=True)
        assert h(table, rows, grads)
        torch.testing.assert_close(table.grad, _dense(V, E, rows, grads), rtol=0, atol=1e-6)
    # kept .grad: the dense path accumulates (the handler declines) ...
    rows2 = torch.randint(0, V, (32,), device="cuda")
    g2 = torch.randn(32, E, device="cuda")
    before = table.grad.clone()
    assert not h(table, rows2, g2)
    table.grad.index_add_(0, rows2, g2)        # what autograd's accumulation does with the dense form
    torch.testing.assert_close(table.grad, before + _dense(V, E, rows2, g2), rtol=0, atol=1e-5)
    # ... and the next set_to_none step starts from an all-zero buffer again
    rows3 = torch.randint(0, V, (32,), device="cuda")
    g3 = torch.randn(32, E, device="cuda")
    table.grad = None
    assert h(table, rows3, g3)
    torch.testing.assert_close(table.grad, _dense(V, E, rows3, g3), rtol=0, atol=1e-6)


def test_adam_skips_untouched_rows_exactly():
    """nr_adam_multi with the handler's per-row flags: bitwise the same parameters and moments as the
    dense update (the flagged-zero rows' gradients are zeros; the kernel only skips reading them),
    including a row width that float4 groups straddle (150)."""
    from newsrec_amd import kernels as K
    torch.manual_seed(1)
    V, E = 3001, 150
    table = torch.nn.Parameter(torch.randn(V, E, device="cuda"))
    h = F._LocalRowGrad()
    rows = torch.randint(0, V, (32,), device="cuda")
    assert h(table, rows, torch.randn(32, E, device="cuda"))
    buf, flags, _ = table._nr_row_touched
    assert int(flags.sum()) == len(set(rows.tolist()))
    m0 = torch.randn(V, E, device="cuda").abs() * 0.01
    v0 = torch.randn(V, E, device="cuda").abs() * 0.001
    outs = []
    for use_flags in (True, False):
        p, m, v = table.detach().clone(), m0.clone(), v0.clone()
        ent = (p, buf, m, v, 1e-3, 3) + ((flags,) if use_flags else ())
        K.adam_multi([ent], 0.9, 0.999, 1e-8, 0.0, 1.0)
        torch.cuda.synchronize()
        outs.append((p, m, v))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rlen", [1, 2, 3, 5])
def test_adam_row_flags_short_rows(rlen):
    """Rows shorter than a float4: a float4 of the gradient spans up to four rows and is
    read when ANY of them is flagged -- bitwise the dense update, one touched row in four."""
    from newsrec_amd import kernels as K
    torch.manual_seed(2)
    rows = 4096
    flags = torch.zeros(rows, dtype=torch.uint8, device="cuda")
    flags[1::4] = 1
    g = torch.randn(rows, rlen, device="cuda") * flags[:, None].float()
    p0 = torch.randn(rows, rlen, device="cuda")
    m0 = torch.randn(rows, rlen, device="cuda").abs() * 0.01
    v0 = torch.randn(rows, rlen, device="cuda").abs() * 0.001
    outs = []
    for use_flags in (True, False):
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        K.adam_multi([(p, g, m, v, 1e-3, 2) + ((flags,) if use_flags else ())], 0.9, 0.999, 1e-8, 0.0, 1.0)
        torch.cuda.synchronize()
        outs.append((p, m, v))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_adam_step_advances_empty_tensors():
    """nr_adam_multi_step (capturable Adam): the device step count of an EMPTY parameter advances
    too, as torch's capturable Adam increments every parameter with a gradient; a launch
    of only empty tensors advances theirs."""
    from newsrec_amd import kernels as K
    p = torch.randn(1000, device="cuda")
    g = torch.randn(1000, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    e = torch.empty(0, device="cuda")
    s_full = torch.zeros((), dtype=torch.int64, device="cuda")
    s_empty = torch.zeros((), dtype=torch.int64, device="cuda")
    lr = torch.full((), 1e-3, device="cuda")
    for _ in range(3):
        K.adam_multi([(p, g, m, v, lr, s_full), (e, e, e.clone(), e.clone(), lr, s_empty)], 0.9, 0.999, 1e-8,
                     0.0, 1.0, advance_steps=True)
    s_only = torch.zeros((), dtype=torch.int64, device="cuda")
    K.adam_multi([(e, e, e.clone(), e.clone(), lr, s_only)], 0.9, 0.999, 1e-8, 0.0, 1.0, advance_steps=True)
    torch.cuda.synchronize()
    assert int(s_full) == 3 and int(s_empty) == 3 and int(s_only) == 1
    assert K.self_cleaning_check("cuda") == []


def test_score_nll_label_semantics():
    """The fused head's loss follows torch.nn.NLLLoss: label -100 is ignored (no term, not
    in the mean's count, no gradient), the mean divides by the counted labels; an out-of-range label
    gives a NaN loss and sets the sticky status (torch raises)."""
    from newsrec_amd import kernels as K
    from newsrec_amd.functions import ScoreNLLFn
    torch.manual_seed(3)
    B, C, H = 8, 5, 64
    cdd = torch.randn(B * C, H, device="cuda", requires_grad=True)
    user = torch.randn(B, H, device="cuda", requires_grad=True)
    label = torch.tensor([0, 1, -100, 4, 0, -100, 2, 3], device="cuda")
    logits, loss = ScoreNLLFn.apply(cdd, user, B, C, label)
    loss.backward()
    c2 = cdd.detach().clone().requires_grad_(True)
    u2 = user.detach().clone().requires_grad_(True)
    s = (c2.view(B, C, H) * u2[:, None]).sum(-1) / H ** 0.5
    want = torch.nn.functional.nll_loss(torch.log_softmax(s, -1), label)
    want.backward()
    torch.testing.assert_close(loss, want, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(cdd.grad, c2.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(user.grad, u2.grad, rtol=1e-4, atol=1e-6)
    assert not K.score_nll_status("cuda")
    _, bad = ScoreNLLFn.apply(cdd.detach(), user.detach(), B, C, torch.tensor([0, 1, 7, 0, 0, 0, 0, 0], device="cuda"))
    assert torch.isnan(bad).item()
    assert K.score_nll_status("cuda")            # seen, and cleared by the read
    assert not K.score_nll_status("cuda")
    assert K.self_cleaning_check("cuda") == []


def test_rows_add_ordered_duplicates_fixed_order():
    """nr_rows_add_ordered (the row-sparse sums of LSTUR's user table, on one process and in GradSync's
    data-parallel exchange): every id's rows summed in ascending position and added once -- equal to the
    float64 sum to fp32 rounding, BITWISE equal to a sequential fp32 sum in that order, and the same
    bits on every run (torch's index_add_ resolves duplicates with atomics).  Half the ids are row 0
    (LSTUR's dropped user ids, RNN.py:100-101), one id repeats across the 'ranks', the padding id is
    skipped, and a leading dimension wider than E is honoured."""
    from newsrec_amd import kernels as K
    torch.manual_seed(3)
    V, E, n = 4000, 150, 256            # 8 ranks x 32 rows
    idx = torch.randint(1, V, (n,), device="cuda")
    idx[::2] = 0
    idx[5] = idx[200] = idx[77] = 1234
    idx[9] = 17                         # the padding id below
    src = torch.randn(n, E + 6, device="cuda")[:, :E]
    base = torch.randn(V, E + 2, device="cuda")[:, :E]
    outs = []
    for _ in range(3):
        dt = base.clone()
        K.rows_add_ordered(src, idx, dt, padding_idx=17)
        outs.append(dt)
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    keep = idx != 17
    want = base.double().index_add(0, idx[keep], src[keep].double())
    torch.testing.assert_close(outs[0].double(), want, rtol=0, atol=1e-5)
    # bitwise: row 0 and row 1234 as fp32 sums in ascending position, added to the base row once
    for t in (0, 1234):
        pos = [j for j in range(n) if int(idx[j]) == t]
        s = src[pos[0]].clone()
        for j in pos[1:]:
            s = s + src[j]
        assert torch.equal(outs[0][t], base[t] + s), t
    assert torch.equal(outs[0][17], base[17])


@pytest.mark.parametrize("rows,cols", [(1152, 768), (1, 5), (130, 67)])
def test_transpose(rows, cols):
    """nr_transpose_f32 (the NRMS table dgrad's k-contiguous weight): exact, ragged tiles, a source
    leading dimension wider than its columns."""
    from newsrec_amd import kernels as K
    src = torch.randn(rows, cols + 3, device="cuda")[:, :cols]
    assert torch.equal(K.transpose(src), src.t().contiguous())


def _word_table_step(cfg, mode, prec=None):
    """The golden model's word-table gradient, FusedAdam stepped once on it; returns the table, its
    gradient, its published row flags (or None) and whether Adam matched the dense update bitwise.
    mode "one": one forward + backward; "passes": a second backward over a batch with other history
    ids accumulated into .grad; "uses": both batches' losses summed, one backward (the table used
    twice in one graph, autograd summing the two gradients)."""
    from golden_util import Golden
    from model_util import build_model, load_golden_params
    from newsrec_amd import kernels as K
    from newsrec_amd.optim import FusedAdam
    g = Golden(cfg)
    model = build_model(g.encN, g.encU, g.hidden, vocab=int(g["meta.vocab"]))
    load_golden_params(model, g)
    if g.encU == "lstur":
        model.encoderU.keep_override = torch.from_numpy(g["in.lstur_keep"])
    model.train()
    x = g.inputs("cuda")
    table = model.embedding.bert_word_embedding.weight
    his = x["his_encoded_index"]
    gen = torch.Generator().manual_seed(5)
    x2 = dict(x, his_encoded_index=torch.randint(1, table.shape[0], his.shape, generator=gen).cuda() * (his != 0))
    import contextlib
    from newsrec_amd import _lib as L
    with (K.gemm_precision(getattr(L, prec)) if prec else contextlib.nullcontext()):
        if mode == "one":
            model.forward_loss(x)[1].backward()
        elif mode == "passes":
            model.forward_loss(x)[1].backward()
            model.forward_loss(x2)[1].backward()
        else:
            (model.forward_loss(x)[1] + model.forward_loss(x2)[1]).backward()
    rt = table._nr_row_touched
    grad = table.grad.detach().clone()
    p0 = table.detach().clone()
    opt = FusedAdam([table], lr=1e-3)
    opt.step()
    st = opt.state[table]
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    K.adam_multi([(p, grad, m, v, 1e-3, 1)], 0.9, 0.999, 1e-8, 0.0, 1.0)
    torch.cuda.synchronize()
    same = (torch.equal(table.detach(), p) and torch.equal(st["exp_avg"], m) and torch.equal(st["exp_avg_sq"], v))
    return table, grad, rt, same


@pytest.mark.parametrize("cfg,prec", [("nrms", None), ("cnn_attn", None), ("cnn_attn", "GEMM_BF16")])
def test_word_table_row_flags(cfg, prec):
    """The word-table gradient's row flags (nr_unique_rows_zero_absent): published for the gradient
    autograd installs as it is, set for every non-zero row and not for the pad row, and FusedAdam
    reading them is bitwise the dense update (bf16: the CNN dgrad's plain scatter stores)."""
    table, grad, rt, same = _word_table_step(cfg, "one", prec)
    assert rt is not None and rt[0]() is table.grad and rt[2] == table.grad._version
    flags = rt[1].bool().cpu()
    nz = (grad != 0).any(1).cpu()
    assert not (nz & ~flags).any()
    assert int(flags[0]) == 0 and int(flags.sum()) >= int(nz.sum()) > 0
    assert same


@pytest.mark.parametrize("mode", ["passes", "uses"])
@pytest.mark.parametrize("cfg", ["nrms", "cnn_attn"])
def test_word_table_row_flags_accumulated(cfg, mode):
    """Gradients of two batches summed into the table's .grad -- a second backward pass (the flags
    are not published: .grad exists), or two uses of the table in one graph (each backward publishes,
    autograd adds the two gradients: a copy changes the address, an in-place add the version) --
    the flags no longer describe .grad, FusedAdam must not use them: bitwise the dense update."""
    table, grad, rt, same = _word_table_step(cfg, mode)
    if rt is not None:
        assert not (rt[0]() is table.grad and rt[2] == table.grad._version)
    assert same


@pytest.mark.parametrize("cfg", ["nrms", "cnn_attn"])
def test_word_table_row_flags_die_with_their_gradient(cfg):
    """flags published for one step's gradient must not outlive it.  zero_grad(set_to_none)
    frees that gradient; a new dense gradient the caching allocator places at the SAME address (version
    0 again) that no backward of ours produced must get the dense Adam update, not the stale flags'
    row skipping."""
    from newsrec_amd.optim import FusedAdam
    from newsrec_amd import kernels as K
    table, grad, rt, same = _word_table_step(cfg, "one")
    assert same and rt is not None
    addr = table.grad.data_ptr()
    flags = rt[1]
    absent = (flags == 0).nonzero().view(-1)
    assert absent.numel() > 0
    opt = FusedAdam([table], lr=1e-3)
    opt.zero_grad(set_to_none=True)
    g2 = torch.empty_like(table)                       # the freed block, reused
    if g2.data_ptr() != addr:
        pytest.skip("allocator did not reuse the gradient's block")
    g2.normal_()
    table.grad = g2
    p0 = table.detach().clone()
    opt.step()
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    K.adam_multi([(p, g2, m, v, 1e-3, 1)], 0.9, 0.999, 1e-8, 0.0, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(table.detach(), p)              # rows the stale flags mark absent moved too
    assert torch.equal(opt.state[table]["exp_avg"], m)
