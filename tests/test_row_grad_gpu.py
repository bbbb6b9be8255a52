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
    buf, flags = table._nr_row_touched
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
