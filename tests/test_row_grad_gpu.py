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
