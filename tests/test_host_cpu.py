"""Host-side step bookkeeping (no GPU): functions.ZERO_ARENA (one zero fill for a step's small
gradients) and GRAD_DEST / SplitRowsFn's offers, on CPU tensors."""
import torch


class _Ctx:
    def __init__(self, needs=True):
        self.needs_input_grad = (needs,)


def test_zero_arena_one_buffer_per_step():
    from newsrec_amd.functions import _ZeroArena
    za = _ZeroArena()
    dev = torch.device("cpu")
    t1 = za.reserve(dev, (3,), (5, 7))
    t2 = za.reserve(dev, (2, 2))
    a, b = za.take(t1, dev, (3,), (5, 7))
    (c,) = za.take(t2, dev, (2, 2))
    assert a.shape == (3,) and b.shape == (5, 7) and c.shape == (2, 2)
    assert a.untyped_storage().data_ptr() == c.untyped_storage().data_ptr()   # one buffer, one fill
    for t in (a, b, c):
        assert t.abs().sum().item() == 0.0
    ptrs = sorted((t.data_ptr(), t.data_ptr() + 4 * t.numel()) for t in (a, b, c))
    assert all(ptrs[i][1] <= ptrs[i + 1][0] for i in range(2))                  # disjoint
    assert all(p % 16 == 0 for p, _ in ptrs)                                     # 16-B aligned views
    b.fill_(1.0)
    # taken once: a second backward over the same graph gets fresh zeros
    a2, b2 = za.take(t1, dev, (3,), (5, 7))
    assert b2.abs().sum().item() == 0.0 and b2.data_ptr() != b.data_ptr()
    # the next step's reservations start a new buffer
    t3 = za.reserve(dev, (4,))
    (d,) = za.take(t3, dev, (4,))
    assert d.untyped_storage().data_ptr() != a.untyped_storage().data_ptr()


def test_zero_arena_fallbacks():
    from newsrec_amd import functions as F
    dev = torch.device("cpu")
    ctx = _Ctx(needs=False)
    F._CALLER_GRAD.on = True   # what _GradAwareFn.apply records
    try:
        F._reserve_zeros(ctx, dev, (8,))
    finally:
        F._CALLER_GRAD.on = None
    assert ctx.zero_tok is None
    (z,) = F._backward_zeros(ctx, dev, (8,))
    assert z.shape == (8,) and z.abs().sum().item() == 0.0
    za = F._ZeroArena()
    big = za.reserve(dev, (za.LIMIT + 4,))
    small = za.reserve(dev, (4,))
    assert small["arena"] is not big["arena"]
    # a shape mismatch falls back to plain zeros
    (w,) = za.take(small, dev, (5,))
    assert w.shape == (5,) and not small["taken"]


def test_split_rows_offers_and_join():
    from newsrec_amd.functions import GRAD_DEST, SplitRowsFn
    x = torch.randn(7, 5, requires_grad=True)
    a, b = SplitRowsFn.apply(x, 3)
    assert torch.equal(a, x[:3]) and torch.equal(b, x[3:])
    da = GRAD_DEST.take(a.detach())
    db = GRAD_DEST.take(b.detach())
    assert da is not None and db is not None and da.shape == (3, 5) and db.shape == (4, 5)
    assert GRAD_DEST.take(a.detach()) is None                                     # one taker per offer

    class Use(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t, dest, scale):
            ctx.dest, ctx.scale = dest, scale
            return t.sum()

        @staticmethod
        def backward(ctx, g):
            ctx.dest.fill_(ctx.scale)
            return ctx.dest, None, None

    SplitRowsFn.stats.update(in_place=0, copied=0)
    (Use.apply(a, da, 2.0) + Use.apply(b, db, 3.0)).backward()
    assert SplitRowsFn.stats == {"in_place": 1, "copied": 0}
    assert torch.equal(x.grad[:3], torch.full((3, 5), 2.0)) and torch.equal(x.grad[3:], torch.full((4, 5), 3.0))
    # consumers that do not write in place: joined by a copy, same values
    x.grad = None
    a, b = SplitRowsFn.apply(x, 3)
    GRAD_DEST.clear()
    (2.0 * a.sum() + 3.0 * b.sum()).backward()
    assert SplitRowsFn.stats["copied"] == 1
    assert torch.equal(x.grad[:3], torch.full((3, 5), 2.0)) and torch.equal(x.grad[3:], torch.full((4, 5), 3.0))
    # one output unused: its half is zero
    x.grad = None
    a, b = SplitRowsFn.apply(x, 3)
    (2.0 * a.sum()).backward()
    assert torch.equal(x.grad[3:], torch.zeros(4, 5)) and torch.equal(x.grad[:3], torch.full((3, 5), 2.0))


def test_backward_possible_sees_the_callers_grad_mode():
    """torch runs Function.forward with grad mode off; _GradAwareFn.apply records the caller's mode, so
    a forward saves backward-only state (the split MHA backward's O rows, the arena's reservations)
    exactly when autograd is recording and an input wants a gradient."""
    from newsrec_amd import functions as F
    seen = []

    class Probe(F._GradAwareFn):
        @staticmethod
        def forward(ctx, t):
            assert not torch.is_grad_enabled()
            seen.append(F._backward_possible(ctx))
            return t * 2

        @staticmethod
        def backward(ctx, g):
            return g * 2

    x = torch.randn(3, requires_grad=True)
    Probe.apply(x).sum().backward()
    with torch.no_grad():
        Probe.apply(x)
    Probe.apply(x.detach())
    with torch.enable_grad():
        with torch.no_grad():
            with torch.enable_grad():
                Probe.apply(x)
    assert seen == [True, False, False, True]
    assert torch.equal(x.grad, torch.full((3,), 2.0))
    assert getattr(F._CALLER_GRAD, "on", None) is None   # restored after each apply
    ctx = _Ctx()
    try:
        F._backward_possible(ctx)
        raise AssertionError("outside a _GradAwareFn forward it must raise")
    except RuntimeError:
        pass
