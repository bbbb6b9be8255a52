"""nr_mha_attn_fwd/bwd against the oracle's tied-QK attention core in fp64
(models/Modules/Attention.py:115-147 with XSoftmax)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import kernels as K
from oracle import restatement as R


def _ref(qk, v, mask, heads, dk, dv):
    n, l, _ = qk.shape
    kp = qk.view(n, l, heads, dk).permute(0, 2, 1, 3)
    vp = v.view(n, l, heads, dv).permute(0, 2, 1, 3)
    s = kp @ kp.transpose(-1, -2) / math.sqrt(dk)
    p = R.xsoftmax(s, R.pairwise_mask(mask))
    return (p @ vp).permute(0, 2, 1, 3).reshape(n, l, heads * dv)


@pytest.mark.parametrize("L,heads,dk,dv,mdt", [(30, 12, 64, 32, torch.int64), (50, 12, 32, 32, torch.float64),
                                               (7, 3, 64, 64, torch.float32), (64, 2, 64, 64, torch.uint8)])
def test_mha_attn(L, heads, dk, dv, mdt):
    g = torch.Generator().manual_seed(L + heads)
    n = 37
    qk = torch.randn(n, L, heads * dk, generator=g, dtype=torch.float64)
    v = torch.randn(n, L, heads * dv, generator=g, dtype=torch.float64)
    lens = torch.randint(0, L + 1, (n,), generator=g)
    lens[0] = 0
    lens[1] = L
    mask = (torch.arange(L)[None] < lens[:, None]).to(mdt)
    qk.requires_grad_(True)
    v.requires_grad_(True)
    want = _ref(qk, v, mask, heads, dk, dv)
    dout = torch.randn(want.shape, generator=g, dtype=torch.float64)
    want.backward(dout)

    # stored with extra columns, as the fused [T, 1152] projection output is
    pad = 8
    qkd = torch.zeros(n * L, heads * dk + pad, device="cuda")
    qkd[:, :heads * dk] = qk.detach().reshape(n * L, -1).float().cuda()
    vd = torch.zeros(n * L, heads * dv + pad, device="cuda")
    vd[:, :heads * dv] = v.detach().reshape(n * L, -1).float().cuda()
    out = torch.empty(n * L, heads * dv, device="cuda")
    md = mask.cuda().contiguous()
    K.mha_attn_fwd(qkd[:, :heads * dk], vd[:, :heads * dv], md, n, L, heads, dk, dv, out)
    torch.testing.assert_close(out.cpu().double().view(n, L, -1), want.detach(), rtol=1e-4, atol=1e-5)
    assert torch.all(out.view(n, L, -1)[0] == 0)          # fully masked sequence -> zeros

    dqk = torch.zeros(n * L, heads * dk, device="cuda")
    dvv = torch.zeros(n * L, heads * dv, device="cuda")
    db = torch.zeros(heads * (dk + dv), device="cuda")
    K.mha_attn_bwd(qkd[:, :heads * dk], vd[:, :heads * dv], md, n, L, heads, dk, dv,
                   dout.reshape(n * L, -1).float().cuda(), dqk, dvv, dbias=db)
    torch.testing.assert_close(dqk.cpu().double().view(n, L, -1), qk.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dvv.cpu().double().view(n, L, -1), v.grad, rtol=1e-4, atol=1e-4)
    # the projection bias gradient folded into the kernel: the column sums of [dqk | dv]
    want_db = torch.cat([qk.grad.sum((0, 1)), v.grad.sum((0, 1))])
    torch.testing.assert_close(db.cpu().double(), want_db, rtol=1e-4, atol=1e-3)
    # without dbias the gradients are the same, bit for bit
    dqk2, dvv2 = torch.zeros_like(dqk), torch.zeros_like(dvv)
    K.mha_attn_bwd(qkd[:, :heads * dk], vd[:, :heads * dv], md, n, L, heads, dk, dv,
                   dout.reshape(n * L, -1).float().cuda(), dqk2, dvv2)
    assert torch.equal(dqk, dqk2) and torch.equal(dvv, dvv2)


@pytest.mark.parametrize("shape,mshape", [((4, 3, 30), (4, 1, 30)), ((2, 12, 30, 30), (2, 1, 30, 30)), ((5, 50), (5, 50))])
def test_xsoftmax_public(shape, mshape):
    """attention.XSoftmax (Attention.py:56-80) on nr_xsoftmax_fwd/bwd against the float64 restatement:
    masked entries exactly zero, a fully masked row all zero, the backward _softmax_backward_data."""
    from newsrec_amd.attention import XSoftmax
    from oracle import restatement as R
    torch.manual_seed(len(shape))
    x = torch.randn(*shape, device="cuda", requires_grad=True)
    mask = (torch.rand(*mshape, device="cuda") > 0.3).long()
    mask.view(-1, mshape[-1])[0] = 0                       # a fully masked row
    y = XSoftmax.apply(x, mask, -1)
    x64 = x.detach().cpu().double().requires_grad_()
    want = R.xsoftmax(x64, mask.cpu().expand(shape), -1)
    torch.testing.assert_close(y.detach().cpu().double(), want, rtol=0, atol=1e-6)
    assert bool((y.detach()[mask.expand(shape) == 0] == 0).all())
    g = torch.randn(*shape, device="cuda")
    y.backward(g)
    want.backward(g.cpu().double())
    torch.testing.assert_close(x.grad.cpu().double(), x64.grad, rtol=0, atol=1e-5)


@pytest.mark.parametrize("sep_key", [False, True])
def test_scaled_dp_attention_public(sep_key):
    """attention.scaled_dp_attention (Attention.py:5-30) in its reference form -- one learned query over
    [..., L, D] keys / values with a [..., 1, L] mask (CNN.py:46, Pooling.py:22-24) -- on the pooling
    kernels: values and every gradient against the float64 restatement."""
    from newsrec_amd.attention import scaled_dp_attention
    from oracle import restatement as R
    torch.manual_seed(7)
    B, n, Lk, D = 3, 4, 30, 150
    q = torch.randn(1, D, device="cuda", requires_grad=True)
    v = torch.randn(B, n, Lk, D, device="cuda", requires_grad=True)
    k = torch.randn(B, n, Lk, D, device="cuda", requires_grad=True) if sep_key else v
    m = (torch.rand(B, n, 1, Lk, device="cuda") > 0.2).long()
    m[0, 0] = 0
    out = scaled_dp_attention(q, k, v, m)
    ts = [t.detach().cpu().double().requires_grad_() for t in (q, k, v)] if sep_key else \
        [t.detach().cpu().double().requires_grad_() for t in (q, v)]
    q64, k64, v64 = (ts[0], ts[1], ts[2]) if sep_key else (ts[0], ts[1], ts[1])
    want = R.scaled_dp_attention(q64, k64, v64, m.cpu())
    torch.testing.assert_close(out.detach().cpu().double(), want, rtol=0, atol=1e-5)
    g = torch.randn_like(out)
    out.backward(g)
    want.backward(g.cpu().double())
    for a, b in zip([q, k, v] if sep_key else [q, v], ts):
        torch.testing.assert_close(a.grad.cpu().double(), b.grad, rtol=0, atol=1e-4)


def test_gather_rows():
    """nr_gather_rows_f32 (the fast-eval history gather): widths with and without float4 rows."""
    from newsrec_amd import kernels as K
    for cols in (150, 384, 3):
        t = torch.randn(500, cols, device="cuda")
        idx = torch.randint(0, 500, (777,), device="cuda")
        assert torch.equal(K.gather_rows(t, idx), t[idx])


@pytest.mark.parametrize("prec", ["bf16x6", "f32", "bf16"])
@pytest.mark.parametrize("L,heads,dk,dv", [(50, 12, 32, 32), (64, 12, 64, 32), (33, 12, 64, 64), (20, 12, 32, 32)])
def test_mha_user_pool(L, heads, dk, dv, prec):
    """nr_mha_user_pool_fwd (the fast eval's MHA user encoder + Attention_Pooling in one launch) against
    the fp64 restatement (tied-QK attention core with the pairwise mask, then query pooling with the
    history mask, MHA.py:58-75 / Pooling.py:12-25), history slots read through a row table; ragged
    histories, an empty one and a full one; the attention products in each GEMM arithmetic."""
    from newsrec_amd import _lib as L_
    g = torch.Generator().manual_seed(L * heads + dk)
    n, nrow = 41, 700
    H = heads * dv
    y = torch.randn(nrow, heads * (dk + dv) + 4, generator=g, dtype=torch.float64)   # padded rows
    rows = torch.randint(0, nrow, (n * L,), generator=g)
    q = torch.randn(H, generator=g, dtype=torch.float64)
    lens = torch.randint(0, L + 1, (n,), generator=g)
    lens[0], lens[1] = 0, L
    mask = (torch.arange(L)[None] < lens[:, None]).to(torch.float64)
    yy = y[rows].view(n, L, -1)
    O = _ref(yy[..., :heads * dk], yy[..., heads * dk:heads * (dk + dv)], mask, heads, dk, dv)
    want = R.scaled_dp_attention(q.view(1, 1, H).expand(n, 1, H), O, O, mask.view(n, 1, L)).view(n, H)
    p_ = {"bf16x6": L_.GEMM_BF16X6, "f32": L_.GEMM_F32, "bf16": L_.GEMM_BF16}[prec]
    out = torch.full((n, H), float("nan"), device="cuda")
    K.mha_user_pool_fwd(y.float().cuda(), rows.cuda(), mask.cuda(), n, L, heads, dk, dv, q.float().cuda(), out,
                        prec=p_)
    err = (out.double().cpu() - want).abs().max().item()
    scale = want.abs().max().item()
    tol = 3e-2 if prec == "bf16" else 2e-5
    print("user pool L=%d dk=%d dv=%d %s: max |err| %.3e of %.3e" % (L, dk, dv, prec, err, scale))
    assert err <= tol * scale
    assert out[0].abs().max().item() == 0.0   # an empty history: zero user vector (XSoftmax)


def test_mha_user_pool_lds_cap_falls_back():
    """At H = 768 the fused user pool's O [L][H + 1] exceeds the 160 KB LDS from L = 54 on: the entry
    refuses the launch (NR_EINVAL(10), never a failed hipFuncSetAttribute), mha_user_pool_supported says
    no, and MHA_User_Encoder.forward_rows takes the two-launch path with the same result as the
    fp64 restatement."""
    from newsrec_amd import _lib as L_
    from newsrec_amd.encoders import MHA_User_Encoder
    L, heads, dk, dv = 64, 12, 64, 64
    H = heads * dv
    assert not K.mha_user_pool_supported(L, heads, dk, dv)
    assert K.mha_user_pool_supported(53, heads, dk, dv) and not K.mha_user_pool_supported(54, heads, dk, dv)
    g = torch.Generator().manual_seed(7)
    n, nrow = 9, 100
    y = torch.randn(nrow, heads * (dk + dv), generator=g, dtype=torch.float64)
    rows = torch.randint(0, nrow, (n * L,), generator=g)
    lens = torch.randint(0, L + 1, (n,), generator=g)
    lens[0], lens[1] = 0, L
    mask = (torch.arange(L)[None] < lens[:, None]).to(torch.float64)
    out = torch.empty(n, H, device="cuda")
    with pytest.raises(L_.HipError):
        K.mha_user_pool_fwd(y.float().cuda(), rows.cuda(), mask.cuda(), n, L, heads, dk, dv,
                            torch.randn(H, device="cuda"), out)

    class _M:
        hidden_dim, head_num, dropout_p = H, heads, 0.2
    enc = MHA_User_Encoder(_M()).cuda()
    assert enc.mha.key_dim == dk and enc.mha.value_dim == dv
    q = enc.query_news.detach().double().cpu().view(-1)
    yy = y[rows].view(n, L, -1)
    O = _ref(yy[..., :heads * dk], yy[..., heads * dk:], mask, heads, dk, dv)
    want = R.scaled_dp_attention(q.view(1, 1, H).expand(n, 1, H), O, O, mask.view(n, 1, L)).view(n, H)
    got = enc.forward_rows(y.float().cuda(), rows.view(n, L).cuda(), mask.view(n, L, 1).cuda(), n, L)
    err = (got.view(n, H).double().cpu() - want).abs().max().item()
    assert err <= 2e-5 * want.abs().max().item()
