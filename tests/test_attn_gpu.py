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
    K.mha_attn_bwd(qkd[:, :heads * dk], vd[:, :heads * dv], md, n, L, heads, dk, dv,
                   dout.reshape(n * L, -1).float().cuda(), dqk, dvv)
    torch.testing.assert_close(dqk.cpu().double().view(n, L, -1), qk.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dvv.cpu().double().view(n, L, -1), v.grad, rtol=1e-4, atol=1e-4)
