"""nr_seq_pool_fwd / nr_seq_pool_bwd (csrc/seq_pool.hip) against a float64 autograd restatement of
Attention_Pooling (models/Encoders/Pooling.py:12-25) and CNN_Encoder's word pooling (CNN.py:46):
s_l = scale q·K_l, p = XSoftmax(s, mask), out = Σ p_l X_l, with K = X (tied) or a tanh key.
Both launch forms: one wave per sequence (many sequences, D <= 256) and one workgroup per sequence
(few sequences, or D up to 512 -- the NRMS user encoder's 32 histories of 50 x 384).  Ragged and
fully masked sequences, zero-padded widths (qn < D) and the extra token gradient dz."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from newsrec_amd import kernels as K


def _ref(x, key, q, mask, scale, tanh_key):
    """float64 restatement: key rows are tanh(pre) when tanh_key (the saved key is the tanh)."""
    k = x if key is None else key
    s = (k @ q) * scale                                   # [nseq, L]
    keep = mask.bool()
    p = torch.softmax(s.masked_fill(~keep, float("-inf")), -1).masked_fill(~keep, 0.0)
    p = torch.nan_to_num(p, nan=0.0)                      # a fully masked sequence pools zeros
    return (p.unsqueeze(-1) * x).sum(1), p


@pytest.mark.parametrize("nseq,L,D,qn,tied", [
    (32, 50, 384, 384, True),      # user encoder: workgroup form, two float4 per lane
    (20, 30, 160, 150, False),     # few CNN titles: workgroup form, one float4 per lane
    (1500, 30, 160, 150, False),   # CNN word pooling: wave per sequence
    (1200, 50, 256, 256, True),    # wave per sequence, L > 32
    (7, 64, 512, 500, True),       # the workgroup form's maxima
])
def test_seq_pool_matches_float64(nseq, L, D, qn, tied):
    g = torch.Generator().manual_seed(nseq + D)
    dev = "cuda"
    x = torch.randn(nseq, L, D, generator=g, dtype=torch.float64)
    x[..., qn:] = 0.0
    key = None if tied else torch.tanh(torch.randn(nseq, L, D, generator=g, dtype=torch.float64))
    if key is not None:
        key[..., qn:] = 0.0
    q = torch.randn(qn, generator=g, dtype=torch.float64)
    qf = torch.cat([q, torch.zeros(D - qn, dtype=torch.float64)])
    lens = torch.randint(1, L + 1, (nseq,), generator=g)
    mask = (torch.arange(L)[None] < lens[:, None]).long()
    mask[0] = 0                                             # fully masked sequence
    mask[1, ::3] = 0                                        # holes
    scale = 1.0 / qn ** 0.5
    dout = torch.randn(nseq, qn, generator=g, dtype=torch.float64)
    dz = torch.randn(nseq, L, D, generator=g, dtype=torch.float64) if not tied else None
    if dz is not None:
        dz[..., qn:] = 0.0

    # reference forward / backward in float64
    xr = x.clone().requires_grad_(True)
    kr = key.clone().requires_grad_(True) if key is not None else None
    qr = qf.clone().requires_grad_(True)
    out_r, p_r = _ref(xr, kr, qr, mask, scale, not tied)
    loss = (out_r[:, :qn] * dout).sum()
    if dz is not None:
        loss = loss + (xr * dz).sum()
    loss.backward()
    dk_want = None if kr is None else kr.grad * (1 - key ** 2)   # through the tanh of the saved key

    f = lambda t: t.float().to(dev).reshape(-1, t.shape[-1]).contiguous()  # noqa: E731
    X, KEY = f(x), (f(key) if key is not None else None)
    Q = q.float().to(dev)
    M = mask.to(dev).reshape(-1)
    out = torch.empty(nseq, D, device=dev)
    probs = torch.empty(nseq * L, device=dev)
    K.seq_pool_fwd(X, Q, M, nseq, L, D, out, probs, key=KEY, scale=scale, qn=qn)
    dx = torch.empty(nseq * L, D, device=dev)
    dk = torch.empty(nseq * L, D, device=dev) if key is not None else None
    dq = torch.zeros(qn, device=dev)
    K.seq_pool_bwd(X, Q, M, nseq, L, D, probs, dout.float().to(dev), dx, dq, key=KEY, dk=dk, key_tanh=not tied,
                   dz=f(dz) if dz is not None else None, scale=scale, qn=qn)
    torch.cuda.synchronize()

    def close(got, want, tol, name):
        err = (got.double().cpu() - want).abs().max().item()
        assert err <= tol * max(1.0, want.abs().max().item()), (name, err)

    close(out, out_r.detach(), 1e-5, "out")
    close(probs.view(nseq, L), p_r.detach(), 1e-5, "probs")
    close(dx.view(nseq, L, D), xr.grad, 1e-5, "dx")
    close(dq, qr.grad[:qn], 1e-4, "dq")
    if dk is not None:
        close(dk.view(nseq, L, D), dk_want, 1e-5, "dk")
    assert out[0].abs().max().item() == 0.0                  # fully masked: exact zeros


@pytest.mark.parametrize("L", [50, 64])
def test_seq_pool_768_wide(L):
    """nr_seq_pool_fwd / bwd at BERT width (D = 768, the workgroup form's NF = 4 instantiation: the
    768-wide MHA user encoder's pooling, Pooling.py:12-25) against float64 autograd."""
    from newsrec_amd import kernels as K
    from oracle import restatement as R
    g = torch.Generator().manual_seed(L)
    n, D = 7, 768
    x = torch.randn(n * L, D, generator=g, dtype=torch.float64)
    q = torch.randn(D, generator=g, dtype=torch.float64)
    lens = torch.randint(1, L + 1, (n,), generator=g)
    lens[0] = L
    mask = (torch.arange(L)[None] < lens[:, None]).to(torch.float64)
    xr, qr = x.clone().requires_grad_(True), q.clone().requires_grad_(True)
    want = R.scaled_dp_attention(qr.view(1, 1, D).expand(n, 1, D), xr.view(n, L, D), xr.view(n, L, D),
                                 mask.view(n, 1, L)).view(n, D)
    dout = torch.randn(n, D, generator=g, dtype=torch.float64)
    want.backward(dout)
    xd, qd, md = x.float().cuda(), q.float().cuda(), mask.cuda()
    out = torch.empty(n, D, device="cuda")
    probs = torch.empty(n * L, device="cuda")
    K.seq_pool_fwd(xd, qd, md, n, L, D, out, probs)
    dx = torch.empty(n * L, D, device="cuda")
    dq = torch.zeros(D, device="cuda")
    K.seq_pool_bwd(xd, qd, md, n, L, D, probs, dout.float().cuda(), dx, dq)
    for got, ref in ((out, want), (dx, xr.grad), (dq, qr.grad)):
        err = (got.double().cpu().view_as(ref) - ref.detach()).abs().max().item()
        assert err <= 2e-5 * max(ref.abs().max().item(), 1e-6)
