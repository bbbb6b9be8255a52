"""Attention primitives with the reference's public interface
(models/Modules/Attention.py): ``scaled_dp_attention``, ``get_attn_mask``, ``XSoftmax`` and
``MultiheadAttention`` (Q and K both from ``keyProject``, no output projection).

``MultiheadAttention`` keeps the reference's parameter names (``keyProject``,
``valueProject``) so checkpoints load unchanged; its forward runs the projections on the
fp32 MFMA GEMM and the attention core in ``nr_mha_attn_fwd``.  The towers do not call it:
they run the whole encoder as one fused autograd Function (functions.py).
"""

import torch
from torch import nn

from . import _lib as L
from . import kernels as K
from .functions import MHAFn, AttnPoolFn


def get_attn_mask(attn_mask):
    """Attention.py:33-53: [N, L] -> pairwise [N, 1, L, L] = m_i * m_j."""
    if attn_mask is None:
        return None
    assert attn_mask.dim() == 2
    return attn_mask[:, None, :, None] * attn_mask[:, None, None, :]


class XSoftmax(torch.autograd.Function):
    """Attention.py:56-80 — masked softmax whose masked (and fully masked) entries are exactly
    zero, on nr_xsoftmax_fwd/bwd (one wave per row of the softmax dimension).  The mask broadcasts
    to the input's shape as in the reference; ``dim`` is the last dimension (every reference call,
    Attention.py:22,139)."""

    @staticmethod
    def forward(ctx, input, mask, dim):
        L.require_gpu(input)
        if dim not in (-1, input.dim() - 1):
            raise L.HipError("XSoftmax: the HIP kernel normalises over the last dimension (dim=-1)")
        x = input.contiguous()
        m = mask.to(x.device)
        m = m if m.shape == x.shape else m.expand(x.shape)
        m = m.contiguous() if m.dtype in (torch.uint8, torch.bool, torch.int64, torch.float64, torch.float32) \
            else m.to(torch.uint8).contiguous()
        out = torch.empty_like(x)
        K.xsoftmax_fwd(x, m, out)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, grad):
        (out,) = ctx.saved_tensors
        dx = torch.empty_like(out)
        K.xsoftmax_bwd(out, grad.contiguous(), dx)
        return dx, None, None


class _QueryPoolFn(torch.autograd.Function):
    """scaled_dp_attention with one learned query (every reference call: CNN.py:46, Pooling.py:22-24,
    MHA.py:38,72): out[s] = Σ_l XSoftmax(q · key[s, l] / sqrt(D), mask[s, l]) value[s, l] on
    nr_attn_pool_fwd/bwd.  rows [S * L, D]; key None = the value rows."""

    @staticmethod
    def forward(ctx, q, key, value, mask, S, Lq):
        D = q.numel()
        probs = torch.empty(S * Lq, device=value.device)
        out = torch.empty(S, D, device=value.device)
        K.attn_pool_fwd(value, q, mask, S, Lq, out, probs, key=key)
        ctx.save_for_backward(q, key, value, mask, probs)
        ctx.cfg = (S, Lq)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, key, value, mask, probs = ctx.saved_tensors
        S, Lq = ctx.cfg
        dv = torch.empty_like(value)
        dk = torch.empty_like(key) if key is not None else None
        dq = torch.zeros(q.numel(), device=q.device)
        K.attn_pool_bwd(value, q, mask, S, Lq, probs, dout.contiguous(), dv, dq, key=key, dk=dk)
        return dq.view_as(q), dk, dv, None, None, None


def scaled_dp_attention(query, key, value, attn_mask=None):
    """Attention.py:5-30: softmax(q kᵀ / sqrt(d)) v with an optional XSoftmax mask, for a learned
    query of one row ([1, D] or [..., 1, D] broadcast over the batch) -- the form every reference
    call site uses (learned-query pooling) -- on the pooling kernels.  Other query shapes raise (the
    encoders run multi-query attention inside their fused kernels)."""
    L.require_gpu(key, value)
    assert query.shape[-1] == key.shape[-1]
    D = query.shape[-1]
    if query.numel() != D or key.shape != value.shape or key.shape[-2] > 64:
        raise L.HipError("scaled_dp_attention: the HIP path takes one query row over <= 64 keys with value "
                         "rows of the key's shape (got q %s, k %s, v %s)" % (tuple(query.shape), tuple(key.shape),
                                                                          tuple(value.shape)))
    lead = key.shape[:-2]
    Lq = key.shape[-2]
    S = int(torch.Size(lead).numel())
    v = value.reshape(S * Lq, D).contiguous()
    k = None if key is value else key.reshape(S * Lq, D).contiguous()
    if attn_mask is None:
        m = torch.ones(S * Lq, dtype=torch.uint8, device=v.device)
    else:
        m = attn_mask.to(v.device).expand(*lead, 1, Lq).reshape(S * Lq)
        m = m.contiguous() if m.dtype in (torch.uint8, torch.bool, torch.int64, torch.float64, torch.float32) \
            else m.to(torch.uint8).contiguous()
    out = _QueryPoolFn.apply(query.reshape(D), k, v, m, S, Lq)
    return out.view(*lead, 1, D)


def _joined_view(a, b):
    """[a; b] as one tensor when b's data directly follows a's in the same storage, else None."""
    if (a.device != b.device or a.dtype != b.dtype or not a.is_contiguous() or not b.is_contiguous()
            or a.shape[1:] != b.shape[1:]):
        return None
    sa, sb = a.untyped_storage(), b.untyped_storage()
    if sa.data_ptr() != sb.data_ptr() or b.storage_offset() != a.storage_offset() + a.numel():
        return None
    return torch.empty(0, dtype=a.dtype, device=a.device).set_(
        sa, a.storage_offset(), (a.shape[0] + b.shape[0],) + tuple(a.shape[1:]))


class _Joined(torch.autograd.Function):
    """The stacked [a; b] of two parameters that live back to back in one buffer, without a copy;
    the backward hands each parameter its rows of the gradient (views, no copy either)."""

    @staticmethod
    def forward(ctx, a, b, joined):
        ctx.n = a.shape[0]
        return joined

    @staticmethod
    def backward(ctx, g):
        return g[:ctx.n], g[ctx.n:], None


class MultiheadAttention(nn.Module):
    """Attention.py:83-147 with the same constructor, parameters and init."""

    def __init__(self, hidden_dim, head_num, key_dim=None, value_dim=None):
        super().__init__()
        self.head_num = head_num
        if not (key_dim and value_dim):
            assert hidden_dim % head_num == 0, "hidden_dim {} must divide head_num {}".format(hidden_dim, head_num)
            head_dim = hidden_dim // head_num
        self.hidden_dim = hidden_dim
        self.key_dim = key_dim if key_dim else head_dim
        self.value_dim = value_dim if value_dim else head_dim
        self.keyProject = nn.Linear(hidden_dim, self.key_dim * head_num)
        self.valueProject = nn.Linear(hidden_dim, self.value_dim * head_num)
        nn.init.xavier_normal_(self.keyProject.weight)
        nn.init.xavier_normal_(self.valueProject.weight)

    def _join_storage(self):
        """Re-home keyProject's and valueProject's weights (and biases) as the two halves of one
        buffer each, so the stacked operand of the projection GEMM is a view, not a per-step cat.
        The parameters stay the reference's (names, shapes, values, state_dict); only their storage
        moves.  Done on first use and again if something (``.to()``) has separated them."""
        kp, vp = self.keyProject, self.valueProject
        with torch.no_grad():
            for name in ("weight", "bias"):
                a, b = getattr(kp, name), getattr(vp, name)
                buf = torch.cat([a.detach(), b.detach()], 0)
                a.data = buf[:a.shape[0]]
                b.data = buf[a.shape[0]:]

    def fused_weight(self):
        """[keyProject; valueProject] stacked for the single projection GEMM (weights and biases):
        views of the joined storage, so no copy per step."""
        kp, vp = self.keyProject, self.valueProject
        jw, jb = _joined_view(kp.weight, vp.weight), _joined_view(kp.bias, vp.bias)
        if jw is None or jb is None:
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                # never re-home storage inside a captured graph: stack by copy
                return (torch.cat([kp.weight, vp.weight], 0), torch.cat([kp.bias, vp.bias], 0))
            self._join_storage()
            jw, jb = _joined_view(kp.weight, vp.weight), _joined_view(kp.bias, vp.bias)
        return _Joined.apply(kp.weight, vp.weight, jw), _Joined.apply(kp.bias, vp.bias, jb)

    def forward(self, hidden_states, attention_mask=None):
        """hidden_states [N, L, D]; attention_mask: the pairwise [N, 1, L, L] mask built by
        ``get_attn_mask`` (only pairwise-product masks are supported: the token mask is read
        off its diagonal, since m_i * m_i = m_i) or None."""
        n, l, d = hidden_states.shape
        L.require_gpu(hidden_states)
        if attention_mask is None:
            tok_mask = torch.ones(n, l, dtype=torch.uint8, device=hidden_states.device)
        else:
            tok_mask = torch.diagonal(attention_mask.reshape(n, l, l), dim1=-2, dim2=-1).contiguous()
        w, b = self.fused_weight()
        x = hidden_states.reshape(n * l, d)
        if x.stride(-1) != 1:
            x = x.contiguous()
        out = MHAFn.apply(x, tok_mask, w, b, n, l, self.head_num, self.key_dim, self.value_dim)
        return out.reshape(n, l, -1)
