"""BERT towers of XFormer / PLM (models/XFormer.py, models/PLM.py) on the HIP kernels.

``BertModel`` mirrors transformers' BertModel as the reference uses it — ``bert(input_ids,
attention_mask)`` returning ``last_hidden_state`` / ``pooler_output`` (``[-1]`` is the pooler
output, PLM.py:102) — with the same module tree and ``state_dict`` names
(``embeddings.word_embeddings.weight``, ``encoder.layer.N.attention.self.query.weight``, …) so
checkpoints load unchanged.  The reference loads pretrained ``bert-base-uncased`` weights
(XFormer.py:45-48), which are not available offline: the default here is transformers' random
init of the same architecture (normal(0, 0.02), zero biases, unit LayerNorms).

The whole encoder is ONE autograd.Function (``BertFn``) over several token segments at once:
XFormer's candidate titles ([B*5, 30]) and user sequence ([B, 501]) share every dense layer, so
their rows are concatenated and each GEMM runs once over all of them (only the attention core
and the position ids are per segment).  Per layer:

  qkv = x [Wq;Wk;Wv]ᵀ + b                 nr_gemm_f32 (one GEMM, N = 3H)
  ctx = attention(qkv, mask)              nr_bert_attn_fwd (online softmax, the GEMM arithmetic)
  h1  = LN(Dropout(ctx Woᵀ + bo) + x)     nr_gemm_f32 + nr_bert_add_ln_fwd
  G   = gelu(h1 Wiᵀ + bi)                 nr_gemm_f32, NR_EPI_STORE_GELU (pre-activation kept)
  h2  = LN(Dropout(G Wo2ᵀ + bo2) + h1)    nr_gemm_f32 + nr_bert_add_ln_fwd
and the pooler is tanh(h[CLS] Wpᵀ + bp): one gather-operand GEMM with a tanh epilogue.
"""
from collections import namedtuple

import torch
from torch import nn

from . import _lib as L
from . import kernels as K
from .functions import _empty, _gemm_backward, _proj_wgrad, _zeros_views, table_grad_buffer


# the bf16-MFMA attention forward stores its dropout keep bits for the backward (False: the backward
# re-hashes every probability's counter, the same masks)
ATTN_KEEP_BITS = True
# input-gradient GEMMs (dX = dY W) on the k-contiguous weight (W transposed per layer and backward by
# nr_transpose_f32) instead of the MN-contiguous one: XFormer step 68.6-68.9 vs 68.1 ms
# (profiles/r05_z_xformer_dgrad_kc_ab.jsonl), off
DGRAD_KC = False


class BertConfig:
    """transformers.BertConfig defaults (bert-base-uncased)."""

    def __init__(self, vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, max_position_embeddings=512, type_vocab_size=2, layer_norm_eps=1e-12,
                 hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1, pad_token_id=0, initializer_range=0.02):
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.intermediate_size = intermediate_size
        self.max_position_embeddings = max_position_embeddings
        self.type_vocab_size = type_vocab_size
        self.layer_norm_eps = layer_norm_eps
        self.hidden_dropout_prob = hidden_dropout_prob
        self.attention_probs_dropout_prob = attention_probs_dropout_prob
        self.pad_token_id = pad_token_id
        self.initializer_range = initializer_range


BertOutput = namedtuple("BertOutput", ["last_hidden_state", "pooler_output"])


class BertEmbeddings(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden_size, padding_idx=c.pad_token_id)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class BertSelfAttention(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.query = nn.Linear(c.hidden_size, c.hidden_size)
        self.key = nn.Linear(c.hidden_size, c.hidden_size)
        self.value = nn.Linear(c.hidden_size, c.hidden_size)
        self.dropout = nn.Dropout(c.attention_probs_dropout_prob)


class BertSelfOutput(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class BertAttention(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.self = BertSelfAttention(c)
        self.output = BertSelfOutput(c)


class BertIntermediate(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.intermediate_size)


class BertLayerOutput(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.intermediate_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class BertLayer(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.attention = BertAttention(c)
        self.intermediate = BertIntermediate(c)
        self.output = BertLayerOutput(c)


class BertEncoder(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])


class BertPooler(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)


class _Segment:
    """One token batch [nseq, L] of the fused pass: ids int64 [nseq*L], mask [nseq*L]."""

    def __init__(self, ids, mask):
        self.nseq, self.L = ids.shape
        self.ids = ids.reshape(-1).contiguous()
        m = mask.reshape(-1)
        self.mask = m if m.is_contiguous() else m.contiguous()


def _wdgrad(w, keep):
    """B operand of dX = dY W for an nn.Linear weight W [out, in]: W itself (MN-contiguous) or its
    transpose (k-contiguous, DGRAD_KC; appended to ``keep``, which holds it until the GEMM is enqueued)."""
    if DGRAD_KC:
        t = K.transpose(w)
        keep.append(t)
        return K.operand(t, L.KCONTIG)
    return K.operand(w, L.MNCONTIG)


class BertFn(torch.autograd.Function):
    """The BertModel forward over concatenated segments -> (last_hidden [T, H], pooled [S, H]).
    ``drop`` = list of per-site (seed, offset, rng, offset inside rng's range) or None (eval / p = 0)."""

    @staticmethod
    def forward(ctx, cfg, segs, drop, *params):
        ctx.prec = K.get_gemm_precision()
        c = cfg
        H, heads, I = c.hidden_size, c.num_attention_heads, c.intermediate_size
        nl = c.num_hidden_layers
        word, pos, typ, elw, elb = params[:5]
        lp = [params[5 + 16 * i: 5 + 16 * (i + 1)] for i in range(nl)]
        pw, pb = params[5 + 16 * nl:]
        dev = word.device
        T = sum(s.nseq * s.L for s in segs)
        S = sum(s.nseq for s in segs)
        r0s, cls = [], []
        r = 0
        for s in segs:
            r0s.append(r)
            cls.append(r + torch.arange(s.nseq, device=dev, dtype=torch.int64) * s.L)
            r += s.nseq * s.L
        cls_idx = torch.cat(cls)
        p_h = c.hidden_dropout_prob if drop is not None else 0.0
        p_a = c.attention_probs_dropout_prob if drop is not None else 0.0

        def dsite(k):
            if drop is None:
                return dict(p_drop=0.0)
            seed, off, rng, rel = drop[k]
            return dict(seed=seed, offset=rel if rng is not None else off, rng=rng)

        def dsite_seg(k, p, extra):
            d = dsite(k)
            if p <= 0.0:
                return dict(p_drop=0.0)
            d["p_drop"] = p
            d["offset"] = d["offset"] + extra
            return d

        x = _empty(T, H, word)
        st_e = torch.empty(T, 2, device=dev)
        for s, r0 in zip(segs, r0s):
            K.bert_embed_fwd(word, pos, typ[0], s.ids, s.nseq, s.L, elw, elb, c.layer_norm_eps,
                             x[r0:r0 + s.nseq * s.L], st_e[r0:r0 + s.nseq * s.L],
                             **dsite_seg(0, p_h, r0 * H))
        saved, keeps_all = [], []
        for li, w in enumerate(lp):
            wq, bq, wk, bk, wv, bv, wo, bo, l1w, l1b, wi, bi, wo2, bo2, l2w, l2b = w
            wqkv = torch.cat([wq, wk, wv], 0)
            bqkv = torch.cat([bq, bk, bv], 0)
            qkv = _empty(T, 3 * H, word)
            K.gemm(T, 3 * H, H, K.operand(x, L.KCONTIG), K.operand(wqkv, L.KCONTIG), qkv, bias=bqkv)
            cx = _empty(T, H, word)
            ml = torch.empty(T * heads * 2, device=dev)
            # the bf16-MFMA attention keeps its dropout bits for the backward (instead of re-hashing
            # every probability's counter twice there): ~12 MB per layer for B = 32's user sequences
            keeps = [K.bert_attn_keep_buffer(s.nseq, s.L, heads, dev)
                     if p_a > 0 and ctx.prec != L.GEMM_F32 and ATTN_KEEP_BITS else None for s in segs]
            for s, r0, kp in zip(segs, r0s, keeps):
                n = s.nseq * s.L
                K.bert_attn_fwd(qkv[r0:r0 + n], heads, s.mask, s.nseq, s.L, cx[r0:r0 + n],
                                ml[r0 * heads * 2:(r0 + n) * heads * 2], keep=kp, **dsite_seg(1 + 3 * li, p_a, r0))
            a = _empty(T, H, word)
            K.gemm(T, H, H, K.operand(cx, L.KCONTIG), K.operand(wo, L.KCONTIG), a, bias=bo)
            h1 = _empty(T, H, word)
            st1 = torch.empty(T, 2, device=dev)
            K.bert_add_ln_fwd(a, x, l1w, l1b, c.layer_norm_eps, h1, st1, **dsite_seg(2 + 3 * li, p_h, 0))
            U = _empty(T, I, word)
            G = _empty(T, I, word)
            K.gemm(T, I, H, K.operand(h1, L.KCONTIG), K.operand(wi, L.KCONTIG), G, bias=bi,
                   epilogue=L.EPI_STORE_GELU, c_rows=K.operand(U, L.KCONTIG))
            o = _empty(T, H, word)
            K.gemm(T, H, I, K.operand(G, L.KCONTIG), K.operand(wo2, L.KCONTIG), o, bias=bo2)
            h2 = _empty(T, H, word)
            st2 = torch.empty(T, 2, device=dev)
            K.bert_add_ln_fwd(o, h1, l2w, l2b, c.layer_norm_eps, h2, st2, **dsite_seg(3 + 3 * li, p_h, 0))
            saved += [x, wqkv, qkv, cx, ml, a, st1, h1, U, G, o, st2]
            keeps_all.append(keeps)
            x = h2
        pooled = _empty(S, H, word)
        K.gemm(S, H, H, K.operand(x, L.KCONTIG, rows=cls_idx, mapping=L.ROWS_GATHER), K.operand(pw, L.KCONTIG),
               pooled, bias=pb, epilogue=L.EPI_STORE_TANH)
        ctx.save_for_backward(*params, st_e, cls_idx, x, pooled, *saved)
        ctx.cfg, ctx.segs, ctx.r0s, ctx.drop = cfg, segs, r0s, drop
        ctx.keeps = keeps_all
        ctx.dsite_seg, ctx.p = dsite_seg, (p_h, p_a)
        ctx.n_params = len(params)
        return x, pooled

    @staticmethod
    @_gemm_backward
    def backward(ctx, dhid, dpooled):
        c = ctx.cfg
        H, heads, I = c.hidden_size, c.num_attention_heads, c.intermediate_size
        nl = c.num_hidden_layers
        sv = ctx.saved_tensors
        npar = ctx.n_params
        params = sv[:npar]
        st_e, cls_idx, hl, pooled = sv[npar:npar + 4]
        saved = sv[npar + 4:]
        word, pos, typ, elw, elb = params[:5]
        lp = [params[5 + 16 * i: 5 + 16 * (i + 1)] for i in range(nl)]
        pw, pb = params[5 + 16 * nl:]
        dev = word.device
        T = hl.shape[0]
        S = pooled.shape[0]
        segs, r0s, dsite_seg = ctx.segs, ctx.r0s, ctx.dsite_seg
        p_h, p_a = ctx.p
        grads = [None] * npar
        z = lambda t: torch.zeros_like(t)   # noqa: E731

        dh = _empty(T, H, word)
        if dhid is not None:
            dh.copy_(dhid)
        else:
            dh.zero_()
        if dpooled is not None:
            dpooled = dpooled.contiguous()
            dpre = _empty(S, H, word)
            K.tanh_bwd(pooled, dpooled, dpre)
            dpw, dpb = z(pw), z(pb)
            _proj_wgrad(dpre, K.operand(hl, L.MNCONTIG, rows=cls_idx, mapping=L.ROWS_GATHER), dpw, dpb, S)
            K.gemm(S, H, H, K.operand(dpre, L.KCONTIG), K.operand(pw, L.MNCONTIG), dh, epilogue=L.EPI_SCATTER,
                   c_rows=K.rows_map(cls_idx, L.ROWS_GATHER), pad_row=-1)
            grads[npar - 2], grads[npar - 1] = dpw, dpb
        for li in reversed(range(nl)):
            x, wqkv, qkv, cx, ml, a, st1, h1, U, G, o, st2 = saved[12 * li: 12 * (li + 1)]
            wq, bq, wk, bk, wv, bv, wo, bo, l1w, l1b, wi, bi, wo2, bo2, l2w, l2b = lp[li]
            # one fill for all 16 gradients of the layer; Q/K/V weight and bias grads are slices of the
            # fused [3H, H] / [3H] wgrad outputs
            dwqkv, dbqkv, *grest = _zeros_views(dev, (3 * H, H), (3 * H,), *[tuple(t.shape) for t in lp[li][6:]])
            g = [dwqkv[:H], dbqkv[:H], dwqkv[H:2 * H], dbqkv[H:2 * H], dwqkv[2 * H:], dbqkv[2 * H:]] + grest
            keep = []   # the layer's transposed weights (DGRAD_KC)
            dh1 = _empty(T, H, word)
            do = _empty(T, H, word)
            K.bert_add_ln_bwd(o, h1, l2w, st2, dh, dh1, do, g[14], g[15], **dsite_seg(3 + 3 * li, p_h, 0))
            dU = _empty(T, I, word)
            K.gemm(T, I, H, K.operand(do, L.KCONTIG), _wdgrad(wo2, keep), dU, epilogue=L.EPI_GELU_GRAD,
                   c_rows=K.operand(U, L.KCONTIG))
            _proj_wgrad(do, K.operand(G, L.MNCONTIG), g[12], g[13], T)
            K.gemm(T, H, I, K.operand(dU, L.KCONTIG), _wdgrad(wi, keep), dh1, epilogue=L.EPI_ACCUM)
            _proj_wgrad(dU, K.operand(h1, L.MNCONTIG), g[10], g[11], T)
            dx = _empty(T, H, word)
            da = _empty(T, H, word)
            K.bert_add_ln_bwd(a, x, l1w, st1, dh1, dx, da, g[8], g[9], **dsite_seg(2 + 3 * li, p_h, 0))
            dcx = _empty(T, H, word)
            K.gemm(T, H, H, K.operand(da, L.KCONTIG), _wdgrad(wo, keep), dcx)
            _proj_wgrad(da, K.operand(cx, L.MNCONTIG), g[6], g[7], T)
            dqkv = _empty(T, 3 * H, word)
            for s, r0, kp in zip(segs, r0s, ctx.keeps[li]):
                n = s.nseq * s.L
                K.bert_attn_bwd(qkv[r0:r0 + n], heads, s.mask, s.nseq, s.L, cx[r0:r0 + n],
                                ml[r0 * heads * 2:(r0 + n) * heads * 2], dcx[r0:r0 + n], dqkv[r0:r0 + n],
                                keep=kp, **dsite_seg(1 + 3 * li, p_a, r0))
            K.gemm(T, H, 3 * H, K.operand(dqkv, L.KCONTIG), _wdgrad(wqkv, keep), dx, epilogue=L.EPI_ACCUM)
            _proj_wgrad(dqkv, K.operand(x, L.MNCONTIG), dwqkv, dbqkv, T)
            for k in range(16):
                grads[5 + 16 * li + k] = g[k]
            dh = dx
        ds = _empty(T, H, word)
        delw, delb, dpos, dtyp = _zeros_views(dev, tuple(elw.shape), tuple(elb.shape), tuple(pos.shape),
                                              tuple(typ.shape))
        ids_all = []
        for s, r0 in zip(segs, r0s):
            n = s.nseq * s.L
            K.bert_embed_bwd(word, pos, typ[0], s.ids, s.nseq, s.L, elw, st_e[r0:r0 + n], dh[r0:r0 + n],
                             ds[r0:r0 + n], delw, delb, **dsite_seg(0, p_h, r0 * H))
            ids_all.append(s.ids)
        dword = table_grad_buffer(word, word.shape[0], word.shape[1], dev, zero=True)   # (dist shard padding)
        K.embedding_bwd(ds, torch.cat(ids_all) if len(ids_all) > 1 else ids_all[0], dword,
                        padding_idx=c.pad_token_id)
        for s, r0 in zip(segs, r0s):
            n = s.nseq * s.L
            K.colsum(ds[r0:r0 + n].view(s.nseq, s.L * H), s.nseq, s.L * H, dpos.view(-1))
        K.colsum(ds, T, H, dtyp[0])
        grads[:5] = [dword, dpos, dtyp, delw, delb]
        return (None, None, None) + tuple(grads)


class BertModel(nn.Module):
    """transformers.BertModel (the parts XFormer / PLM use) on the HIP kernels."""

    def __init__(self, config=None):
        super().__init__()
        self.config = config or BertConfig()
        c = self.config
        if c.hidden_size % c.num_attention_heads or c.hidden_size // c.num_attention_heads != 64:
            raise ValueError("the HIP attention kernels take 64-dim heads (hidden %d / %d heads)"
                             % (c.hidden_size, c.num_attention_heads))
        self.embeddings = BertEmbeddings(c)
        self.encoder = BertEncoder(c)
        self.pooler = BertPooler(c)
        self._init_weights()
        from .encoders import _DropoutStream
        self._rng = _DropoutStream()

    def _init_weights(self):
        """BertPreTrainedModel._init_weights: normal(0, 0.02) weights, zero biases, padding row 0,
        LayerNorm (1, 0)."""
        r = self.config.initializer_range
        with torch.no_grad():
            for m in self.modules():
                if isinstance(m, nn.Linear):
                    m.weight.normal_(0.0, r)
                    m.bias.zero_()
                elif isinstance(m, nn.Embedding):
                    m.weight.normal_(0.0, r)
                    if m.padding_idx is not None:
                        m.weight[m.padding_idx].zero_()
                elif isinstance(m, nn.LayerNorm):
                    m.weight.fill_(1.0)
                    m.bias.zero_()

    def flat_params(self):
        e = self.embeddings
        ps = [e.word_embeddings.weight, e.position_embeddings.weight, e.token_type_embeddings.weight,
              e.LayerNorm.weight, e.LayerNorm.bias]
        for l in self.encoder.layer:
            a = l.attention
            ps += [a.self.query.weight, a.self.query.bias, a.self.key.weight, a.self.key.bias,
                   a.self.value.weight, a.self.value.bias, a.output.dense.weight, a.output.dense.bias,
                   a.output.LayerNorm.weight, a.output.LayerNorm.bias, l.intermediate.dense.weight,
                   l.intermediate.dense.bias, l.output.dense.weight, l.output.dense.bias,
                   l.output.LayerNorm.weight, l.output.LayerNorm.bias]
        ps += [self.pooler.dense.weight, self.pooler.dense.bias]
        return ps

    def _drop_sites(self, T, device):
        c = self.config
        if not self.training or (c.hidden_dropout_prob <= 0 and c.attention_probs_dropout_prob <= 0):
            return None
        H = c.hidden_size
        # counter ranges of the 1 + 3 x layers sites (attention: per (seq, head) keys, q*L + k), taken
        # as ONE snapshot (one nr_rng_take launch per step instead of 37); a site's kernels add its
        # start inside the range to the snapshot's device offset -- the same counters, hence masks,
        # as one take per site
        sizes = [T * H] + [T * 64, T * H, T * H] * c.num_hidden_layers
        seed, off, snap = self._rng.take(sum(sizes), device)
        sites, rel = [], 0
        for n in sizes:
            sites.append((seed, off + rel, snap, rel))
            rel += n
        return sites

    def encode_segments(self, segments):
        """[(input_ids [n, L], attention_mask [n, L]), ...] -> [BertOutput per segment] from ONE
        fused pass (every dense layer runs once over the rows of all segments)."""
        dev = self.embeddings.word_embeddings.weight.device
        segs = []
        for ids, mask in segments:
            L.require_gpu(ids.to(dev))
            segs.append(_Segment(ids.to(dev), mask.to(dev)))
        T = sum(s.nseq * s.L for s in segs)
        hid, pooled = BertFn.apply(self.config, segs, self._drop_sites(T, dev), *self.flat_params())
        outs, r, q = [], 0, 0
        for s in segs:
            n = s.nseq * s.L
            outs.append(BertOutput(hid[r:r + n].view(s.nseq, s.L, -1), pooled[q:q + s.nseq]))
            r += n
            q += s.nseq
        return outs

    def forward(self, input_ids, attention_mask=None):
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        return self.encode_segments([(input_ids, attention_mask)])[0]
