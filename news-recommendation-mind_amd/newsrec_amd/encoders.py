"""News and user encoders with the reference's constructors, parameter names, init and
forward signatures (models/Encoders/{CNN,MHA,Pooling,RNN}.py), computing in HIP kernels.

News encoders expose two entry points:
  forward(news_embedding, attn_mask)            the reference contract (embeddings given)
  encode_tokens(table, token_ids, attn_mask)    the fused path TwoTower uses: the embedding
                                                gather is folded into the first GEMM
Both return (token_repr, news_repr) shaped like the reference's.
"""
import math

import torch
from torch import nn

from . import _lib as L
from .attention import MultiheadAttention
from . import functions as F
from .functions import AttnPoolFn, CNNNewsFn, CNNNewsRowsFn, MHAFn, MHANewsFn, RNNUserFn

# fast eval: the MHA user encoder and its pooling in one launch (nr_mha_user_pool_fwd); False runs the
# attention core and the pooling as two launches (the form the parity tests compare it with)
USER_POOL_FUSED = True


def _identity_rows(n, device):
    return torch.arange(n, device=device, dtype=torch.int64)


def _mask_rows(mask, rows):
    m = mask.reshape(rows)
    return m if m.is_contiguous() else m.contiguous()


class _DropoutStream:
    """Stateless counter RNG bookkeeping for the fused dropout: a fixed seed and an offset that
    advances by the number of elements each training forward consumes.  The pair lives on the
    device: each forward snapshots it (the kernels read the snapshot; the backward reuses it)
    and advances it with a device add, so a captured train step replayed as a graph draws a
    fresh mask every replay."""

    def __init__(self):
        self.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFF
        self.offset = 0
        self.state = None

    def take(self, n, device):
        """-> (seed, offset, rng): rng = int64 CUDA (seed, offset) snapshot for the kernels."""
        if self.state is None or self.state.device != device:
            self.state = torch.tensor([self.seed, self.offset], dtype=torch.int64, device=device)
        snap = torch.empty_like(self.state)
        L.call("nr_rng_take", L.ptr(self.state), L.ptr(snap), int(n), L.stream_ptr(self.state))
        off = self.offset
        self.offset += int(n)   # host mirror (eager bookkeeping; replays advance only the device pair)
        return self.seed, off, snap


class CNN_Encoder(nn.Module):
    """models/Encoders/CNN.py:5-50."""

    def __init__(self, manager):
        super().__init__()
        self.hidden_dim = manager.hidden_dim
        self.embedding_dim = manager.bert_dim
        self.cnn = nn.Conv1d(self.embedding_dim, self.hidden_dim, kernel_size=3, padding=1)
        nn.init.xavier_normal_(self.cnn.weight)
        self.query_words = nn.Parameter(torch.randn((1, self.hidden_dim), requires_grad=True))
        nn.init.xavier_normal_(self.query_words)
        self.wordQueryProject = nn.Linear(self.hidden_dim, self.hidden_dim)
        nn.init.xavier_normal_(self.wordQueryProject.weight)
        self.Tanh = nn.Tanh()
        self.Relu = nn.ReLU()

    def _w3(self):
        # Conv1d weight [H, E, 3] -> [H][tap*E + e] (the K = 3E GEMM operand)
        return self.cnn.weight.permute(0, 2, 1).reshape(self.hidden_dim, 3 * self.embedding_dim)

    def _rows_operands(self):
        """The distinct-row path's operands: the conv weight as [3*Hp, E] (row tap*Hp + h =
        weight[h, :, tap]) and the key projection zero-padded to Hp = ceil32(H) (K % 32 == 0)."""
        H = self.hidden_dim
        Hp = (H + 31) // 32 * 32
        return F.CNNWeightsFn.apply(self.cnn.weight, self.wordQueryProject.weight, self.wordQueryProject.bias, Hp)

    def encode_tokens(self, table, token_ids, attn_mask, pad_row=0):
        lead = token_ids.shape[:-1]
        seq_len = token_ids.shape[-1]
        T = token_ids.numel()
        ids = token_ids.reshape(T)
        if F.DEDUP_ROWS:
            w3t, wq, bq, w3tt = self._rows_operands()
            news, tok = CNNNewsRowsFn.apply(table, ids, _mask_rows(attn_mask, T), w3t, self.cnn.bias, wq, bq,
                                            self.query_words, seq_len, pad_row, self.hidden_dim, w3tt)
            return tok.reshape(*lead, seq_len, self.hidden_dim), news.reshape(*lead, self.hidden_dim)
        news, tok = CNNNewsFn.apply(table, ids, _mask_rows(attn_mask, T), self._w3().contiguous(), self.cnn.bias,
                                    self.wordQueryProject.weight, self.wordQueryProject.bias, self.query_words,
                                    seq_len, pad_row)
        return tok.reshape(*lead, seq_len, self.hidden_dim), news.reshape(*lead, self.hidden_dim)

    def forward(self, news_embedding, attn_mask=None):
        L.require_gpu(news_embedding)
        lead = news_embedding.shape[:-2]
        seq_len, e = news_embedding.shape[-2:]
        rows = news_embedding.reshape(-1, e)
        if attn_mask is None:
            attn_mask = torch.ones(lead + (seq_len,), dtype=torch.uint8, device=rows.device)
        return self.encode_tokens(rows.contiguous(), _identity_rows(rows.shape[0], rows.device).view(*lead, seq_len),
                                  attn_mask, pad_row=-1)


class MHA_Encoder(nn.Module):
    """models/Encoders/MHA.py:5-39 (tied-QK 12-head attention, LayerNorm, Dropout, pooling)."""

    def __init__(self, manager):
        super().__init__()
        self.hidden_dim = manager.hidden_dim
        self.embedding_dim = manager.bert_dim
        self.head_num = manager.head_num
        value_dim, x = divmod(self.hidden_dim, self.head_num)
        assert x == 0, "hidden_dim {} must divide head_num {}".format(self.hidden_dim, self.head_num)
        self.mha = MultiheadAttention(self.embedding_dim, self.head_num, value_dim=value_dim)
        self.query_words = nn.Parameter(torch.randn(1, self.hidden_dim))
        self.layerNorm = nn.LayerNorm(self.hidden_dim)
        self.dropOut = nn.Dropout(p=manager.dropout_p)
        self._rng = _DropoutStream()

    def encode_tokens(self, table, token_ids, attn_mask, pad_row=0, want_tokens=False):
        lead = token_ids.shape[:-1]
        seq_len = token_ids.shape[-1]
        T = token_ids.numel()
        p = float(self.dropOut.p) if self.training else 0.0
        seed, off, rng = self._rng.take(T * self.hidden_dim, table.device) if p > 0 else (0, 0, None)
        w, b = self.mha.fused_weight()
        news, tok = MHANewsFn.apply(table, token_ids.reshape(T), _mask_rows(attn_mask, T), w, b,
                                    self.layerNorm.weight, self.layerNorm.bias, self.query_words, self.head_num,
                                    self.mha.key_dim, self.mha.value_dim, seq_len, pad_row, p, seed, off,
                                    want_tokens, rng)
        tok = tok.reshape(*lead, seq_len, self.hidden_dim) if tok is not None else None
        return tok, news.reshape(*lead, self.hidden_dim)

    def forward(self, news_embedding, attn_mask=None):
        L.require_gpu(news_embedding)
        lead = news_embedding.shape[:-2]
        seq_len, e = news_embedding.shape[-2:]
        rows = news_embedding.reshape(-1, e).contiguous()
        if attn_mask is None:
            attn_mask = torch.ones(lead + (seq_len,), dtype=torch.uint8, device=rows.device)
        return self.encode_tokens(rows, _identity_rows(rows.shape[0], rows.device).view(*lead, seq_len),
                                  attn_mask, pad_row=-1, want_tokens=True)


def _his_mask_rows(his_mask, B, N, device):
    """[B, N, 1] (f64, possibly on the CPU as the reference feeds it, TwoTower.py:47) -> [B*N]."""
    m = his_mask.to(device, non_blocking=True).reshape(B * N)
    return m if m.is_contiguous() else m.contiguous()


def _rows_view(news_reprs):
    B, N, H = news_reprs.shape
    x = news_reprs.reshape(B * N, H)
    if x.stride(-1) != 1 or x.stride(0) < H:
        x = x.contiguous()
    return x


class Attention_Pooling(nn.Module):
    """models/Encoders/Pooling.py:5-25."""

    def __init__(self, manager):
        super().__init__()
        self.query_news = nn.Parameter(torch.randn(1, manager.hidden_dim))
        nn.init.xavier_normal_(self.query_news)

    def forward(self, news_reprs, his_mask=None, *args, **kargs):
        L.require_gpu(news_reprs)
        B, N, H = news_reprs.shape
        if his_mask is None:
            mask = torch.ones(B * N, dtype=torch.uint8, device=news_reprs.device)
        else:
            mask = _his_mask_rows(his_mask, B, N, news_reprs.device)
        return AttnPoolFn.apply(_rows_view(news_reprs), self.query_news, mask, B, N).unsqueeze(1)


class Average_Pooling(nn.Module):
    """models/Encoders/Pooling.py:28-42: mean over all N slots (the mask is ignored, as in
    the reference)."""

    def __init__(self, manager):
        super().__init__()

    def forward(self, news_reprs, *args, **kargs):
        return news_reprs.mean(dim=1, keepdim=True)


class MHA_User_Encoder(nn.Module):
    """models/Encoders/MHA.py:42-75.  The pooling mask is transposed to [B,1,N] as
    Attention_Pooling does (the reference passes [B,N,1] and returns [B,N,H], SURVEY
    Appendix A.3).  The reference's unused layerNorm / dropOut are kept as BUFFERS with the
    same state_dict keys, so checkpoints load and DDP sees no unused parameters."""

    def __init__(self, manager):
        super().__init__()
        self.name = "mha-u"
        self.hidden_dim = manager.hidden_dim
        head_num = manager.head_num
        value_dim, x = divmod(self.hidden_dim, head_num)
        assert x == 0, "hidden_dim {} must divide head_num {}".format(self.hidden_dim, head_num)
        self.mha = MultiheadAttention(self.hidden_dim, manager.head_num, value_dim=value_dim)
        self.query_news = nn.Parameter(torch.randn(1, self.hidden_dim))
        ln = nn.Module()
        ln.register_buffer("weight", torch.ones(self.hidden_dim))
        ln.register_buffer("bias", torch.zeros(self.hidden_dim))
        self.layerNorm = ln
        self.dropOut = nn.Dropout(p=manager.dropout_p)

    def forward(self, news_repr, his_mask=None, **kargs):
        L.require_gpu(news_repr)
        B, N, H = news_repr.shape
        if his_mask is None:
            mask = torch.ones(B * N, dtype=torch.uint8, device=news_repr.device)
        else:
            mask = _his_mask_rows(his_mask, B, N, news_repr.device)
        w, b = self.mha.fused_weight()
        h = MHAFn.apply(_rows_view(news_repr), mask, w, b, B, N, self.mha.head_num, self.mha.key_dim,
                        self.mha.value_dim)
        return AttnPoolFn.apply(h, self.query_news, mask, B, N).unsqueeze(1)

    @torch.no_grad()
    def project_rows(self, x):
        """keyProject / valueProject (Attention.py:107-108) of every row of x [R, H] ->
        [R, heads*(dk+dv)].  Fast eval projects the news table once; forward_rows gathers."""
        from . import kernels as K
        w, b = self.mha.fused_weight()
        x = x if x.stride(-1) == 1 and x.stride(0) % 4 == 0 else x.contiguous()
        Y = torch.empty(x.shape[0], w.shape[0], device=x.device)
        K.gemm(x.shape[0], w.shape[0], x.shape[1], K.operand(x, L.KCONTIG), K.operand(w, L.KCONTIG), Y, bias=b)
        return Y

    @torch.no_grad()
    def forward_rows(self, Y, rows, his_mask, B, N):
        """forward() (eval, no autograd) with the projections precomputed per distinct news:
        history slot t reads Y[rows[t]] inside the attention kernel.  Same per-row GEMM, so the
        result equals forward(table[rows])."""
        from . import kernels as K
        mha = self.mha
        mask = _his_mask_rows(his_mask, B, N, Y.device)
        NQ = mha.head_num * mha.key_dim
        if USER_POOL_FUSED and K.mha_user_pool_supported(N, mha.head_num, mha.key_dim, mha.value_dim):
            # attention + pooling in one launch per impression (the attention output never leaves the CU)
            out = torch.empty(B, mha.head_num * mha.value_dim, device=Y.device)
            K.mha_user_pool_fwd(Y, rows.reshape(-1).contiguous(), mask, B, N, mha.head_num, mha.key_dim,
                                mha.value_dim, self.query_news.reshape(-1).contiguous(), out)
            return out.unsqueeze(1)
        O = torch.empty(B * N, mha.head_num * mha.value_dim, device=Y.device)
        K.mha_attn_fwd(Y[:, :NQ], Y[:, NQ:], mask, B, N, mha.head_num, mha.key_dim, mha.value_dim, O,
                       rows=rows.reshape(-1).contiguous())
        return AttnPoolFn.apply(O, self.query_news, mask, B, N).unsqueeze(1)


class RNN_User_Encoder(nn.Module):
    """models/Encoders/RNN.py:36-73 (LSTM or GRU, packed by the history length)."""

    def __init__(self, manager):
        super().__init__()
        self.hidden_dim = manager.hidden_dim
        self.descend_history = manager.descend_history
        self.cell = L.CELL_GRU if manager.encoderU == "gru" else L.CELL_LSTM
        if manager.encoderU == "gru":
            self.rnn = nn.GRU(self.hidden_dim, self.hidden_dim, batch_first=True)
        elif manager.encoderU == "lstm":
            self.rnn = nn.LSTM(self.hidden_dim, self.hidden_dim, batch_first=True)
        for name, param in self.rnn.named_parameters():
            if "weight" in name:
                nn.init.orthogonal_(param)

    def forward(self, news_repr, **kwargs):
        L.require_gpu(news_repr)
        B, N, H = news_repr.shape
        mask = _his_mask_rows(kwargs["his_mask"], B, N, news_repr.device) if "his_mask" in kwargs else None
        r = self.rnn
        h = RNNUserFn.apply(_rows_view(news_repr), r.weight_ih_l0, r.weight_hh_l0, r.bias_ih_l0, r.bias_hh_l0,
                            None, self.cell, mask, B, N, bool(self.descend_history), None)
        return h.unsqueeze(1)


class LSTUR_User_Encoder(nn.Module):
    """models/Encoders/RNN.py:76-104: LSTM over the flipped history, h0 = userEmbedding[u] with
    u = Bernoulli(0.5) * user id (the id drop applies in eval too, as in the reference).
    Accepts ``user_index`` (the reference's name) or ``user_id`` (what TwoTower passes)."""

    def __init__(self, manager):
        super().__init__()
        self.hidden_dim = manager.hidden_dim
        self.rnn = nn.LSTM(self.hidden_dim, self.hidden_dim, batch_first=True)
        self.userEmbedding = nn.Embedding(manager.get_user_num() + 1, self.hidden_dim)
        nn.init.zeros_(self.userEmbedding.weight[0])
        for name, param in self.rnn.named_parameters():
            if "weight" in name:
                nn.init.orthogonal_(param)
        self.keep_override = None   # tests: an injected Bernoulli draw

    def forward(self, news_repr, his_mask=None, user_index=None, user_id=None):
        L.require_gpu(news_repr)
        if user_index is None:
            user_index = user_id
        B, N, H = news_repr.shape
        user_index = user_index.to(news_repr.device)
        if self.keep_override is not None:
            keep = self.keep_override.to(news_repr.device, torch.long)
        else:
            keep = torch.zeros(B, dtype=torch.long, device=news_repr.device).bernoulli_()
        u = (keep * user_index).contiguous()
        r = self.rnn
        h = RNNUserFn.apply(_rows_view(news_repr), r.weight_ih_l0, r.weight_hh_l0, r.bias_ih_l0, r.bias_hh_l0,
                            self.userEmbedding.weight, L.CELL_LSTM, None, B, N, True, u)
        return h.unsqueeze(1)
