"""models/TwoTowerBaseModel.py + models/TwoTower.py with the same methods and semantics.

Fast path (both towers' news through one fused launch sequence): when the embedding is this
package's BERT_Embedding and the news encoder has ``encode_tokens``, candidate and history
titles are concatenated into ONE token batch, the gather is fused into the encoder's first
GEMM, and the scorer + head is one kernel.  Otherwise the reference composition
``encoderN(embedding(tokens), mask)`` runs (still on the HIP kernels).
"""
import contextlib
import math

import torch
from torch import nn

from . import _lib as L
from . import kernels as K
from .attention import _joined_view
from .functions import GRAD_DEST, ScoreFn, ScoreNLLFn, SplitRowsFn


class TwoTowerBaseModel(nn.Module):
    """models/TwoTowerBaseModel.py:6-83."""

    def __init__(self, manager):
        super().__init__()
        self.scale = manager.scale
        self.cdd_size = manager.cdd_size
        self.mode = "test" if manager.mode == "test" else "dev"
        self.impr_size = manager.impr_size
        self.batch_size_news = manager.batch_size_news
        self.encoding = False
        self.his_size = manager.his_size
        self.signal_length = manager.signal_length
        self.device = manager.device
        self.hidden_dim = manager.bert_dim
        self.news_reprs = None
        # GEMM arithmetic of this model's forward AND backward (the autograd Functions record it):
        # None = the thread default (NR_GEMM_PREC, bf16x6); L.GEMM_BF16 = the bf16 configuration
        self.gemm_prec = None

    def arithmetic(self):
        return K.gemm_precision(self.gemm_prec) if self.gemm_prec is not None else contextlib.nullcontext()

    def init_encoding(self):
        self.encoding = True

    def init_embedding(self, news_table=None):
        """TwoTowerBaseModel.py:34-39.  The reference reloads news.pt from disk; a table
        produced in memory (Manager.encode_news_table) can be passed directly."""
        if news_table is None:
            path = "data/cache/tensors/{}/{}/{}/news.pt".format(self.name, self.scale, self.mode)
            news_table = torch.load(path, map_location=torch.device(self.device), weights_only=True)
        self.news_reprs = nn.Embedding.from_pretrained(news_table)

    def destroy_encoding(self):
        self.encoding = False

    def destroy_embedding(self):
        self.news_reprs = None

    def compute_score(self, cdd_news_repr, user_repr, mode=L.SCORE_RAW):
        """[B, C, H] x [B, 1, H] -> [B, C] scores / sqrt(H) (TwoTowerBaseModel.py:51-62),
        optionally with the log_softmax / sigmoid head fused."""
        B, C, H = cdd_news_repr.shape
        cdd = cdd_news_repr.reshape(B * C, H)
        user = user_repr.reshape(B, H)
        if cdd.stride(-1) != 1:
            cdd = cdd.contiguous()
        if user.stride(-1) != 1:
            user = user.contiguous()
        return ScoreFn.apply(cdd, user, B, C, mode)

    def forward(self, x):
        """TwoTowerBaseModel.py:65-75: (log_softmax logits when training, sigmoid otherwise, kid)."""
        try:
            with self.arithmetic():
                cdd_repr, user_repr, kid = self._encode_both(x)
                mode = L.SCORE_LOG_SOFTMAX if self.training else L.SCORE_SIGMOID
                return self.compute_score(cdd_repr, user_repr, mode), kid
        finally:
            GRAD_DEST.clear()   # the split's gradient offers are good for this forward only

    def forward_loss(self, x):
        """Training forward with the loss of Manager._train (utils/Manager.py:641, NLLLoss on
        forward(x)'s log-softmax logits) fused into the head: -> (logits, loss).  The same numbers
        as ``nll_loss(self(x)[0], x["label"])``, one kernel each way instead of three and two."""
        if not self.training:
            raise RuntimeError("forward_loss is the training head (log-softmax logits)")
        try:
            with self.arithmetic():
                cdd_repr, user_repr, _ = self._encode_both(x)
                B, C, H = cdd_repr.shape
                cdd = cdd_repr.reshape(B * C, H)
                user = user_repr.reshape(B, H)
                if cdd.stride(-1) != 1:
                    cdd = cdd.contiguous()
                if user.stride(-1) != 1:
                    user = user.contiguous()
                return ScoreNLLFn.apply(cdd, user, B, C, x["label"])
        finally:
            GRAD_DEST.clear()   # an offer no consumer took must not outlive this forward

    def _encode_both(self, x):
        cdd_repr = self.encode_news(x)
        user_repr, kid = self.encode_user(x)
        return cdd_repr, user_repr, kid

    def predict_fast(self, x):
        """TwoTowerBaseModel.py:78-83: candidates gathered from the news table inside the
        scorer kernel, the user encoded in full."""
        with self.arithmetic():
            user_repr, _ = self.encode_user(x)
        cdd_id = x["cdd_id"].to(user_repr.device)
        if cdd_id.dim() == 1:
            cdd_id = cdd_id.unsqueeze(0)
        B, C = cdd_id.shape
        H = user_repr.shape[-1]
        from . import kernels as K
        logits = torch.empty(B, C, device=user_repr.device)
        user = user_repr.reshape(B, H)
        if user.stride(-1) != 1:
            user = user.contiguous()
        ids = cdd_id.reshape(-1).contiguous()
        K.score_fwd(self.news_reprs.weight, user, B, C, H, L.SCORE_SIGMOID, logits, cdd_idx=ids)
        return logits


class TwoTower(TwoTowerBaseModel):
    """models/TwoTower.py:4-49."""

    def __init__(self, manager, embedding, encoderN, encoderU):
        super().__init__(manager)
        self.embedding = embedding
        self.encoderN = encoderN
        self.encoderU = encoderU
        self.hidden_dim = manager.hidden_dim
        manager.name = "__".join(["twotower", manager.encoderN, manager.encoderU])
        self.name = manager.name

    def _dev(self):
        return next(self.parameters()).device

    def _fused(self):
        return hasattr(self.encoderN, "encode_tokens") and hasattr(self.embedding, "table")

    def _news(self, tokens, mask):
        dev = self._dev()
        tokens = tokens.to(dev, non_blocking=True)
        mask = mask.to(dev, non_blocking=True)
        if self._fused():
            return self.encoderN.encode_tokens(self.embedding.table, tokens, mask)[1]
        return self.encoderN(self.embedding(tokens), mask)[1]

    def encode_news(self, x):
        """TwoTower.py:21-33."""
        with self.arithmetic():
            return self._news(x["cdd_encoded_index"], x["cdd_attn_mask"])

    def _user_from_his(self, his_news_repr, x):
        dev = his_news_repr.device
        return self.encoderU(his_news_repr, his_mask=x["his_mask"], user_id=x["user_id"].to(dev))

    def encode_user(self, x):
        """TwoTower.py:36-49."""
        with self.arithmetic():
            his = self._news(x["his_encoded_index"], x["his_attn_mask"])
            return self._user_from_his(his, x), None

    def _encode_both(self, x):
        if not self._fused():
            return super()._encode_both(x)
        dev = self._dev()
        cdd_t = x["cdd_encoded_index"].to(dev, non_blocking=True)
        his_t = x["his_encoded_index"].to(dev, non_blocking=True)
        B, C, Lq = cdd_t.shape
        N = his_t.shape[1]
        cdd_m = x["cdd_attn_mask"].to(dev, non_blocking=True)
        his_m = x["his_attn_mask"].to(dev, non_blocking=True)
        # one encoder pass over candidates + history: the device batch former lays both out back to
        # back (joined views, no copy); other callers' batches are stacked
        tokens = _joined_view(cdd_t.reshape(B * C, Lq), his_t.reshape(B * N, Lq))
        if tokens is None:
            tokens = torch.cat([cdd_t.reshape(B * C, Lq), his_t.reshape(B * N, Lq)], 0)
        masks = _joined_view(cdd_m.reshape(B * C, Lq), his_m.reshape(B * N, Lq))
        if masks is None:
            masks = torch.cat([cdd_m.reshape(B * C, Lq), his_m.reshape(B * N, Lq)], 0)
        news = self.encoderN.encode_tokens(self.embedding.table, tokens, masks)[1]
        # split, not two slices (two slices' backwards would zero-fill and copy a full-size gradient
        # each, then add them); SplitRowsFn's consumers write their input gradients straight into
        # its joined gradient buffer, so the join costs no copy either
        cdd, his = SplitRowsFn.apply(news, B * C)
        cdd = cdd.reshape(B, C, -1)
        his = his.reshape(B, N, -1)
        return cdd, self._user_from_his(his, x), None
