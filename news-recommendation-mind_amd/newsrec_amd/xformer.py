"""models/XFormer.py and models/PLM.py (the BERT branch) on the HIP BERT tower.

Both keep the reference's constructors (a ``manager``), attribute and parameter names
(``bert.*``, ``userBias``, ``encoderU.*``; state_dicts load unchanged), and methods
(``encode_news``, ``encode_user``, ``forward`` via TwoTowerBaseModel).  ``forward`` runs the
candidate titles and the user side through ONE fused BERT pass (``BertModel.encode_segments``).

Out of scope: the reformer / longformer / bigbird / deberta / funnel /
synthesizer / distill / newsbert variants (XFormer.py:19-41, PLM.py:20-78) — only ``bert``.
"""
import torch
from torch import nn

from .bert import BertConfig, BertModel
from .twotower import TwoTowerBaseModel

# Manager.get_max_length_for_truncating (utils/Manager.py:1013-1027), "bert" entry
MAX_LENGTH = {"bert": (512, 10)}


def _bert_for(manager, bert, bert_config):
    name = getattr(manager, "bert", "bert")
    if name != "bert":
        raise NotImplementedError("only the 'bert' tower is built (got %r)" % name)
    if bert is not None:
        return bert
    if bert_config is None:
        bert_config = BertConfig(hidden_size=manager.bert_dim, num_attention_heads=manager.bert_dim // 64)
    return BertModel(bert_config)


def _user_bias(manager):
    if not getattr(manager, "debias", True):
        return None
    p = nn.Parameter(torch.randn(1, manager.bert_dim))
    nn.init.xavier_normal_(p)
    return p


class XFormer(TwoTowerBaseModel):
    """models/XFormer.py:8-100 (bert branch): one-tower user modelling — the user is BERT's
    pooler output over [CLS] + the first 10 tokens of each history title (501 tokens)."""

    def __init__(self, manager, bert=None, bert_config=None):
        super().__init__(manager)
        self.bert_name = getattr(manager, "bert", "bert")
        self.max_length, self.max_length_per_history = MAX_LENGTH[self.bert_name]
        self.bert = _bert_for(manager, bert, bert_config)
        ub = _user_bias(manager)
        if ub is not None:
            self.userBias = ub
        manager.name = "__".join(["xformer", self.bert_name])
        self.name = manager.name

    def _dev(self):
        return self.bert.embeddings.word_embeddings.weight.device

    def user_tokens(self, x):
        """XFormer.py:80-89: [CLS] + his[:, :, 1:11] flattened, cut to max_length - 1."""
        dev = self._dev()
        his = x["his_encoded_index"].to(dev, non_blocking=True)
        hm = x["his_attn_mask"].to(dev, non_blocking=True)
        B = his.shape[0]
        k = self.max_length_per_history
        t = his[:, :, 1:k + 1].reshape(B, -1)[:, :self.max_length - 1]
        m = hm[:, :, 1:k + 1].reshape(B, -1)[:, :self.max_length - 1]
        return torch.cat([his[:, 0, :1], t], -1), torch.cat([hm[:, 0, :1], m], -1)

    def _cdd(self, x):
        dev = self._dev()
        c = x["cdd_encoded_index"].to(dev, non_blocking=True)
        return c.reshape(-1, c.shape[-1]), x["cdd_attn_mask"].to(dev, non_blocking=True).reshape(-1, c.shape[-1])

    def _finish_user(self, pooled):
        user = pooled.unsqueeze(1)
        if hasattr(self, "userBias"):
            user = user + self.userBias
        return user

    def encode_news(self, x):
        """XFormer.py:59-77."""
        B = x["cdd_encoded_index"].shape[0]
        return self.bert(*self._cdd(x)).pooler_output.view(B, -1, self.hidden_dim)

    def encode_user(self, x):
        """XFormer.py:80-100."""
        return self._finish_user(self.bert(*self.user_tokens(x)).pooler_output), None

    def _encode_both(self, x):
        B = x["cdd_encoded_index"].shape[0]
        oc, ou = self.bert.encode_segments([self._cdd(x), self.user_tokens(x)])
        return oc.pooler_output.view(B, -1, self.hidden_dim), self._finish_user(ou.pooler_output), None


class PLM(TwoTowerBaseModel):
    """models/PLM.py:8-132 (bert branch): every title through BERT (pooler output), an L3 user
    encoder over the history vectors, + userBias.  With a news table installed
    (init_embedding, the fast-eval path) the history is read from it (PLM.py:95-97)."""

    def __init__(self, manager, encoderU, bert=None, bert_config=None):
        super().__init__(manager)
        self.encoderU = encoderU
        ub = _user_bias(manager)
        if ub is not None:
            self.userBias = ub
        self.bert = _bert_for(manager, bert, bert_config)
        manager.name = "__".join(["plm", getattr(manager, "bert", "bert"), manager.encoderU])
        self.name = manager.name

    def _dev(self):
        return self.bert.embeddings.word_embeddings.weight.device

    def _titles(self, x, key):
        dev = self._dev()
        t = x[key + "_encoded_index"].to(dev, non_blocking=True)
        m = x[key + "_attn_mask"].to(dev, non_blocking=True)
        return t.reshape(-1, t.shape[-1]), m.reshape(-1, t.shape[-1])

    def encode_news(self, x):
        """PLM.py:89-104."""
        B = x["cdd_encoded_index"].shape[0]
        return self.bert(*self._titles(x, "cdd")).pooler_output.view(B, -1, self.hidden_dim)

    def _user(self, his, x):
        dev = his.device
        user = self.encoderU(his, his_mask=x["his_mask"], user_id=x["user_id"].to(dev) if "user_id" in x else None)
        if hasattr(self, "userBias"):
            user = user + self.userBias
        return user

    def encode_user(self, x):
        """PLM.py:107-132."""
        B = x["his_encoded_index"].shape[0]
        if self.news_reprs is not None:
            his = self.news_reprs(x["his_id"].to(self._dev()))
        else:
            his = self.bert(*self._titles(x, "his")).pooler_output.view(B, -1, self.hidden_dim)
        return self._user(his, x), None

    def _encode_both(self, x):
        if self.news_reprs is not None:
            return super()._encode_both(x)
        B, C = x["cdd_encoded_index"].shape[:2]
        ct, cm = self._titles(x, "cdd")
        ht, hm = self._titles(x, "his")
        # candidates and history share L: one segment, one pass
        out = self.bert.encode_segments([(torch.cat([ct, ht], 0), torch.cat([cm, hm], 0))])[0]
        pooled = out.pooler_output
        cdd = pooled[:B * C].view(B, C, self.hidden_dim)
        his = pooled[B * C:].view(B, -1, self.hidden_dim)
        return cdd, self._user(his, x), None
