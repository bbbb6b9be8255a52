"""models/Embeddings/BERT.py: the BERT word-embedding table as a drop-in module.

The reference loads ``bert-base-uncased``'s ``embeddings.word_embeddings`` by name
(BERT.py:16-21), which needs the network.  Here the table is an ``nn.Embedding(30522, 768,
padding_idx=0)`` (same module type, same state_dict key ``bert_word_embedding.weight``),
initialised N(0, 0.02²) like BERT's initializer unless a pretrained tensor is given.
"""
import torch
from torch import nn

from . import _lib as L
from .functions import EmbeddingFn

BERT_VOCAB = 30522


class BERT_Embedding(nn.Module):
    def __init__(self, manager, vocab_size=BERT_VOCAB, weight=None):
        super().__init__()
        self.hidden_dim = manager.bert_dim
        self.bert_word_embedding = nn.Embedding(vocab_size, self.hidden_dim, padding_idx=0)
        with torch.no_grad():
            if weight is not None:
                self.bert_word_embedding.weight.copy_(weight)
            else:
                self.bert_word_embedding.weight.normal_(0.0, 0.02)

    @property
    def table(self):
        return self.bert_word_embedding.weight

    def forward(self, news_batch):
        """[batch, *, L] int64 -> [batch, *, L, E] (BERT.py:24-40; the 4-D bag-of-words branch
        of the reference needs a ``freq_embedding`` that never exists and is not supported)."""
        L.require_gpu(news_batch)
        if news_batch.dim() == 4:
            raise NotImplementedError("bag-of-words input (BERT.py:35-36) has no freq_embedding")
        ids = news_batch.reshape(-1)
        ids = ids if ids.is_contiguous() else ids.contiguous()
        out = EmbeddingFn.apply(self.table, ids, self.bert_word_embedding.padding_idx)
        return out.view(*news_batch.shape, self.hidden_dim)
