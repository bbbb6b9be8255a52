"""Build newsrec_amd models with the golden fixtures' configuration and parameters."""
import torch


class Cfg:
    """The Manager attributes the model constructors read (utils/Manager.py:38-147)."""

    def __init__(self, encN, encU, hidden, device="cuda", user_num=40, dropout_p=0.0):
        self.scale = "demo"; self.mode = "train"; self.cdd_size = 5
        self.impr_size = 2000; self.batch_size_news = 500
        self.his_size = 50; self.signal_length = 30; self.device = device
        self.bert_dim = 768; self.embedding_dim = 768; self.hidden_dim = hidden
        self.head_num = 12; self.dropout_p = dropout_p; self.descend_history = False
        self.encoderN = encN; self.encoderU = encU
        self.user_num = user_num

    def get_user_num(self):
        return self.user_num


def build_model(encN, encU, hidden, vocab=30522, device="cuda", user_num=40, dropout_p=0.0):
    from newsrec_amd.embedding import BERT_Embedding
    from newsrec_amd import encoders as E
    from newsrec_amd.twotower import TwoTower
    m = Cfg(encN, encU, hidden, device, user_num, dropout_p)
    emb = BERT_Embedding(m, vocab_size=vocab)
    en = E.CNN_Encoder(m) if encN == "cnn" else E.MHA_Encoder(m)
    eu = {"attn": E.Attention_Pooling, "avg": E.Average_Pooling, "lstm": E.RNN_User_Encoder,
          "gru": E.RNN_User_Encoder, "lstur": E.LSTUR_User_Encoder, "mha": E.MHA_User_Encoder}[encU](m)
    return TwoTower(m, emb, en, eu).to(device)


def load_golden_params(model, g):
    """Copy the golden's regenerated parameters into the model by reference state_dict name."""
    sd = model.state_dict()
    with torch.no_grad():
        for n in g.names:
            assert n in sd, "missing %s" % n
            sd[n].copy_(torch.from_numpy(g.params[n]))
