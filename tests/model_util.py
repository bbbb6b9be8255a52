"""Build newsrec_amd models with the golden fixtures' configuration and parameters."""
import torch

from newsrec_amd.manager import ManagerConfig as Cfg, build_model  # noqa: F401


def load_golden_params(model, g):
    """Copy the golden's regenerated parameters into the model by reference state_dict name."""
    sd = model.state_dict()
    with torch.no_grad():
        for n in g.names:
            assert n in sd, "missing %s" % n
            sd[n].copy_(torch.from_numpy(g.params[n]))


def build_bert_model(g, device="cuda"):
    """XFormer / PLM (bert branch) shaped like the golden's reduced BertConfig
    (tests/golden/make_bert_golden.py), parameters copied from the golden's stream."""
    from newsrec_amd.bert import BertConfig
    from newsrec_amd.xformer import PLM, XFormer
    from newsrec_amd import encoders as E
    H = g.hidden
    bc = BertConfig(vocab_size=int(g["meta.vocab"]), hidden_size=H, num_hidden_layers=2,
                    num_attention_heads=g.heads, intermediate_size=512, max_position_embeddings=512,
                    hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = Cfg("bert", g.encU, H, device=device, bert_dim=H)
    m.bert, m.debias = "bert", True
    if g.encU == "xformer":
        model = XFormer(m, bert_config=bc)
    else:
        eu = {"attn": E.Attention_Pooling, "avg": E.Average_Pooling}[g.encU](m)
        model = PLM(m, eu, bert_config=bc)
    model = model.to(device)
    load_golden_params(model, g)
    return model
