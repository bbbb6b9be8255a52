"""Model assembly and train-step plumbing mirroring twotower.py:7-59 and utils/Manager.py.

``ManagerConfig`` carries the attributes the reference's model constructors read from its
``Manager`` (Manager.py:38-147, defaults as its argparse block); ``build_model`` is
twotower.py's encoder dispatch (:17-47); ``get_optim`` is Manager._get_optim (:389-422)
on the HIP Adam; ``train_step`` is one iteration of Manager._train (:636-647).
"""
import torch

USER_NUM = {"demo": 2146, "small": 94057, "large": 876956, "whole": 876956}       # Manager.py:874-881
NEWS_NUM = {"demo": 42416, "small": 42416, "large": 72023, "whole": 72023}        # Manager.py:884-914 (dev)


class ManagerConfig:
    def __init__(self, encoderN="cnn", encoderU="lstm", hidden_dim=150, scale="large", mode="train",
                 device="cuda", dropout_p=0.2, head_num=12, his_size=50, signal_length=30, npratio=4,
                 bert_dim=768, descend_history=False, user_num=None, lr=1e-4, bert_lr=6e-6):
        self.scale = scale; self.mode = mode; self.npratio = npratio; self.cdd_size = npratio + 1
        self.impr_size = 2000; self.batch_size_news = 500
        self.his_size = his_size; self.signal_length = signal_length; self.device = device
        self.bert_dim = bert_dim; self.embedding_dim = bert_dim; self.hidden_dim = hidden_dim
        self.head_num = head_num; self.dropout_p = dropout_p; self.descend_history = descend_history
        self.encoderN = encoderN; self.encoderU = encoderU
        self.user_num = USER_NUM[scale] if user_num is None else user_num
        self.lr = lr; self.bert_lr = bert_lr

    def get_user_num(self):
        return self.user_num

    def get_news_num(self):
        return NEWS_NUM[self.scale]


PRECISIONS = {"f32": 0, "bf16x6": 1, "bf16": 2}   # enum nr_gemm_precision


def build_model(encN, encU, hidden, vocab=30522, device="cuda", user_num=40, dropout_p=0.0, cfg=None,
                precision=None):
    """twotower.py:17-47 dispatch (incl. the 'lstur' choice whose import is broken in the
    reference, twotower.py:44 / SURVEY Appendix A.2).  ``precision``: the model's GEMM arithmetic
    ("f32", "bf16x6" or "bf16"; None = NR_GEMM_PREC, default bf16x6)."""
    from .embedding import BERT_Embedding
    from . import encoders as E
    from .twotower import TwoTower
    m = cfg or ManagerConfig(encN, encU, hidden, device=device, dropout_p=dropout_p, user_num=user_num)
    emb = BERT_Embedding(m, vocab_size=vocab)
    en = E.CNN_Encoder(m) if encN == "cnn" else E.MHA_Encoder(m)
    eu = {"attn": E.Attention_Pooling, "avg": E.Average_Pooling, "lstm": E.RNN_User_Encoder,
          "gru": E.RNN_User_Encoder, "lstur": E.LSTUR_User_Encoder, "mha": E.MHA_User_Encoder}[encU](m)
    model = TwoTower(m, emb, en, eu).to(device)
    if precision is not None:
        model.gemm_prec = PRECISIONS[precision]
    return model


def get_optim(model, lr=1e-4, bert_lr=6e-6, capturable=False):
    """Manager._get_optim: names containing 'bert' -> bert_lr, the rest -> lr.  ``capturable``:
    step counts on the device (the step can be captured in a graph)."""
    from .optim import FusedAdam
    import re
    base, bert = [], []
    for name, p in model.named_parameters():
        (bert if re.search("bert", name) else base).append(p)
    return FusedAdam([{"params": base, "lr": lr}, {"params": bert, "lr": bert_lr}], capturable=capturable)


def train_step(model, optimizer, x, grad_sync=None, check_labels=True):
    """Manager._train :636-647 (zero_grad(set_to_none), forward, NLLLoss, backward, step);
    ``grad_sync`` averages gradients over data-parallel ranks before the step.  ``check_labels``: raise,
    as torch's NLLLoss does, when the fused head saw a label outside [0, C) (its sticky status word;
    reading it synchronises, as the reference's per-step ``float(loss)`` at Manager.py:642 does)."""
    optimizer.zero_grad(set_to_none=True)
    if hasattr(model, "forward_loss") and model.training:
        loss = model.forward_loss(x)[1]   # NLLLoss fused into the head (same numbers)
        if check_labels:
            from . import kernels as K
            if K.score_nll_status(loss.device):
                raise IndexError("NLLLoss: a label is outside [0, C) and not the ignored -100")
    else:
        logits = model(x)[0]
        loss = torch.nn.functional.nll_loss(logits, x["label"].to(logits.device))
    loss.backward()
    scale = grad_sync() if grad_sync is not None else 1.0
    if scale != 1.0 and not hasattr(optimizer, "sync_lr"):
        # a torch optimizer: DDP's mean by hand (FusedAdam folds it into its kernel)
        with torch.no_grad():
            for g in optimizer.param_groups:
                for p in g["params"]:
                    if p.grad is not None:
                        p.grad.mul_(scale)
        scale = 1.0
    if scale != 1.0:
        optimizer.step(grad_scale=scale)
    else:
        optimizer.step()
    if grad_sync is not None:
        grad_sync.after_step()   # sharded tables: gather the updated slabs (no-op otherwise)
    return loss
