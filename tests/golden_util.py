"""Load a golden fixture written by tests/golden/make_golden.py and regenerate its
parameters from the seeded stream (tests/golden/params.py)."""
import os

import numpy as np
import torch

from params import regen_params

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONFIG_ENCODERS = {
    "cnn_attn": ("cnn", "attn"), "cnn_avg": ("cnn", "avg"), "cnn_lstm": ("cnn", "lstm"),
    "cnn_gru": ("cnn", "gru"), "cnn_lstur": ("cnn", "lstur"), "nrms": ("mha", "mha"),
}
# BERT-tower goldens (tests/golden/make_bert_golden.py): XFormer (one-tower user sequence) and
# PLM (bert branch) with an Attention_Pooling user encoder.
BERT_CONFIGS = {"xformer": ("bert", "xformer"), "plm": ("bert", "attn")}


class Golden:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"))
        self.z = {k: z[k] for k in z.files}
        self.names = [k[len("grad."):] for k in z.files if k.startswith("grad.")]
        shapes = [(n, self.z["grad." + n].shape) for n in self.names]
        self.params = regen_params(shapes, int(self.z["meta.seed"]))
        self.encN, self.encU = {**CONFIG_ENCODERS, **BERT_CONFIGS}[name]
        self.heads = int(self.z["meta.heads"]) if "meta.heads" in self.z else 12
        self.hidden = int(self.z["meta.hidden_dim"])
        for n in self.names:
            p = self.params[n].astype(np.float64)
            want = self.z["pcheck." + n]
            got = np.asarray([p.sum(), np.abs(p).sum()])
            assert np.allclose(got, want, rtol=1e-6, atol=1e-6), f"param stream drift on {n}"

    def inputs(self, device="cpu"):
        x = {}
        for k, v in self.z.items():
            if k.startswith("in."):
                x[k[3:]] = torch.from_numpy(v).to(device)
        return x

    def torch_params(self, device="cpu", requires_grad=False):
        return {n: torch.tensor(self.params[n], device=device, requires_grad=requires_grad)
                for n in self.names}

    def __getitem__(self, k):
        return self.z[k]
