"""Throughput probe of the BERT towers (XFormer / PLM, bert-base, 12 layers, dropout 0.1) on
synthetic MIND-large-shaped batches: train step (fwd + NLL + bwd + Adam) and eval forward.

    python tools/bench_bert.py [--model xformer|plm] [--batch 32] [--steps 5] [--warmup 2] [--layers 12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def synth(gen, B, C=5, N=50, Lt=30, V=30522):
    def titles(n):
        t = torch.randint(1000, V, (n, Lt), generator=gen)
        t[:, 0] = 101
        t[:, -1] = 102
        return t, torch.ones(n, Lt, dtype=torch.long)
    ct, cm = titles(B * C)
    ht, hm = titles(B * N)
    return {"cdd_encoded_index": ct.view(B, C, Lt), "cdd_attn_mask": cm.view(B, C, Lt),
            "his_encoded_index": ht.view(B, N, Lt), "his_attn_mask": hm.view(B, N, Lt),
            "his_mask": torch.ones(B, N, 1, dtype=torch.float64), "user_id": torch.randint(1, 1000, (B,)),
            "label": torch.zeros(B, dtype=torch.long)}


def build(kind, layers, dev):
    from newsrec_amd.bert import BertConfig
    from newsrec_amd.manager import ManagerConfig
    from newsrec_amd.xformer import PLM, XFormer
    from newsrec_amd import encoders as E
    torch.manual_seed(42)
    bc = BertConfig(num_hidden_layers=layers)
    m = ManagerConfig("bert", "attn", 768, bert_dim=768)
    if kind == "xformer":
        return XFormer(m, bert_config=bc).to(dev)
    return PLM(m, E.Attention_Pooling(m), bert_config=bc).to(dev)


def flops_per_impression(kind, layers, C=5, N=50, Lt=30):
    """Algorithmic forward FLOPs (dense layers 2*7.08 M MAC-weights per token per layer + attention
    4*L^2*768 per sequence per layer + pooler)."""
    dense = 2 * (4 * 768 * 768 + 2 * 768 * 3072) * layers
    if kind == "xformer":
        seqs = [(Lt, C), (501, 1)]
    else:
        seqs = [(Lt, C + N)]
    f = 0
    for L, n in seqs:
        f += n * (L * dense + layers * 4 * L * L * 768 + 2 * 768 * 768)
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xformer", choices=["xformer", "plm"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layers", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from newsrec_amd.manager import get_optim
    model = build(a.model, a.layers, dev)
    opt = get_optim(model)
    gen = torch.Generator().manual_seed(0)
    x = {k: v.to(dev) for k, v in synth(gen, a.batch).items()}

    def step():
        opt.zero_grad(set_to_none=True)
        logits, _ = model(x)
        loss = torch.nn.functional.nll_loss(logits, x["label"])
        loss.backward()
        opt.step()
        return loss
    model.train()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    model.eval()
    with torch.no_grad():
        model(x)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(a.steps):
            model(x)
        torch.cuda.synchronize()
        ev = (time.perf_counter() - t1) / a.steps
    f = flops_per_impression(a.model, a.layers) * a.batch
    print(json.dumps({"model": a.model, "layers": a.layers, "batch": a.batch, "train_ms": round(el * 1e3, 2),
                      "train_impr_per_s": round(a.batch / el, 1), "train_tflops": round(3 * f / el / 1e12, 1),
                      "eval_ms": round(ev * 1e3, 2), "eval_impr_per_s": round(a.batch / ev, 1),
                      "eval_tflops": round(f / ev / 1e12, 1), "loss": float(loss),
                      "mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
