"""GEMM throughput, exact-f32 MFMA vs bf16x6, on the step's shapes (NRMS projection, BERT-base
layers at XFormer B=32).  python tools/split_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
import torch  # noqa: E402
from newsrec_amd import _lib as L, kernels as K  # noqa: E402
from newsrec_amd import functions as F  # noqa: E402


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = "cuda"
    torch.manual_seed(0)
    out = {}
    V, E = 30522, 768
    table = torch.randn(V, E, device=dev)
    U = 24576
    ids = torch.randint(1, V, (U,), device=dev)
    W = torch.randn(1152, E, device=dev) / 30
    Y = torch.empty(U, 1152, device=dev)
    dY = torch.randn(U, 1152, device=dev)
    dX = torch.empty(U, E, device=dev)
    dW = torch.zeros(1152, E, device=dev)
    T = 20832
    x = torch.randn(T, 768, device=dev)
    wqkv = torch.randn(2304, 768, device=dev) / 30
    qkv = torch.empty(T, 2304, device=dev)
    wi = torch.randn(3072, 768, device=dev) / 30
    Ub = torch.empty(T, 3072, device=dev)
    G = torch.empty(T, 3072, device=dev)
    wo2 = torch.randn(768, 3072, device=dev) / 50
    o = torch.empty(T, 768, device=dev)
    dWi = torch.zeros(3072, 768, device=dev)
    cases = {
        "nrms_proj_fwd": (2 * U * E * 1152, lambda: K.gemm_dyn(U, 1152, E, K.operand(table, L.KCONTIG, rows=ids, mapping=L.ROWS_GATHER),
                                                               K.operand(W, L.KCONTIG), Y)),
        "nrms_proj_dgrad": (2 * U * E * 1152, lambda: K.gemm_dyn(U, E, 1152, K.operand(dY, L.KCONTIG), K.operand(W, L.MNCONTIG), dX)),
        "nrms_proj_wgrad": (2 * U * E * 1152, lambda: K.gemm_dyn(1152, E, U, K.operand(dY, L.MNCONTIG),
                                                                 K.operand(table, L.MNCONTIG, rows=ids, mapping=L.ROWS_GATHER), dW,
                                                                 epilogue=L.EPI_ATOMIC, split_k=F._split_k(1152, E, U))),
        "bert_qkv": (2 * T * 768 * 2304, lambda: K.gemm(T, 2304, 768, K.operand(x, L.KCONTIG), K.operand(wqkv, L.KCONTIG), qkv)),
        "bert_ffn1_gelu": (2 * T * 768 * 3072, lambda: K.gemm(T, 3072, 768, K.operand(x, L.KCONTIG), K.operand(wi, L.KCONTIG), G,
                                                              epilogue=L.EPI_STORE_GELU, c_rows=K.operand(Ub, L.KCONTIG))),
        "bert_ffn2": (2 * T * 768 * 3072, lambda: K.gemm(T, 768, 3072, K.operand(G, L.KCONTIG), K.operand(wo2, L.KCONTIG), o)),
        "bert_ffn1_dgrad": (2 * T * 768 * 3072, lambda: K.gemm(T, 768, 3072, K.operand(G, L.KCONTIG), K.operand(wi, L.MNCONTIG), o)),
        "bert_ffn1_wgrad": (2 * T * 768 * 3072, lambda: K.gemm(3072, 768, T, K.operand(G, L.MNCONTIG), K.operand(x, L.MNCONTIG), dWi,
                                                               epilogue=L.EPI_ATOMIC, split_k=F._split_k(3072, 768, T))),
    }
    for prec, name in ((L.GEMM_F32, "f32"), (L.GEMM_BF16X6, "bf16x6")):
        K.set_gemm_precision(prec)
        for k, (fl, fn) in cases.items():
            ms = bench(fn)
            out.setdefault(k, {})[name] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
    for k, v in out.items():
        v["speedup"] = round(v["f32"]["ms"] / v["bf16x6"]["ms"], 2)
    # accuracy on the projection shape: max |C - C_fp64| / (sqrt(K) max|a| max|b|)
    a = torch.randn(4096, 768, device=dev)
    b = torch.randn(1152, 768, device=dev)
    ref = (a.double() @ b.double().t())
    scale = 768 ** 0.5 * a.abs().max().item() * b.abs().max().item()
    for prec, name in ((L.GEMM_F32, "f32"), (L.GEMM_BF16X6, "bf16x6")):
        K.set_gemm_precision(prec)
        C = torch.empty(4096, 1152, device=dev)
        K.gemm_dyn(4096, 1152, 768, K.operand(a, L.KCONTIG), K.operand(b, L.KCONTIG), C)
        d = (C.double() - ref).abs()
        out.setdefault("accuracy", {})[name] = {"max_abs_err": d.max().item(), "rel_to_bound": d.max().item() / scale,
                                                "mean_abs_err": d.mean().item()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
