"""Time nr_gemm_f32 on the NRMS news-tower shapes (B=32: T=52,800 tokens)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
import torch
from newsrec_amd import _lib as L
from newsrec_amd import kernels as K

T, E, NQKV, V = 52800, 768, 1152, 30522
table = torch.randn(V, E, device="cuda") * 0.05
tok = torch.randint(1000, V, (T,), device="cuda")
W = torch.randn(NQKV, E, device="cuda") * 0.03
b = torch.zeros(NQKV, device="cuda")
Y = torch.empty(T, NQKV, device="cuda")
dY = torch.randn(T, NQKV, device="cuda")
dtab = torch.zeros(V, E, device="cuda")
dW = torch.zeros(NQKV, E, device="cuda")
Hc = 150
W3 = torch.randn(Hc, 3 * E, device="cuda") * 0.02
C3 = torch.empty(T, Hc, device="cuda")


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def fwd():
    K.gemm(T, NQKV, E, K.operand(table, L.KCONTIG, rows=tok, mapping=L.ROWS_GATHER), K.operand(W, L.KCONTIG), Y, bias=b)


def dgrad():
    K.gemm(T, E, NQKV, K.operand(dY, L.KCONTIG), K.operand(W, L.MNCONTIG), dtab,
           epilogue=L.EPI_SCATTER, c_rows=K.rows_map(tok, L.ROWS_GATHER), pad_row=0)


def wgrad(s):
    def f():
        K.gemm(NQKV, E, T, K.operand(dY, L.MNCONTIG), K.operand(table, L.MNCONTIG, rows=tok, mapping=L.ROWS_GATHER),
               dW, epilogue=L.EPI_ATOMIC, split_k=s)
    return f


def conv():
    K.gemm(T, Hc, 3 * E, K.operand(table, L.KCONTIG, rows=tok, mapping=L.ROWS_CONV3, seq_len=30, seg=E),
           K.operand(W3, L.KCONTIG), C3, bias=b, epilogue=L.EPI_STORE_RELU)


fl = 2 * T * NQKV * E
ONLY = os.environ.get("PROBE_ONLY")
if ONLY == "fwd":
    ms = timeit(fwd, n=int(os.environ.get("ITERS", "20")))
    print("%-22s %8.3f ms  %7.1f TF/s" % ("proj fwd gather", ms, fl / ms / 1e9), flush=True)
    sys.exit(0)
for name, fn, flops in [("proj fwd gather", fwd, fl), ("proj dgrad scatter", dgrad, fl),
                        ("proj wgrad sk6", wgrad(6), fl), ("proj wgrad sk9", wgrad(9), fl),
                        ("proj wgrad sk12", wgrad(12), fl), ("proj wgrad sk19", wgrad(19), fl),
                        ("proj wgrad sk24", wgrad(24), fl), ("proj wgrad sk28", wgrad(28), fl),
                        ("proj wgrad sk38", wgrad(38), fl), ("proj wgrad sk48", wgrad(48), fl), ("conv3 fwd H150", conv, 2 * T * Hc * 3 * E)]:
    ms = timeit(fn)
    print("%-22s %8.3f ms  %7.1f TF/s" % (name, ms, flops / ms / 1e9), flush=True)
ref = lambda: torch.matmul(table[tok], W.t())
ms = timeit(ref)
print("%-22s %8.3f ms  %7.1f TF/s" % ("torch gather+mm", ms, fl / ms / 1e9))
