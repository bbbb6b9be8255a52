"""Sweep the fast GEMM over M/N/K to separate steady-state k-loop rate from per-block
prologue/epilogue and wave-quantization effects; torch.matmul (hipBLASLt fp32) beside it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
import torch
from newsrec_amd import _lib as L
from newsrec_amd import kernels as K


def timeit(fn, n=10):
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


shapes = [(24608, 1152, 768), (24608, 1152, 3072), (24576, 1024, 768), (32768, 1152, 768), (49152, 1152, 768),
          (24608, 768, 1152), (65536, 1024, 768), (65536, 1024, 3072), (4096, 4096, 4096)]
if os.environ.get("SWEEP_SHAPES"):
    shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["SWEEP_SHAPES"].split(",")]
for M, N, Kd in shapes:
    A = torch.randn(M, Kd, device="cuda")
    B = torch.randn(N, Kd, device="cuda")
    C = torch.empty(M, N, device="cuda")
    fl = 2 * M * N * Kd
    f = lambda: K.gemm(M, N, Kd, K.operand(A, L.KCONTIG), K.operand(B, L.KCONTIG), C)
    ms = timeit(f)
    g = lambda: torch.matmul(A, B.t(), out=C)
    ms2 = timeit(g)
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    print("M=%6d N=%5d K=%5d tiles=%5d rounds=%.2f  nr %7.3f ms %6.1f TF   torch %7.3f ms %6.1f TF"
          % (M, N, Kd, tiles, tiles / 512, ms, fl / ms / 1e9, ms2, fl / ms2 / 1e9), flush=True)
    del A, B, C
    torch.cuda.empty_cache()
