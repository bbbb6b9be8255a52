"""Time the distinct-row GEMM shapes (NRMS B=32: U_pad ~ 24.6k rows); NR_PKG_ROOT points at
another checkout to A/B two builds on one box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# NR_PKG_ROOT: time another checkout's package (A/B of two builds)
sys.path.insert(0, os.path.join(os.environ.get("NR_PKG_ROOT", ROOT), "news-recommendation-mind_amd"))
import torch
from newsrec_amd import _lib as L
from newsrec_amd import kernels as K


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


U, E, NY, V = 24608, 768, 1152, 30522
table = torch.randn(V, E, device="cuda") * 0.05
uids = torch.randperm(V, device="cuda")[:U].sort().values
W = torch.randn(NY, E, device="cuda") * 0.03
b = torch.zeros(NY, device="cuda")
Y = torch.empty(U, NY, device="cuda")
dYu = torch.randn(U, NY, device="cuda")
dtab = torch.zeros(V, E, device="cuda")
m_dev = torch.tensor([U], dtype=torch.int32, device="cuda")
import inspect
has_split = "tail_split" in inspect.signature(K.gemm_dyn).parameters
for split in ((False, True) if has_split else (False,)):
    kw = {"tail_split": split} if has_split else {}
    fwd = lambda: K.gemm_dyn(U, NY, E, K.operand(table, L.KCONTIG, rows=uids, mapping=L.ROWS_GATHER),
                             K.operand(W, L.KCONTIG), Y, m_dev=m_dev, bias=b, **kw)
    dgr = lambda: K.gemm_dyn(U, E, NY, K.operand(dYu, L.KCONTIG), K.operand(W, L.MNCONTIG), dtab, m_dev=m_dev,
                             epilogue=L.EPI_SCATTER_STORE, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, **kw)
    fl = 2 * U * NY * E
    t1, t2 = timeit(fwd), timeit(dgr)
    print("tail_split=%d  fwd %.3f ms %.1f TF   dgrad %.3f ms %.1f TF" % (split, t1, fl / t1 / 1e9, t2, fl / t2 / 1e9),
          flush=True)
