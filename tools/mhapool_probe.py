"""Time nr_mha_pool_fwd/bwd on the NRMS news shape (1760 titles x 30 tokens, 12 heads)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
import torch
from newsrec_amd import kernels as K

n, L, heads, dk, dv = 1760, 30, 12, 64, 32
H = heads * dv
T = n * L
y = torch.randn(T, heads * (dk + dv), device="cuda")
mask = torch.ones(T, dtype=torch.int64, device="cuda")
gamma = torch.ones(H, device="cuda"); beta = torch.zeros(H, device="cuda"); q = torch.randn(H, device="cuda")
news = torch.empty(n, H, device="cuda"); stats = torch.empty(T, 2, device="cuda"); probs = torch.empty(T, device="cuda")
dy = torch.empty_like(y); db = torch.zeros(heads * (dk + dv), device="cuda")
dq = torch.zeros(H, device="cuda"); dg = torch.zeros(H, device="cuda"); dbt = torch.zeros(H, device="cuda")
dnews = torch.randn(n, H, device="cuda")


def timeit(fn, n=int(os.environ.get("ITERS", "20"))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


O = torch.empty(T, H, device="cuda")
dob = torch.empty(T, H, device="cuda")
for p in (0.0, 0.2):
    f2 = lambda: K.mha_pool_fwd(y, mask, n, L, heads, dk, dv, gamma, beta, q, news, stats, probs, p_drop=p, seed=1,
                                oout=O)
    b2 = lambda: K.mha_pool_bwd(y, mask, n, L, heads, dk, dv, gamma, beta, q, stats, probs, dnews, dy, db, dq, dg,
                                dbt, p_drop=p, seed=1, o=O, dob=dob)
    print("p=%.1f split: fwd+O %.1f us  bwd %.1f us" % (p, timeit(f2), timeit(b2)), flush=True)
for p in (0.0, 0.2):
    f = lambda: K.mha_pool_fwd(y, mask, n, L, heads, dk, dv, gamma, beta, q, news, stats, probs, p_drop=p, seed=1)
    b = lambda: K.mha_pool_bwd(y, mask, n, L, heads, dk, dv, gamma, beta, q, stats, probs, dnews, dy, db, dq, dg, dbt,
                               p_drop=p, seed=1)
    print("p=%.1f fwd %.1f us  bwd %.1f us  (env dbg=%s)" % (p, timeit(f), timeit(b), os.environ.get("NR_DEBUG_MHAPOOL")), flush=True)
