"""Times the NRMS news-encoder attention kernels at the bench's size (1,760 titles x 30 tokens, 12
heads of 64 / 32, distinct-row projections through yrows): the fused forward, the split backward
(kernel 1 = pooling / LN backward, kernel 2 = per-head attention backward) and the per-kernel split
measured by running kernel 1 alone.  python tools/attn_probe.py [--reps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "news-recommendation-mind_amd"))
from newsrec_amd import kernels as K  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    n, L, heads, dk, dv = 1760, 30, 12, 64, 32
    H, NY, T, U = heads * dv, heads * (dk + dv), 1760 * 30, 24600
    Y = torch.randn(U, NY, device=dev) * 0.3
    yrows = torch.randint(0, U, (T,), device=dev)
    lens = torch.randint(5, L + 1, (n,), device=dev)
    mask = (torch.arange(L, device=dev)[None] < lens[:, None]).to(torch.uint8).reshape(-1)
    gamma = torch.rand(H, device=dev) + 0.5
    beta = torch.randn(H, device=dev) * 0.1
    q = torch.randn(H, device=dev)
    news = torch.empty(n, H, device=dev)
    stats = torch.empty(T, 2, device=dev)
    probs = torch.empty(T, device=dev)
    O = torch.empty(T, H, device=dev)
    kw = dict(p_drop=0.2, seed=1, offset=0, yrows=yrows)
    fwd = lambda: K.mha_pool_fwd(Y, mask, n, L, heads, dk, dv, gamma, beta, q, news, stats, probs, oout=O, **kw)  # noqa
    t_fwd = timed(fwd, a.reps)
    dnews = torch.randn(n, H, device=dev)
    dY = torch.empty(T, NY, device=dev)
    dob = torch.empty(T, 8, device=dev)
    db, dq, dg, dbt = (torch.zeros(NY, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev),
                       torch.zeros(H, device=dev))
    from newsrec_amd.functions import GRAD_COPIES, _grad_copies
    ws = _grad_copies(torch.device(dev, 0), 3 * H + NY) if os.environ.get("NR_PROBE_WS", "1") == "1" else None
    bwd = lambda: K.mha_pool_bwd(Y, mask, n, L, heads, dk, dv, gamma, beta, q, stats, probs, dnews, dY, db, dq, dg,  # noqa
                                 dbt, o=O, dob=dob, ws=ws, ws_copies=GRAD_COPIES if ws is not None else 0, **kw)
    t_bwd = timed(bwd, a.reps)
    print(json.dumps({"mha_pool_fwd_us": round(t_fwd, 1), "split_bwd_us": round(t_bwd, 1)}))


if __name__ == "__main__":
    main()
