"""Time nr_cnn_keypool_fwd / _bwd at the bench's CNN shape (B = 32: 1,760 titles x 30 tokens, H = 150)
in each arithmetic, and the unfused key GEMM + pooling path it replaces.  python tools/keypool_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "news-recommendation-mind_amd"))
import torch  # noqa: E402
from newsrec_amd import _lib as L  # noqa: E402
from newsrec_amd import kernels as K  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = "cuda"
    n, Lq, H, Hp = 1760, 30, 150, 160
    T = n * Lq
    torch.manual_seed(0)
    C = torch.zeros(T, Hp, device=dev)
    C[:, :H] = torch.relu(torch.randn(T, H, device=dev))
    wq = torch.zeros(Hp, Hp, device=dev)
    wq[:H, :H] = torch.randn(H, H, device=dev) * 0.1
    bq = torch.zeros(Hp, device=dev)
    q = torch.randn(H, device=dev)
    mask = torch.ones(T, dtype=torch.int64, device=dev)
    news = torch.empty(n, Hp, device=dev)
    probs = torch.empty(T, device=dev)
    dnews = torch.randn(n, H, device=dev)
    dc = torch.empty(T, Hp, device=dev)
    dwq, dbq, dq, dcb = (torch.empty(Hp, Hp, device=dev), torch.empty(Hp, device=dev), torch.empty(H, device=dev),
                         torch.empty(H, device=dev))
    out = {}
    for name, prec in (("f32", L.GEMM_F32), ("bf16x6", L.GEMM_BF16X6), ("bf16", L.GEMM_BF16)):
        out[name] = {
            "fwd_us": timed(lambda: K.cnn_keypool_fwd(C, wq, bq, q, mask, n, Lq, news, probs, qn=H, prec=prec)),
            "bwd_us": timed(lambda: K.cnn_keypool_bwd(C, wq, bq, q, n, Lq, H, probs, dnews, dc, dwq, dbq, dq, dcb,
                                                      prec=prec)),
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
