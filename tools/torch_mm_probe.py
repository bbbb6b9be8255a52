"""Calibration: torch.matmul (hipBLASLt) in bf16 and fp32 on the step's GEMM shapes and a square one,
timed with HIP events — what the vendor library reaches on the same hardware.
python tools/torch_mm_probe.py"""
import json

import torch


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


out = {}
for name, (M, N, K) in {"nrms_proj_fwd": (24576, 1152, 768), "nrms_proj_dgrad": (24576, 768, 1152),
                        "nrms_proj_wgrad": (1152, 768, 24576), "bert_ffn1": (20832, 3072, 768),
                        "square_8192": (8192, 8192, 8192)}.items():
    for dt in (torch.bfloat16, torch.float32):
        A = torch.randn(M, K, device="cuda", dtype=dt)
        B = torch.randn(N, K, device="cuda", dtype=dt)
        ms = bench(lambda: torch.matmul(A, B.t()))
        out.setdefault(name, {})[str(dt).split(".")[-1]] = {"us": round(ms * 1e3, 1),
                                                             "tflops": round(2 * M * N * K / ms / 1e9, 1)}
print(json.dumps(out))
