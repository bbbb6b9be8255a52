"""Times nr_adam_multi on the NRMS parameter set (the 30522 x 768 word table + ~1.2 M dense
parameters in 20 tensors): host step counts vs device step counts / learning rates (the graphed
step's form), against the 28 B per parameter HBM floor.  python tools/adam_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "news-recommendation-mind_amd"))
from newsrec_amd import kernels as K  # noqa: E402


def main():
    dev = "cuda"
    shapes = [(30522, 768), (1152, 768), (1152,), (384,), (384,), (384,), (768, 384), (768,), (384,)]
    shapes += [(384, 384)] * 2 + [(384,)] * 9
    ts = []
    for sh in shapes:
        p = torch.randn(sh, device=dev)
        ts.append((p, torch.randn(sh, device=dev), torch.zeros(sh, device=dev), torch.zeros(sh, device=dev)))
    n = sum(t[0].numel() for t in ts)
    step_dev = torch.ones((), dtype=torch.int64, device=dev)
    lr_dev = torch.full((), 1e-4, dtype=torch.float32, device=dev)
    out = {"params": n, "floor_us": round(28 * n / 8e12 * 1e6, 1)}
    for name, mk in (("host_step", lambda: [(p, g, m, v, 1e-4, 3) for p, g, m, v in ts]),
                     ("device_step", lambda: [(p, g, m, v, lr_dev, step_dev) for p, g, m, v in ts])):
        ent = mk()
        K.adam_multi(ent, 0.9, 0.999, 1e-8, 0.0)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        s.record()
        for _ in range(reps):
            K.adam_multi(ent, 0.9, 0.999, 1e-8, 0.0)
        e.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(s.elapsed_time(e) * 1e3 / reps, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
