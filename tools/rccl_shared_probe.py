"""Probe: can RCCL ("nccl" backend) run two ranks on ONE GPU?  (If it can, the one-GPU lease can
run the data-parallel GPU tests over RCCL itself instead of gloo.)  Prints one JSON line per rank."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

if "WORLD_SIZE" not in os.environ:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "news-recommendation-mind_amd"))
    from newsrec_amd.dist import spawn_ranks
    sys.exit(spawn_ranks(2, [os.path.abspath(__file__)], timeout=90))
rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
t0 = time.time()
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
ok = bool((x == 3.0).all().item())
print(json.dumps({"rank": rank, "ok": ok, "s": round(time.time() - t0, 2)}), flush=True)
dist.destroy_process_group()
