import os, sys, json
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import torch, torch.multiprocessing as mp
import test_dist_gpu as T

def main():
    world, port = 2, T._port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=T._shard_worker, args=(r, world, port, sys.argv[1], sys.argv[2], q)) for r in range(world)]
    for p in ps: p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps: p.join(timeout=60)
    for rank, err, diffs in res:
        if err: print(rank, err); continue
        bad = {n: v for n, v in diffs.items() if v[1] > 0 or v[3] > 0}
        print(rank, json.dumps({n: [float('%.3g' % v[0]), v[1], v[2], v[3]] for n, v in bad.items()}))

if __name__ == "__main__":
    main()
