"""Benchmark of the north-star path: NRMS (MHA news encoder + MHA user encoder, H=384,
12 heads) two-tower TRAIN step on synthetic MIND-large-shaped impressions.

One step = one batch of B=32 impressions per GPU (1 clicked + 4 negative candidates, a
50-click history, 30-token titles), FORMED ON THE DEVICE from a MIND-large-shaped
train split resident in HBM (nr_form_train_batch: sampler indices -> impression -> news ids ->
token rows, negative sampling from a device RNG; --data resident feeds pre-formed batches
instead), through forward (fused embedding gather,
news tower over 55 titles per impression, user tower, scorer + log-softmax), NLL loss,
backward, gradient all-reduce (N > 1) and Adam (two groups, lr 1e-4 / 6e-6 for the 23.4 M
parameter word table), exactly as utils/Manager.py:636-647.  Inputs are resident in HBM
before the timed region.  fp32 storage and arithmetic (the reference's precision).

The eval leg is the fast-eval pipeline (Manager._eval_fast): the 72,024-row MIND-large dev news
table encoded (sharded over ranks + RCCL all-gather), batched predict_fast over a synthetic
MIND-large-shaped dev split (376,471 impressions, ~37 candidates each), and cal_metric on the GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--data device|resident]

Rank 0 prints ONE JSON line.  N > 1: either launch with torch.distributed.run (one rank/GPU), or
run ``bench.py --gpus N`` directly and it spawns the N ranks itself (twotower.py:62-73).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "news-recommendation-mind_amd"))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist

B, C, NH, L, V, E, H, HEADS = 32, 5, 50, 30, 30522, 768, 384, 12
USERS_LARGE, NEWS_LARGE_DEV, NEWS_LARGE_TRAIN = 876956, 72023, 101527
DEV_IMPR_LARGE = 376471            # MIND-large dev impressions
TRAIN_IMPR_SYNTH = 262144          # train impressions resident for the synthetic split (a subset of 2.23 M)
FP32_MFMA_PEAK_TF = 157.3          # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 = f32 vector peak
BF16_MFMA_PEAK_TF = 2500.0         # MI355X_MICROARCH.md: bf16 dense MFMA peak (no sparsity)
HBM_PEAK_GBS = 8000.0
EVAL_BATCH_IMPR = 16384            # impressions per fast-eval predict batch (the host loop's launches amortised)


def synth_batch(gen, device, b=B, c=C, nh=NH, l=L, full=True):
    """MIND-shaped train batch (MIND.py:311-365 keys).  Token ids U[1000, V) with [CLS]=101 at
    position 0 and [SEP]=102 at the last real position; throughput runs use full titles."""
    def titles(n):
        tok = torch.randint(1000, V, (n, l), generator=gen)
        if full:
            lens = torch.full((n,), l)
        else:
            lens = torch.randint(5, l + 1, (n,), generator=gen)
        pos = torch.arange(l)[None]
        mask = (pos < lens[:, None]).long()
        tok = tok * mask
        tok[:, 0] = 101
        tok[torch.arange(n), lens - 1] = 102
        return tok, mask
    ct, cm = titles(b * c)
    ht, hm = titles(b * nh)
    x = {
        "cdd_encoded_index": ct.view(b, c, l), "cdd_attn_mask": cm.view(b, c, l),
        "his_encoded_index": ht.view(b, nh, l), "his_attn_mask": hm.view(b, nh, l),
        "his_mask": torch.ones(b, nh, 1, dtype=torch.float64),
        "user_id": torch.randint(1, USERS_LARGE + 1, (b,), generator=gen),
        "label": torch.zeros(b, dtype=torch.long),
        "cdd_id": torch.randint(1, NEWS_LARGE_DEV + 1, (b, c), generator=gen),
    }
    return {k: v.to(device) for k, v in x.items()}


DROPOUT_P = 0.2   # the headline's dropout (tools/ab_step.py may set bench.DROPOUT_P for an A/B)


def build(device):
    from newsrec_amd.manager import build_model
    torch.manual_seed(42)
    return build_model("mha", "mha", H, vocab=V, device=device, user_num=USERS_LARGE, dropout_p=DROPOUT_P)


def make_optim(model, capturable=False):
    from newsrec_amd.manager import get_optim
    return get_optim(model, capturable=capturable)


class ResidentFeed:
    """Pre-formed synthetic batches already in HBM; step i copies batch i into the static inputs."""

    def __init__(self, batches):
        self.batches = batches
        self.x = {k: v.clone() for k, v in batches[0].items()}

    def feed(self, i):
        for k, v in self.batches[i % len(self.batches)].items():
            self.x[k].copy_(v, non_blocking=True)

    def form(self):
        return self.x


class DeviceFeed:
    """Batches formed on the device each step from a MIND-large-shaped train split in HBM
    (MINDStore + nr_form_train_batch).  The sampler's epoch order (DistributedSampler: shuffled,
    strided over ranks) is uploaded once; form() launches the formation kernel, which takes the
    next B indices of that order at a device cursor and draws negatives from the device RNG pair,
    advancing both itself (captured in the graph: every replay forms the next batch with fresh
    negatives, no per-step copy)."""

    def __init__(self, device, world, rank, b=B, n_impr=TRAIN_IMPR_SYNTH):
        from newsrec_amd.dist import shard_train
        from newsrec_amd.mind import MINDStore, synthetic_arrays
        self.store = MINDStore.from_arrays(
            synthetic_arrays("train", NEWS_LARGE_TRAIN + 1, n_impr, vocab=V, users=USERS_LARGE, seed=99),
            "train", seed=1234 + rank, device=device)
        order = shard_train(len(self.store), world, rank, shuffle=True, seed=0)
        self.order = torch.tensor(order, dtype=torch.int64, device=device)
        self.b = b
        self.x = self.store.train_batch(self.order, device_rng=True, epoch_batch=b)

    def feed(self, i):
        pass   # the formation kernel walks the epoch order itself

    def form(self):
        return self.store.train_batch(self.order, out=self.x, device_rng=True, epoch_batch=self.b)


class GraphedStep:
    """The whole train step (batch formation, forward, NLL, backward, Adam) captured once as a
    HIP graph and replayed: the ~80 kernels of a step launch back to back with no host work
    between them.  Each step first feeds its sampler indices (or resident batch) into the
    captured input buffers; dropout draws, negative sampling and Adam step counts advance on the
    device, so replays are real training steps.

    Data parallel (``sync`` = a GradSync, N > 1): three graphs per step, the RCCL collectives issued
    eagerly between them (no collective is ever captured; GradSync's docstring):
      graph 1   forward + backward up to the word-table gradient (the projection weight-gradient GEMM
                deferred, WGRAD_DEFER_HOOK);
      issue     the word-table all-reduce starts on RCCL's stream;
      graph W   the deferred weight-gradient GEMM on all but GradSync.collective_cus CUs + bucket
                packing -- it runs BESIDE the all-reduce (twotower.py:49-50: DDP overlaps its bucket
                all-reduces with the rest of the backward);
      exchange  the remaining bucket all-reduces and the sparse exchange; wait for all;
      graph 2   bucket unpacking + Adam."""

    def __init__(self, model, opt, feed, sync, warmup):
        self.feed = feed
        self.opt = opt
        self.sync = sync
        if sync is not None:
            sync.deferred = True
        # warm-up as ordinary eager steps on the current stream (allocator, lazy init, optimizer
        # state); the capture then runs on torch.cuda.graph's own stream
        for i in range(max(2, warmup)):
            feed.feed(i)
            train_step(model, opt, feed.form(), sync)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        if sync is None:
            with torch.cuda.graph(self.graph):
                # detached: the captured loss must not keep the capture's autograd graph (and its
                # AccumulateGrad nodes, bound to the capture stream) alive
                self.loss = train_step(model, opt, feed.form(), sync).detach()
            self.opt_graph = None
        else:
            pool = torch.cuda.graph_pool_handle()   # the graphs share one memory pool
            with torch.cuda.graph(self.graph, pool=pool):
                self.loss = forward_backward(model, opt, feed.form()).detach()
                self.rec = sync.take_sparse()
            self.wgraph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.wgraph, pool=pool):
                outs = sync.run_deferred()
                self.early, self.packed = sync.pack(self.rec, outs)
            self.kept = sync.kept   # the deferred GEMMs' operands (graph 1's outputs) stay allocated
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph, pool=pool):
                sync.unpack(self.packed)
                opt.step(grad_scale=sync.scale)
        torch.cuda.synchronize()

    def __call__(self, i):
        self.feed.feed(i)
        self.opt.sync_lr()   # a scheduler's lr changes reach the captured Adam
        self.graph.replay()
        if self.opt_graph is not None:
            works = self.sync.issue(self.early)
            self.wgraph.replay()
            self.sync.exchange(self.packed, self.rec, works)
            self.opt_graph.replay()
            self.sync.after_step()   # shard_tables: all-gather the updated table slabs (else nothing)


_ONES = {}


def _one(t):
    """A persistent 1.0 on t's device as the loss gradient: autograd's implicit ones_like would be a
    fill launch per step (created by the eager warm-up, so a captured step reads it)."""
    one = _ONES.get(t.device)
    if one is None:
        one = _ONES[t.device] = torch.ones((), device=t.device)
    return one


def forward_backward(model, opt, x):
    """Manager._train :636-644: zero_grad, forward, NLLLoss, backward (the two-tower models fuse the
    loss into their head: TwoTowerBaseModel.forward_loss)."""
    opt.zero_grad(set_to_none=True)
    if hasattr(model, "forward_loss"):
        _, loss = model.forward_loss(x)
    else:
        logits, _ = model(x)
        loss = torch.nn.functional.nll_loss(logits, x["label"])
    loss.backward(_one(loss))
    return loss


def train_step(model, opt, x, sync):
    """utils/Manager.py:636-647 with the DDP gradient mean (GradSync: the word-table gradient's
    all-reduce starts inside the backward; 1/world folded into Adam)."""
    loss = forward_backward(model, opt, x)
    scale = sync() if sync is not None else 1.0
    opt.step(grad_scale=scale)
    if sync is not None:
        sync.after_step()
    return loss


def fast_eval_leg(model, dev, world, rank, n_impr):
    """Manager._eval_fast + evaluate on a synthetic MIND-large-shaped dev split resident in HBM:
    (1) encode the 72,024-row news table (rank shards + all-gather), (2) batched predict_fast over
    the rank's Partition_Sampler chunks (history representations read from the table), predictions
    gathered to rank 0, (3) cal_metric (auc, mean_mrr, ndcg@5;10) on the GPU.  Every phase is
    bracketed by a barrier + synchronize; times are rank 0's (phases end in collectives)."""
    from newsrec_amd import evaluate as EV
    from newsrec_amd.mind import MINDStore, synthetic_arrays
    st = MINDStore.from_arrays(synthetic_arrays("dev", NEWS_LARGE_DEV + 1, n_impr, vocab=V, users=USERS_LARGE,
                                                seed=2024), "dev", device=dev)
    n_cand = int(st.cand_off_host[-1])

    def sync():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # warm-up: kernels, allocator
    small = MINDStore.from_arrays(synthetic_arrays("dev", 2048, 256, vocab=V, seed=1), "dev", device=dev)
    EV.evaluate(model, small, batch_impr=128)
    sync()
    t0 = time.perf_counter()
    table = EV.encode_news_table(model, st)
    sync()
    t1 = time.perf_counter()
    preds, labels, grp = EV.eval_fast(model, st, batch_impr=EVAL_BATCH_IMPR, news_table=table)
    sync()
    t2 = time.perf_counter()
    res = EV.cal_metric_packed(preds, labels, grp, ["auc", "mean_mrr", "ndcg@5;10"]) if rank == 0 else None
    t3 = time.perf_counter()
    enc, pred, met = t1 - t0, t2 - t1, t3 - t2
    return {"mode": "fast eval (Manager._eval_fast + evaluate): sharded news-table encode + RCCL all-gather, "
                    "batched predict_fast (ragged scorer), cal_metric on the GPU",
            "news": st.n_news, "impressions": n_impr, "candidates": n_cand,
            "news_encode_ms": round(enc * 1e3, 2), "news_per_s": round(st.n_news / enc, 1),
            "predict_ms": round(pred * 1e3, 2), "candidates_per_s": round(n_cand / pred, 1),
            "metric_ms": round(met * 1e3, 2),
            "end_to_end_ms": round((enc + pred + met) * 1e3, 2),
            "end_to_end_candidates_per_s": round(n_cand / (enc + pred + met), 1),
            "metrics_random_model": res}


SHARD_TABLES = False   # --shard-table: the word tables' Adam sharded by rows across ranks (GradSync)


def _dp_setup(model, world):
    """Data parallel (N > 1): rank 0's parameters broadcast (DDP's construction, twotower.py:49-50) and
    a GradSync for the model (its gradient hooks are process-wide: one live GradSync at a time)."""
    if world == 1:
        return None
    from newsrec_amd.dist import GradSync
    with torch.no_grad():
        for p in model.parameters():
            dist.broadcast(p, 0)
    return GradSync(model, shard_tables=SHARD_TABLES)


def _timed(step_fn, steps, world, dev):
    """Time exactly ``steps`` calls bracketed by a barrier + synchronize on both sides; the max over
    ranks (seconds per step)."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el / steps


def xformer_leg(dev, steps=5, warmup=2, b=B, world=1, rank=0):
    """configs[4] beside the headline: XFormer (bert-base news encoder + 501-token user sequence,
    12 layers, dropout 0.1, Adam) train steps and eval forwards on synthetic MIND-shaped batches;
    the train step replayed as HIP graphs like the headline (dropout draws advance on the device).
    N > 1: every rank trains on its own batch and GradSync forms the DDP gradient mean between the
    graphs (xformer.py:19-20; the 94 MB word table in place, the other 344 MB of BERT gradients in
    128 MB buckets); the replicas are checked after the timed steps (dp_check).  FLOPs are
    algorithmic (dense layers + attention + pooler, train = 3x fwd)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_bert as BB
    from newsrec_amd.manager import get_optim
    model = BB.build("xformer", 12, dev)
    sync = _dp_setup(model, world)
    opt = get_optim(model, capturable=True)
    gen = torch.Generator().manual_seed(3 + rank)
    x = {k: v.to(dev) for k, v in BB.synth(gen, b).items()}
    model.train()
    step = GraphedStep(model, opt, ResidentFeed([x]), sync, warmup)
    el = _timed(step, steps, world, dev)
    chk = dp_check(model, opt, world, dev) if world > 1 else {}
    if sync is not None:
        sync.close()
    model.eval()
    with torch.no_grad():
        model(x)
        ev = _timed(lambda i: model(x), steps, world, dev)
    f = BB.flops_per_impression("xformer", 12) * b
    del step, model, opt
    torch.cuda.empty_cache()
    out = {"workload": "XFormer train step: bert-base (12 layers, 768, 12 heads) over 5x30-token candidates + "
                       "501-token user sequence, dropout 0.1, Adam; synthetic batches, random init",
           "launch": "hipGraph replay of the train step" + (" (three graphs, RCCL collectives between them)"
                                                            if world > 1 else ""),
           "n_gpus": world, "per_gpu_batch": b, "impressions_per_s": round(world * b / el, 1),
           "ms_per_step": round(el * 1e3, 2), "train_tflops": round(world * 3 * f / el / 1e12, 1),
           "eval_impressions_per_s": round(world * b / ev, 1), "eval_tflops": round(world * f / ev / 1e12, 1),
           "roofline": {"bound": "mfma", "peak_tflops": round(BF16_MFMA_PEAK_TF / 6, 1),
                        "peak_basis": "fp32-equivalent bf16x6 (2.5 PF bf16 dense / 6), per GPU",
                        "frac": round(3 * f / el / 1e12 / (BF16_MFMA_PEAK_TF / 6), 4)}}
    out.update(chk)
    return out


# algorithmic train FLOPs per impression (token-wise count, fwd x 3) and the
# parameter count of the dense Adam per configuration (H = 150, V = 30522)
LEG_FLOPS_BASIS = ("token-wise algorithmic FLOPs (the reference's Conv1d and key projection over every token, "
                   "fwd x 3); the distinct-row CNN encoder executes about half of them (the tap projection and its "
                   "two gradient GEMMs over the batch's U distinct word rows instead of T tokens)")
LEG_FLOPS = {"cnn_attn": 3.65e9, "cnn_attn_bf16": 3.65e9, "cnn_lstur": 3.70e9, "cnn_gru": 3.60e9}


def _leg_floor(name, model, ms):
    """Roofline of one config leg: the step's floor = max(algorithmic FLOPs / MFMA peak, HBM bytes /
    HBM peak) with bytes = the dense Adam's 28 B per parameter + the dense word-table gradient's zero
    fill and store (2 x 4 B x V x E); frac = floor / measured."""
    bf16 = name.endswith("bf16")
    peak_tf = BF16_MFMA_PEAK_TF if bf16 else BF16_MFMA_PEAK_TF / 6
    n_params = sum(p.numel() for p in model.parameters())
    flops = LEG_FLOPS[name] * B
    bytes_ = 28 * n_params + 2 * 4 * V * E
    t_mfma = flops / (peak_tf * 1e12) * 1e3
    t_hbm = bytes_ / (HBM_PEAK_GBS * 1e9) * 1e3
    floor = max(t_mfma, t_hbm)
    return {"bound": "mfma" if t_mfma >= t_hbm else "hbm", "floor_ms": round(floor, 4),
            "frac": round(floor / ms, 4), "achieved_tflops": round(flops / (ms * 1e-3) / 1e12, 1),
            "peak_tflops": round(peak_tf, 1), "flop_basis": LEG_FLOPS_BASIS, "adam_params": n_params,
            "hbm_bytes_floor": bytes_,
            "gemm_arithmetic": "bf16 (operands rounded to bf16, fp32 accumulate)" if bf16 else "bf16x6 (fp32-class)"}


def config_legs(dev, feed, steps=20, warmup=3, only=None, world=1):
    """The other two-tower configurations of BASELINE.json beside the headline: configs[1] CNN news +
    additive-attention user (fp32-class and the bf16 configuration), configs[3] LSTUR (CNN news +
    LSTM with user embedding, MIND-large user table) and the GRU variant.  Train steps (batch
    formation on the device, fwd, NLL, bwd, Adam) of B = 32 per GPU, H = 150, V = 30522, each leg's
    whole step replayed as HIP graphs like the headline.  N > 1 (configs[3] is quoted on 8 GPUs):
    every rank forms its own batches (its DistributedSampler shard), GradSync forms the DDP mean (the
    LSTUR user table by the exact row-sparse exchange) and the replicas are checked after the timed
    steps (dp_check)."""
    from newsrec_amd.manager import build_model, get_optim
    out = {}
    for name, encN, encU, prec in (("cnn_attn", "cnn", "attn", None), ("cnn_attn_bf16", "cnn", "attn", "bf16"),
                                   ("cnn_lstur", "cnn", "lstur", None), ("cnn_gru", "cnn", "gru", None)):
        if only is not None and name not in only:
            continue
        torch.manual_seed(42)
        model = build_model(encN, encU, 150, vocab=V, device=dev, user_num=USERS_LARGE, precision=prec)
        model.train()
        sync = _dp_setup(model, world)
        opt = get_optim(model, capturable=True)
        step = GraphedStep(model, opt, feed, sync, warmup)
        el = _timed(step, steps, world, dev)
        ms = el * 1e3
        out[name] = {"n_gpus": world, "impressions_per_s": round(world * B / el, 1), "ms_per_step": round(ms, 3),
                     "roofline": _leg_floor(name, model, ms)}
        if world > 1:
            out[name].update(dp_check(model, opt, world, dev))
            sync.close()
        del step, model, opt
        torch.cuda.empty_cache()
    out["note"] = ("hipGraph replay of the whole train step (device batch formation, fwd, NLL, bwd, Adam), B=32 per "
                   "GPU, H=150, V=30522 trainable table, MIND-large user table for LSTUR (876,957 rows); cnn_attn_bf16 = "
                   "configs[1]'s bf16 configuration (GEMM operands rounded to bf16, fp32 accumulation, fp32 master "
                   "weights); lstur = the reference's LSTUR_User_Encoder (LSTM, RNN.py:76-104); impressions_per_s is "
                   "the whole job's over n_gpus ranks, the roofline per GPU")
    return out


def gather_probe(dev, reps=20):
    """BERT_Embedding.forward (BERT.py:39) as the standalone gather (nr_embedding_fwd, the unfused
    contract): the step's T = 52,800 token rows of the 30522 x 768 fp32 table, read + write bytes ÷
    time (HIP events on the launch stream)."""
    from newsrec_amd import kernels as Kn
    g = torch.Generator().manual_seed(3)
    table = torch.randn(V, E, device=dev)
    ids = torch.randint(0, V, (B * (C + NH) * L,), generator=g).to(dev)
    out = torch.empty(ids.numel(), E, device=dev)
    for _ in range(3):
        Kn.embedding_fwd(table, ids, out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        Kn.embedding_fwd(table, ids, out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    nbytes = 2 * ids.numel() * E * 4 + ids.numel() * 8
    return {"kernel": "nr_embedding_fwd (standalone gather)", "rows": ids.numel(), "ms": round(ms, 4),
            "achieved_gbs": round(nbytes / (ms * 1e-3) / 1e9, 1), "peak_gbs": HBM_PEAK_GBS,
            "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bytes": nbytes}


def host_cores():
    """The cores this process may actually use: len(sched_getaffinity(0)), capped by
    the cgroup CPU quota when one is set (a GPU box exposes every core of the machine to affinity
    but grants a 16-core share; more threads than that only oversubscribe it)."""
    n = len(os.sched_getaffinity(0))
    try:   # cgroup v2
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        try:   # cgroup v1
            quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if quota > 0:
                n = min(n, max(1, quota // period))
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:   # the box's own share (16 on the GPU pool)
        n = min(n, int(omp))
    return n


def cpu_baseline(seconds=20.0):
    """The oracle (oracle/restatement.py, torch fp32 CPU) on the same NRMS step, timed on this
    host's cores over a bounded sample (steps of B=32 until ~`seconds` elapse)."""
    from oracle import restatement as R
    threads = host_cores()
    torch.set_num_threads(threads)
    model = build("cpu")
    P = {n: p.detach().clone().requires_grad_(True) for n, p in model.named_parameters()}
    gen = torch.Generator().manual_seed(7)
    x = synth_batch(gen, "cpu")
    kw = {"p_drop": 0.2}      # the reference's nn.Dropout(0.2) in training (MHA.py:19,37)
    _, _, opt = R.train_step(P, x, "mha", "mha", None, cdd_kw=kw, his_kw=kw)      # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        _, _, opt = R.train_step(P, x, "mha", "mha", opt, cdd_kw=kw, his_kw=kw)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 50:
            break
    # eval: the forward in eval mode (sigmoid), candidates scored per second
    with torch.no_grad():
        Pn = {n: p.detach() for n, p in P.items()}
        R.forward(Pn, x, "mha", "mha", False)
        ne, t1 = 0, time.perf_counter()
        while True:
            R.forward(Pn, x, "mha", "mha", False)
            ne += 1
            el_e = time.perf_counter() - t1
            if el_e >= seconds / 4 or ne >= 50:
                break
    return {"value": round(steps * B / el, 2), "unit": "impressions/s", "cores": threads, "kind": "port",
            "sample": "%d NRMS train steps of B=32 (fwd+bwd+Adam, fp32) after 1 warm-up, oracle/restatement.py" % steps,
            "eval_candidates_per_s": round(ne * B * C / el_e, 1),
            "eval_sample": "%d eval-mode forwards of B=32 x 5 candidates (sigmoid), oracle/restatement.py" % ne}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment this process "
                         "spawns them itself (default 1, or WORLD_SIZE under torch.distributed.run)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--data", choices=["device", "resident"], default="device",
                    help="device: form each batch on the GPU from a resident MIND split; resident: pre-formed")
    ap.add_argument("--eval-impr", type=int, default=DEV_IMPR_LARGE,
                    help="dev impressions of the fast-eval leg (0 skips it)")
    ap.add_argument("--config-legs", type=int, default=1, help="1: time configs[1]/[3] beside the headline")
    ap.add_argument("--legs", default="", help="comma list of config legs to run (default: all of "
                                               "cnn_attn, cnn_attn_bf16, cnn_lstur, cnn_gru)")
    ap.add_argument("--xformer-steps", type=int, default=5,
                    help="timed XFormer (configs[4]) train steps reported beside the headline (0 skips)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the train step as HIP graphs (auto = on; N > 1: forward/backward and "
                         "optimizer graphs with the RCCL collectives between them)")
    ap.add_argument("--shard-table", action="store_true",
                    help="N > 1: shard the word tables' Adam by rows (reduce-scatter + slab Adam + all-gather) "
                         "instead of the DDP all-reduce + replicated Adam")
    a = ap.parse_args()
    global SHARD_TABLES
    SHARD_TABLES = bool(a.shard_table)

    # one rank per GPU over RCCL; NR_DIST_BACKEND=gloo lets a 1-GPU box rehearse the N > 1 path
    backend = os.environ.get("NR_DIST_BACKEND", "nccl")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        world = a.gpus if a.gpus is not None else 1
        if world > 1:
            # twotower.py:62-73 (mp.spawn, one process per GPU): this process only launches and
            # joins the ranks -- it must not touch the GPU (device_count() does not initialise it)
            if backend == "nccl" and torch.cuda.device_count() < world:
                print("bench.py: --gpus %d needs %d GPUs, %d visible" % (world, world, torch.cuda.device_count()),
                      file=sys.stderr)
                sys.exit(2)
            from newsrec_amd.dist import spawn_ranks
            sys.exit(spawn_ranks(world, [os.path.abspath(__file__)] + sys.argv[1:]))
    else:
        world = int(env_world)
        if a.gpus is not None and a.gpus != world:
            print("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world), file=sys.stderr)
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and backend == "nccl" and torch.cuda.device_count() < world:
        print("bench.py: WORLD_SIZE=%d needs %d GPUs under nccl, %d visible" % (world, world, torch.cuda.device_count()),
              file=sys.stderr)
        sys.exit(2)
    dev_index = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        kw = {"device_id": torch.device("cuda", dev_index)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        if dist.get_world_size() != world:
            raise RuntimeError("process group has %d ranks, expected %d" % (dist.get_world_size(), world))
    dev = torch.device("cuda", dev_index)
    from newsrec_amd.dist import GradSync
    torch.cuda.set_device(dev)

    from newsrec_amd import functions as F
    model = build(dev)
    model.train()
    if world > 1:
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p, 0)
    use_graph = a.graph in ("on", "auto")
    opt = make_optim(model, capturable=use_graph)
    sync = GradSync(model, shard_tables=SHARD_TABLES) if world > 1 else None
    gen = torch.Generator().manual_seed(1234 + rank)
    feed = DeviceFeed(dev, world, rank) if a.data == "device" else \
        ResidentFeed([synth_batch(gen, dev) for _ in range(4)])

    if use_graph:
        step_fn = GraphedStep(model, opt, feed, sync, a.warmup)
    else:
        def step_fn(i):
            feed.feed(i)
            train_step(model, opt, feed.form(), sync)
        for i in range(a.warmup):
            step_fn(i)
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step_fn(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if a.data == "device":
        feed.store.check_status()
    from newsrec_amd import kernels as Kn
    if Kn.score_nll_status(dev):
        raise RuntimeError("the training head saw a label outside [0, C) (NaN loss)")

    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # data parallel: every rank must hold the same parameters and Adam moments after the timed steps
    in_sync = dp_check(model, opt, world, dev) if world > 1 else None
    if in_sync is not None and not in_sync["dp_in_sync"]:
        print("bench.py: ranks diverged after the timed steps: %s" % json.dumps(in_sync), file=sys.stderr)

    # per-launch timing of the step's projection GEMMs: the launches of one eager step kept as
    # closures over their real operands, each replayed back to back between HIP events on its stream
    # (events cannot sit inside a graph replay; rocprofv3's trace of the graphed step agrees)
    F.PROBE.enable()
    feed.feed(a.steps)
    train_step(model, opt, feed.form(), sync)
    probe = F.PROBE.time(reps=20)
    F.PROBE.disable()

    # eval (a): forward in eval mode (sigmoid) over train-shaped batches -> candidates scored/s
    model.eval()
    evb = []
    for i in range(4):
        feed.feed(i)
        evb.append({k: v.clone() for k, v in feed.form().items()})
    with torch.no_grad():
        for i in range(3):
            model(evb[i % len(evb)])
        torch.cuda.synchronize()
        ne = max(5, a.steps // 2)
        t1 = time.perf_counter()
        for i in range(ne):
            model(evb[i % len(evb)])
        torch.cuda.synchronize()
        el_eval = time.perf_counter() - t1
    del evb
    if sync is not None:
        sync.close()   # the legs below install their own GradSync (the hooks are process-wide)
    # eval (b): the fast-eval pipeline over a MIND-large-shaped dev split
    fast = fast_eval_leg(model, dev, world, rank, a.eval_impr) if a.eval_impr > 0 else None
    # configs[4] (XFormer) and configs[1]/[3] at every N: the 8-GPU configurations are measured on N ranks
    xf = xformer_leg(dev, a.xformer_steps, world=world, rank=rank) if a.xformer_steps > 0 else None
    only = [n for n in a.legs.split(",") if n] or None
    legs = config_legs(dev, feed, world=world, only=only) if (a.config_legs and a.data == "device") else None
    gather = gather_probe(dev) if world == 1 else None

    if rank == 0:
        ms = el / a.steps * 1e3
        value = world * B * a.steps / el
        from newsrec_amd import _lib as Lb, kernels as Kn
        split = Kn.get_gemm_precision() == Lb.GEMM_BF16X6
        # bf16x6: six bf16 MFMAs per fp32 multiply-add -> fp32-equivalent peak = bf16 dense peak / 6
        peak = BF16_MFMA_PEAK_TF / 6 if split else FP32_MFMA_PEAK_TF
        # the news tower's three projection GEMMs, each timed per launch (F.PROBE.time): forward
        # (gathered table rows x [Wk; Wv]^T), table dgrad (dY W -> distinct table rows), weight
        # gradient (dY^T x gathered rows: the split-K GEMM + its ordered reduction, one unit).  Each
        # is 2 x rows x 768 x 1152 FLOP with rows = the batch's distinct word rows U_pad (read back
        # from the device)
        gemms = {}
        for name, what in (("proj_fwd", "forward: gathered rows x [Wk;Wv]^T"),
                           ("proj_dgrad", "table dgrad: dY x [Wk;Wv] -> distinct table rows"),
                           ("proj_wgrad", "weight gradient: dY^T x gathered rows (split-K GEMM + splitk_reduce)")):
            g_ms = probe.get(name + "_ms")
            if not g_ms:
                continue
            rows = probe.get(name + "_rows", float(B * (C + NH) * L))
            fl = 2.0 * rows * E * (E + H)
            ach = fl / (g_ms * 1e-3) / 1e12
            tr = None
            pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % name)
            if os.path.exists(pmc):
                tr = json.load(open(pmc)).get("hbm_bytes_per_launch")
            gemms[name] = {"what": what, "launch_ms": round(g_ms, 4), "rows_per_launch": rows,
                           "flops_per_launch": fl, "achieved": round(ach, 2), "frac": round(ach / peak, 4),
                           "traffic": tr, "traffic_source": ("profiles/pmc_%s.json (rocprofv3 --pmc passes of "
                                                             "this build: FETCH_SIZE x 2 + WRITE_SIZE)" % name)
                           if tr else None}
        # the roofline line names the DOMINANT kernel of the step: the longest of the three
        dom = max(gemms, key=lambda k: gemms[k]["launch_ms"]) if gemms else None
        gd = gemms.get(dom, {})
        achieved = gd.get("achieved")
        traffic = gd.get("traffic")
        gemm_ms = gd.get("launch_ms")
        gemm_flops = gd.get("flops_per_launch")
        gemm_rows = gd.get("rows_per_launch")
        out = {
            "metric": "impressions/sec (train) + candidates scored/sec (eval), NRMS MIND-large 1/8 GPU",
            "value": round(value, 1), "unit": "impressions/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (MIND-large-shaped, random-init weights)",
            "gemm_arithmetic": ("bf16x6: fp32 operands split into 3 bf16 terms, 6 products on the bf16 MFMA, "
                                "fp32 accumulate (measured as accurate as the f32 MFMA)") if split else
                               "f32 MFMA (exact fp32 products)",
            "config": {"workload": "NRMS train step: MHA news encoder + MHA user encoder, H=384, 12 heads, "
                                   "V=30522 word table (trainable), dropout 0.2, Adam",
                       "launch": "hipGraph replay of the whole step" if use_graph else "eager",
                       "batches": ("formed on the device each step from a synthetic MIND-large-shaped train split "
                                   "in HBM (%d impressions, 101,528-news token table)" % TRAIN_IMPR_SYNTH)
                       if a.data == "device" else "pre-formed synthetic batches resident in HBM",
                       "global_batch": B * world, "per_gpu_batch": B, "candidates": C, "history": NH,
                       "seq_len": L, "parallelism": "dp%d" % world},
            "eval": dict(fast or {}, forward={"candidates_per_s": round(world * B * C * ne / el_eval, 1),
                                              "impressions_per_s": round(world * B * ne / el_eval, 1),
                                              "mode": "model(x) in eval mode (sigmoid) on train-shaped batches"}),
            "roofline": {"kernel": "%s GEMM of the news-tower key/value projection (%s)"
                                   % (dom, gd.get("what")) if dom else None, "bound": "mfma",
                         "achieved": round(achieved, 2) if achieved else None, "peak": round(peak, 1),
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4) if achieved else None,
                         "peak_basis": ("fp32-equivalent: 2.5 PF bf16 dense MFMA / 6 (bf16x6 split arithmetic)"
                                        if split else "fp32 MFMA (v_mfma_f32_32x32x2_f32)"),
                         "frac_of_fp32_peak": round(achieved / FP32_MFMA_PEAK_TF, 4) if achieved else None,
                         "traffic": traffic, "launch_ms": round(gemm_ms, 4) if gemm_ms else None,
                         "flops_per_launch": gemm_flops, "rows_per_launch": gemm_rows,
                         "tokens_per_launch": B * (C + NH) * L,
                         "timing": "per-launch average of 20 replays of the step's own launch, each after a 512 MB cache-evicting write "
                                   "(HIP events on its stream)", "projection_gemms": gemms},
        }
        if in_sync is not None:
            out.update(in_sync)
        if xf is not None:
            out["xformer"] = xf
        if legs is not None:
            out["other_configs"] = legs
        if gather is not None:
            out["gather"] = gather
        if not a.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    diverged = [k for k, v in [("headline", in_sync), ("xformer", xf)] + list((legs or {}).items())
                if isinstance(v, dict) and v.get("dp_in_sync") is False]
    if diverged:
        print("bench.py: replicas diverged in %s" % ", ".join(diverged), file=sys.stderr)
        sys.exit(3)


def dp_check(model, opt, world, dev):
    """After the timed data-parallel steps: each rank's float64 checksums (sum and sum of squares) of
    every parameter and both Adam moments, all-gathered over the process group and compared with
    rank 0's.  DDP semantics (twotower.py:49-50, Manager.py:167) keep the replicas identical: every
    rank applies the same all-reduced gradients through the same Adam, so the sums agree bitwise."""
    sums = []
    with torch.no_grad():
        for p in model.parameters():
            # a sharded table's moments exist for the rank's own rows only (GradSync shard_tables):
            # nothing to compare across ranks; its parameter is
            sharded = getattr(p, "_nr_shard", None) is not None
            ts = [p] + [opt.state[p][k] for k in ("exp_avg", "exp_avg_sq")
                        if k in opt.state.get(p, {}) and not sharded]
            for t in ts:
                d = t.detach().double()
                sums.append(d.sum())
                sums.append((d * d).sum())
    vec = torch.stack(sums)
    allv = torch.empty(world, vec.numel(), dtype=vec.dtype, device=dev)
    dist.all_gather_into_tensor(allv.view(-1), vec)
    ref = allv[0]
    diff = (allv - ref).abs() / ref.abs().clamp_min(1e-30)
    rel = float(diff.max().item())
    exact = bool((allv == ref).all().item())
    return {"dp_in_sync": rel <= 1e-9, "dp_bitwise_equal": exact, "dp_max_rel_diff": rel,
            "dp_checksums": int(vec.numel()), "dp_world_size": dist.get_world_size(),
            "dp_shard_tables": any(getattr(p, "_nr_shard", None) is not None for p in model.parameters())}


if __name__ == "__main__":
    main()
