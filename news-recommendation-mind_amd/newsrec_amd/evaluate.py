"""Fast evaluation pipeline: Manager._eval_fast (utils/Manager.py:474-541),
Manager.evaluate (:544-590) and cal_metric (:1205-1345), MI355X-first.

The reference encodes the news table on rank 0 only, saves it with torch.save, barriers, reloads
it on every rank, then scores one impression at a time (loader batch size 1) and gathers Python
lists with all_gather_object.  Here:

  encode_news_table   every rank encodes a contiguous shard of the news rows (fused gather +
                      encoder kernels, eval mode) and one RCCL all_gather_into_tensor assembles
                      the [N+1, H] table on every GPU -- no disk round trip
  predict_fast_batch  a batch of impression chunks at once: the user tower over the chunks'
                      histories, then ONE ragged scorer launch over all their candidates
                      (nr_score_ragged: table row . user row / sqrt(H), sigmoid)
  eval_fast           the rank's Partition_Sampler chunk range, then one padded RCCL all-gather
                      of the predictions to rank 0 (instead of all_gather_object of lists)
  cal_metric          per-impression AUC / MRR / nDCG@k / hit@k in one HIP launch
                      (nr_impression_metrics), then the reference's np.mean + round(4)

history_from_table: the reference re-encodes each impression's history titles inside
predict_fast (TwoTowerBaseModel.py:78-83 calls encode_user).  In eval mode the encoder is
deterministic and row-independent, so the history representations equal the news table's rows
for the same news ids; reading them from the table is the same result without re-running the
news tower (test_mind_gpu.py checks the two paths agree).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L
from . import kernels as K


def _chunk_range(n_chunks, world, rank):
    """Partition_Sampler (utils.py:267-283): contiguous chunks, the last rank takes the rest."""
    per, extra = divmod(n_chunks, world)
    lo = per * rank
    return lo, lo + per + (extra if rank + 1 == world else 0)


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


@torch.no_grad()
def encode_news_table(model, store, batch_news=8192, group=None):
    """Manager._eval_fast step 1 (Manager.py:490-509): news_reprs[cdd_id] = encode_news(x) for every
    row of the split's news table (row 0 included, as MIND_news yields it, MIND.py:471-491),
    sharded over the ranks of ``group`` and all-gathered.  -> [N+1, H] fp32 on every rank."""
    world, rank = _world(group)
    was_training = model.training
    model.eval()
    model.init_encoding()
    N = store.n_news
    H = model.hidden_dim
    per = -(-N // world)
    lo, hi = rank * per, min((rank + 1) * per, N)
    shard = torch.zeros(per, H, dtype=torch.float32, device=store.device)
    for s in range(lo, hi, batch_news):
        e = min(s + batch_news, hi)
        x = {"cdd_encoded_index": store.tok[s:e].to(torch.int64).unsqueeze(1),
             "cdd_attn_mask": store.attn[s:e].to(torch.int64).unsqueeze(1)}
        shard[s - lo:e - lo] = model.encode_news(x).squeeze(-2)
    model.destroy_encoding()
    model.train(was_training)
    return gather_shards(shard, N, group)


def gather_shards(shard, n, group=None):
    """Equal row shards (rank r holds rows [r*per, (r+1)*per)) -> the first n rows on every rank:
    one all_gather_into_tensor."""
    world, _ = _world(group)
    if world == 1:
        return shard[:n]
    full = torch.empty((shard.shape[0] * world,) + tuple(shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    dist.all_gather_into_tensor(full, shard.contiguous(), group=group)
    return full[:n]


def score_ragged(table, user, cand_ids, cand_seg, seg_base, out=None, mode=L.SCORE_SIGMOID):
    """out[c] = sigmoid(table[cand_ids[c]] . user[cand_seg[c] - seg_base] / sqrt(H))."""
    n = cand_ids.numel()
    H = table.shape[1]
    for t, name in ((table, "table"), (user, "user")):
        if t.dtype != torch.float32 or not t.is_cuda or t.stride(-1) != 1 or t.dim() != 2:
            raise L.HipError("score_ragged: %s must be a row-major 2-D float32 CUDA tensor" % name)
    if user.shape[1] != H:
        raise L.HipError("score_ragged: user width %d != table width %d" % (user.shape[1], H))
    if cand_ids.dtype != torch.int64 or cand_seg.dtype != torch.int32 or cand_seg.numel() != n:
        raise L.HipError("score_ragged: cand_ids int64 [n] and cand_seg int32 [n] expected")
    cand_ids, cand_seg = cand_ids.contiguous(), cand_seg.contiguous()
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=table.device)
    status = torch.zeros(1, dtype=torch.int32, device=table.device)
    L.call("nr_score_ragged", L.ptr(table), table.stride(0), table.shape[0], L.ptr(cand_ids), L.ptr(cand_seg),
           int(seg_base), n, L.ptr(user), user.stride(0), user.shape[0], H, mode, L.ptr(out), L.ptr(status),
           L.stream_ptr(table))
    return out, status


@torch.no_grad()
def user_reprs(model, table, batch, history_from_table=True, cache=None):
    """User representations [B, H] of a MINDStore.eval_batch.  history_from_table: the history
    news representations are the table's rows; an MHA user encoder then reads its key / value
    projections of the TABLE (computed once per table, kept in ``cache``) through the attention
    kernel's row indirection instead of projecting B*N gathered rows."""
    if not history_from_table:
        user = model.encode_user(batch)[0]
    else:
        enc = model.encoderU
        B, NH = batch["his_id"].shape
        if hasattr(enc, "forward_rows"):
            cache = {} if cache is None else cache
            if cache.get("Y") is None:
                cache["Y"] = enc.project_rows(table)
            user = enc.forward_rows(cache["Y"], batch["his_id"], batch["his_mask"], B, NH)
        else:
            his = K.gather_rows(table, batch["his_id"].reshape(-1).contiguous()).view(B, NH, -1)
            user = model._user_from_his(his, batch)
    user = user.reshape(user.shape[0], -1)
    if user.stride(-1) != 1 or user.stride(0) != user.shape[1]:
        user = user.contiguous()
    return user


@torch.no_grad()
def predict_fast_batch(model, batch, history_from_table=True, cache=None):
    """TwoTowerBaseModel.predict_fast (:78-83) for a batch of impression chunks from
    MINDStore.eval_batch: user representations for the chunks, then the ragged scorer over all
    their candidates.  -> sigmoid scores [n] aligned with batch["cdd_id"]."""
    table = model.news_reprs.weight
    user = user_reprs(model, table, batch, history_from_table, cache)
    preds, _ = score_ragged(table, user, batch["cdd_id"], batch["cand_seg"], batch["chunk0"])
    return preds


@torch.no_grad()
def eval_fast(model, store, batch_impr=1024, group=None, history_from_table=True, news_table=None):
    """Manager._eval_fast (:474-541): -> (preds, labels, grp_off) for the whole split on rank 0
    (packed, device tensors; labels None for test), (None, None, None) on other ranks."""
    world, rank = _world(group)
    was_training = model.training
    model.eval()
    if news_table is None:
        news_table = encode_news_table(model, store, group=group)
    model.init_embedding(news_table)
    c_lo, c_hi = _chunk_range(len(store), world, rank)
    o_lo, o_hi = int(store.cand_off_host[c_lo]), int(store.cand_off_host[c_hi])
    preds = torch.empty(o_hi - o_lo, dtype=torch.float32, device=store.device)
    cache = {}
    for c0 in range(c_lo, c_hi, batch_impr):
        b = min(batch_impr, c_hi - c0)
        x = store.eval_batch(c0, b, with_tokens=not history_from_table)
        o0, o1 = x["cand_range"]
        table = model.news_reprs.weight
        user = user_reprs(model, table, x, history_from_table, cache)
        score_ragged(table, user, x["cdd_id"], x["cand_seg"], c0, out=preds[o0 - o_lo:o1 - o_lo])
    model.destroy_embedding()
    model.train(was_training)
    if world > 1:
        rng = [_chunk_range(len(store), world, r) for r in range(world)]
        sizes = [int(store.cand_off_host[h] - store.cand_off_host[l]) for l, h in rng]
        preds = gather_ranges(preds, sizes, group)
        if preds is None:
            return None, None, None
    return preds, store.cand_labels, store.grp_off


def gather_ranges(local, sizes, group=None):
    """Ranks hold consecutive ranges of one packed vector (rank r: sizes[r] entries): one padded
    all_gather_into_tensor (RCCL on GPUs, gloo on CPUs) -> the whole vector on rank 0, None on
    the other ranks (replaces all_gather_object of Python lists, Manager.py:522-535)."""
    world, rank = _world(group)
    if local.numel() != sizes[rank]:
        raise ValueError("rank %d holds %d entries, sizes says %d" % (rank, local.numel(), sizes[rank]))
    cap = max(max(sizes), 1)
    buf = torch.zeros(cap, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    allp = torch.empty(cap * world, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(allp, buf, group=group)
    if rank != 0:
        return None
    return torch.cat([allp[r * cap:r * cap + sizes[r]] for r in range(world)])


def _parse_metrics(metrics):
    """Manager.py:1279-1345 metric names -> (wants, ndcg ks, hit ks)."""
    wants, nd, hit = [], [], []
    for m in metrics:
        if m in ("auc", "mean_mrr"):
            wants.append((m, None))
        elif m.startswith("ndcg") or m.startswith("hit"):
            ks = m.split("@")
            lst = [int(t) for t in ks[1].split(";")] if len(ks) > 1 else [1, 2]
            kind = "ndcg" if m.startswith("ndcg") else "hit"
            for k in lst:
                wants.append((kind, k))
                (nd if kind == "ndcg" else hit).append(k)
        elif m in ("rmse", "logloss", "acc", "f1"):
            raise ValueError("metric {0} is a flat (ungrouped) metric; the grouped device path computes "
                             "auc, mean_mrr, ndcg@k and hit@k".format(m))
        else:
            raise ValueError("not define this metric {0}".format(m))
    return wants, sorted(set(nd) | set(hit))


def cal_metric_packed(preds, labels, grp_off, metrics):
    """cal_metric (Manager.py:1276-1345) over packed groups: preds fp32 [n], labels int [n], group
    offsets int64 [G+1] (device tensors).  Per-group terms on the GPU, then np.mean and round(4)
    on the host exactly as the reference."""
    wants, ks = _parse_metrics(metrics)
    if len(ks) > 8:
        raise ValueError("at most 8 distinct cutoffs k per call")
    dev = preds.device
    G = grp_off.numel() - 1
    if labels.dtype != torch.int32:
        labels = labels.to(torch.int32)
    preds, labels, grp_off = preds.contiguous(), labels.contiguous(), grp_off.to(torch.int64).contiguous()
    if preds.dtype != torch.float32:
        preds = preds.float()
    ks_t = torch.tensor(ks if ks else [1], dtype=torch.int32, device=dev)
    W = 2 + 2 * len(ks)
    out = torch.empty(max(G, 1), W, dtype=torch.float64, device=dev)
    flags = torch.zeros(max(G, 1), dtype=torch.int32, device=dev)
    L.call("nr_impression_metrics", L.ptr(preds), L.ptr(labels), L.ptr(grp_off), G, L.ptr(ks_t), len(ks),
           L.ptr(out), L.ptr(flags), L.stream_ptr(preds))
    per = out[:G].cpu().numpy()
    fl = flags[:G].cpu().numpy()
    res = {}
    for kind, k in wants:
        if kind == "auc":
            if (fl & L.METRIC_ONE_CLASS).any():
                raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
            if (fl & L.METRIC_NONBINARY).any():
                raise ValueError("multiclass format is not supported")
            res["auc"] = round(np.mean(per[:, 0]), 4)
        elif kind == "mean_mrr":
            res["mean_mrr"] = round(np.mean(per[:, 1]), 4)
        elif kind == "ndcg":
            res["ndcg@{0}".format(k)] = round(np.mean(per[:, 2 + ks.index(k)]), 4)
        else:
            res["hit@{0}".format(k)] = round(np.mean(per[:, 2 + len(ks) + ks.index(k)]), 4)
    return res


def cal_metric(labels, preds, metrics, device="cuda"):
    """cal_metric(labels, preds, metrics) with the reference's signature (Manager.py:1276):
    labels / preds are lists of per-impression lists.  Packs them and runs on the GPU."""
    sizes = [len(p) for p in preds]
    if [len(l) for l in labels] != sizes:
        raise ValueError("labels and preds differ in shape")
    off = np.zeros(len(sizes) + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    p = torch.tensor([v for x in preds for v in x], dtype=torch.float32, device=device)
    y = torch.tensor([int(v) for x in labels for v in x], dtype=torch.int32, device=device)
    return cal_metric_packed(p, y, torch.from_numpy(off).to(device), metrics)


def evaluate(model, store, metrics=("auc", "mean_mrr", "ndcg@5;10"), batch_impr=1024, group=None,
             history_from_table=True):
    """Manager.evaluate (:544-590) with fast=True on a dev split: the metrics dict on rank 0,
    None elsewhere."""
    if store.mode != "dev":
        raise ValueError("evaluate needs a dev split with labels")
    preds, labels, grp_off = eval_fast(model, store, batch_impr, group, history_from_table)
    if preds is None:
        return None
    return cal_metric_packed(preds, labels, grp_off, list(metrics))

