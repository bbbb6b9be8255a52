"""Device-resident MIND dataset and batch formation.

The reference builds every impression on the host (utils/MIND.py:296-449 with newsample,
utils/utils.py:83-98), collates with the DataLoader (num_workers=0, Manager.py:79) and copies the
batch to the GPU (TwoTower.py:26-27,40-41).  Here the whole split lives in HBM:

  tok, attn     [N+1, L] int32   encoded_news / attn_mask truncated to L columns, last column
                                 forced to [SEP] when it is not [PAD] (MIND.py:100-108)
  his_off/ids   CSR click histories (behaviors.pkl "histories")
  neg_off/ids   CSR unclicked news per train impression ("negatives")
  imprs         [P, 2] int32 (impression index, clicked news) train samples ("imprs")
  chunks        dev/test: impression chunks of <= impr_size candidates ("imprs"), packed:
                cand_ids / cand_labels / cand_seg (chunk of each candidate), cand_off (CSR)

and one HIP launch (csrc/mind_batch.hip) forms a collated batch: the news-id -> token-row gather
and the negative sampling run on the device.  The batch dict has the reference's keys, shapes
and dtypes (int64 ids / tokens / masks, float64 his_mask / cdd_mask).

Negative sampling draws from a counter RNG (seed, offset) instead of Python's ``random``: the
structure (uniform npratio-subset of the impression's negatives in uniform random order, zero
padding and cdd_mask when there are fewer, label = 0 or the shuffled position) is the
reference's; the draws are not the same numbers.
"""
import numpy as np
import torch

from . import _lib as L
from .dist import Partition_Sampler, shard_train

PAD_TOKEN_ID, SEP_TOKEN_ID = 0, 102       # Manager.get_special_token_id for bert-base-uncased


def prepare_token_table(encoded_news, attn_mask, signal_length, pad_token_id=PAD_TOKEN_ID,
                        sep_token_id=SEP_TOKEN_ID):
    """MINDBaseDataset.__init__ news branch (utils/MIND.py:100-108): keep signal_length columns of
    the 512-column news.pkl arrays and put [SEP] in the last column when it is not [PAD]."""
    tok = np.array(np.asarray(encoded_news)[:, :signal_length], dtype=np.int64, copy=True)
    msk = np.array(np.asarray(attn_mask)[:, :signal_length], dtype=np.int64, copy=True)
    sep_pos = tok[:, -1] != pad_token_id
    tok[:, -1] = sep_token_id * sep_pos
    return tok, msk


def _csr(lists):
    off = np.zeros(len(lists) + 1, np.int64)
    if lists:
        off[1:] = np.cumsum([len(x) for x in lists])
    ids = np.fromiter((v for x in lists for v in x), dtype=np.int64, count=int(off[-1]))
    return off, ids


def _i32(a, name, lo=None, hi=None):
    a = np.asarray(a, dtype=np.int64)
    if a.size and ((lo is not None and a.min() < lo) or (hi is not None and a.max() >= hi)):
        raise ValueError("%s: values outside [%s, %s)" % (name, lo, hi))
    if a.size and (a.min() < -2 ** 31 or a.max() >= 2 ** 31):
        raise ValueError("%s: does not fit int32" % name)
    return a.astype(np.int32)


class MINDStore:
    """One MIND split (train / dev / test) resident in HBM, with the reference's __getitem__
    semantics for whole batches.

    news       dict with the news.pkl arrays {"encoded_news", "attn_mask"} ([N+1, >= L])
    behaviors  dict with the behaviors.pkl lists of the split (MIND.py:154-275):
               train {"imprs": [(impr_index, pos)], "histories", "negatives", "uindexes"},
               dev   {"imprs": [(impr_index, news, labels)], "histories", "uindexes"},
               test  {"imprs": [(impr_index, news)], "histories", "uindexes"}
    Options are the Manager attributes MINDBaseDataset reads (MIND.py:16-24)."""

    def __init__(self, news, behaviors, mode, his_size=50, signal_length=30, npratio=4, impr_size=2000,
                 shuffle_pos=False, descend_history=False, device="cuda", seed=None,
                 pad_token_id=PAD_TOKEN_ID, sep_token_id=SEP_TOKEN_ID):
        if mode not in ("train", "dev", "test"):
            raise ValueError("Mode {} not defined".format(mode))
        self.mode, self.his_size, self.signal_length = mode, int(his_size), int(signal_length)
        self.npratio, self.impr_size = int(npratio), int(impr_size)
        self.shuffle_pos, self.descend_history = bool(shuffle_pos), bool(descend_history)
        self.device = torch.device(device)
        tok, msk = prepare_token_table(news["encoded_news"], news["attn_mask"], self.signal_length,
                                       pad_token_id, sep_token_id)
        arrays = {"tok": tok, "attn": msk, "uindex": behaviors["uindexes"]}
        arrays["his_off"], arrays["his_ids"] = _csr(behaviors["histories"])
        imprs = behaviors["imprs"]
        if mode == "train":
            arrays["imprs"] = np.asarray([(i, p) for i, p in imprs], dtype=np.int64).reshape(-1, 2)
            arrays["neg_off"], arrays["neg_ids"] = _csr(behaviors["negatives"])
        else:
            arrays["chunk_impr"] = [c[0] for c in imprs]
            arrays["cand_off"], arrays["cand_ids"] = _csr([c[1] for c in imprs])
            if mode == "dev":
                arrays["cand_labels"] = _csr([c[2] for c in imprs])[1]
        self._upload(arrays, seed)

    @classmethod
    def from_arrays(cls, arrays, mode, seed=None, device="cuda", **opts):
        """A store from CSR arrays directly (the layout of ``save``; no per-impression Python
        lists): tok / attn [N+1, L] (already prepared), his_off / his_ids, uindex, and
        train: imprs [P, 2], neg_off / neg_ids; dev/test: chunk_impr, cand_off / cand_ids
        (+ cand_labels for dev)."""
        self = cls.__new__(cls)
        self.mode = mode
        self.his_size, self.signal_length = int(opts.get("his_size", 50)), int(np.asarray(arrays["tok"]).shape[1])
        self.npratio, self.impr_size = int(opts.get("npratio", 4)), int(opts.get("impr_size", 2000))
        self.shuffle_pos = bool(opts.get("shuffle_pos", False))
        self.descend_history = bool(opts.get("descend_history", False))
        self.device = torch.device(device)
        self._upload(arrays, seed)
        return self

    def save(self, path):
        """np.savez of the store's arrays (loads back with ``load``, no pickle)."""
        keys = ["tok", "attn", "his_off", "his_ids", "uindex"] + (
            ["imprs", "neg_off", "neg_ids"] if self.mode == "train" else
            ["chunk_impr", "cand_off", "cand_ids"] + (["cand_labels"] if self.mode == "dev" else []))
        meta = np.array([self.his_size, self.npratio, self.impr_size, int(self.shuffle_pos),
                         int(self.descend_history), ("train", "dev", "test").index(self.mode)], np.int64)
        np.savez(path, meta=meta, **{k: getattr(self, k).cpu().numpy() for k in keys})

    @classmethod
    def from_reference_cache(cls, news_pkl, behaviors_pkl, mode, device="cuda", seed=None, **opts):
        """A store from the caches the reference's MIND dataset writes:
        ``news.pkl`` = {"encoded_news": i64 [N+1, 512], "attn_mask": i64 [N+1, 512]}
        (utils/MIND.py:144-151) and the split's ``behaviors.pkl`` (:199-207 train, dev/test
        below it).  These are pickles: load only caches your own reference run wrote."""
        import pickle
        with open(news_pkl, "rb") as f:
            news = pickle.load(f)
        with open(behaviors_pkl, "rb") as f:
            behaviors = pickle.load(f)
        return cls(news, behaviors, mode, device=device, seed=seed, **opts)

    @classmethod
    def load(cls, path, device="cuda", seed=None):
        with np.load(path, allow_pickle=False) as z:
            meta = z["meta"]
            arrays = {k: z[k] for k in z.files if k != "meta"}
        mode = ("train", "dev", "test")[int(meta[5])]
        return cls.from_arrays(arrays, mode, seed=seed, device=device, his_size=meta[0], npratio=meta[1],
                               impr_size=meta[2], shuffle_pos=bool(meta[3]), descend_history=bool(meta[4]))

    def _upload(self, a, seed):
        mode, dev = self.mode, self.device
        tok = np.asarray(a["tok"])
        self.n_news = tok.shape[0]
        self.tok = torch.from_numpy(_i32(tok, "encoded_news")).to(dev)
        self.attn = torch.from_numpy(_i32(a["attn"], "attn_mask")).to(dev)
        his_off = np.asarray(a["his_off"], np.int64)
        if his_off.size == 0 or his_off[0] != 0 or (np.diff(his_off) < 0).any():
            raise ValueError("his_off is not a CSR offset array")
        self.n_impr = his_off.shape[0] - 1
        self.his_off = torch.from_numpy(his_off).to(dev)
        self.his_ids = torch.from_numpy(_i32(a["his_ids"], "histories", 0, self.n_news)).to(dev)
        uidx = _i32(a["uindex"], "uindexes")
        if uidx.shape[0] != self.n_impr:
            raise ValueError("uindexes has %d entries for %d impressions" % (uidx.shape[0], self.n_impr))
        self.uindex = torch.from_numpy(uidx).to(dev)
        # flags of the kernel: descend_history reverses train/dev histories; the test branch
        # applies the flag the other way round (MIND.py:339-342 vs :433-436)
        reverse = self.descend_history if mode != "test" else not self.descend_history
        self.flags = (L.BATCH_REVERSE_HISTORY if reverse else 0) | \
                     (L.BATCH_SHUFFLE_POS if (self.shuffle_pos and mode == "train") else 0)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = int(torch.initial_seed() if seed is None else seed) & 0xFFFFFFFFFFFF
        self.offset = 0
        if mode == "train":
            arr = np.asarray(a["imprs"], dtype=np.int64).reshape(-1, 2)
            _i32(arr[:, 0], "imprs impression index", 0, self.n_impr)
            _i32(arr[:, 1], "imprs clicked news", 0, self.n_news)
            self.imprs = torch.from_numpy(arr.astype(np.int32)).to(dev)
            neg_off = np.asarray(a["neg_off"], np.int64)
            if neg_off.shape[0] != self.n_impr + 1 or neg_off[0] != 0 or (np.diff(neg_off) < 0).any():
                raise ValueError("negatives: CSR offsets for %d impressions expected" % self.n_impr)
            self.neg_off = torch.from_numpy(neg_off).to(dev)
            self.neg_ids = torch.from_numpy(_i32(a["neg_ids"], "negatives", 0, self.n_news)).to(dev)
            self.n_samples = arr.shape[0]
        else:
            chunk_impr = _i32(a["chunk_impr"], "imprs impression index", 0, self.n_impr)
            n_chunks = chunk_impr.shape[0]
            self.chunk_impr = torch.from_numpy(chunk_impr).to(dev)
            cand_off = np.asarray(a["cand_off"], np.int64)
            if cand_off.shape[0] != n_chunks + 1 or cand_off[0] != 0 or (np.diff(cand_off) < 0).any():
                raise ValueError("candidates: CSR offsets for %d chunks expected" % n_chunks)
            cand_ids = np.asarray(a["cand_ids"], np.int64)
            _i32(cand_ids, "candidate news", 0, self.n_news)
            self.cand_off_host = cand_off
            self.cand_off = torch.from_numpy(cand_off).to(dev)
            self.cand_ids = torch.from_numpy(cand_ids).to(dev)
            seg = np.repeat(np.arange(n_chunks, dtype=np.int32), np.diff(cand_off))
            self.cand_seg = torch.from_numpy(seg).to(dev)
            if mode == "dev":
                self.cand_labels = torch.from_numpy(_i32(a["cand_labels"], "labels")).to(dev)
            else:
                self.cand_labels = None
            # impressions cut into several chunks regroup by impression index (_group_lists,
            # utils.py:60-80): consecutive chunks of one impression form one metric group
            starts = np.ones(n_chunks, bool)
            starts[1:] = chunk_impr[1:] != chunk_impr[:-1]
            first = np.flatnonzero(starts)
            if len(np.unique(chunk_impr)) != len(first):
                raise ValueError("chunks of one impression must be consecutive")
            grp = np.append(cand_off[first], cand_off[-1]).astype(np.int64)
            self.grp_off_host = grp
            self.grp_off = torch.from_numpy(grp).to(dev)
            self.n_samples = n_chunks

    def __len__(self):
        """MIND.__len__ (utils/MIND.py:289-294): train samples or dev/test chunks."""
        return self.n_samples

    # ------------------------------------------------------------------ batches
    def check_status(self):
        """Raise if a launch saw an out-of-range index (syncs the stream)."""
        s = int(self.status.item())
        if s:
            self.status.zero_()
            raise IndexError("MIND batch formation: %s" % ", ".join(
                m for b, m in ((1, "sample index out of range"), (2, "news id out of range"),
                               (4, "candidate/user row out of range")) if s & b))

    def train_batch(self, sample_idx, out=None, device_rng=False, epoch_batch=None):
        """Collated MIND.__getitem__ train outputs for the samples sample_idx (int64 [B],
        device or host).

        out: a dict from an earlier call to fill in place (a captured graph's static inputs).
        device_rng: draw from the device-resident (seed, offset) pair ``rng_state`` and advance
        it on the device (graph-capturable: every replay draws fresh negatives) instead of the
        host-side offset.
        epoch_batch = B (with device_rng): sample_idx is a whole epoch order on the device and each
        call forms its next batch of B from it (the cursor lives in ``rng_state`` and the launch
        advances it: a replayed graph walks the epoch with no copy per step)."""
        if self.mode != "train":
            raise ValueError("train_batch on a %s split" % self.mode)
        dev = self.device
        idx = torch.as_tensor(sample_idx, dtype=torch.int64)
        if not idx.is_cuda:
            if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= self.n_samples):
                raise IndexError("sample index out of range [0, %d)" % self.n_samples)
            idx = idx.to(dev, non_blocking=True)
        idx = idx.contiguous()
        if epoch_batch is not None and not device_rng:
            raise ValueError("epoch_batch needs device_rng (the cursor lives in rng_state)")
        B = idx.numel() if epoch_batch is None else int(epoch_batch)
        if epoch_batch is not None and not 0 < B <= idx.numel():
            raise ValueError("epoch_batch must be in (0, len(order)]")
        C, NH, Ls = self.npratio + 1, self.his_size, self.signal_length
        shapes = {"user_id": ((B,), torch.int64), "cdd_id": ((B, C), torch.int64), "his_id": ((B, NH), torch.int64),
                  "cdd_encoded_index": ((B, C, Ls), torch.int64), "his_encoded_index": ((B, NH, Ls), torch.int64),
                  "cdd_attn_mask": ((B, C, Ls), torch.int64), "his_attn_mask": ((B, NH, Ls), torch.int64),
                  "cdd_mask": ((B, C, 1), torch.float64), "his_mask": ((B, NH, 1), torch.float64),
                  "label": ((B,), torch.int64)}
        if out is None:
            x = {k: torch.empty(sh, dtype=dt, device=dev) for k, (sh, dt) in shapes.items()}
            # candidate and history titles back to back (one buffer each for tokens and masks): the
            # two-tower encoder reads them as one [B*(C+NH), Ls] batch without stacking them
            for a, b in (("cdd_encoded_index", "his_encoded_index"), ("cdd_attn_mask", "his_attn_mask")):
                buf = torch.empty(B * (C + NH) * Ls, dtype=torch.int64, device=dev)
                x[a] = buf[:B * C * Ls].view(B, C, Ls)
                x[b] = buf[B * C * Ls:].view(B, NH, Ls)
        else:
            x = out
            want_dev = torch.device(dev)
            for k, (sh, dt) in shapes.items():
                t = x[k]
                same_dev = t.device.type == want_dev.type and (want_dev.index is None or t.device.index == want_dev.index)
                if tuple(t.shape) != sh or t.dtype != dt or not t.is_contiguous() or not same_dev:
                    raise ValueError("out[%r]: expected contiguous %s %s on %s" % (k, sh, dt, dev))
        rng = None
        if device_rng:
            if getattr(self, "rng_state", None) is None:
                # {seed, offset, ticket, cursor, n_order, 0}: nr_form_train_batch advances the offset
                # (and, walking an epoch order, the cursor) itself
                self.rng_state = torch.tensor([self.seed, self.offset, 0, 0, 0, 0], dtype=torch.int64, device=dev)
                self._rng_order = None
            if epoch_batch is not None and getattr(self, "_rng_order", None) != idx.numel():
                self.rng_state[3:5] = torch.tensor([0, idx.numel()], dtype=torch.int64)
                self._rng_order = idx.numel()
            rng = self.rng_state
        seed, off = self.seed, self.offset
        self.offset += B * 4 * C
        P = L.ptr
        L.call("nr_form_train_batch", P(idx), B, P(self.imprs), self.n_samples, P(self.his_off), P(self.his_ids),
               P(self.neg_off), P(self.neg_ids), P(self.uindex), P(self.tok), P(self.attn), self.n_news, Ls,
               self.npratio, NH, self.flags | (L.BATCH_CURSOR if epoch_batch is not None else 0), seed, off, P(rng),
               P(x["cdd_id"]), P(x["his_id"]),
               P(x["cdd_encoded_index"]), P(x["cdd_attn_mask"]), P(x["his_encoded_index"]), P(x["his_attn_mask"]),
               P(x["cdd_mask"]), P(x["his_mask"]), P(x["user_id"]), P(x["label"]), P(self.status),
               L.stream_ptr(idx))
        return x

    def eval_batch(self, chunk0, n_chunks, with_tokens=False):
        """Dev/test chunks [chunk0, chunk0 + n_chunks) (MIND.__getitem__ dev/test branches,
        utils/MIND.py:367-449), batched: history side per chunk ([B, his_size] like the reference)
        and the chunks' candidates packed (cdd_id [n] int64 with cand_seg [n] = chunk index,
        label [n] for dev).  with_tokens: also the history token rows (the non-fast path)."""
        if self.mode == "train":
            raise ValueError("eval_batch on a train split")
        if chunk0 < 0 or n_chunks < 0 or chunk0 + n_chunks > self.n_samples:
            raise IndexError("chunks [%d, %d) outside [0, %d)" % (chunk0, chunk0 + n_chunks, self.n_samples))
        dev = self.device
        B, NH, Ls = n_chunks, self.his_size, self.signal_length
        i64 = dict(dtype=torch.int64, device=dev)
        x = {"impr_index": torch.empty(B, **i64), "user_id": torch.empty(B, **i64),
             "his_id": torch.empty(B, NH, **i64),
             "his_mask": torch.empty(B, NH, 1, dtype=torch.float64, device=dev)}
        if with_tokens:
            x["his_encoded_index"] = torch.empty(B, NH, Ls, **i64)
            x["his_attn_mask"] = torch.empty(B, NH, Ls, **i64)
        P = L.ptr
        L.call("nr_form_eval_batch", chunk0, B, P(self.chunk_impr), self.n_samples, P(self.his_off),
               P(self.his_ids), P(self.uindex), P(self.tok), P(self.attn), self.n_news, Ls, NH, self.flags,
               P(x["his_id"]), P(x.get("his_encoded_index")), P(x.get("his_attn_mask")), P(x["his_mask"]),
               P(x["user_id"]), P(x["impr_index"]), P(self.status), L.stream_ptr(self.tok))
        o0, o1 = int(self.cand_off_host[chunk0]), int(self.cand_off_host[chunk0 + n_chunks])
        x["cdd_id"] = self.cand_ids[o0:o1]
        x["cand_seg"] = self.cand_seg[o0:o1]
        x["chunk0"] = chunk0
        x["cand_range"] = (o0, o1)
        if self.cand_labels is not None:
            x["label"] = self.cand_labels[o0:o1]
        return x

    def news_rows(self, ids):
        """(encoded_news[ids], attn_mask[ids]) as int64 [len(ids), L] (MIND.py:340-343)."""
        ids = torch.as_tensor(ids, dtype=torch.int64).to(self.device).contiguous()
        n, Ls = ids.numel(), self.signal_length
        tok = torch.empty(n, Ls, dtype=torch.int64, device=self.device)
        msk = torch.empty(n, Ls, dtype=torch.int64, device=self.device)
        L.call("nr_gather_news_rows", L.ptr(ids), n, L.ptr(self.tok), L.ptr(self.attn), self.n_news, Ls,
               L.ptr(tok), L.ptr(msk), L.ptr(self.status), L.stream_ptr(ids))
        return tok, msk


class DeviceLoader:
    """DataLoader(MIND, batch_size, sampler=...) over a MINDStore (Manager.py:208-228): train
    splits follow DistributedSampler's strided, padded order (optionally shuffled per epoch);
    dev/test splits follow Partition_Sampler's contiguous chunk ranges (utils.py:267-283).
    Yields device batch dicts; nothing is formed on the host."""

    def __init__(self, store, batch_size, world_size=1, rank=0, shuffle=False, seed=0, drop_last=False):
        self.store, self.batch_size = store, int(batch_size)
        self.world_size, self.rank, self.shuffle, self.seed = world_size, rank, shuffle, seed
        self.drop_last, self.epoch = drop_last, 0

    def set_epoch(self, epoch):
        self.epoch = epoch

    def _indices(self):
        if self.store.mode == "train":
            if self.world_size > 1:
                return shard_train(len(self.store), self.world_size, self.rank, self.shuffle, self.seed, self.epoch)
            if self.shuffle:
                g = torch.Generator().manual_seed(self.seed + self.epoch)
                return torch.randperm(len(self.store), generator=g).tolist()
            return list(range(len(self.store)))
        part = Partition_Sampler(self.store, self.world_size, self.rank)
        return range(part.start, part.end)

    def __len__(self):
        n = len(self._indices())
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        idx = self._indices()
        n = len(idx)
        stop = n - n % self.batch_size if self.drop_last else n
        if self.store.mode == "train":
            dev_idx = torch.tensor(idx, dtype=torch.int64).to(self.store.device)   # one upload per epoch
            for s in range(0, stop, self.batch_size):
                yield self.store.train_batch(dev_idx[s:s + self.batch_size])
        else:
            for s in range(0, stop, self.batch_size):
                c0 = idx[s]
                yield self.store.eval_batch(c0, min(self.batch_size, stop - s))


def synthetic_arrays(mode, n_news, n_impr, his_len=(50, 100), neg_len=(4, 60), cand_len=(2, 75),
                     signal_length=30, vocab=30522, users=876956, full_titles=True, seed=0):
    """MIND-shaped synthetic split as ``MINDStore.from_arrays`` input: token ids
    U[1000, vocab) with [CLS]=101 first and [SEP]=102 at the last real position (all positions
    real when full_titles), row 0 = the padded "" news; histories / negatives / candidate lists
    with lengths drawn from the given ranges; dev chunks get at least one click each."""
    rng = np.random.default_rng(seed)
    Ls = signal_length
    tok = rng.integers(1000, vocab, (n_news, Ls), dtype=np.int64)
    lens = np.full(n_news, Ls) if full_titles else rng.integers(5, Ls + 1, n_news)
    msk = (np.arange(Ls)[None] < lens[:, None]).astype(np.int64)
    tok *= msk
    tok[:, 0] = 101
    tok[np.arange(n_news), lens - 1] = 102
    tok[0], msk[0] = 0, 0
    tok[0, :2], msk[0, :2] = (101, 102), 1

    def csr(lo_hi, n):
        ln = rng.integers(lo_hi[0], lo_hi[1] + 1, n)
        off = np.zeros(n + 1, np.int64)
        off[1:] = np.cumsum(ln)
        return off, rng.integers(1, n_news, int(off[-1]))

    a = {"tok": tok, "attn": msk, "uindex": rng.integers(1, users + 1, n_impr)}
    a["his_off"], a["his_ids"] = csr(his_len, n_impr)
    if mode == "train":
        a["neg_off"], a["neg_ids"] = csr(neg_len, n_impr)
        a["imprs"] = np.stack([np.arange(n_impr), rng.integers(1, n_news, n_impr)], 1)
    else:
        a["chunk_impr"] = np.arange(n_impr)
        a["cand_off"], a["cand_ids"] = csr(cand_len, n_impr)
        if mode == "dev":
            lab = (rng.random(int(a["cand_off"][-1])) < 0.04).astype(np.int64)
            first = a["cand_off"][:-1] + rng.integers(0, np.diff(a["cand_off"]))
            lab[first] = 1
            off = a["cand_off"]
            full = np.flatnonzero(np.add.reduceat(lab, off[:-1]) == np.diff(off))   # keep one unclicked
            lab[off[full] + (first[full] - off[full] + 1) % (off[full + 1] - off[full])] = 0
            a["cand_labels"] = lab
    return a


def write_reference_cache(news_pkl, behaviors_pkl, encoded_news, attn_mask, behaviors):
    """Write caches in the reference's on-disk format (utils/MIND.py:144-151 and :199-207) so the
    reference's own Manager / MIND dataset can run on them offline (the tokenizer is skipped when
    the caches exist).  ``behaviors`` is the split's dict ("imprs", "histories", "negatives" for
    train, "uindexes")."""
    import pickle
    with open(news_pkl, "wb") as f:
        pickle.dump({"encoded_news": np.asarray(encoded_news), "attn_mask": np.asarray(attn_mask)}, f)
    with open(behaviors_pkl, "wb") as f:
        pickle.dump(behaviors, f)
