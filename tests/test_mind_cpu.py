"""CPU checks of the device-side MIND data path's oracle and host logic.

The oracle (oracle/restatement.py mind_* / cal_metric) is pinned against what the reference's own
MIND dataset and cal_metric returned on a synthetic split (tests/golden/make_mind_golden.py):
every deterministic field exactly; the sampled negatives through the reference's recorded choice
(its draws come from Python's `random`, the device's from a counter RNG)."""
import json
import os
import socket

import numpy as np
import pytest
import torch

from mind_util import GOLDEN, load_data, load_ref
from oracle import restatement as R
from newsrec_amd.mind import DeviceLoader, MINDStore, prepare_token_table


@pytest.fixture(scope="module")
def data():
    return load_data()


@pytest.fixture(scope="module")
def ref():
    return load_ref()


def test_token_table_matches_reference(data, ref):
    news, _, opts = data
    tok, msk = prepare_token_table(news["encoded_news"], news["attn_mask"], opts["signal_length"])
    np.testing.assert_array_equal(tok, ref["table_tok"])
    np.testing.assert_array_equal(msk, ref["table_attn"])
    assert (tok[:, -1][tok[:, -1] != 0] == 102).all()


@pytest.mark.parametrize("key,desc", [("train_s0_d0", False), ("train_s0_d1", True)])
def test_oracle_train_items_match_reference(data, ref, key, desc):
    news, beh, opts = data
    tr = beh["train"]
    tok, msk = ref["table_tok"], ref["table_attn"]
    k = opts["npratio"]
    for i in range(len(tr["imprs"])):
        rec_cdd = ref[key + "/cdd_id"][i]
        neg_num = int(ref[key + "/cdd_mask"][i].sum()) - 1
        negs = tr["negatives"][tr["imprs"][i][0]]
        # the reference's draw: distinct negatives of this impression, or all of them + zeros
        if k > len(negs):
            assert list(rec_cdd[1:]) == negs + [0] * (k - len(negs))
        else:
            assert len(set(rec_cdd[1:].tolist())) == k and set(rec_cdd[1:].tolist()) <= set(negs)
        x = R.mind_train_item(tr["imprs"], tr["histories"], tr["negatives"], tr["uindexes"], tok, msk, i, k,
                              opts["his_size"], reverse=desc,
                              choose=lambda n, kk, c=rec_cdd, m=neg_num: (list(c[1:]), m))
        np.testing.assert_array_equal(x["cdd_id"], rec_cdd)
        np.testing.assert_array_equal(x["his_id"], ref[key + "/his_id"][i])
        np.testing.assert_array_equal(x["his_mask"], ref[key + "/his_mask"][i])
        np.testing.assert_array_equal(x["cdd_mask"], ref[key + "/cdd_mask"][i])
        assert x["label"] == ref[key + "/label"][i] == 0
        assert x["user_id"] == ref[key + "/user_id"][i]


def test_oracle_shuffle_pos_matches_reference(data, ref):
    news, beh, opts = data
    tr = beh["train"]
    key = "train_s1_d0"
    k = opts["npratio"]
    for i in range(len(tr["imprs"])):
        rec = ref[key + "/cdd_id"][i]
        lab = int(ref[key + "/label"][i])
        assert rec[lab] == tr["imprs"][i][1]
        negs_in_order = [v for j, v in enumerate(rec.tolist()) if j != lab]
        perm, nxt = [], 1
        for j in range(k + 1):
            perm.append(0 if j == lab else nxt)
            nxt += j != lab
        neg_num = int(ref[key + "/cdd_mask"][i].sum()) - 1
        x = R.mind_train_item(tr["imprs"], tr["histories"], tr["negatives"], tr["uindexes"], ref["table_tok"],
                              ref["table_attn"], i, k, opts["his_size"], shuffle_pos=True, perm=perm,
                              choose=lambda n, kk, v=negs_in_order, m=neg_num: (v, m))
        np.testing.assert_array_equal(x["cdd_id"], rec)
        assert x["label"] == lab
        np.testing.assert_array_equal(x["cdd_mask"], ref[key + "/cdd_mask"][i])


@pytest.mark.parametrize("key", ["dev_s0_d0", "dev_s0_d1", "test_s0_d0", "test_s0_d1"])
def test_oracle_eval_items_match_reference(data, ref, key):
    news, beh, opts = data
    split = key.split("_")[0]
    desc = key.endswith("d1")
    b = beh[split]
    chunk_impr = [c[0] for c in b["imprs"]]
    cands = [c[1] for c in b["imprs"]]
    labels = [c[2] for c in b["imprs"]] if split == "dev" else None
    reverse = desc if split == "dev" else not desc
    lens = ref[key + "/cdd_id_len"]
    off = np.concatenate([[0], np.cumsum(lens)])
    for c in range(len(chunk_impr)):
        x = R.mind_eval_item(chunk_impr, cands, labels, b["histories"], b["uindexes"], c, opts["his_size"], reverse)
        np.testing.assert_array_equal(x["cdd_id"], ref[key + "/cdd_id"][off[c]:off[c + 1]])
        np.testing.assert_array_equal(x["his_id"], ref[key + "/his_id"][c])
        np.testing.assert_array_equal(x["his_mask"], ref[key + "/his_mask"][c])
        assert x["impr_index"] == ref[key + "/impr_index"][c]
        assert x["user_id"] == ref[key + "/user_id"][c]
        if labels is not None:
            np.testing.assert_array_equal(x["label"], ref[key + "/label"][off[c]:off[c + 1]])


def test_oracle_metrics_match_reference():
    for case in json.load(open(os.path.join(GOLDEN, "cal_metric.json"))):
        got = R.cal_metric(case["labels"], case["preds"], ["auc", "mean_mrr", "ndcg@5;10"])
        for k, v in got.items():
            assert v == case["res"][k], k
    for case in json.load(open(os.path.join(GOLDEN, "metric_ref.json"))):
        gl, gp = R.group_lists(case["impr_index"], case["labels"], case["preds"])
        got = R.cal_metric(gl, gp, ["auc", "mean_mrr", "ndcg@1;3;5;10"])
        assert got == case["res"]


def test_oracle_metric_ties_and_errors():
    # stable-reversed tie order: of two equal scores the later index ranks first
    assert R._mrr([1, 0], [0.5, 0.5]) == pytest.approx(0.5)
    assert R._mrr([0, 1], [0.5, 0.5]) == pytest.approx(1.0)
    assert R._auc([1, 0, 0], [0.5, 0.5, 0.1]) == pytest.approx(0.75)
    assert R._hit([0, 1, 0], [0.9, 0.8, 0.1], 1) == 0 and R._hit([0, 1, 0], [0.9, 0.8, 0.1], 2) == 1
    with pytest.raises(ValueError):
        R._auc([1, 1], [0.2, 0.3])
    with pytest.raises(ValueError):
        R.cal_metric([[1, 0]], [[0.1, 0.2]], ["bogus"])


def test_oracle_sampler_is_uniform():
    """Floyd subset + Fisher-Yates order: every negative appears with frequency k/n, every slot
    is uniform, picks are distinct."""
    negs = list(range(100, 110))
    n, k, trials = len(negs), 4, 6000
    cnt = np.zeros((k, n))
    for t in range(trials):
        picks, m = R.mind_sample_negatives(negs, k, 12345, t * 64)
        assert m == k and len(set(picks)) == k
        for s, v in enumerate(picks):
            cnt[s, v - 100] += 1
    expect = trials / n
    assert np.abs(cnt - expect).max() < 6 * np.sqrt(expect)
    assert R.mind_sample_negatives([7, 8], 4, 1, 0) == ([7, 8, 0, 0], 2)
    assert R.mind_sample_negatives([], 4, 1, 0) == ([0, 0, 0, 0], 0)


def test_store_layout_cpu(data, tmp_path):
    news, beh, opts = data
    dv = MINDStore(news, beh["dev"], "dev", device="cpu", **opts)
    chunk_impr = [c[0] for c in beh["dev"]["imprs"]]
    assert len(dv) == len(chunk_impr)
    # groups = impressions (chunks of one impression merged), _group_lists order
    sizes = {}
    for c, (imp, cand, _) in enumerate(beh["dev"]["imprs"]):
        sizes[imp] = sizes.get(imp, 0) + len(cand)
    np.testing.assert_array_equal(np.diff(dv.grp_off_host), list(sizes.values()))
    np.testing.assert_array_equal(dv.cand_seg.numpy(), np.repeat(np.arange(len(chunk_impr)),
                                                                 [len(c[1]) for c in beh["dev"]["imprs"]]))
    p = str(tmp_path / "dev.npz")
    dv.save(p)
    dv2 = MINDStore.load(p, device="cpu")
    for k in ("tok", "attn", "his_off", "his_ids", "cand_ids", "cand_labels", "grp_off"):
        assert torch.equal(getattr(dv, k), getattr(dv2, k)), k
    tr = MINDStore(news, beh["train"], "train", device="cpu", **opts)
    assert len(tr) == len(beh["train"]["imprs"])
    assert tr.flags == 0 and MINDStore(news, beh["test"], "test", device="cpu", **opts).flags == 1


def test_store_rejects_bad_ids(data):
    news, beh, opts = data
    bad = dict(beh["train"])
    bad["histories"] = [list(h) for h in bad["histories"]]
    bad["histories"][0] = [10 ** 6]
    with pytest.raises(ValueError):
        MINDStore(news, bad, "train", device="cpu", **opts)
    bad = dict(beh["dev"])
    bad["imprs"] = list(bad["imprs"])
    bad["imprs"][0] = (0, [-1], [0])
    with pytest.raises(ValueError):
        MINDStore(news, bad, "dev", device="cpu", **opts)


def test_device_loader_indices(data):
    from newsrec_amd.dist import shard_train
    news, beh, opts = data
    tr = MINDStore(news, beh["train"], "train", device="cpu", **opts)
    for r in range(2):
        ld = DeviceLoader(tr, 8, world_size=2, rank=r, shuffle=True, seed=3)
        assert ld._indices() == shard_train(len(tr), 2, r, True, 3, 0)
    dv = MINDStore(news, beh["dev"], "dev", device="cpu", **opts)
    parts = [DeviceLoader(dv, 4, world_size=3, rank=r)._indices() for r in range(3)]
    assert [i for p in parts for i in p] == list(range(len(dv)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    from newsrec_amd.evaluate import gather_ranges, gather_shards
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = [5, 0, 7][:world]
    start = sum(sizes[:rank])
    local = torch.arange(start, start + sizes[rank], dtype=torch.float32)
    full = gather_ranges(local, sizes)
    shard = torch.full((4, 3), float(rank))
    table = gather_shards(shard, 4 * world - 2)
    q.put((rank, None if full is None else full.tolist(), table[:, 0].tolist()))
    dist.destroy_process_group()


def test_eval_gathers_gloo():
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, full, col = q.get(timeout=120)
        out[r] = (full, col)
    for p in procs:
        p.join(30)
    assert out[0][0] == list(range(12)) and out[1][0] is None
    for r in range(world):
        assert out[r][1] == [0.0] * 4 + [1.0] * 4 + [2.0] * 2


def test_reference_cache_round_trip(tmp_path):
    """news.pkl / behaviors.pkl in the reference's format (MIND.py:144-151, :199-207) -> MINDStore:
    the token table is truncated to L with [SEP] forced (MIND.py:103-108), CSR arrays match."""
    import numpy as np
    from newsrec_amd.mind import MINDStore, write_reference_cache
    rng = np.random.default_rng(0)
    enc = rng.integers(1000, 30000, (7, 512))
    enc[:, 0] = 101
    msk = np.ones((7, 512), np.int64)
    enc[0, 2:] = 0
    msk[0, 2:] = 0
    beh = {"imprs": [(0, 3), (1, 5)], "histories": [[1, 2], []], "negatives": [[4, 6], [1]], "uindexes": [7, 9]}
    write_reference_cache(tmp_path / "news.pkl", tmp_path / "behaviors.pkl", enc, msk, beh)
    st = MINDStore.from_reference_cache(tmp_path / "news.pkl", tmp_path / "behaviors.pkl", "train", device="cpu",
                                        signal_length=30)
    tok = st.tok.numpy()
    assert tok.shape == (7, 30)
    assert (tok[1:, -1] == 102).all() and tok[0, -1] == 0
    assert (tok[1:, :-1] == enc[1:, :29]).all()
    assert st.his_off.tolist() == [0, 2, 2] and st.his_ids.tolist() == [1, 2]
    assert st.neg_off.tolist() == [0, 2, 3] and st.neg_ids.tolist() == [4, 6, 1]
    assert st.imprs.tolist() == [[0, 3], [1, 5]] and st.uindex.tolist() == [7, 9]
