"""The synthetic MIND split of tests/golden/mind_data.npz (written by make_mind_golden.py from the
reference's own dataset code) as the behaviors.pkl / news.pkl dicts the reference reads, plus the
reference's recorded __getitem__ outputs (mind_ref.npz)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _lists(off, ids):
    return [[int(v) for v in ids[off[i]:off[i + 1]]] for i in range(len(off) - 1)]


def load_data():
    z = np.load(os.path.join(GOLDEN, "mind_data.npz"))
    d = {k: z[k] for k in z.files}
    n_news, L, his, npratio, impr_size, sep, pad = (int(v) for v in d["meta"])
    news = {"encoded_news": d["raw_tok"], "attn_mask": d["raw_attn"]}
    train = {"imprs": [tuple(int(v) for v in r) for r in d["tr_imprs"]],
             "histories": _lists(d["tr_his_off"], d["tr_his_ids"]),
             "negatives": _lists(d["tr_neg_off"], d["tr_neg_ids"]),
             "uindexes": [int(v) for v in d["tr_uindex"]]}
    cands = _lists(d["dv_cand_off"], d["dv_cand_ids"])
    labels = _lists(d["dv_cand_off"], d["dv_cand_labels"])
    chunk_impr = [int(v) for v in d["dv_chunk_impr"]]
    dev = {"imprs": [(i, c, l) for i, c, l in zip(chunk_impr, cands, labels)],
           "histories": _lists(d["dv_his_off"], d["dv_his_ids"]),
           "uindexes": [int(v) for v in d["dv_uindex"]]}
    test = {"imprs": [(i, c) for i, c in zip(chunk_impr, cands)], "histories": dev["histories"],
            "uindexes": dev["uindexes"]}
    opts = {"his_size": his, "signal_length": L, "npratio": npratio, "impr_size": impr_size}
    return news, {"train": train, "dev": dev, "test": test}, opts


def load_ref():
    z = np.load(os.path.join(GOLDEN, "mind_ref.npz"))
    return {k: z[k] for k in z.files}


def store_arrays(store):
    """A MINDStore's arrays as numpy (the oracle's input)."""
    keys = ["tok", "attn", "his_off", "his_ids", "uindex", "imprs", "neg_off", "neg_ids"]
    return {k: getattr(store, k).cpu().numpy() for k in keys if hasattr(store, k)}
