"""Distinct-row projection path: nr_unique_rows / nr_segment_rows_sum / nr_gemm_f32_dyn and the
yrows indirection of the fused MHA pool kernels, each against a plain torch / numpy statement
of the same operation; then the MHA news Function with and without dedup on the same inputs."""
import numpy as np
import pytest
import torch

from newsrec_amd import _lib as L
from newsrec_amd import functions as F
from newsrec_amd import kernels as K

pytestmark = pytest.mark.gpu


def _ids(T, V, seed, pad_frac=0.4):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, V, (T,), generator=g)
    ids[torch.rand(T, generator=g) < pad_frac] = 0
    return ids


# V <= 65536: count + fused scan (one launch); 200000: the multi-tile scan (two more launches)
@pytest.mark.parametrize("T,V", [(1, 5), (37, 7), (1000, 30522), (52800, 30522), (4096, 100), (60000, 200000),
                                 (20000, 65536), (5000, 900000), (3000, 1200000)])
def test_unique_rows(T, V):
    ids = _ids(T, V, T + V)
    ur = K.UniqueRows(ids.cuda(), V, fill_row=0)
    torch.cuda.synchronize()
    U, Up, bad, Tc = ur.counts.tolist()
    ref = np.unique(ids.numpy())
    assert bad == 0 and U == len(ref) and Up == (U + 31) // 32 * 32
    uids = ur.uids.cpu().numpy()
    assert (uids[:U] == ref).all() and (uids[U:Up] == 0).all()
    inv = ur.inv.cpu().numpy()
    assert (uids[inv] == ids.numpy()).all()
    off = ur.seg_off.cpu().numpy()
    tok = ur.seg_tok.cpu().numpy()
    assert off[0] == 0 and off[Up] == T and (off[U:Up + 1] == T).all()
    for u in np.random.default_rng(0).choice(U, size=min(U, 200), replace=False):
        seg = np.sort(tok[off[u]:off[u + 1]])
        assert (seg == np.nonzero(ids.numpy() == uids[u])[0]).all()


def test_unique_rows_grad_mask_segments():
    T, V = 5000, 700
    ids = _ids(T, V, 99)
    gm = (torch.rand(T, generator=torch.Generator().manual_seed(5)) < 0.6)
    gm[ids == 0] = False
    ur = K.UniqueRows(ids.cuda(), V, fill_row=0, grad_mask=gm.long().cuda())
    torch.cuda.synchronize()
    U, Up, bad, Tc = ur.counts.tolist()
    assert U == len(np.unique(ids.numpy())) and Tc == int(gm.sum())
    uids, off, tok = ur.uids.cpu().numpy(), ur.seg_off.cpu().numpy(), ur.seg_tok.cpu().numpy()
    assert off[Up] == Tc
    for u in range(U):
        seg = np.sort(tok[off[u]:off[u + 1]])
        want = np.nonzero((ids.numpy() == uids[u]) & gm.numpy())[0]
        assert (seg == want).all()
    src = torch.randn(T, 64, device="cuda")
    dst = torch.full((ur.cap, 64), float("nan"), device="cuda")
    ur.segment_sum(src, dst)
    ref = torch.zeros(ur.cap, 64, dtype=torch.float64, device="cuda")
    g = gm.cuda()
    ref.index_add_(0, ur.inv[g], src[g].double())
    torch.cuda.synchronize()
    torch.testing.assert_close(dst[:Up].double(), ref[:Up], rtol=1e-5, atol=1e-5)   # empty segments: 0


@pytest.mark.parametrize("V", [5, 100000])
def test_unique_rows_flags_bad_ids(V):
    ids = torch.tensor([0, 3, V + 4, 2], dtype=torch.int64)
    ur = K.UniqueRows(ids.cuda(), V)
    torch.cuda.synchronize()
    U, Up, bad, Tc = ur.counts.tolist()
    assert bad == 1 and U == 3 and Tc == 3
    # the workspace is self-cleaning: the next call on the same buffer starts from zero counters
    ur2 = K.UniqueRows(torch.tensor([1, 1, 2], dtype=torch.int64).cuda(), V)
    torch.cuda.synchronize()
    assert ur2.counts.tolist() == [2, 32, 0, 3]


@pytest.mark.parametrize("V", [30522, 100000])
def test_unique_rows_repeated_calls_and_empty(V):
    """Back-to-back calls on the one persistent workspace (its counters and control words must come
    back zero after every call), an empty batch among them."""
    for i, T in enumerate([5000, 0, 1, 30000, 5000]):
        ids = _ids(T, V, 1000 + i)
        ur = K.UniqueRows(ids.cuda(), V, fill_row=0)
        torch.cuda.synchronize()
        U, Up, bad, Tc = ur.counts.tolist()
        ref = np.unique(ids.numpy())
        assert (U, Up, bad, Tc) == (len(ref), (len(ref) + 31) // 32 * 32, 0, T)
        assert (ur.uids[:U].cpu().numpy() == ref).all()
        if T:
            assert (ur.uids.cpu().numpy()[ur.inv.cpu().numpy()] == ids.numpy()).all()
    ws = K._SELF_CLEANING[(torch.device("cuda", 0), f"nr_unique_rows/{V}")]
    V4 = (V + 3) // 4 * 4
    assert int(ws[:4 + 2 * V4].abs().sum()) == 0   # ctrl words + both counters back to zero
    assert int(ws[4 + 4 * V4:].abs().sum()) == 0    # the vocabulary tiles' totals too
    assert K.self_cleaning_check("cuda") == []


def test_unique_rows_dirty_tile_totals_detected():
    """The tile totals (tot, after the scratch arrays) must be zero on entry like the counters: a call
    stopped between count and fill would leave them set.  self_cleaning_check reports that and
    reset=True clears them, after which the next call is exact again."""
    V = 30522
    K.UniqueRows(_ids(100, V, 1).cuda(), V)
    ws = K._SELF_CLEANING[(torch.device("cuda", 0), f"nr_unique_rows/{V}")]
    V4 = (V + 3) // 4 * 4
    ws[4 + 4 * V4] = 7                                  # a stale tile total
    assert f"nr_unique_rows/{V}" in K.self_cleaning_check("cuda", reset=True)
    assert K.self_cleaning_check("cuda") == []
    ids = _ids(5000, V, 2)
    ur = K.UniqueRows(ids.cuda(), V)
    torch.cuda.synchronize()
    ref = np.unique(ids.numpy())
    assert ur.counts.tolist()[0] == len(ref) and (ur.uids[:len(ref)].cpu().numpy() == ref).all()


@pytest.mark.parametrize("T,V,W", [(300, 50, 1152), (52800, 30522, 1152), (33, 4, 4)])
def test_segment_sum(T, V, W):
    ids = _ids(T, V, 7 * T)
    ur = K.UniqueRows(ids.cuda(), V)
    src = torch.randn(T, W, device="cuda")
    dst = torch.full((ur.cap, W), float("nan"), device="cuda")
    ur.segment_sum(src, dst)
    torch.cuda.synchronize()
    U, Up, _, _ = ur.counts.tolist()
    ref = torch.zeros(ur.cap, W, dtype=torch.float64, device="cuda")
    ref.index_add_(0, ur.inv, src.double())
    # fp32 sums of n unit-variance terms: tolerance grows with the segment length n
    n = torch.bincount(ur.inv, minlength=ur.cap)[:U].double()[:, None]
    err = (dst[:U].double() - ref[:U]).abs()
    assert (err <= 1e-5 + 1e-6 * n).all(), float((err - 1e-6 * n).max())
    assert (dst[U:Up] == 0).all()


def test_gemm_dyn_rows_and_k():
    torch.manual_seed(0)
    V, E, N = 2000, 256, 384
    table = torch.randn(V, E, device="cuda")
    W = torch.randn(N, E, device="cuda") * 0.05
    b = torch.randn(N, device="cuda")
    ids = _ids(5000, V, 3).cuda()
    ur = K.UniqueRows(ids, V)
    Y = torch.full((ur.cap, N), float("nan"), device="cuda")
    K.gemm_dyn(ur.cap, N, E, K.operand(table, L.KCONTIG, rows=ur.uids, mapping=L.ROWS_GATHER),
               K.operand(W, L.KCONTIG), Y, m_dev=ur.u_pad, bias=b)
    torch.cuda.synchronize()
    Up = int(ur.counts[1])
    ref = table[ur.uids[:Up]].double() @ W.double().t() + b.double()
    torch.testing.assert_close(Y[:Up].double(), ref, rtol=1e-4, atol=1e-4)
    assert torch.isnan(Y[Up:]).all()   # rows past the device extent untouched
    # K from the device: dW = dYuᵀ table[uids] over U_pad rows, split-K atomic
    dYu = torch.randn(ur.cap, N, device="cuda")
    dW = torch.zeros(N, E, device="cuda")
    K.gemm_dyn(N, E, ur.cap, K.operand(dYu, L.MNCONTIG), K.operand(table, L.MNCONTIG, rows=ur.uids,
               mapping=L.ROWS_GATHER), dW, k_dev=ur.u_pad, epilogue=L.EPI_ATOMIC, split_k=7)
    torch.cuda.synchronize()
    ref = dYu[:Up].double().t() @ table[ur.uids[:Up]].double()
    torch.testing.assert_close(dW.double(), ref, rtol=1e-4, atol=1e-3)
    # scatter dgrad into a table gradient over the distinct rows
    dtab = torch.zeros(V, E, device="cuda")
    K.gemm_dyn(ur.cap, E, N, K.operand(dYu, L.KCONTIG), K.operand(W, L.MNCONTIG), dtab, m_dev=ur.u_pad,
               epilogue=L.EPI_SCATTER, c_rows=K.rows_map(ur.uids, L.ROWS_GATHER), pad_row=0)
    torch.cuda.synchronize()
    ref = torch.zeros(V, E, dtype=torch.float64, device="cuda")
    ref.index_add_(0, ur.uids[:Up], dYu[:Up].double() @ W.double())
    ref[0] = 0
    torch.testing.assert_close(dtab.double(), ref, rtol=1e-4, atol=1e-4)
    # the same through plain row stores over the U distinct rows
    dtab2 = torch.zeros(V, E, device="cuda")
    K.gemm_dyn(ur.cap, E, N, K.operand(dYu, L.KCONTIG), K.operand(W, L.MNCONTIG), dtab2, m_dev=ur.n_rows,
               epilogue=L.EPI_SCATTER_STORE, c_rows=K.rows_map(ur.uids, L.ROWS_GATHER), pad_row=0)
    torch.cuda.synchronize()
    torch.testing.assert_close(dtab2.double(), ref, rtol=1e-4, atol=1e-4)


def test_mha_pool_yrows_matches_gathered():
    torch.manual_seed(1)
    n, Lq, heads, dk, dv = 64, 30, 12, 64, 32
    T, NY, H = n * Lq, heads * (dk + dv), heads * dv
    ids = _ids(T, 500, 11).cuda()
    ur = K.UniqueRows(ids, 500)
    Yu = torch.randn(ur.cap, NY, device="cuda") * 0.3
    Yt = Yu[ur.inv].contiguous()
    mask = (torch.rand(n, Lq, device="cuda") < 0.8).long()
    mask[:, 0] = 1
    gamma = 1 + 0.1 * torch.randn(H, device="cuda")
    beta = 0.1 * torch.randn(H, device="cuda")
    q = torch.randn(H, device="cuda")
    outs = []
    for Y, yrows in ((Yt, None), (Yu, ur.inv)):
        news = torch.empty(n, H, device="cuda")
        stats = torch.empty(T, 2, device="cuda")
        probs = torch.empty(T, device="cuda")
        K.mha_pool_fwd(Y, mask, n, Lq, heads, dk, dv, gamma, beta, q, news, stats, probs, p_drop=0.2, seed=5,
                       offset=9, yrows=yrows)
        dnews = torch.ones(n, H, device="cuda")
        dy = torch.empty(T, NY, device="cuda")
        db, dq, dg, dbt = (torch.zeros(NY, device="cuda"), torch.zeros(H, device="cuda"),
                           torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda"))
        K.mha_pool_bwd(Y, mask, n, Lq, heads, dk, dv, gamma, beta, q, stats, probs, dnews, dy, db, dq, dg, dbt,
                       p_drop=0.2, seed=5, offset=9, yrows=yrows)
        outs.append((news, dy))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])   # same rows, same arithmetic: bitwise
    assert torch.equal(outs[0][1], outs[1][1])


def test_mha_news_dedup_vs_tokenwise(monkeypatch):
    torch.manual_seed(2)
    V, E, heads, dk, dv, Lq, n = 3000, 768, 12, 64, 32, 30, 96
    H, NY = heads * dv, heads * (dk + dv)
    table = (torch.randn(V, E, device="cuda") * 0.5).requires_grad_()
    ids = _ids(n * Lq, V, 21).cuda()
    mask = (ids != 0).long().view(n, Lq)
    mask[:, 0] = 1
    w = (torch.randn(NY, E, device="cuda") * 0.03).requires_grad_()
    b = (torch.randn(NY, device="cuda") * 0.1).requires_grad_()
    gamma = torch.ones(H, device="cuda", requires_grad=True)
    beta = torch.zeros(H, device="cuda", requires_grad=True)
    q = torch.randn(1, H, device="cuda", requires_grad=True)
    res = []
    for dedup in (False, True):
        monkeypatch.setattr(F, "DEDUP_ROWS", dedup)
        for t in (table, w, b, gamma, beta, q):
            t.grad = None
        news, _ = F.MHANewsFn.apply(table, ids, mask, w, b, gamma, beta, q, heads, dk, dv, Lq, 0, 0.2, 3, 4, False)
        (news * torch.linspace(-1, 1, H, device="cuda")).sum().backward()
        res.append([news.detach().clone()] + [t.grad.clone() for t in (table, w, b, gamma, beta, q)])
    torch.cuda.synchronize()
    from newsrec_amd import _lib as Lb
    if K.get_gemm_precision() == Lb.GEMM_F32:
        assert torch.equal(res[0][0], res[1][0])   # forward: identical rows, identical arithmetic
    else:   # bf16x6: the small token-wise GEMM runs on the f32 64x64 kernel, the distinct-row one on bf16x6
        torch.testing.assert_close(res[1][0], res[0][0], rtol=1e-5, atol=1e-5)
    for a, c in zip(res[0][1:], res[1][1:]):   # backward: same sums, different fp32 order
        torch.testing.assert_close(c, a, rtol=1e-4, atol=5e-5)


def test_segment_sum_multi_leaves_single_rows():
    """nr_segment_rows_sum_multi: the rows of two or more CSR tokens are summed as by
    nr_segment_rows_sum (same order: bitwise), a one-token row keeps what its producer wrote; pad rows
    and rows without a gradient-carrying token are zero."""
    g = torch.Generator().manual_seed(4)
    T, V, W = 3000, 900, 1152
    ids = torch.randint(0, V, (T,), generator=g).cuda()
    gm = (torch.rand(T, generator=g) < 0.7).long().cuda()
    ur = K.UniqueRows(ids, V, grad_mask=gm)
    src = torch.randn(T, W, device="cuda")
    full = torch.empty(ur.cap, W, device="cuda")
    ur.segment_sum(src, full)
    dst = torch.full((ur.cap, W), 7.0, device="cuda")
    ur.segment_sum_multi(src, dst)
    torch.cuda.synchronize()
    up = int(ur.counts[1].item())   # rows [0, U_pad) are the sums' extent
    seg = ur.seg_off[:up + 1].long()
    single = (seg[1:] - seg[:-1]) == 1
    assert single.any() and (~single).any()
    assert torch.equal(dst[:up][~single], full[:up][~single])
    assert (dst[:up][single] == 7.0).all()


@pytest.mark.parametrize("form", ["split", "fused_saved", "recompute"])
def test_mha_pool_bwd_single_rows_direct(form):
    """nr_mha_pool_bwd with seg_off: a token alone in its distinct row's segment writes its gradient
    row straight to the per-distinct-row sums; with nr_segment_rows_sum_multi the sums equal the
    per-token backward + nr_segment_rows_sum, bitwise -- ragged masks, dropout, the three backward
    forms."""
    torch.manual_seed(3)
    n, Lq, heads, dk, dv = 80, 30, 12, 64, 32
    T, NY, H = n * Lq, heads * (dk + dv), heads * dv
    ids = _ids(T, 700, 13).cuda()
    mask = (torch.rand(n, Lq, device="cuda") < 0.75).long()
    mask[:, 0] = 1
    ur = K.UniqueRows(ids, 700, grad_mask=mask)
    Yu = torch.randn(ur.cap, NY, device="cuda") * 0.3
    gamma = 1 + 0.1 * torch.randn(H, device="cuda")
    beta = 0.1 * torch.randn(H, device="cuda")
    q = torch.randn(H, device="cuda")
    news = torch.empty(n, H, device="cuda")
    stats = torch.empty(T, 2, device="cuda")
    probs = torch.empty(T, device="cuda")
    O = torch.empty(T, H, device="cuda") if form != "recompute" else None
    K.mha_pool_fwd(Yu, mask, n, Lq, heads, dk, dv, gamma, beta, q, news, stats, probs, p_drop=0.2, seed=5,
                   offset=9, yrows=ur.inv, oout=O)
    dnews = torch.randn(n, H, device="cuda")
    outs = []
    for direct in (False, True):
        dyall = torch.full((T + ur.cap, NY), float("nan"), device="cuda")
        dob = torch.empty(T, 8, device="cuda") if form == "split" else None
        db, dq, dg, dbt = (torch.zeros(NY, device="cuda"), torch.zeros(H, device="cuda"),
                           torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda"))
        K.mha_pool_bwd(Yu, mask, n, Lq, heads, dk, dv, gamma, beta, q, stats, probs, dnews,
                       dyall if direct else dyall[:T], db, dq, dg, dbt, p_drop=0.2, seed=5, offset=9, yrows=ur.inv,
                       o=O, dob=dob, seg=ur if direct else None, dyu_row0=T)
        dyu = dyall[T:]
        (ur.segment_sum_multi if direct else ur.segment_sum)(dyall[:T], dyu)
        outs.append((dyu.clone(), db, dq, dg, dbt))
    torch.cuda.synchronize()
    U = int(ur.counts[1].item())
    assert not torch.isnan(outs[1][0][:U]).any()
    assert torch.equal(outs[0][0][:U], outs[1][0][:U])
    for a, b in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)   # atomics: order-level differences


def test_zero_absent_rows():
    """UniqueRows.zero_absent_rows: rows of ids absent from the batch and the pad row become zero,
    present rows keep their contents; after another nr_unique_rows call on the same vocabulary the
    presence scan is gone and the whole matrix is zeroed instead."""
    g = torch.Generator().manual_seed(8)
    V, W, T = 5000, 768, 4000
    ids = torch.randint(0, V, (T,), generator=g).cuda()
    ids[:7] = 0
    ur = K.UniqueRows(ids, V, fill_row=0)
    dst = torch.full((V, W), 3.0, device="cuda")
    ur.zero_absent_rows(dst, 0)
    torch.cuda.synchronize()
    present = torch.zeros(V, dtype=torch.bool)
    present[ids.cpu()] = True
    present[0] = False
    d = dst.cpu()
    assert (d[present] == 3.0).all() and (d[~present] == 0.0).all()
    K.UniqueRows(ids[:100].contiguous(), V)   # replaces the workspace's scan
    dst.fill_(3.0)
    ur.zero_absent_rows(dst, 0)
    torch.cuda.synchronize()
    assert (dst == 0.0).all()
