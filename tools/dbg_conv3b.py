import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "news-recommendation-mind_amd"))
import torch
from newsrec_amd import _lib as L
from newsrec_amd import kernels as K
g = torch.Generator().manual_seed(5)
V, E, Lq, nn_, H = 100, 64, 7, 9, 40
table = torch.randn(V, E, generator=g)
tok = torch.randint(0, V, (nn_, Lq), generator=g)
w = torch.randn(H, E, 3, generator=g)
b = torch.zeros(H)
x = table[tok].transpose(1, 2)
wr = w.permute(0, 2, 1).reshape(H, 3 * E).contiguous()
tc, tokc = table.cuda(), tok.reshape(-1).cuda()
# host im2col
xp = torch.nn.functional.pad(table[tok], (0, 0, 1, 1))  # [n, L+2, E]
A = torch.cat([xp[:, 0:Lq], xp[:, 1:Lq + 1], xp[:, 2:Lq + 2]], -1).reshape(-1, 3 * E)
want = A.double() @ wr.double().t()
for tap in (None, 0, 1, 2):
    wt = wr.clone()
    if tap is not None:
        for j in range(3):
            if j != tap:
                wt[:, j * E:(j + 1) * E] = 0
    wa = A.double() @ wt.double().t()
    outs = []
    for rep in range(4):
        Y = torch.full((nn_ * Lq, H), 99.0, device="cuda")
        K.gemm(nn_ * Lq, H, 3 * E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Lq, seg=E),
               K.operand(wt.cuda(), L.KCONTIG), Y, bias=b.cuda(), epilogue=L.EPI_STORE)
        outs.append(Y.cpu())
    Yp = torch.full((nn_ * Lq, H), 99.0, device="cuda")
    K.gemm(nn_ * Lq, H, 3 * E, K.operand(A.cuda(), L.KCONTIG), K.operand(wt.cuda(), L.KCONTIG), Yp, bias=b.cuda())
    torch.cuda.synchronize()
    for rep, Y in enumerate(outs):
        d = (Y.double() - wa).abs()
        bad = (d > 1e-3).nonzero()
        print("tap", tap, "rep", rep, "nbad", len(bad), "cols", sorted(set(bad[:, 1].tolist()))[:10], "rows", bad[:12, 0].tolist())
    print("plain im2col nbad", int(((Yp.cpu().double() - wa).abs() > 1e-3).sum()))
