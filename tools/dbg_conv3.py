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
b = torch.randn(H, generator=g)
x = table[tok].transpose(1, 2)
want = (torch.nn.functional.conv1d(x.double(), w.double(), b.double(), padding=1)).transpose(1, 2).reshape(-1, H)
wr = w.permute(0, 2, 1).reshape(H, 3 * E).contiguous()
tc, tokc = table.cuda(), tok.reshape(-1).cuda()
for epi in (L.EPI_STORE, L.EPI_STORE_RELU):
    Y = torch.empty(nn_ * Lq, H, device="cuda")
    K.gemm(nn_ * Lq, H, 3 * E, K.operand(tc, L.KCONTIG, rows=tokc, mapping=L.ROWS_CONV3, seq_len=Lq, seg=E),
           K.operand(wr.cuda(), L.KCONTIG), Y, bias=b.cuda(), epilogue=epi)
    w2 = want.clamp_min(0) if epi == L.EPI_STORE_RELU else want
    d = (Y.cpu().double() - w2).abs()
    bad = (d > 1e-3).nonzero()
    print("epi", epi, "nbad", len(bad), bad[:40].tolist())
    print(Y.cpu()[bad[:5,0], bad[:5,1]].tolist(), w2[bad[:5,0], bad[:5,1]].tolist())
