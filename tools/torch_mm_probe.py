"""torch.matmul fp32 on the NRMS projection shapes (to read hipBLASLt's kernel choice)."""
import torch
for M, N, K in [(52800, 1152, 768), (4096, 4096, 4096)]:
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda")
    for _ in range(5):
        C = torch.matmul(A, B.t())
    torch.cuda.synchronize()
