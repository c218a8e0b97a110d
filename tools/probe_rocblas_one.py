"""One fp64 AᵀA torch.matmul at the C3 Gram shape (m = 16384, K = 65536), for rocprofv3 kernel names."""
import torch

A = torch.randn(65536, 16384, dtype=torch.float64, device="cuda") / 128.0
for _ in range(2):
    torch.matmul(A.t(), A)
torch.cuda.synchronize()
