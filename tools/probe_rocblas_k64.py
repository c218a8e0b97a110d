"""One fp64 AᵀA torch.matmul at m = 16384, K = 65536 (rocprofv3 --pmc comparison with the Gram)."""
import torch

A = torch.randn(65536, 16384, dtype=torch.float64, device="cuda") / 128.0
torch.matmul(A.t(), A)
torch.cuda.synchronize()
