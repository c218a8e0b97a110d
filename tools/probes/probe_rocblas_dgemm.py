"""Reference point for the fp64 MFMA Gram: rocBLAS/hipBLASLt DGEMM (torch.matmul, fp64) on the
Gram's shape AᵀA with A (K x m), and the same flops as a square GEMM.  Prints TF/s per shape
(2·m²·K flops for the full product; our Gram computes the symmetric half: N·m·(m+1))."""
import json
import sys
import time

import torch


def bench(a, b, reps):
    torch.matmul(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    out = []
    for (m, K) in ((16384, 65536), (8192, 100000), (16384, 16384), (8192, 8192)):
        A = torch.randn(K, m, dtype=torch.float64, device=dev) / m ** 0.5
        ms = bench(A.t(), A, 3)
        out.append({"op": "A^T A (torch.matmul fp64)", "m": m, "K": K, "ms": ms,
                    "tflops_full": 2.0 * m * m * K / ms / 1e9})
        print(json.dumps(out[-1]), flush=True)
        del A
        torch.cuda.empty_cache()
    print(json.dumps({"device": torch.cuda.get_device_name(0), "results": out}))


if __name__ == "__main__":
    sys.exit(main())
