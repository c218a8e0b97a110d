"""CPU baseline for bench.py --config c5 -- TEST/MEASUREMENT INFRASTRUCTURE ONLY.

Times one ProxLQNSCORE iterate!() epoch of BASELINE configs[4] (box-constrained
least squares, sparse A with density ρ, m = 2^16, mem = 20, fp64) with the
reference's own call structure restated in NumPy/SciPy (oracle "port"; Julia
is absent here and on the GPU box).  The reference evaluates, per epoch:

  f(x)                 A*x, 1/2N‖Ax − y‖²                      iterate.jl:189
  ∇f(x)  in step!      A*x, Aᵀ(Ax − y)/N                       prox-L-BFGS-SCORE.jl:101
  two-loop recursion   2·mem dots + axpys over m               prox-L-BFGS-SCORE.jl:47-68,105
  smoother, prox       O(m)                                    prox-L-BFGS-SCORE.jl:84-99,135-141
  ∇f(x_new)            A*x, Aᵀ(…)/N                            prox-L-BFGS-SCORE.jl:150
  memory update        O(m)                                    prox-L-BFGS-SCORE.jl:151-162

i.e. 3 products with A and 2 with Aᵀ (SparseMatrixCSC mul!, single-threaded).
Bounded sample: the sparse products are timed on N_s of the N rows (same m and
ρ; cost linear in nnz) and scaled by N / N_s; the O(mem·m) vector work runs at
the full m.  Prints one JSON line.

    python oracle/cpu_baseline_lqn.py --N 1048576 --m 65536 --rho 0.01 --Ns 65536
"""
import argparse
import json
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--m", type=int, default=1 << 16)
    ap.add_argument("--rho", type=float, default=0.01)
    ap.add_argument("--Ns", type=int, default=1 << 16)
    ap.add_argument("--mem", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import scipy.sparse as sp

    rng = np.random.default_rng(0)
    N, m, Ns = a.N, a.m, a.Ns
    k = max(1, round(a.rho * m))
    cols = rng.integers(0, m, size=(Ns, k), dtype=np.int32).reshape(-1)
    vals = rng.standard_normal(Ns * k) / np.sqrt(k)
    A = sp.csr_matrix((vals, cols, np.arange(0, Ns * k + 1, k, dtype=np.int64)), shape=(Ns, m))
    y = rng.standard_normal(Ns)
    x = np.clip(rng.standard_normal(m), -1, 1)
    c = 1.0 / N

    def sparse_part():
        r = A @ x - y                       # f(x)
        f = 0.5 * c * float(r @ r)
        r = A @ x - y                       # ∇f(x)
        g = c * (A.T @ r)
        r = A @ x - y                       # ∇f(x_new)
        g2 = c * (A.T @ r)
        return f, g, g2

    S = rng.standard_normal((a.mem, m))
    Y = rng.standard_normal((a.mem, m))
    g = rng.standard_normal(m)

    def vector_part():
        q = g.copy()                        # two-loop (prox-L-BFGS-SCORE.jl:47-68)
        al = np.empty(a.mem)
        rho = np.empty(a.mem)
        for i in range(a.mem - 1, -1, -1):
            rho[i] = 1.0 / (Y[i] @ S[i])
            al[i] = rho[i] * (S[i] @ q)
            q -= al[i] * Y[i]
        r = q
        for i in range(a.mem):
            beta = rho[i] * (Y[i] @ r)
            r += S[i] * (al[i] - beta)
        mu = 0.6                            # PHuberSmootherIndBox grad/hess + box prox, O(m)
        xa = x + 1.0
        xb = 1.0 - x
        gr = xa * (mu * mu + xa * xa) ** -0.5 - xb * (mu * mu + xb * xb) ** -0.5
        Hr = mu * mu * (mu * mu + xa * xa) ** -1.5 + mu * mu * (mu * mu + xb * xb) ** -1.5
        xn = np.clip(x - r / Hr, -1.0, 1.0)
        return float(np.linalg.norm(xn - x) + gr[0])

    sparse_part()
    vector_part()
    ts, tv = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        sparse_part()
        ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        vector_part()
        tv.append(time.perf_counter() - t0)
    t_sparse, t_vec = float(np.median(ts)), float(np.median(tv))
    t_iter = t_sparse * (N / Ns) + t_vec
    print(json.dumps({
        "value": 1.0 / t_iter, "unit": "iterations/s", "cores": 1, "kind": "port",
        "t_iter_s": t_iter, "t_sparse_sample_s": t_sparse, "t_vector_s": t_vec, "reps": a.reps, "stat": "median",
        "threads_note": "1 thread: the reference's SparseMatrixCSC products (SparseArrays mul!) are single-threaded, "
                        "and SciPy's CSR/CSC matvec holds the GIL (measured: 8 threads over row chunks = 1.0x)",
        "sample": f"oracle port (SciPy CSR, single thread, reference call structure: 3 A*x + 2 Aᵀ*r per epoch) "
                  f"of one ProxLQNSCORE(mem={a.mem}) epoch: sparse products on {Ns} of {N} rows "
                  f"(rho={a.rho}, nnz {Ns * k}) scaled x{N // Ns}, two-loop/smoother/prox at full m={m}",
    }))


if __name__ == "__main__":
    main()
