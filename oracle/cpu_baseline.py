"""CPU baseline for bench.py -- TEST/MEASUREMENT INFRASTRUCTURE ONLY.

Times one ProxGGNSCORE iterate!() epoch of the BASELINE workload (sparse
logistic regression, N = 2^20 samples, m = 2^14 features, fp64) with the
reference's own BLAS/LAPACK call structure, restated in NumPy/SciPy
(oracle "port": Julia is absent here and on the GPU box):

  f(x)            z = A*x, CE loss                         iterate.jl:189
  out_fn / J      ŷ = σ(A*x); J = diag(s)*A  (N x m copy)   prox-GGN-SCORE.jl:45-46
  Jt*Q*Jt'        full dgemm on the (m x N) scaled copy      prox-GGN-SCORE.jl:121,129
  Je = Jt*[r;1]   dgemv                                      prox-GGN-SCORE.jl:130
  qr(JQJ) \\ Je    dgeqrf + dormqr + dtrtrs (QRCompactWY \\)  prox-GGN-SCORE.jl:131
  smoother / prox O(m)

A bounded sample: the sample-dependent part (everything above except the QR)
is timed on N_s rows of the same m = 2^14 columns and scaled by N / N_s (its
cost is linear in N); the QR solve is timed once on an m x m system of the
full size m (or on m_s with m^3 scaling when requested).  Prints one JSON line.

    OPENBLAS_NUM_THREADS=16 python oracle/cpu_baseline.py --N 1048576 --m 16384 --Ns 2048
"""
import argparse
import json
import os
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--m", type=int, default=1 << 14)
    ap.add_argument("--Ns", type=int, default=2048)
    ap.add_argument("--ms", type=int, default=0, help="QR timed at ms and scaled by (m/ms)^3 (0: full m)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--method", default="ggn", choices=["ggn", "ggn_ls", "nscore"],
                    help="ggn: C3 (CE + sigmoid out_fn, QR); ggn_ls: C4 (least squares, J = A, QR); "
                         "nscore: C2 (logistic margin, hess_fx Gram, LU)")
    a = ap.parse_args()
    import scipy.linalg.lapack as lapack

    rng = np.random.default_rng(0)
    N, m, Ns = a.N, a.m, a.Ns
    A = np.asfortranarray(rng.standard_normal((Ns, m)) / np.sqrt(m))
    y = (rng.random(Ns) < 0.5).astype(np.float64)
    x = rng.standard_normal(m) * 0.1
    c = 1.0 / N
    lam = 1e-3

    def sample_part():
        z = A @ x                                                    # f(x) pass
        yh = 1.0 / (1.0 + np.exp(-z))
        f = -c * np.sum(y * np.log(yh) + (1 - y) * np.log(1 - yh))
        z = A @ x                                                    # out_fn pass in step!
        e = np.exp(-z)
        yh = 1.0 / (1.0 + e)
        s = e / ((1.0 + e) * (1.0 + e))
        r = -c * (y / yh - (1 - y) / (1 - yh))
        q = c * (y / (yh * yh) + (1 - y) / ((1 - yh) * (1 - yh)))
        J = s[:, None] * A                                            # jac_yx: N x m
        Jt = np.ascontiguousarray(J.T)                                # hcat([J' λ gr]) copy
        JtQ = Jt * q[None, :]                                         # Jt * Q (sparse diagonal)
        JQJ = JtQ @ Jt.T                                              # full dgemm
        Je = Jt @ r
        return f, JQJ, Je

    def sample_nscore():
        # prox-N-SCORE.jl:51-70 with closed-form callbacks: f pass, grad_fx, hess_fx = Aᵀ diag(h) A
        ys = 2 * y - 1
        z = A @ x                                                    # f(x) pass
        f = c * np.sum(np.log1p(np.exp(-ys * z)))
        z = A @ x                                                    # grad_fx
        e = np.exp(-ys * z)
        g = A.T @ (c * (-ys * e / (1.0 + e)))
        z = A @ x                                                    # hess_fx
        e = np.exp(-ys * z)
        h = c * e / ((1.0 + e) * (1.0 + e))
        H = A.T @ (h[:, None] * A)                                    # full dgemm
        return f, g, H

    def sample_ggn_ls():
        # prox-GGN-SCORE.jl:44-56,121-130 with out_fn = A*x, least squares: J = A (copy), Q = c I
        z = A @ x                                                    # f(x) pass
        f = 0.5 * c * np.sum((z - y) ** 2)
        z = A @ x                                                    # out_fn
        r = c * (z - y)
        Jt = np.ascontiguousarray(A.T)                                # jac_yx + hcat copy
        JtQ = Jt * c
        JQJ = JtQ @ Jt.T
        Je = Jt @ r
        return f, JQJ, Je

    if a.method == "nscore":
        sample_part = sample_nscore  # noqa: F811
    elif a.method == "ggn_ls":
        sample_part = sample_ggn_ls  # noqa: F811

    def solve_part(msz):
        M = rng.standard_normal((msz, msz)) / np.sqrt(msz)
        M = np.asfortranarray(M @ M.T + np.eye(msz))
        b = rng.standard_normal(msz)
        t0 = time.perf_counter()
        if a.method == "nscore":   # `\` on a dense Matrix: dgetrf + dgetrs (prox-N-SCORE.jl:70)
            lu, piv, info = lapack.dgetrf(M, overwrite_a=True)
            d, info = lapack.dgetrs(lu, piv, b)
        else:                      # qr(JQJ) \ Je: dgeqrf + dormqr + dtrtrs (prox-GGN-SCORE.jl:131)
            qr, tau, work, info = lapack.dgeqrf(M, overwrite_a=True)
            qtb, work, info = lapack.dormqr("L", "T", qr, tau, b, max(1, msz * 64))
            d, info = lapack.dtrtrs(qr, qtb, lower=0)
        return time.perf_counter() - t0

    sample_part()  # warm-up (page-in, threads)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        sample_part()
        ts.append(time.perf_counter() - t0)
    t_sample = float(np.median(ts))
    msz = a.ms if a.ms else m
    t_qr = float(np.median([solve_part(msz) for _ in range(a.reps)]))
    t_qr_full = t_qr * (m / msz) ** 3
    t_iter = t_sample * (N / Ns) + t_qr_full
    threads = int(os.environ.get("OPENBLAS_NUM_THREADS", os.environ.get("OMP_NUM_THREADS", os.cpu_count())))
    print(json.dumps({
        "value": 1.0 / t_iter, "unit": "iterations/s", "cores": threads, "kind": "port",
        "t_iter_s": t_iter, "t_sample_s": t_sample, "t_qr_s": t_qr, "qr_m": msz, "reps": a.reps, "stat": "median",
        "sample": f"oracle port (NumPy/OpenBLAS, reference BLAS call structure) of one "
                  f"{'ProxNSCORE' if a.method == 'nscore' else 'ProxGGNSCORE'} epoch ({a.method}): "
                  f"sample part on {Ns} of {N} rows x m={m} scaled x{N / Ns:.0f}, "
                  f"{'dgetrf/dgetrs' if a.method == 'nscore' else 'dgeqrf/dormqr/dtrtrs'} solve at "
                  f"m={msz}" + (f" scaled x{(m / msz) ** 3:.0f}" if msz != m else ""),
        "threads_note": (f"{threads} BLAS threads = this job's CPU share on the GPU box (OMP_NUM_THREADS is set to 16 "
                         "per GPU there; os.cpu_count() and the affinity mask report the whole multi-GPU host, "
                         "whose other cores belong to the other GPUs' jobs)"),
    }))


if __name__ == "__main__":
    main()
