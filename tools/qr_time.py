"""Wall time and residual of the reference-solver QR (scs_solve_eval mode 2) against the default
Cholesky path (mode 0) on (Aᵀ diag(w) A + diag d) x = rhs at the given orders."""
import sys
import time

import numpy as np

sys.path.insert(0, "selfconcordantsmoothoptimization.jl_amd")
import scsopt  # noqa: E402
from scsopt import losses  # noqa: E402

for m in [int(v) for v in (sys.argv[1:] or ["2048", "8192"])]:
    N = m + 512
    p = scsopt.Problem.synthetic(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1.0, kind=3, seed=5)
    rng = np.random.default_rng(6)
    w = (rng.random(N) + 0.5) / N
    d = (rng.random(m) + 0.5) * 1e-2
    rhs = rng.standard_normal(m)
    for mode in (0, 2, 2):
        t0 = time.perf_counter()
        x, _ = p.solve_eval(w, d, rhs, mode=mode)
        t = time.perf_counter() - t0
        r = p.gemv_t(w * p.gemv_n(x)) + d * x - rhs
        print(f"m={m} mode={mode} wall={t * 1e3:.1f} ms  |r|/|b| = {np.linalg.norm(r) / np.linalg.norm(rhs):.2e}",
              flush=True)
    p.ctx.close()
