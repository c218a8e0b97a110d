"""Where the sparse Gram's time goes (C5 shape: N = 2^20, m = 2^16, rho = 0.01): the production walk
(variant 8) against its timing builds (SCS_SPARSE_GRAM_DIAG=1: every LDS atomic to the lane's own
slot -- the same ds_add_f64 count without bank conflicts; 2: no LDS accumulation at all; 3: as 2 with
two rows per load instruction, 16-B value and 4-B index loads per lane).
(Variant 9 -- that load structure with the real accumulation -- was measured once and dropped,
profiles/r04/v9/.)  The timing
builds' G is wrong; only the T_GRAM time per launch is reported.  Usage: python3 tools/sgram_diag.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "selfconcordantsmoothoptimization.jl_amd"))
import scsopt  # noqa: E402
from scsopt import losses  # noqa: E402

N, m = 1 << 20, 1 << 16
t0 = time.time()
x0 = np.random.default_rng(1234).standard_normal(m)
p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), 1e-4, density=0.01, seed=2026,
                                    C_set=[-1.0, 1.0])
print(f"problem built in {time.time() - t0:.1f} s", flush=True)
rng = np.random.default_rng(5)
w, v = rng.random(N) + 0.5, rng.standard_normal(N)
lib, h = scsopt._lib.lib, p.ctx.h
p.ctx.check(lib.scs_timing_enable(h, 1))
p.gram_atv_sample(w, v, [(0, 0)])   # builds the segment structure
cases = [("8", d) for d in ("0", "1", "2", "3")]   # (variant, timing build)
for rep in range(2):
    for var, diag in cases:
        os.environ["SCS_SPARSE_GRAM_KERNEL"] = var
        os.environ["SCS_SPARSE_GRAM_DIAG"] = diag
        p.ctx.check(lib.scs_timing_reset(h))
        for _ in range(2):
            p.gram_atv_sample(w, v, [(0, 0)])
        t = p.ctx.timing()
        print(f"variant {var} diag {diag} run {rep}: {t['gram_ms'] / max(1, t['gram_calls']):.1f} ms per Gram "
              f"({t['gram_calls']} calls)", flush=True)
os.environ.pop("SCS_SPARSE_GRAM_DIAG")
os.environ.pop("SCS_SPARSE_GRAM_KERNEL")
p.ctx.close()
