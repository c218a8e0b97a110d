"""Time the hand-written blocked LU (lu.hip) at n = 8192 / 16384 through scs_lu_eval: device time of
factor + solve (hipEvent, the context's T_SOLVE accumulator), backward error, one JSON line per n."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "selfconcordantsmoothoptimization.jl_amd"))
import scsopt  # noqa: E402

ctx = scsopt._lib.Context(0)
ctx.check(scsopt._lib.lib.scs_timing_enable(ctx.h, 1))
for n in [int(a) for a in (sys.argv[1:] or ["8192"])]:
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    scsopt.lu_solve(A, b, ctx=ctx)   # warm-up: code objects, aux buffers
    ctx.check(scsopt._lib.lib.scs_timing_reset(ctx.h))
    reps = 3
    for _ in range(reps):
        x, ipiv, info = scsopt.lu_solve(A, b, ctx=ctx)
    tm = ctx.timing()
    bwd = float(np.linalg.norm(A @ x - b, np.inf) / (np.linalg.norm(A, np.inf) * np.linalg.norm(x, np.inf)))
    ms = tm["solve_ms"] / tm["solve_calls"]
    print(json.dumps({"n": n, "info": info, "factor_plus_solve_ms": ms, "tflops": (2 / 3 * n ** 3) / (ms * 1e-3) / 1e12,
                      "backward_error": bwd, "reps": reps}))
