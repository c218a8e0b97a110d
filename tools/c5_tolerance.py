"""C5 fp32-vs-fp64 tolerance study at full size (BASELINE configs[4]).

Both arms solve the same generated problem -- sparse A (N = 2^20, m = 2^16, rho = 0.01), box least
squares, ProxLQNSCORE(mem = 20) + indbox + PHuberSmootherIndBox(mu = 0.6), lambda = 1e-4 -- from the
same x0 for 50 epochs with x_tol = f_tol = 0.  Two studies against the fp64 arm:
  --arm storage (r03): A's VALUES stored fp32 (rounded from the same draws), every product still
      accumulated in fp64 -- storage rounding only;
  --arm compute (r04): fp32-stored values AND fp32 arithmetic in the sparse products (A x and Aᵀ r:
      fp32 products, lane sums, scans and row sums) and in the L-BFGS two-loop (fp32 dots, axpys,
      α, ρ, β) -- scs_set_compute_f32; f, η, the step, the prox and the loop stay fp64.

Per epoch (the iterate! history pushes, iterate.jl:214): |obj64 - obj32| / |obj64|, ||x64 - x32||_inf
and the number of coordinates whose box-active status (x_i = -1 or +1, the indbox prox clamps exactly)
differs between the arms.  Output: one JSON file (profiles/r03/c5/tolerance.json for the storage arm,
profiles/r04/c5/tolerance_f32compute.json for the compute arm).

    python tools/c5_tolerance.py [--arm storage|compute] [--epochs 50] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd"))


def run_arm(f32, N, m, rho, epochs, compute=False):
    import numpy as np
    import scsopt
    from scsopt import losses
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), 1e-4, density=rho, seed=2026,
                                        f32=f32, C_set=[-1.0, 1.0])
    if compute:
        p.set_compute_f32(True)
    xs = []
    t0 = time.perf_counter()
    sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", scsopt.PHuberSmootherIndBox(-1.0, 1.0, 0.6),
                         max_epoch=epochs, x_tol=0.0, f_tol=0.0, verbose=0,
                         metrics={"x": lambda model, x: xs.append(np.array(x, dtype=np.float64)) or 0.0})
    dt = time.perf_counter() - t0
    p.ctx.close()
    return sol, xs, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--m", type=int, default=1 << 16)
    ap.add_argument("--rho", type=float, default=0.01)
    ap.add_argument("--arm", choices=("storage", "compute"), default="storage")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.out is None:
        args.out = os.path.join(ROOT, "profiles", *(("r03", "c5", "tolerance.json") if args.arm == "storage" else
                                                    ("r04", "c5", "tolerance_f32compute.json")))
    import numpy as np
    s64, x64, t64 = run_arm(False, args.N, args.m, args.rho, args.epochs)
    s32, x32, t32 = run_arm(True, args.N, args.m, args.rho, args.epochs, compute=args.arm == "compute")
    import math
    n = min(len(s64.obj), len(s32.obj))
    rows = []
    for e in range(n):
        a, b = x64[e], x32[e]
        act64 = (a == -1.0) | (a == 1.0)
        act32 = (b == -1.0) | (b == 1.0)
        rows.append({"entry": e, "obj64": s64.obj[e], "obj32": s32.obj[e],
                     "rel_dobj": abs(s64.obj[e] - s32.obj[e]) / abs(s64.obj[e]),
                     "dx_inf": float(np.max(np.abs(a - b))), "active64": int(act64.sum()),
                     "active32": int(act32.sum()), "active_diff": int((act64 != act32).sum())})
    out = {"config": {"N": args.N, "m": args.m, "rho": args.rho, "epochs": args.epochs, "method": "ProxLQNSCORE(m=20)",
                      "reg": "indbox [-1, 1]", "smoother": "PHuberSmootherIndBox(mu=0.6)", "lambda": 1e-4,
                      "x_tol": 0.0, "f_tol": 0.0},
           "arms": {"fp64": "A values fp64, fp64 arithmetic",
                    "fp32": ("A values stored fp32 (rounded from the same draws), widened on load, fp64 arithmetic"
                             if args.arm == "storage" else
                             "A values stored fp32; fp32 arithmetic in A x, A'r (spmv_blk32_kernel) and the L-BFGS "
                             "two-loop (two_loop / tl_* kernels <float>); f, eta, step, prox, loop in fp64")},
           "study": args.arm,
           "wall_s": {"fp64": t64, "fp32": t32},
           # entries where both arms' objective is Inf (x0 outside the box: get_reg(indbox) = Inf) carry no
           # relative difference; they are listed, not folded into the maximum
           "max_rel_dobj": max(r["rel_dobj"] for r in rows if math.isfinite(r["obj64"]) and math.isfinite(r["obj32"])),
           "entries_inf_both_arms": [r["entry"] for r in rows if not math.isfinite(r["obj64"])],
           "max_dx_inf": max(r["dx_inf"] for r in rows),
           "max_active_diff": max(r["active_diff"] for r in rows),
           "final": rows[-1], "per_entry": rows}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("max_rel_dobj", "max_dx_inf", "max_active_diff", "wall_s")}))


if __name__ == "__main__":
    main()
