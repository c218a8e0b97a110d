"""CPU baseline for bench.py --config c1 -- TEST/MEASUREMENT INFRASTRUCTURE ONLY.

BASELINE configs[0]: the README quick start (README.md:43-70), ProxLQNSCORE(m = 10) +
PHuberSmootherL1L2(1) on the 2-variable Rosenbrock with l1, λ = 1e-8, run through the oracle's
iterate!() restatement (oracle "port": Julia is absent here and on the GPU box; single thread).
Prints one JSON line with iterations/s over the whole solve.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import scsopt_oracle as O  # noqa: E402

X0 = [0.5908446386657102, 0.7667970365022592]   # test/test_algs.jl:4 (Julia's randn stream is not reproducible)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    best = None
    for _ in range(reps):
        model = O.Problem(None, None, np.array(X0), O.Loss("rosenbrock"), 1e-8)
        t0 = time.perf_counter()
        sol = O.iterate(O.ProxLQNSCORE(m=10), model, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=1000)
        dt = time.perf_counter() - t0
        rate = (sol.epochs + 1) / dt
        best = rate if best is None else max(best, rate)
    print(json.dumps({"value": best, "unit": "iterations/s", "cores": 1, "kind": "port",
                      "sample": f"oracle iterate!() restatement of the C1 solve ({sol.epochs + 1} epochs, best of "
                                f"{reps}), NumPy scalar path, one thread"}))


if __name__ == "__main__":
    main()
