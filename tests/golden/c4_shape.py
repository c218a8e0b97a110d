"""The C4-shape ProxGGNSCORE group-lasso case (tests/test_gpu_default_path.py::
test_c4_shape_ggn_group_lasso) and the script that makes its committed oracle fixture
tests/golden/c4_shape_oracle.npz.

The oracle (oracle/scsopt_oracle.py, FAST_LINALG: dsyrk Gram and LU in place of the QR, the same
systems) needs ~2.5 min of host BLAS at this shape (N·m² = 4e13 flop per Gram, an m = 32768 solve per
epoch) -- a quarter of the GPU suite, whose driver step has a time limit.  Its trajectory is a fixed
function of the data, so it is computed once and committed: obj / fval / rel histories, the final x,
λ, and a fingerprint of the data it ran on (the exactly rounded sums, math.fsum, of three columns of
A), which the test checks before comparing.  The data comes from the library's on-device
counter-based generator (Problem.synthetic kind 3, seed 2026): the same A on every run and box, so
making the fixture needs a GPU:

    python tests/golden/c4_shape.py          # writes tests/golden/c4_shape_oracle.npz

Provenance: "restatement of prox-GGN-SCORE.jl:34-135 / iterate.jl:100-267 (oracle), not
reference-executed", as every golden trajectory here.
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "c4_shape_oracle.npz")
N, M, GS, MU, SEED = 36864, 32768, 32, 1e-2, 2026
FP_COLS = (0, 12345, M - 1)
EPOCHS = 2


def groups():
    ng = M // GS
    return np.array([[1 + GS * g for g in range(ng)], [GS * (g + 1) for g in range(ng)], [1] * ng])


def setup():
    """The device problem: A N(0,1) (kind 3), y = A x_true + 0.1ε, least squares + sparse-group lasso,
    λ = [1e-8, 0.1·max_g ‖∇_g f(0)‖] from the device gradient at 0.  Returns (problem, x0, λ)."""
    import scsopt
    from scsopt import losses
    x0 = np.random.default_rng(1234).standard_normal(M)
    f, out = losses.least_squares(1.0 / N), losses.linear_ls(1.0 / N)
    p = scsopt.Problem.synthetic(N, M, x0, f, 1.0, kind=3, seed=SEED, out_fn=out)
    g0 = p.gradx(np.zeros(M))
    lam = [1e-8, 0.1 * float(np.max(np.linalg.norm(g0.reshape(M // GS, GS), axis=1)))]
    p.λ = lam
    p.P = scsopt.get_P(M, np.arange(1, M + 1), groups())
    return p, x0, lam


def fingerprint(p):
    cols = p.get_columns(np.array(FP_COLS))
    return np.array([math.fsum(cols[:, i]) for i in range(len(FP_COLS))])


def main():
    root = os.path.dirname(os.path.dirname(HERE))
    for d in (os.path.join(root, "selfconcordantsmoothoptimization.jl_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, d)
    import scsopt_oracle as O
    O.FAST_LINALG = True
    p, x0, lam = setup()
    fp = fingerprint(p)
    A, y = p.get_data()
    om = O.Problem(A, y, x0, O.Loss("least_squares", 1.0 / N, ggn="linear_ls"), lam,
                   P=O.GroupP(M, groups(), np.arange(1, M + 1)))
    del A
    osol = O.iterate(O.ProxGGNSCORE(), om, "gl", O.PHuberSmootherGL(MU, om), max_epoch=EPOCHS, x_tol=0.0, f_tol=0.0)
    np.savez(FIXTURE, obj=np.asarray(osol.obj, dtype=np.float64), fval=np.asarray(osol.fval, dtype=np.float64),
             rel=np.asarray(osol.rel, dtype=np.float64), x=np.asarray(osol.x, dtype=np.float64),
             lam=np.asarray(lam, dtype=np.float64), fp=fp, epochs=np.int64(osol.epochs),
             shape=np.array([N, M, GS, SEED], dtype=np.int64), mu=np.float64(MU))
    print(f"wrote {FIXTURE}: epochs {osol.epochs}, obj {osol.obj}")


if __name__ == "__main__":
    main()
