"""Parity at the shapes the headline numbers are quoted on, with NO env overrides.

The other GPU tests force each kernel variant at small sizes (SCS_GRAM_TALL=1, SCS_GRAM_FUSE=2,
m <= 3200 ...).  These run the library's default choices at the BASELINE shapes (SURVEY.md §8:
C2 m = 8192, C3 m = 16384, C4 m = 32768, C5 m = 65536), against the oracle:

  * C3 shape: ProxGGNSCORE logistic + l1, m = 16384, N = 20480 (N + 1 > m: the feature branch):
    256 x 128 Gram tiles with the Aᵀv fused into the Gram pass, the tail-balanced K-split
    schedule, the 256-workgroup SCORE tail (m >= 16384) and the two-level Cholesky (128 inner
    blocks = 16 outer blocks of 8) with its second-stream lookahead -- 3 epochs at rtol 1e-8;
  * C2 shape: ProxNSCORE logistic (margin) + l1, m = 8192 (128 x 128 tiles, 8 outer blocks);
  * C4 shape: the m = 32768 Cholesky solve (256 inner blocks) by its backward error, with the
    residual formed by the independent streaming GEMV kernels; the m = 32768 LU likewise; the
    2-epoch group-lasso trajectory against the oracle's, committed as tests/golden/c4_shape_oracle.npz;
  * C5 shape: ProxLQNSCORE(mem 20) box least squares on a sparse A with m = 65536 (4 LDS column
    blocks of the CSR product, the multi-workgroup two-loop / tail / L-BFGS update) and
    N = 2^17 (8 row blocks of the CSC product), 10 epochs at rtol 1e-8.

The oracle runs its literal restatement except for FAST_LINALG (dsyrk Gram, LU in place of the
QR: the same systems, equal to O(cond·eps) -- oracle/scsopt_oracle.py).
"""
import os

import numpy as np
import pytest

import scsopt
import scsopt_oracle as O
from scsopt import losses

pytestmark = pytest.mark.gpu


@pytest.fixture
def clean_env(monkeypatch):
    for k in list(os.environ):
        if k.startswith("SCS_"):
            monkeypatch.delenv(k)
    monkeypatch.setattr(O, "FAST_LINALG", True)


def _lam_rule(p, m):
    """BASELINE's λ = 0.1·‖∇f(0)‖∞ (bench.py)."""
    return 0.1 * float(np.max(np.abs(p.gradx(np.zeros(m)))))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("shape", ["c3", "c2"])
def test_default_path_newton_methods(shape, clean_env):
    if shape == "c3":
        N, m, kind = 20480, 16384, 1
        f, out = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N)
        of = O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce")
        meth, ometh = scsopt.ProxGGNSCORE(), O.ProxGGNSCORE()
    else:
        N, m, kind = 12288, 8192, 2
        f, out = losses.logistic_margin(1.0 / N), None
        of = O.Loss("logistic_margin", 1.0 / N)
        meth, ometh = scsopt.ProxNSCORE(), O.ProxNSCORE()
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic(N, m, x0, f, 1.0, kind=kind, seed=2026, out_fn=out)
    lam = _lam_rule(p, m)
    p.λ = lam
    A, y = p.get_data()
    if shape == "c3":   # the configuration under test really is the fused 256 x 128 launch
        rng = np.random.default_rng(5)
        cols = rng.choice(m, 6, replace=False)
        w, v = rng.random(N), rng.standard_normal(N)
        pairs = [(i, j) for i in cols for j in cols]
        g, atv, fused = p.gram_atv_sample(w, v, pairs)
        assert fused
        for (i, j), gv in zip(pairs, g):
            terms = float(np.abs(A[:, i] * w * A[:, j]).sum())
            assert abs(gv - float((A[:, i] * w) @ A[:, j])) <= 1e-13 * terms
        bound = 1e-13 * (np.abs(A[:, cols]).T @ np.abs(v))
        assert np.all(np.abs(atv[cols] - A[:, cols].T @ v) <= bound)
    om = O.Problem(A, y, x0, of, lam)
    sol = scsopt.iterate(meth, p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=3, x_tol=0.0, f_tol=0.0,
                         verbose=0)
    osol = O.iterate(ometh, om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=3, x_tol=0.0, f_tol=0.0)
    assert sol.epochs == osol.epochs and len(sol.obj) == len(osol.obj)
    np.testing.assert_allclose(sol.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.fval, osol.fval, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.x, osol.x, rtol=1e-6, atol=1e-9)
    assert sol.obj[-1] < sol.obj[0]


def _gemv_residual(p, w, d, x, rhs):
    """(Aᵀ diag(w) A + diag d) x - rhs through the streaming GEMV kernels (not the Gram)."""
    return p.gemv_t(w * p.gemv_n(x)) + d * x - rhs


def _norm2_est(p, w, d, m, iters=12):
    v = np.random.default_rng(0).standard_normal(m)
    for _ in range(iters):
        v = p.gemv_t(w * p.gemv_n(v)) + d * v
        v /= np.linalg.norm(v)
    return float(np.linalg.norm(p.gemv_t(w * p.gemv_n(v)) + d * v))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", [0, 1])
def test_c4_shape_solve_backward_error(mode, clean_env):
    """m = 32768: the two-level Cholesky (mode 0, 256 inner blocks, lookahead) and the blocked LU
    (mode 1) on (Aᵀ diag(w) A + diag d), N = m + 4096: ||r|| <= 1e-12 ||G|| ||x||."""
    N, m = 32768 + 4096, 32768
    p = scsopt.Problem.synthetic(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1.0, kind=3, seed=11)
    rng = np.random.default_rng(12)
    w = (rng.random(N) + 0.5) / N
    d = (rng.random(m) + 0.5) * 1e-2
    rhs = rng.standard_normal(m)
    x, used_lu = p.solve_eval(w, d, rhs, mode=mode)
    assert used_lu == (mode == 1)
    r = _gemv_residual(p, w, d, x, rhs)
    gn = _norm2_est(p, w, d, m)
    assert np.linalg.norm(r) <= 1e-12 * gn * np.linalg.norm(x), (np.linalg.norm(r), gn, np.linalg.norm(x))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("m", [16384, 8192])
def test_c3_c2_shape_cholesky_backward_error(m, clean_env):
    """The m = 16384 (C3) and m = 8192 (C2) default factor + one-launch solves (mode 0) -- the sizes
    where round 3 saw a wrong-result race (the diagonal kernel's intra-wave LDS exchange, fenced
    since; DESIGN §3 lists every intra-wave hand-off) -- by the backward error through the
    independent GEMV kernels: ||r|| <= 1e-12 ||G|| ||x||, on two right-hand sides."""
    N = m + 2048
    p = scsopt.Problem.synthetic(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1.0, kind=3, seed=m + 1)
    rng = np.random.default_rng(m)
    w = (rng.random(N) + 0.5) / N
    d = (rng.random(m) + 0.5) * 1e-2
    gn = _norm2_est(p, w, d, m)
    for _ in range(2):
        rhs = rng.standard_normal(m)
        x, used_lu = p.solve_eval(w, d, rhs, mode=0)
        assert not used_lu
        r = _gemv_residual(p, w, d, x, rhs)
        assert np.linalg.norm(r) <= 1e-12 * gn * np.linalg.norm(x), (np.linalg.norm(r), gn, np.linalg.norm(x))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("f32", [False, True])
def test_c5_shape_lqn_sparse(f32, clean_env):
    """C5 with N = 2^17 (m = 2^16 as configured): ProxLQNSCORE(mem 20) + indbox + PHuberSmootherIndBox(0.6),
    fp64 or fp32-stored values (the oracle runs on the values read back, widened to fp64)."""
    N, m, rho = 1 << 17, 1 << 16, 0.01
    x0 = np.random.default_rng(1234).standard_normal(m)
    lam, mu = 1e-4, 0.6
    p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), lam, density=rho, seed=2026,
                                        C_set=[-1.0, 1.0], f32=f32)
    A, y = p.get_sparse()
    om = O.Problem(A, y, x0, O.Loss("least_squares", 1.0 / N), lam, C_set=[-1.0, 1.0])
    sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", scsopt.PHuberSmootherIndBox(-1.0, 1.0, mu),
                         max_epoch=10, x_tol=0.0, f_tol=0.0, verbose=0)
    osol = O.iterate(O.ProxLQNSCORE(m=20), om, "indbox", O.PHuberSmootherIndBox(-1.0, 1.0, mu), max_epoch=10,
                     x_tol=0.0, f_tol=0.0)
    assert sol.epochs == osol.epochs and len(sol.obj) == len(osol.obj)
    np.testing.assert_allclose(sol.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.x, osol.x, rtol=1e-6, atol=1e-9)
    assert np.all(sol.x >= -1.0) and np.all(sol.x <= 1.0)


@pytest.mark.timeout(600)
def test_c5_shape_lqn_sparse_fp32_compute(clean_env, record_property):
    """The fp32-COMPUTE arm (scs_set_compute_f32: fp32 arithmetic in A x, Aᵀ r and the two-loop) on the
    C5 shape above against the fp64 oracle on the same fp32-stored values.

    Asserted, each bound stated before any run (BASELINE configs[4] is a tolerance STUDY):
      * every finite history entry within rtol 1e-4 of the oracle's objective -- an fp32 sum of the
        ~655 terms of a row / ~1300 of a column carries at most n·2⁻²⁴ ≈ 8e-5 relative error
        (n ≤ 1300), the objective itself is evaluated in fp64 on top of it;
      * the iterates stay in the box [-1, 1] exactly (the clamp prox, prox-operators.jl:27-46);
      * the fp32 SpMV kernel is the one that ran;
      * two REGRESSION GUARDS, not accuracy bounds (r06): max |x_dev − x_oracle| <= 0.1
        (5 % of the box width, ~50x the 2.07e-3 measured in r04) and at most m/100 coordinates whose
        box-active state differs -- a drift of the fp32 path in x by an order of magnitude fails.
    Reported (the measured values beside the guards) (record_property + stdout): max |x_dev − x_oracle|, the count of
    coordinates whose box-active state differs and their distance to the bound, the worst relative
    objective gap.  No a-priori bound on x exists here: after 10 L-BFGS epochs neither arm is near
    the optimum, and the two-loop's curvature pairs amplify the fp32 perturbation by the inverse of
    the smallest curvature they sample (AᵀA/N ≈ I/m · [0.09, 2.9] at N = 2m), so the
    x gap is a measured statistic of the study: 2.07e-3 on the r04 box (gpurun_out/r04/t1.log:124),
    which an earlier version of this test then asserted against a bound fitted to it (r04 verdict)."""
    N, m, rho = 1 << 17, 1 << 16, 0.01
    x0 = np.random.default_rng(1234).standard_normal(m)
    lam, mu = 1e-4, 0.6
    p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), lam, density=rho, seed=2026,
                                        C_set=[-1.0, 1.0], f32=True)
    p.set_compute_f32(True)
    A, y = p.get_sparse()
    om = O.Problem(A, y, x0, O.Loss("least_squares", 1.0 / N), lam, C_set=[-1.0, 1.0])
    sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", scsopt.PHuberSmootherIndBox(-1.0, 1.0, mu),
                         max_epoch=10, x_tol=0.0, f_tol=0.0, verbose=0)
    assert p.ctx.kernel_names()[1] == "spmv_blk32_kernel"
    osol = O.iterate(O.ProxLQNSCORE(m=20), om, "indbox", O.PHuberSmootherIndBox(-1.0, 1.0, mu), max_epoch=10,
                     x_tol=0.0, f_tol=0.0)
    assert sol.epochs == osol.epochs and len(sol.obj) == len(osol.obj)
    fin = [i for i, v in enumerate(osol.obj) if np.isfinite(v)]   # entry 0: x0 outside the box, Inf
    np.testing.assert_allclose(np.array(sol.obj)[fin], np.array(osol.obj)[fin], rtol=1e-4, atol=0)
    assert np.all(sol.x >= -1.0) and np.all(sol.x <= 1.0)
    ad = (np.abs(sol.x) == 1.0) != (np.abs(osol.x) == 1.0)
    dist = np.minimum(np.abs(np.abs(sol.x) - 1), np.abs(np.abs(osol.x) - 1))[ad]
    stats = {"max_abs_dx": float(np.max(np.abs(sol.x - osol.x))),
             "active_set_differences": int(ad.sum()),
             "max_bound_distance_of_differences": float(dist.max()) if dist.size else 0.0,
             "max_rel_dobj": float(np.max(np.abs(np.array(sol.obj)[fin] - np.array(osol.obj)[fin])
                                          / np.abs(np.array(osol.obj)[fin])))}
    for k, v in stats.items():
        record_property(k, v)
    print("fp32-compute study (reported):", stats)
    assert stats["max_abs_dx"] <= 0.1, stats
    assert stats["active_set_differences"] <= m // 100, stats


@pytest.mark.timeout(900)
def test_c4_shape_ggn_group_lasso(clean_env):
    """C4 shape (BASELINE configs[3]) on one GPU: ProxGGNSCORE least squares + sparse-group lasso,
    m = 32768 in 1024 groups of 32, N = 36864 (N + 1 > m: the feature branch), μ = 1e-2,
    λ = [1e-8, 0.1·max_g ‖∇_g f(0)‖] -- the 256 x 128 Gram with the fused Jᵀr, the m = 32768
    two-level Cholesky (no CU reserve above m = 16384), the multi-workgroup PHuberSmootherGL with its
    global dot(Dg, Dg) (phuber-smooth.jl:137-164) and the group prox over 1024 groups
    (prox-operators.jl:48-66, prox-reg-utils.jl:84-119).  2 epochs vs the oracle at rtol 1e-8 on
    obj / fval and on rel (the mean_square_error of reg "gl", iterate.jl:171-175).  The oracle's
    trajectory on this data is the committed fixture tests/golden/c4_shape_oracle.npz (made by
    tests/golden/c4_shape.py: ~2.5 min of host BLAS, r06 moved it out of the suite); the data's
    fingerprint (exact sums of three columns of A) and λ are checked against it first."""
    import c4_shape as C
    fx = np.load(C.FIXTURE)
    assert tuple(fx["shape"]) == (C.N, C.M, C.GS, C.SEED) and int(fx["epochs"]) == C.EPOCHS
    p, x0, lam = C.setup()
    assert np.array_equal(C.fingerprint(p), fx["fp"]), "the device data is not the fixture's"
    np.testing.assert_allclose(lam, fx["lam"], rtol=1e-14, atol=0)
    p.λ = [float(v) for v in fx["lam"]]
    sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "gl", scsopt.PHuberSmootherGL(C.MU, p), max_epoch=C.EPOCHS,
                         x_tol=0.0, f_tol=0.0, verbose=0)
    assert sol.epochs == int(fx["epochs"]) and len(sol.obj) == len(fx["obj"])
    np.testing.assert_allclose(sol.obj, fx["obj"], rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.fval, fx["fval"], rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.rel, fx["rel"], rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.x, fx["x"], rtol=1e-6, atol=1e-9)
    # the group prox zeroes whole groups: the support pattern is group-aligned on both sides
    ng = C.M // C.GS
    zd = (sol.x.reshape(ng, C.GS) == 0).all(axis=1)
    zo = (fx["x"].reshape(ng, C.GS) == 0).all(axis=1)
    assert np.array_equal(zd, zo)
