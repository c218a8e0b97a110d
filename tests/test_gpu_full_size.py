"""GPU: parity at the FULL BASELINE sizes, default code path (no env overrides).

The other default-path tests (tests/test_gpu_default_path.py) run the BASELINE m at reduced N.  Here:
  * C2 (BASELINE configs[1]: ProxNSCORE logistic (margin) + l1, N = 100000, m = 8192), the whole
    problem: 2 epochs of the device loop against the oracle's restatement on the downloaded A at rtol
    1e-8 (obj, fval) -- a full-size trajectory;
  * C3 (configs[2]: N = 2^20, m = 2^14, A = 128 GiB on the device): the production Gram launch (fused
    Aᵀv) on 36 column pairs and 8 Aᵀv entries against host fp64 dots of downloaded columns (bound
    1e-11·Σ|terms|: the summation order differs, a wrong tile / weight / panel is an O(1) error), then
    two epochs of the default loop (the objective decreases, the iterate is finite);
  * C4's per-rank shape at 8 GPUs (configs[3]: N = 2^22 / 8 = 2^19 rows, m = 2^15, least squares +
    sparse-group lasso, 1024 groups of 32; A = 128 GiB): the production Gram sampled like C3, then two
    epochs of the default loop (objective decreases, iterate finite);
  * C3 and C4's per-rank shape also get a whole-length f(x) / ∇f(x) check at the run's final x (C3 at
    x0 too): the device's GEMV passes and loss epilogue against a host fp64 evaluation of A streamed
    down in row blocks (host_f_grad: bounds from 1e-11·Σ|terms|, z-propagation included);
  * C5 (configs[4]: sparse A, N = 2^20, m = 2^16, ρ = 0.01, 6.9e8 nonzeros): 3 epochs, then f(x) and
    ∇f(x) at the final x through the production SpMV kernels against a host SciPy evaluation of the
    whole downloaded CSR (1e-11 relative on f, 1e-11·Σ|terms| per gradient entry).
The oracle runs with FAST_LINALG (dsyrk Gram, LU for the QR: the same systems, equal to O(cond·eps)).
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
    import gc
    gc.collect()   # contexts left in reference cycles by earlier tests: free their device memory first
    for k in list(os.environ):
        if k.startswith("SCS_"):
            monkeypatch.delenv(k)
    monkeypatch.setattr(O, "FAST_LINALG", True)


@pytest.mark.timeout(900)
def test_c2_full_size_trajectory(clean_env):
    N, m = 100_000, 8192
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic(N, m, x0, losses.logistic_margin(1.0 / N), 1.0, kind=2, seed=2026)
    lam = 0.1 * float(np.max(np.abs(p.gradx(np.zeros(m)))))   # bench.py's λ rule
    p.λ = lam
    A, y = p.get_data()
    sol = scsopt.iterate(scsopt.ProxNSCORE(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=2, x_tol=0.0,
                         f_tol=0.0, verbose=0)
    p.ctx.close()
    om = O.Problem(A, y, x0, O.Loss("logistic_margin", 1.0 / N), lam)
    osol = O.iterate(O.ProxNSCORE(), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=2, x_tol=0.0, f_tol=0.0)
    assert sol.epochs == osol.epochs and len(sol.obj) == len(osol.obj)
    np.testing.assert_allclose(sol.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.fval, osol.fval, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.x, osol.x, rtol=1e-6, atol=1e-9)
    assert sol.obj[-1] < sol.obj[0]


def host_f_grad(p, x, kind, chunk_bytes=4 << 30):
    """f(x), ∇f(x) and their error bounds evaluated on the host in fp64 from the device's A, streamed
    down in row blocks (scs_get_data, column-major: no host copy of the whole A).  One pass: per block
    z = A_b x, then the loss terms and the block's share of Aᵀ(s⊙r) (logistic CE: s = σ'(z) and r the
    CE residual, as prox-GGN-SCORE.jl:44-49 / the oracle's Loss.grad form them; least squares:
    s = 1, r = c(z − y)).  Bounds (summation orders differ; an error in z moves a CE term by at most
    c·|δz| and s⊙r by at most c·|δz|/4 for |σ'| <= 1/4): f: 1e-11·(Σ|terms| + c·Σ_i Σ_j |A_ij x_j|);
    ∇f_j: 1e-11·(Σ_i |A_ij s_i r_i| + c·Σ_i |A_ij| Σ_k |A_ik x_k|)."""
    import ctypes as C
    from scsopt import _lib
    N, m = p.N, p.m
    c = 1.0 / p.N_global
    nr = max(16, (chunk_bytes // (8 * m)) // 16 * 16)
    buf = np.empty((nr, m), dtype=np.float64)   # buf[:n].ravel() holds an (m, n) column-major block
    yb = np.empty(nr)
    f = fterms = fz = 0.0
    g = np.zeros(m)
    gb = np.zeros(m)
    xa = np.abs(x)
    for r0 in range(0, N, nr):
        n = min(nr, N - r0)
        Acm = buf.reshape(-1)[: m * n].reshape(m, n)   # Acm.T = rows r0 .. r0+n of A
        p.ctx.check(_lib.lib.scs_get_data(p.ctx.h, r0, n, Acm.ctypes.data_as(_lib.c_dp), n,
                                          yb.ctypes.data_as(_lib.c_dp)))
        y = yb[:n]
        Ab = np.abs(Acm)
        z = Acm.T @ x
        zabs = Ab.T @ xa
        if kind == "logistic_ce":
            s, yhat = O.sigmoid_jac(z)
            terms = -c * (y * np.log(yhat) + (1.0 - y) * np.log(1.0 - yhat))
            sr = s * O.ce_r(y, yhat, c)
        else:
            res = z - y
            terms = 0.5 * c * res * res
            sr = c * res
        f += float(terms.sum())
        fterms += float(np.abs(terms).sum())
        fz += c * float(zabs.sum())
        g += Acm @ sr
        gb += Ab @ np.abs(sr) + c * (Ab @ zabs)
    return f, 1e-11 * (fterms + fz), g, 1e-11 * gb


def check_f_grad(p, x, kind):
    """The device's f(x) / ∇f(x) -- the production GEMV passes and the loss epilogue -- at full size
    against host_f_grad."""
    f_dev, g_dev = p.fx(x), p.gradx(x)
    f_ref, f_bnd, g_ref, g_bnd = host_f_grad(p, x, kind)
    assert abs(f_dev - f_ref) <= f_bnd, (f_dev, f_ref, f_bnd)
    worst = float(np.max(np.abs(g_dev - g_ref) / (g_bnd + 1e-300)))
    assert worst <= 1.0, worst


@pytest.mark.timeout(600)
def test_c3_full_size_gram_and_step(clean_env):
    N, m = 1 << 20, 1 << 14
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic(N, m, x0, losses.logistic_ce(1.0 / N), 1.0, kind=1, seed=2026,
                                 out_fn=losses.sigmoid_ce(1.0 / N))
    p.λ = 0.1 * float(np.max(np.abs(p.gradx(np.zeros(m)))))
    rng = np.random.default_rng(7)
    cols = np.sort(rng.choice(m, 8, replace=False))
    w, v = rng.random(N) + 0.5, rng.standard_normal(N)
    pairs = [(int(i), int(j)) for a, i in enumerate(cols) for j in cols[a:]]
    g, atv, fused = p.gram_atv_sample(w, v, pairs)
    assert fused   # the production configuration at this shape: 256 x 128 tiles with the fused Aᵀv
    Ac = p.get_columns(cols)
    k = {int(c): n for n, c in enumerate(cols)}
    for (i, j), gv in zip(pairs, g):
        a, b = Ac[:, k[i]], Ac[:, k[j]]
        assert abs(gv - float((a * w) @ b)) <= 1e-11 * float(np.abs(a * w * b).sum())
    assert np.all(np.abs(atv[cols] - Ac.T @ v) <= 1e-11 * (np.abs(Ac).T @ np.abs(v)))
    sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=2, x_tol=0.0,
                         f_tol=0.0, verbose=0)
    # obj holds the pre-step objective of each epoch (+ the duplicated last push): obj[1] is f + λg at x1
    assert sol.epochs == 2 and np.all(np.isfinite(sol.x)) and sol.obj[1] < sol.obj[0]
    # the whole-length f / ∇f through the sigmoid / CE epilogue at the run's final x (and at x0)
    check_f_grad(p, sol.x, "logistic_ce")
    check_f_grad(p, x0, "logistic_ce")
    p.ctx.close()


@pytest.mark.timeout(600)
def test_c4_rank_shape_gram_and_steps(clean_env):
    N, m, gs, mu = 1 << 19, 1 << 15, 32, 1e-2
    ng = m // gs
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic(N, m, x0, losses.least_squares(1.0 / N), 1.0, kind=3, seed=2026,
                                 out_fn=losses.linear_ls(1.0 / N))
    g0 = p.gradx(np.zeros(m))
    p.λ = [1e-8, 0.1 * float(np.max(np.linalg.norm(g0.reshape(ng, gs), axis=1)))]
    ind = np.array([[1 + gs * g for g in range(ng)], [gs * (g + 1) for g in range(ng)], [1] * ng])
    p.P = scsopt.get_P(m, np.arange(1, m + 1), ind)
    rng = np.random.default_rng(11)
    cols = np.sort(rng.choice(m, 8, replace=False))
    w, v = rng.random(N) + 0.5, rng.standard_normal(N)
    pairs = [(int(i), int(j)) for a, i in enumerate(cols) for j in cols[a:]]
    g, atv, fused = p.gram_atv_sample(w, v, pairs)
    assert fused
    Ac = p.get_columns(cols)
    k = {int(c): n for n, c in enumerate(cols)}
    for (i, j), gv in zip(pairs, g):
        a, b = Ac[:, k[i]], Ac[:, k[j]]
        assert abs(gv - float((a * w) @ b)) <= 1e-11 * float(np.abs(a * w * b).sum())
    assert np.all(np.abs(atv[cols] - Ac.T @ v) <= 1e-11 * (np.abs(Ac).T @ np.abs(v)))
    sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "gl", scsopt.PHuberSmootherGL(mu, p), max_epoch=2, x_tol=0.0,
                         f_tol=0.0, verbose=0)
    assert sol.epochs == 2 and np.all(np.isfinite(sol.x)) and sol.obj[1] < sol.obj[0]
    check_f_grad(p, sol.x, "least_squares")
    p.ctx.close()


@pytest.mark.timeout(900)
def test_c5_full_size_f_and_gradient(clean_env):
    N, m = 1 << 20, 1 << 16
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), 1e-4, density=0.01, seed=2026,
                                        C_set=[-1.0, 1.0])
    sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", scsopt.PHuberSmootherIndBox(-1.0, 1.0, 0.6),
                         max_epoch=3, x_tol=0.0, f_tol=0.0, verbose=0)
    x = sol.x
    f_dev, g_dev = p.fx(x), p.gradx(x)
    A, y = p.get_sparse()
    p.ctx.close()
    scale = 1.0 / N
    r = A @ x - y
    f_ref = 0.5 * scale * float(r @ r)
    g_ref = scale * (A.T @ r)
    assert abs(f_dev - f_ref) <= 1e-11 * abs(f_ref)
    assert np.all(np.abs(g_dev - g_ref) <= 1e-11 * scale * (abs(A).T @ np.abs(r)) + 1e-300)
