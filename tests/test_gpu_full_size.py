"""GPU: parity at the FULL BASELINE sizes, default code path (no env overrides).

The other default-path tests (tests/test_gpu_default_path.py) run the BASELINE m at reduced N.  Here:
  * C2 (BASELINE configs[1]: ProxNSCORE logistic (margin) + l1, N = 100000, m = 8192), the whole
    problem: 2 epochs of the device loop against the oracle's restatement on the downloaded A at rtol
    1e-8 (obj, fval) -- a full-size trajectory;
  * C3 (configs[2]: N = 2^20, m = 2^14, A = 128 GiB on the device) and C4's per-rank shape at 8 GPUs
    (configs[3]: N = 2^22 / 8 = 2^19 rows, m = 2^15, least squares + sparse-group lasso, 1024 groups of
    32; A = 128 GiB): ONE default step! checked as a whole (r06; r05 sampled 36 Gram entries): the
    device's direction d = dx / safe_α must solve the whole feature-space GGN system, verified
    matrix-free on the host in ONE streamed pass over A in row blocks (host_ggn_pass: residual of
    (Aᵀ diag(w) A + λ diag Hr) d + Aᵀ(s⊙r) + λ gr against a bound stated before the run -- every Gram
    tile, the fused Aᵀv, the XCD work order and the factor / solves at the stated size), f and ∇f at
    x0 in the same pass, then the elementwise tail (η, α, the l1 / gl prox) against the oracle's
    functions on that d (sign / support pattern equal outside an 8-ulp near-threshold band); then
    two epochs of the default loop (objective decreases, iterate finite);
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


TAU = 1e-11   # the bound's relative unit, stated before any run (see host_ggn_pass)


def host_ggn_pass(p, x, d, kind, lam, Hr, gr, chunk_bytes=2 << 30):
    """ONE streamed pass over the device's A (scs_get_data, row blocks, column-major; no host copy
    of the whole A) that evaluates in fp64, at the step's x and for the device's direction d:
      * f(x) and ∇f(x) = Aᵀ(s⊙r) (the loss epilogue and the GEMV passes);
      * the whole feature-space GGN system of ggn_score_step (prox-GGN-SCORE.jl:121-131), matrix-free:
        res = (Aᵀ diag(w) A + λ diag Hr) d + (Aᵀ(s⊙r) + λ gr) = Aᵀ(w⊙(A d) + s⊙r) + λ(Hr⊙d + gr),
        with J = diag(s)A, Q = diag(q), w = s²q (logistic CE + sigmoid) or s = 1, r = c(z − y), w = c
        (least squares) -- every Gram entry enters through (G d)_j, every Aᵀv entry through e_j;
      * the diagonal M_jj = Σ_i w_i A_ij² + λ Hr_j of the system.
    Bounds (τ = TAU = 1e-11, stated before any run):
      f:    τ·(Σ|terms| + c·Σ_i (|A||x|)_i)
      ∇f_j: τ·(|A|ᵀ(|s r| + c·|A||x|))_j
      res_j: τ·( (|A|ᵀ(|w|⊙|A||d| + |s r| + c(|A d| + 1)⊙|A||x|))_j + λ(|Hr_j d_j| + |gr_j|)
               + sqrt(M_jj)·Σ_k sqrt(M_kk)|d_k| )
    The first group covers the summation orders (device Gram / GEMV vs host BLAS) and the host z
    differing from the device z in the last bits (|∂(s r)/∂z| <= c/4, |∂w/∂z| <= c/2); the last term
    is the Cholesky backward error |ΔM| <= γ_{3m+1}|Rᵀ||R| with (|Rᵀ||R|)_jk <= sqrt(M_jj M_kk)
    (γ_{3m+1} = 5.5e-12 at m = 16384, 1.1e-11 at 32768 -- Higham Thm 10.4; the blocked MFMA factor's
    error constant is the same order)."""
    from scsopt import _lib
    N, m = p.N, p.m
    c = 1.0 / p.N_global
    nr = max(16, (chunk_bytes // (8 * m)) // 16 * 16)
    buf = np.empty(nr * m)
    abuf = np.empty(nr * m)
    yb = np.empty(nr)
    X2 = np.stack([x, d], axis=1)
    X2a = np.abs(X2)
    f = fterms = fz = 0.0
    G2 = np.zeros((m, 2))      # [∇f | res without the λ terms]
    B2 = np.zeros((m, 2))      # their bound sums
    diag = np.zeros(m)
    for r0 in range(0, N, nr):
        n = min(nr, N - r0)
        Acm = buf[: m * n].reshape(m, n)   # Acm.T = rows r0 .. r0+n of A
        p.ctx.check(_lib.lib.scs_get_data(p.ctx.h, r0, n, Acm.ctypes.data_as(_lib.c_dp), n,
                                          yb.ctypes.data_as(_lib.c_dp)))
        y = yb[:n]
        Ab = np.abs(Acm, out=abuf[: m * n].reshape(m, n))
        Z = Acm.T @ X2
        ZA = Ab.T @ X2a
        z, u, zabs, uabs = Z[:, 0], Z[:, 1], ZA[:, 0], ZA[:, 1]
        if kind == "logistic_ce":
            s, yhat = O.sigmoid_jac(z)
            terms = -c * (y * np.log(yhat) + (1.0 - y) * np.log(1.0 - yhat))
            r = O.ce_r(y, yhat, c)
            w = s * s * O.ce_q(y, yhat, c)
            sr = s * r
        else:
            res = z - y
            terms = 0.5 * c * res * res
            sr = c * res
            w = np.full(n, c)
        f += float(terms.sum())
        fterms += float(np.abs(terms).sum())
        fz += c * float(zabs.sum())
        G2 += Acm @ np.stack([sr, w * u + sr], axis=1)
        asr = np.abs(sr)
        B2 += Ab @ np.stack([asr + c * zabs, np.abs(w) * uabs + asr + c * (np.abs(u) + 1.0) * zabs], axis=1)
        np.multiply(Ab, Ab, out=Ab)
        diag += Ab @ w
    res = G2[:, 1] + lam * (Hr * d + gr)
    M = diag + lam * Hr
    sq = np.sqrt(np.maximum(M, 0.0))
    rbnd = TAU * (B2[:, 1] + lam * (np.abs(Hr * d) + np.abs(gr)) + sq * float(sq @ np.abs(d)))
    return dict(f=f, fbnd=TAU * (fterms + fz), g=G2[:, 0], gbnd=TAU * B2[:, 0], res=res, rbnd=rbnd, M=M)


def whole_step_check(p, hm_dev, osm, om, reg, x0, lam, kind, record_property):
    """One default step! at x0 on the device (scs_step, iter 1), then: d = dx / safe_α (η, α from the
    oracle's smoother at x0, prox-GGN-SCORE.jl:89-97), the whole GGN system residual, f and ∇f at x0
    (host_ggn_pass), and the elementwise tail -- the oracle's prox applied to x0 + dx with the
    oracle's Hr -- against the device's x_new: equal sign / support pattern outside a stated
    near-threshold band (8 ulp of the threshold), values within 4 ulp of |x0 + dx| + threshold."""
    from scsopt.iterate import init_method, step
    m = x0.shape[0]
    M = scsopt.ProxGGNSCORE()
    p.configure(reg, hm_dev)
    init_method(M, p)
    x1, dx, pri = step(M, p, reg, hm_dev, x0, x0, 1, return_dx=True)
    Cmat = om.P if reg == "gl" else None
    gr, Hr = osm.grad(Cmat, x0), osm.hess(Cmat, x0)
    lgr = lam * gr
    Hinv = 1.0 / Hr
    Mg = O.get_Mg(osm.Mh, osm.nu, osm.mu, m)
    eta = np.sqrt(float(np.dot(lgr, Hinv * lgr)))
    step_size = 0.5                                     # ss_type 1, L === nothing
    safe_a = min(1.0, step_size / (1 + Mg * eta))
    d = dx / safe_a
    h = host_ggn_pass(p, x0, d, kind, lam, Hr, gr)
    f_dev, g_dev = p.fx(x0), p.gradx(x0)
    assert abs(f_dev - h["f"]) <= h["fbnd"], (f_dev, h["f"], h["fbnd"])
    gw = float(np.max(np.abs(g_dev - h["g"]) / (h["gbnd"] + 1e-300)))
    rw = float(np.max(np.abs(h["res"]) / (h["rbnd"] + 1e-300)))
    # the residual against the system's size: ‖res‖∞ / (‖diag M‖∞‖d‖∞ + ‖e‖∞), reported
    rel = float(np.max(np.abs(h["res"]))) / (float(np.max(h["M"])) * float(np.max(np.abs(d))) +
                                            float(np.max(np.abs(h["g"] + lgr))))
    record_property("grad_worst_over_bound", gw)
    record_property("residual_worst_over_bound", rw)
    record_property("residual_rel", rel)
    print(f"[whole-step] grad worst/bound {gw:.3e}  residual worst/bound {rw:.3e}  residual rel {rel:.3e}")
    assert gw <= 1.0, gw
    assert rw <= 1.0, rw
    # the tail: the oracle's prox on z = x0 + dx with the oracle's Hr
    z = x0 + dx
    x1h = O.invoke_prox(om, reg, z, Hinv, lam if reg != "gl" else om.lam, step_size)
    thr = step_size * lam * Hr if reg == "l1" else om.lam[0] * Hr
    eps = np.finfo(np.float64).eps
    near = np.abs(np.abs(z) - thr) <= 8 * eps * thr
    if reg == "gl":   # a group is zeroed when ‖u_g‖ <= α λ2 w_g Hr_k: flag groups near that threshold too
        u = np.sign(z) * np.maximum(np.abs(z) - thr, 0.0)
        ng = om.P.grpNUM
        gs = m // ng
        un = np.linalg.norm(u.reshape(ng, gs), axis=1)
        gthr = step_size * om.lam[1] * Hr.reshape(ng, gs)
        gnear = np.any(np.abs(un[:, None] - gthr) <= 1e-12 * gthr, axis=1)
        near |= np.repeat(gnear, gs)
    pat_dev = np.sign(x1) + 2.0 * np.signbit(x1)
    pat_host = np.sign(x1h) + 2.0 * np.signbit(x1h)
    bad = (pat_dev != pat_host) & ~near
    record_property("tail_near_threshold", int(near.sum()))
    assert not bad.any(), (int(bad.sum()), np.flatnonzero(bad)[:8])
    assert int(near.sum()) <= m // 1000, int(near.sum())
    ok = ~near
    vb = 4 * eps * (np.abs(z) + thr)   # the soft threshold: |z| − t and its sign, a few roundings
    if reg == "gl":
        # plus the group factor f = max(1 − a/‖u_g‖, 0), a = α λ2 w_g Hr_k, on u_k: ‖u_g‖ over gs squares
        # and a sqrt carries <= (gs/2 + 1) eps relative (worst case, any summation order), so
        # |δf| <= eps·(2 + (gs/2 + 1)·a/‖u_g‖).  (The first r06 run asserted the soft-threshold term
        # alone, 4 ulp, and measured 4.5 ulp at C4: that bound had left this factor out.)
        a = gthr.reshape(-1)
        vb = vb + np.abs(u) * eps * (2.0 + (gs / 2 + 1) * a / np.maximum(np.repeat(un, gs), 1e-300))
    worst = float(np.max(np.abs(x1[ok] - x1h[ok]) / vb[ok]))
    record_property("tail_worst_over_bound", worst)
    print(f"[whole-step] tail worst/bound {worst:.3e}  near-threshold coordinates {int(near.sum())}")
    assert worst <= 1.0, worst
    assert abs(pri - float(np.linalg.norm(x1 - x0))) <= 1e-12 * max(pri, 1e-300)
    return x1


@pytest.mark.timeout(600)
def test_c3_full_size_whole_step(clean_env, record_property):
    """C3 at its stated size (N = 2^20, m = 2^14, 128 GiB on the device): one default ProxGGNSCORE
    step! checked as a WHOLE -- the GGN system over every Gram tile, the fused Aᵀv, the XCD work
    order, the factor and the solves (host_ggn_pass), the damping and the l1 prox -- then two epochs
    of the default device loop (objective decreases, iterate finite)."""
    N, m = 1 << 20, 1 << 14
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic(N, m, x0, losses.logistic_ce(1.0 / N), 1.0, kind=1, seed=2026,
                                 out_fn=losses.sigmoid_ce(1.0 / N))
    lam = 0.1 * float(np.max(np.abs(p.gradx(np.zeros(m)))))
    p.λ = lam
    om = O.Problem(None, None, x0, O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce"), lam)
    whole_step_check(p, scsopt.PHuberSmootherL1L2(1.0), O.PHuberSmootherL1L2(1.0), om, "l1", x0, lam, "logistic_ce", record_property)
    sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=2, x_tol=0.0,
                         f_tol=0.0, verbose=0)
    # obj holds the pre-step objective of each epoch (+ the duplicated last push): obj[1] is f + λg at x1
    assert sol.epochs == 2 and np.all(np.isfinite(sol.x)) and sol.obj[1] < sol.obj[0]
    p.ctx.close()


@pytest.mark.timeout(600)
def test_c4_rank_shape_whole_step(clean_env, record_property):
    """C4's per-rank shape at 8 GPUs (N = 2^22 / 8 = 2^19 rows, m = 2^15, least squares + sparse-group
    lasso, 1024 groups of 32, μ = 1e-2): one default ProxGGNSCORE step! checked as a whole (the
    system at λ1 with PHuberSmootherGL's Hr, then the gl prox), then two epochs of the default loop."""
    N, m, gs, mu = 1 << 19, 1 << 15, 32, 1e-2
    ng = m // gs
    x0 = np.random.default_rng(1234).standard_normal(m)
    p = scsopt.Problem.synthetic(N, m, x0, losses.least_squares(1.0 / N), 1.0, kind=3, seed=2026,
                                 out_fn=losses.linear_ls(1.0 / N))
    g0 = p.gradx(np.zeros(m))
    lam = [1e-8, 0.1 * float(np.max(np.linalg.norm(g0.reshape(ng, gs), axis=1)))]
    p.λ = lam
    ind = np.array([[1 + gs * g for g in range(ng)], [gs * (g + 1) for g in range(ng)], [1] * ng])
    p.P = scsopt.get_P(m, np.arange(1, m + 1), ind)
    om = O.Problem(None, None, x0, O.Loss("least_squares", 1.0 / N, ggn="linear_ls"), lam,
                   P=O.GroupP(m, ind, np.arange(1, m + 1)))
    whole_step_check(p, scsopt.PHuberSmootherGL(mu, p), O.PHuberSmootherGL(mu, om), om, "gl", x0, lam[0], "least_squares", record_property)
    sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "gl", scsopt.PHuberSmootherGL(mu, p), max_epoch=2, x_tol=0.0,
                         f_tol=0.0, verbose=0)
    assert sol.epochs == 2 and np.all(np.isfinite(sol.x)) and sol.obj[1] < sol.obj[0]
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
