"""CPU: pin the oracle against the reference's own tests, analytic known answers and
the committed golden fixtures (tests/golden/make_golden.py)."""
import math

import numpy as np
import pytest

import scsopt_oracle as O
from make_golden import LOGI_A, LOGI_Y, X0, QP_A, QP_Y, QP_X0, QP_XS


def logistic_model(ggn=True):
    return O.Problem(np.array(LOGI_A), np.array(LOGI_Y, float), X0,
                     O.Loss("logistic_margin", 1 / 5, ggn="sigmoid_ce" if ggn else None), 1)


@pytest.mark.parametrize("meth", [O.ProxNSCORE, O.ProxGGNSCORE, O.ProxLQNSCORE])
@pytest.mark.parametrize("reg", ["l1", "l2"])
def test_reference_logistic_assertions(meth, reg):
    """test/test_algs.jl:22-51 (and the batch/slice_samples copies :54-78)."""
    model = logistic_model()
    sol = O.iterate(meth(), model, reg, O.PHuberSmootherL1L2(1))
    assert np.allclose(model.sol, 0.0)
    assert sol.epochs + 1 >= 1
    assert sol.rel[-1] <= 1e-6
    assert sol.objrel[-1] <= 1e-6


@pytest.mark.parametrize("smoother,alpha", [("phuber", 0.8), ("exp", 1.0)])
def test_reference_indbox_assertions(smoother, alpha):
    """test/test_algs.jl:82-108."""
    sm = (O.PHuberSmootherIndBox(-1.0, 1.0, 0.6) if smoother == "phuber"
          else O.ExponentialSmootherIndBox(-1.0, 1.0, 0.6))
    model = O.Problem(np.array(QP_A), np.array(QP_Y), QP_X0, O.Loss("quadratic"), 1e-4, C_set=[-1.0, 1.0],
                      sol=np.array(QP_XS))
    sol = O.iterate(O.ProxNSCORE(), model, "indbox", sm, alpha=alpha)
    assert sol.rel[-1] <= 1e-3
    assert sol.objrel[-1] <= 1e-3


def test_smoother_constants():
    """test/test_smooth.jl:7-8, 13-14."""
    h = O.PHuberSmootherL1L2(1)
    assert h.Mh == 2.0 and h.nu == 2.6
    h = O.PHuberSmootherIndBox(-1.0, 1.0, 1)
    assert h.Mh == 2.0 and h.nu == 2.6


def test_kat_boxqp_interior_optimum():
    """x_star of test_algs.jl:85 is the unconstrained optimum A⁻¹(−y) (interior of the box)."""
    xs = np.linalg.solve(np.array(QP_A), -np.array(QP_Y))
    assert np.max(np.abs(xs - np.array(QP_XS))) < 3e-6
    assert np.all(np.abs(xs) < 1)


def test_kat_l1_logistic_zero():
    """λ = 1 ≥ ‖∇f(0)‖∞ ⇒ x* = 0 exactly; the prox lands on exact zeros."""
    model = logistic_model()
    g0 = model.gradx(np.zeros(2))
    assert np.max(np.abs(g0)) <= 1
    sol = O.iterate(O.ProxNSCORE(), model, "l1", O.PHuberSmootherL1L2(1))
    assert np.all(sol.x == 0.0)


def test_kat_rosenbrock():
    model = O.Problem(None, None, X0, O.Loss("rosenbrock"), 1e-8)
    sol = O.iterate(O.ProxLQNSCORE(m=10), model, "l1", O.PHuberSmootherL1L2(1.0))
    assert np.allclose(sol.x, [1.0, 1.0], atol=1e-6)


def test_history_semantics_max_epoch():
    """iterate.jl:219-231: with no early stop the pre-step x is pushed twice at max_epoch."""
    model = O.Problem(None, None, X0, O.Loss("rosenbrock"), 1e-8)
    sol = O.iterate(O.ProxLQNSCORE(m=10), model, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=5)
    assert len(sol.obj) == 6
    assert sol.obj[-1] == sol.obj[-2]
    assert sol.pri_res_norm[0] is None
    assert sol.epochs == 5


def test_julia_scalar_semantics():
    assert math.copysign(1, float(O.jl_max(-0.0, 0.0))) == 1.0
    assert math.copysign(1, float(O.jl_max(0.0, -0.0))) == 1.0
    assert math.copysign(1, float(O.jl_min(0.0, -0.0))) == -1.0
    assert math.isnan(float(O.jl_max(np.nan, 1.0))) and math.isnan(float(O.jl_max(1.0, np.nan)))
    assert math.copysign(1, float(O.jl_sign(-0.0))) == -1.0 and float(O.jl_sign(-3.0)) == -1.0
    # prox l1 keeps signed zeros: sign(z)*max(|z|-t, 0)
    out = O.prox_l1(np.array([-0.1, 0.1, -0.0, 0.0]), np.ones(4), 1.0, 1.0)
    assert list(np.signbit(out)) == [True, False, True, False]


def test_get_Mg_values():
    """get_Mg(2, 2.6, 1, m) for the config sizes."""
    assert O.get_Mg(2.0, 2.6, 1.0, 8192) == pytest.approx(12.1257, abs=1e-4)
    assert O.get_Mg(2.0, 2.6, 1.0, 16384) == pytest.approx(13.9288, abs=1e-4)
    assert O.get_Mg(2.0, 2.6, 1.0, 65536) == pytest.approx(18.3792, abs=1e-4)
    with pytest.raises(ValueError, match="μ must be positive"):
        O.get_Mg(2.0, 2.6, 0.0, 5)


def test_phuber_indbox_kat():
    """the `-x < a` quirk (phuber-smooth.jl:89) at x ∈ {−2,…,2}, μ = 0.6, box [−1, 1]."""
    x = np.array([-2.0, -1.0, 0.0, 1.0, 2.0])
    g = O.huber_grad_indbox(x, 0.6, -1.0, 1.0)
    h = O.huber_hess_indbox(x, 0.6, -1.0, 1.0)
    assert list(g[:3]) == [O.EPS] * 3 and g[3] == 0.0
    assert g[4] == pytest.approx(-0.98058, abs=1e-5)
    assert h[0] == pytest.approx(0.22698, abs=1e-5) and h[4] == pytest.approx(0.22698, abs=1e-5)
    assert h[1] == pytest.approx(1 / 0.6, rel=1e-12) and h[3] == pytest.approx(1 / 0.6, rel=1e-12)
    assert h[2] == O.EPS


def test_golden_fixtures_reproduce(golden):
    """The committed trajectories are what this oracle produces (regression pin)."""
    import make_golden
    fresh = make_golden.cases()
    for name, ref in golden["cases"].items():
        got = fresh[name]
        assert got["epochs"] == ref["epochs"], name
        assert len(got["obj"]) == len(ref["obj"]), name
        np.testing.assert_allclose(got["obj"], ref["obj"], rtol=1e-13, atol=0, err_msg=name)
        np.testing.assert_allclose(got["x"], ref["x"], rtol=1e-12, atol=1e-300, err_msg=name)
        assert len(got["fvaltest"]) == len(ref["fvaltest"]), name
        np.testing.assert_allclose(got["fvaltest"], ref["fvaltest"], rtol=1e-13, atol=0, err_msg=name)
        if name.endswith("_heldout"):
            assert len(got["fvaltest"]) == len(got["obj"]) > 0, name
        else:
            assert got["fvaltest"] == [], name


def test_golden_kernel_vectors(golden):
    k = golden["kernels"]
    x = np.array(k["x"])
    np.testing.assert_array_equal(O.huber_grad(x, 1.0), np.array(k["phuber_l1l2_mu1"]["grad"]))
    p = k["prox_in"]
    out = O.prox_l1(np.array(p["z"]), 1.0 / np.array(p["Hr"]), p["lam"], p["alpha"])
    np.testing.assert_array_equal(out, np.array(k["prox_l1"]))


@pytest.mark.parametrize("mu", [0.3, 1.0])
def test_new_smoothers_derivative_consistency(mu):
    """LogExp indbox / Ostrovskii-Bach restatements (log-exp-smooth.jl:36-61,
    ostrovskii-bach-smooth.jl:28-36): central differences of val reproduce grad, of grad reproduce
    hess (away from the branch points; the reference ships no vectors for these smoothers, so this
    pins the restatement against its own value functions)."""
    x = np.linspace(-3.0, 3.0, 61)
    x = x[np.abs(x) > 0.04]
    h = 1e-6
    # Ostrovskii-Bach (l1 smoothing)
    g_fd = (O.osba_val(x + h, mu) - O.osba_val(x - h, mu)) / (2 * h)
    np.testing.assert_allclose(O.osba_grad(x, mu), g_fd, rtol=1e-6, atol=1e-8)
    H_fd = (O.osba_grad(x + h, mu) - O.osba_grad(x - h, mu)) / (2 * h)
    np.testing.assert_allclose(O.osba_hess(x, mu), H_fd, rtol=1e-5, atol=1e-7)
    assert np.isnan(O.osba_grad(np.array([0.0]), mu)[0])          # 0/0 at x = 0, as in Julia
    # LogExp indbox on [-1, 1]: both pieces, away from x = a, a + μ, b - μ, b
    lb, ub = -1.0, 1.0
    kinks = np.array([lb, lb + mu, ub - mu, ub])
    xs = np.linspace(-0.999, 0.999, 200)
    xs = xs[np.min(np.abs(xs[:, None] - kinks[None, :]), axis=1) > 1e-3]
    g_fd = (O.logexp_val_indbox(xs + h, mu, lb, ub) - O.logexp_val_indbox(xs - h, mu, lb, ub)) / (2 * h)
    np.testing.assert_allclose(O.logexp_grad_indbox(xs, mu, lb, ub), g_fd, rtol=1e-6, atol=1e-8)
    H_fd = (O.logexp_grad_indbox(xs + h, mu, lb, ub) - O.logexp_grad_indbox(xs - h, mu, lb, ub)) / (2 * h)
    np.testing.assert_allclose(O.logexp_hess_indbox(xs, mu, lb, ub), H_fd, rtol=1e-5, atol=1e-7)
    # outside the box: the barrier part μ/(a-x), μ/(a-x)^2
    xo = np.array([-1.5, 1.5])
    np.testing.assert_allclose(O.logexp_grad_indbox(xo, mu, lb, ub),
                               [(-1.5 + 1 - 2 * mu) / mu + mu / 0.5, (1.5 - 1 + 2 * mu) / mu - mu / -0.5])


def test_new_smoother_constants():
    """Mh / ν of the added smoothers (log-exp-smooth.jl:25-26, ostrovskii-bach-smooth.jl:3-4) and
    the get_Mg branch they select (smoothing.jl:12-25: ν = 3 -> n^0 μ^-0.5 Mh; ν = 2 -> n^0.5 μ^-1 Mh)."""
    import scsopt
    h = scsopt.OsBaSmootherL1L2(0.5)
    assert (h.Mh, h.ν) == (2 * np.sqrt(2), 3.0)
    assert O.get_Mg(h.Mh, h.ν, 0.5, 1000) == pytest.approx(2 * np.sqrt(2) * 0.5 ** -0.5)
    h = scsopt.LogExpSmootherIndBox(-1.0, 1.0, 0.5)
    assert (h.Mh, h.ν) == (1.0, 2.0)
    assert O.get_Mg(h.Mh, h.ν, 0.5, 100) == pytest.approx(10.0 * 0.5 ** -1.0)


def test_loader_batches_semantics():
    """iterate.jl:124-146 / utils.jl:14-25: ceil(N/b) batches with a partial last one, batch_size
    wins over slice_samples, slice_samples keeps only the first sample (max_iter stays 1),
    local_max_iter truncates; the product's host restatement builds the identical list."""
    from scsopt.iterate import loader_batches as host_batches
    perm = np.random.default_rng(0).permutation(10)
    cases = [dict(batch_size=4, shuffle_batch=False), dict(batch_size=4, shuffle_batch=True, perm=perm),
             dict(batch_size=10), dict(batch_size=3, local_max_iter=2.9), dict(slice_samples=True),
             dict(batch_size=5, slice_samples=True, shuffle_batch=False), dict()]
    for kw in cases:
        kw.setdefault("perm", perm)
        ob = O.loader_batches(10, **kw)
        hb = host_batches(10, **kw)
        if ob is None:
            assert hb is None
            continue
        assert [list(b) for b in ob] == [list(b) for b in hb], kw
    b = O.loader_batches(10, 4, shuffle_batch=False)
    assert [len(t) for t in b] == [4, 4, 2] and list(np.concatenate(b)) == list(range(10))
    assert [list(t) for t in O.loader_batches(10, slice_samples=True)] == [[0]]
    assert len(O.loader_batches(10, 3, shuffle_batch=False, local_max_iter=2.9)) == 2
    assert O.loader_batches(10) is None
    assert [list(t) for t in O.loader_batches(10, 5, slice_samples=True, shuffle_batch=False)] == \
        [[0, 1, 2, 3, 4], [5, 6, 7, 8, 9]]


@pytest.mark.parametrize("meth", [O.ProxNSCORE, O.ProxGGNSCORE, O.ProxLQNSCORE])
def test_batched_loop_semantics(meth):
    """One unshuffled full batch == the full-batch loop (bitwise); two batches per epoch keep the
    history rules (one push per epoch + the max_epoch entry, iterate.jl:219-231, taken before the
    epoch's last batch) and step on each batch's rows."""
    model = logistic_model()
    full = O.iterate(meth(), model, "l1", O.PHuberSmootherL1L2(1))
    one = O.iterate(meth(), logistic_model(), "l1", O.PHuberSmootherL1L2(1),
                    batches=O.loader_batches(5, 5, shuffle_batch=False))
    assert full.obj == one.obj and np.array_equal(full.x, one.x) and full.epochs == one.epochs
    small = lambda: O.Problem(np.array(LOGI_A), np.array(LOGI_Y, float), X0,  # noqa: E731
                              O.Loss("logistic_margin", 1 / 5, ggn="sigmoid_ce"), 0.1)
    two = O.iterate(meth(), small(), "l1", O.PHuberSmootherL1L2(1), max_epoch=4, x_tol=0.0, f_tol=0.0,
                    batches=O.loader_batches(5, 3, shuffle_batch=False))
    assert len(two.obj) == 5 and two.epochs == 4   # the max_epoch entry is taken before the last batch
    assert not np.array_equal(two.x, O.iterate(meth(), small(), "l1", O.PHuberSmootherL1L2(1),
                                               max_epoch=4, x_tol=0.0, f_tol=0.0).x)


def test_set_name_plain_labels():
    """set_name! without the prox: the literal names / labels of prox-N-SCORE.jl:24-33,
    prox-GGN-SCORE.jl:24-33 and prox-L-BFGS-SCORE.jl:37-46."""
    for M, name, label in ((O.ProxNSCORE, "newtonscore", "Newton-SCORE"), (O.ProxGGNSCORE, "ggnscore", "GGN-SCORE"),
                           (O.ProxLQNSCORE, "lbfgsscore", "LBFGS-SCORE")):
        algs = []
        m = M(use_prox=False)
        O.set_name(m, algs)
        assert (m.name, m.label) == (name, label) and algs[-1] == name
        p = M()
        O.set_name(p, algs)
        assert p.name.startswith("prox-") and p.label.startswith("Prox-")


def test_oracle_fvaltest_history():
    """iterate.jl:169-175 / utils.jl:55-57: with Atest AND ytest every stats push appends
    ftest(x) = f(Atest, ytest, x) of the pushed point (same f, same scale), so len(fvaltest) ==
    len(obj), including the duplicated max-epoch push.  One of the two alone (the xor case,
    iterate.jl:170-171) logs the @info and leaves `ftest` unassigned, so the first show_stat!
    (:201) raises UndefVarError; a ProblemGeneric records nothing."""
    A = np.array([[-0.560501, 0.0], [0.0, 1.85278], [-0.0192918, -0.827763], [0.128064, 0.110096],
                  [0.0, -0.251176]])
    y = np.array([-1.0, -1.0, -1.0, 1.0, -1.0])
    At = np.array([[0.3, -0.2], [-1.1, 0.4], [0.7, 0.9]])
    yt = np.array([1.0, -1.0, 1.0])
    x0 = np.array([0.5908446386657102, 0.7667970365022592])
    loss = O.Loss("logistic_margin", 1 / 5)
    for max_epoch in (2, 1000):
        om = O.Problem(A, y, x0, loss, 1.0, Atest=At, ytest=yt)
        sol = O.iterate(O.ProxNSCORE(), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=max_epoch)
        assert len(sol.fvaltest) == len(sol.obj)
        assert sol.fvaltest[0] == loss.f(At, yt, x0)
        if max_epoch == 1000:   # the termination push is of x_new = the returned x (iterate.jl:235-247)
            assert sol.fvaltest[-1] == pytest.approx(loss.f(At, yt, sol.x), rel=1e-12)
        else:   # 2 epoch pushes + the duplicated max-epoch push (iterate.jl:219-231)
            assert len(sol.obj) == 3 and sol.fvaltest[-1] == sol.fvaltest[-2] and sol.obj[-1] == sol.obj[-2]
    for kw in ({"Atest": At}, {"ytest": yt}):
        om = O.Problem(A, y, x0, loss, 1.0, **kw)
        assert not om.test_model
        with pytest.raises(O.UndefVarError, match="ftest"):
            O.iterate(O.ProxNSCORE(), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=3)


def test_oracle_ggn_ss3_grad_fx_one_argument():
    """SURVEY Appendix A #8 (prox-GGN-SCORE.jl:58-59,83-84): ProxGGNSCORE's grad_f is
    x -> model.grad_fx(x), one argument, called only by the ss_type 3 line search (utils.jl:31,
    after f(x + αd) and f(x)).  A data problem's grad_fx(A, y, x) raises MethodError at the first
    trial; a one-argument grad_fx is applicable and gives the same steps as the loss kind (whose
    gradient plays ForwardDiff's part, grad_fx === nothing); ss_type 1 never calls it."""
    rng = np.random.default_rng(4)
    N, m = 40, 6
    A = rng.standard_normal((N, m)) / np.sqrt(m)
    y = (rng.random(N) < 0.5).astype(np.float64)
    x0 = rng.standard_normal(m) * 0.3
    kind = O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce")
    sig = lambda z: 1.0 / (1.0 + np.exp(-z))  # noqa: E731
    calls = []

    def f(A, y, x):
        calls.append("f")
        return kind.f(A, y, x)

    def g3(A, y, x):
        return kind.grad(A, y, x)

    pieces = dict(out_fn=lambda A, x: sig(A @ x),
                  jac_yx=lambda A, y, yh, x: (yh * (1 - yh))[:, None] * A,
                  grad_fy=lambda A, y, yh: (-(y / yh) + (1 - y) / (1 - yh)) / N,
                  hess_fy=lambda A, y, yh: (y / yh ** 2 + (1 - y) / (1 - yh) ** 2) / N)
    hm = O.PHuberSmootherL1L2(1.0)
    p3 = O.Problem(A, y, x0, O.CallbackLoss(f, g3, **pieces), 1e-2)
    with pytest.raises(O.MethodError, match=r"no method matching grad_fx\(::Vector\{Float64\}\)"):
        O.iterate(O.ProxGGNSCORE(ss_type=3), p3, "l1", hm, max_epoch=3)
    assert calls.count("f") >= 2      # f(x + αd) and f(x) ran before grad_f (utils.jl:31 order)
    a = O.iterate(O.ProxGGNSCORE(ss_type=1), p3, "l1", hm, max_epoch=3)
    b = O.iterate(O.ProxGGNSCORE(ss_type=1), O.Problem(A, y, x0, kind, 1e-2), "l1", hm, max_epoch=3)
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-9)
    g1 = lambda x: kind.grad(A, y, x)  # noqa: E731
    c = O.iterate(O.ProxGGNSCORE(ss_type=3), O.Problem(A, y, x0, O.CallbackLoss(f, g1, **pieces), 1e-2), "l1", hm,
                  max_epoch=4)
    d = O.iterate(O.ProxGGNSCORE(ss_type=3), O.Problem(A, y, x0, kind, 1e-2), "l1", hm, max_epoch=4)
    assert c.epochs == d.epochs
    np.testing.assert_allclose(c.obj, d.obj, rtol=1e-9)
