"""GPU: held-out data -- Problem(...; Atest, ytest) (problems.jl:27-28,67-68) and the per-push
test loss ftest(x) = f(Atest, ytest, x) that becomes Solution.fvaltest (iterate.jl:169-175,
utils.jl:55-57).

Every case runs the HIP path through the C ABI and compares the whole fvaltest history with the
oracle's restatement of the same loop (oracle/scsopt_oracle.py `iterate`) at rtol 1e-8; the
history has one entry per obj entry (the epoch pushes, the duplicated max-epoch push and the
termination push).  Parity of the held-out loss against the reference itself is unpinned: the
reference's tests never pass Atest / ytest.
"""
import logging

import numpy as np
import pytest
import scipy.sparse as sp

import scsopt
import scsopt_oracle as O
from scsopt import losses

pytestmark = pytest.mark.gpu

RT = 1e-8


def _kinds(method, N):
    if method == "ggn":
        return (losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N), O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce"),
                scsopt.ProxGGNSCORE, O.ProxGGNSCORE)
    if method == "nscore":
        return (losses.logistic_margin(1.0 / N), None, O.Loss("logistic_margin", 1.0 / N), scsopt.ProxNSCORE,
                O.ProxNSCORE)
    return (losses.least_squares(1.0 / N), None, O.Loss("least_squares", 1.0 / N), scsopt.ProxLQNSCORE,
            O.ProxLQNSCORE)


def _data(method, N, Nt, m, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((N + Nt, m)) / np.sqrt(m)
    xt = rng.standard_normal(m) * (rng.random(m) < 0.2)
    z = A @ xt
    if method == "ggn":
        y = (rng.random(N + Nt) < 1 / (1 + np.exp(-z))).astype(float)
    elif method == "nscore":
        y = np.where(rng.random(N + Nt) < 1 / (1 + np.exp(-z)), 1.0, -1.0)
    else:
        y = z + 0.1 * rng.standard_normal(N + Nt)
    return A[:N], y[:N], A[N:], y[N:]


def _check(sol, osol):
    assert sol.epochs == osol.epochs
    assert len(sol.fvaltest) == len(sol.obj) == len(osol.fvaltest) == len(osol.obj)
    np.testing.assert_allclose(sol.obj, osol.obj, rtol=RT, atol=0)
    np.testing.assert_allclose(sol.fvaltest, osol.fvaltest, rtol=RT, atol=0)


@pytest.mark.parametrize("method", ["ggn", "nscore", "lqn"])
@pytest.mark.parametrize("device_loop", [True, False])
def test_fvaltest_matches_oracle(method, device_loop):
    """All three methods, both loops (scs_iterate and the host restatement), a max-epoch run (the
    duplicated last push) and a terminating run (the post-step push of x_new)."""
    N, Nt, m, lam = 2048, 640, 192, 2e-3
    A, y, At, yt = _data(method, N, Nt, m, 11)
    x0 = np.random.default_rng(3).standard_normal(m) * 0.5
    f, out, of, meth, ometh = _kinds(method, N)
    p = scsopt.Problem(A, y, x0, f, lam, out_fn=out, Atest=At, ytest=yt)
    om = O.Problem(A, y, x0, of, lam, Atest=At, ytest=yt)
    assert p.test_model and om.test_model
    for max_epoch, x_tol in ((7, 1e-10), (300, 1e-4)):   # the second run terminates at 15-22 epochs
        sol = scsopt.iterate(meth(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=max_epoch, x_tol=x_tol,
                             verbose=0, device_loop=device_loop)
        osol = O.iterate(ometh(), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=max_epoch, x_tol=x_tol)
        _check(sol, osol)
        # the value is ftest of the pushed point: the first entry is f(Atest, ytest, x0)
        assert sol.fvaltest[0] == pytest.approx(of.f(At, yt, x0), rel=1e-12)
        if max_epoch == 7:   # 7 epoch pushes + the duplicated max-epoch push (iterate.jl:219-231)
            assert len(sol.obj) == 8 and sol.fvaltest[-1] == sol.fvaltest[-2]


def test_fused_lqn_loop_fvaltest():
    """ProxLQNSCORE at m >= 16384 runs scs_iterate's fused, one-epoch-pipelined loop: the held-out
    loss of x_new is enqueued behind the epoch's tail and rides the epoch's scalar hand-off."""
    N, Nt, m, lam = 1024, 384, 16384, 1e-4
    A, y, At, yt = _data("lqn", N, Nt, m, 5)
    x0 = np.clip(np.random.default_rng(8).standard_normal(m) * 0.3, -1, 1)
    p = scsopt.Problem(A, y, x0, losses.least_squares(1.0 / N), lam, C_set=[-1.0, 1.0], Atest=At, ytest=yt)
    om = O.Problem(A, y, x0, O.Loss("least_squares", 1.0 / N), lam, C_set=[-1.0, 1.0], Atest=At, ytest=yt)
    hm, ohm = scsopt.PHuberSmootherIndBox(-1.0, 1.0, 0.6), O.PHuberSmootherIndBox(-1.0, 1.0, 0.6)
    for max_epoch, x_tol in ((9, 1e-10), (400, 1e-5)):
        sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", hm, max_epoch=max_epoch, x_tol=x_tol, verbose=0)
        host = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", hm, max_epoch=max_epoch, x_tol=x_tol,
                              verbose=0, device_loop=False)
        osol = O.iterate(O.ProxLQNSCORE(m=20), om, "indbox", ohm, max_epoch=max_epoch, x_tol=x_tol)
        _check(sol, osol)
        assert sol.fvaltest == host.fvaltest and sol.obj == host.obj


def test_sparse_test_set():
    """A sparse A with a sparse held-out set (the C5 problem class in miniature): CSR test rows,
    fp64 and fp32-stored values."""
    N, Nt, m, lam = 4096, 1024, 512, 1e-4
    rng = np.random.default_rng(21)
    A = sp.random(N + Nt, m, density=0.02, format="csr", random_state=rng, data_rvs=rng.standard_normal)
    y = A @ rng.uniform(-1.5, 1.5, m) + 0.1 * rng.standard_normal(N + Nt)
    Atr, Ate = A[:N], A[N:]
    x0 = np.clip(rng.standard_normal(m), -1, 1)
    om = O.Problem(Atr, y[:N], x0, O.Loss("least_squares", 1.0 / N), lam, C_set=[-1.0, 1.0], Atest=Ate,
                   ytest=y[N:])
    osol = O.iterate(O.ProxLQNSCORE(m=20), om, "indbox", O.PHuberSmootherIndBox(-1.0, 1.0, 0.6), max_epoch=12)
    for f32 in (False, True):
        p = scsopt.Problem(Atr, y[:N], x0, losses.least_squares(1.0 / N), lam, C_set=[-1.0, 1.0], sparse_f32=f32)
        p.set_test(Ate, y[N:], sparse_f32=f32)
        sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=20), p, "indbox", scsopt.PHuberSmootherIndBox(-1.0, 1.0, 0.6),
                             max_epoch=12, verbose=0)
        if not f32:
            _check(sol, osol)
        else:   # fp32-stored values of both sets: the storage rounding only
            np.testing.assert_allclose(sol.fvaltest, osol.fvaltest, rtol=1e-5)
            assert len(sol.fvaltest) == len(sol.obj)


def test_callback_loss_test_set():
    """A callback loss keeps the held-out data on the host: SCS_CB_FTEST calls the caller's own
    f(Atest, ytest, x)."""
    N, Nt, m, lam = 600, 200, 40, 1e-3
    A, y, At, yt = _data("lqn", N, Nt, m, 2)
    x0 = np.random.default_rng(1).standard_normal(m)

    def f(A_, y_, x):
        r = A_ @ x - y_
        return 0.5 * float(r @ r) / N

    def g(A_, y_, x):
        return A_.T @ (A_ @ x - y_) / N

    p = scsopt.Problem(A, y, x0, losses.callback(f, g), lam, Atest=At, ytest=yt)
    om = O.Problem(A, y, x0, O.CallbackLoss(f, g), lam, Atest=At, ytest=yt)
    sol = scsopt.iterate(scsopt.ProxLQNSCORE(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=10, verbose=0)
    osol = O.iterate(O.ProxLQNSCORE(), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=10)
    _check(sol, osol)


def test_generated_test_rows_and_skip(caplog):
    """gen_test: the held-out rows are rows [N, N + Nt) of the same generator (same x_true); one of
    Atest / ytest alone logs the reference's message and then raises the reference's UndefVarError at
    the first stats push (iterate.jl:170-171,201), in both loops and in the multi-device context."""
    N, Nt, m = 2048, 512, 128
    x0 = np.random.default_rng(4).standard_normal(m)
    f, out, of, meth, ometh = _kinds("ggn", N)
    p = scsopt.Problem.synthetic(N, m, x0, f, 1e-3, kind=1, seed=17, out_fn=out, test_N=Nt)
    big = scsopt.Problem.synthetic(N + Nt, m, x0, f, 1e-3, kind=1, seed=17, out_fn=out)
    Ab, yb = big.get_data()
    A, y = p.get_data()
    np.testing.assert_array_equal(A, Ab[:N])
    np.testing.assert_array_equal(y, yb[:N])
    assert p.ftest(x0) == pytest.approx(of.f(Ab[N:], yb[N:], x0), rel=1e-13)
    om = O.Problem(A, y, x0, of, 1e-3, Atest=Ab[N:], ytest=yb[N:])
    sol = scsopt.iterate(meth(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=6, verbose=0)
    osol = O.iterate(ometh(), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=6)
    _check(sol, osol)
    for kw in ({"Atest": Ab[N:]}, {"ytest": yb[N:]}):
        for devices in (None, [0]):
            q = scsopt.Problem(A, y, x0, f, 1e-3, out_fn=out, devices=devices, **kw)
            assert not q.test_model and q.test_xor
            for device_loop in (True, False):
                caplog.clear()
                with caplog.at_level(logging.INFO, logger="scsopt"):
                    with pytest.raises(scsopt.ScsReferenceError, match="UndefVarError: `ftest` not defined"):
                        scsopt.iterate(meth(), q, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=3, verbose=0,
                                       device_loop=device_loop)
                assert "Will skip testing" in caplog.text
        with pytest.raises(O.UndefVarError):
            O.iterate(ometh(), O.Problem(A, y, x0, of, 1e-3, **kw), "l1", O.PHuberSmootherL1L2(1.0), max_epoch=3)
    # both given again: the same problem runs (a new set_test clears the xor state)
    q.set_test(Ab[N:], yb[N:])
    assert q.test_model and not q.test_xor
    assert len(scsopt.iterate(meth(), q, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=2, verbose=0).fvaltest) == 3


def test_multi_device_context_test_set():
    """scs_create_multi at one device splits the held-out rows like the data; same history."""
    N, Nt, m = 1500, 333, 96
    A, y, At, yt = _data("nscore", N, Nt, m, 9)
    x0 = np.random.default_rng(6).standard_normal(m) * 0.2
    f, out, of, meth, ometh = _kinds("nscore", N)
    a = scsopt.Problem(A, y, x0, f, 1e-3, Atest=At, ytest=yt)
    b = scsopt.Problem(A, y, x0, f, 1e-3, Atest=At, ytest=yt, devices=[0])
    sa = scsopt.iterate(meth(), a, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=5, verbose=0)
    sb = scsopt.iterate(meth(), b, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=5, verbose=0)
    assert sa.fvaltest == sb.fvaltest and sa.obj == sb.obj and len(sa.fvaltest) == len(sa.obj)


def test_six_field_scs_iterate_refuses_test_data():
    """ABI note: scs_iterate reads the six-field (r03) history and never writes fvaltest,
    so with test data held it refuses (SCS_ERR_STATE, pointing at scs_iterate_ex) instead of returning
    a Solution whose fvaltest was silently dropped; without test data it runs as before."""
    import ctypes as C
    from scsopt import _lib
    from scsopt.iterate import init_method
    N, Nt, m = 400, 120, 30
    A, y, At, yt = _data("lqn", N, Nt, m, 5)
    f, out = _kinds("lqn", N)[:2]
    x0 = np.random.default_rng(6).standard_normal(m) * 0.2
    hm = scsopt.PHuberSmootherL1L2(1.0)
    for with_test in (True, False):
        kw = dict(Atest=At, ytest=yt) if with_test else {}
        p = scsopt.Problem(A, y, x0, f, 1e-3, out_fn=out, **kw)
        M = scsopt.ProxLQNSCORE(m=5)
        p.configure("l1", hm)
        init_method(M, p)
        hist = {k: np.empty(9) for k in ("obj", "fval", "pri_res_norm", "rel", "objrel", "times", "fvaltest")}
        h = _lib.History(*(hist[k].ctypes.data_as(_lib.c_dp) for k in hist))
        xo, nh, ep = np.empty(m), C.c_int64(), C.c_int64()
        x0c, xs = np.ascontiguousarray(x0), np.zeros(m)
        rc = _lib.lib.scs_iterate(p.ctx.h, x0c.ctypes.data_as(_lib.c_dp), xs.ctypes.data_as(_lib.c_dp), 4, 0.0, 0.0, 0,
                                  xo.ctypes.data_as(_lib.c_dp), C.byref(h), C.byref(nh), C.byref(ep))
        if with_test:
            assert rc == _lib.SCS_ERR_STATE
            assert "scs_iterate_ex" in _lib.lib.scs_last_error(p.ctx.h).decode()
        else:
            assert rc == _lib.SCS_OK and ep.value == 4
