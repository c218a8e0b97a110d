"""GPU parity of the minibatch path (iterate.jl:124-146,204-255; utils.jl:14-25): the collected
DataLoader batches gathered on the device (scs_set_batches / scs_select_batch) against the
oracle's optim_loop! over the same row lists.

The shuffled loader's permutation is passed explicitly (Julia's global RNG stream is not
reproducible outside Julia), so these trajectories are parity-unpinned by the reference below
its own tests (it has no minibatch test); they pin the device path to the restatement.
Tolerances as tests/test_gpu_parity.py: objective history rtol 1e-8, same history length and
epochs; device loop vs host loop bit-identical.
"""
import numpy as np
import pytest

import scsopt
import scsopt_oracle as O
from scsopt import losses

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


def _pair(method, N, m, lam=2e-3, seed=99):
    x0 = np.random.default_rng(1234).standard_normal(m) * 0.5
    if method == "ggn":
        f, out, kind, of = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N), 1, \
            O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce")
    elif method == "nscore":
        f, out, kind, of = losses.logistic_margin(1.0 / N), None, 2, O.Loss("logistic_margin", 1.0 / N)
    else:
        f, out, kind, of = losses.least_squares(1.0 / N), None, 3, O.Loss("least_squares", 1.0 / N)
    p = scsopt.Problem.synthetic(N, m, x0, f, lam, kind=kind, seed=seed, out_fn=out)
    A, y = p.get_data()
    return p, O.Problem(A, y, x0, of, lam)


METHODS = {"ggn": (scsopt.ProxGGNSCORE, O.ProxGGNSCORE), "nscore": (scsopt.ProxNSCORE, O.ProxNSCORE),
           "lqn": (scsopt.ProxLQNSCORE, O.ProxLQNSCORE)}


@pytest.mark.parametrize("method,batch_size", [("ggn", 384), ("ggn", 100), ("nscore", 384), ("lqn", 384),
                                               ("lqn", 2000)])
def test_minibatch_trajectory(method, batch_size):
    """Shuffled batches with a partial last one (N = 2000); GGN at batch 100 < m takes the
    sample-space branch on every batch; batch_size = N is one shuffled full-size batch."""
    N, m, max_epoch = 2000, 192, 6
    p, om = _pair(method, N, m)
    perm = np.random.default_rng(3).permutation(N)
    kw = dict(batch_size=batch_size, shuffle_batch=True, batch_perm=perm, max_epoch=max_epoch, verbose=0)
    a = scsopt.iterate(METHODS[method][0](), p, "l1", scsopt.PHuberSmootherL1L2(1.0), device_loop=True, **kw)
    b = scsopt.iterate(METHODS[method][0](), p, "l1", scsopt.PHuberSmootherL1L2(1.0), device_loop=False, **kw)
    batches = O.loader_batches(N, batch_size, shuffle_batch=True, perm=perm)
    assert len(batches) == -(-N // batch_size)
    o = O.iterate(METHODS[method][1](), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=max_epoch, batches=batches)
    for s in (a, b):
        assert s.epochs == o.epochs and len(s.obj) == len(o.obj)
        np.testing.assert_allclose(s.obj, o.obj, rtol=1e-8, atol=0)
        np.testing.assert_allclose(s.x, o.x, rtol=1e-6, atol=1e-9)
    assert a.obj == b.obj and a.pri_res_norm == b.pri_res_norm and np.array_equal(bits(a.x), bits(b.x))


def test_unshuffled_batches_and_local_max_iter():
    """shuffle_batch=false keeps row order; local_max_iter = 2 forces max_epoch = 1 and runs only
    the first two batches (iterate.jl:66,124-128)."""
    N, m = 1000, 128
    p, om = _pair("lqn", N, m)
    for kw, okw in (({"max_epoch": 4}, {"max_epoch": 4}), ({"local_max_iter": 2.7}, {"max_epoch": 1})):
        s = scsopt.iterate(scsopt.ProxLQNSCORE(m=5), p, "l1", scsopt.PHuberSmootherL1L2(1.0), batch_size=256,
                           shuffle_batch=False, verbose=0, **kw)
        batches = O.loader_batches(N, 256, shuffle_batch=False, local_max_iter=kw.get("local_max_iter"))
        o = O.iterate(O.ProxLQNSCORE(m=5), om, "l1", O.PHuberSmootherL1L2(1.0), batches=batches, **okw)
        assert s.epochs == o.epochs and len(s.obj) == len(o.obj)
        np.testing.assert_allclose(s.obj, o.obj, rtol=1e-8)
    assert len(O.loader_batches(N, 256, shuffle_batch=False, local_max_iter=2.7)) == 2


@pytest.mark.parametrize("method", ["nscore", "lqn"])
def test_slice_samples_first_row_only(method):
    """slice_samples=true: one-sample batches, and with max_iter = 1 only sample 1 ever steps
    (iterate.jl:127,136-138,146)."""
    N, m = 512, 64
    p, om = _pair(method, N, m, lam=1e-2)
    s = scsopt.iterate(METHODS[method][0](), p, "l1", scsopt.PHuberSmootherL1L2(1.0), slice_samples=True,
                       max_epoch=5, verbose=0)
    o = O.iterate(METHODS[method][1](), om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=5,
                  batches=O.loader_batches(N, slice_samples=True))
    assert s.epochs == o.epochs and len(s.obj) == len(o.obj)
    np.testing.assert_allclose(s.obj, o.obj, rtol=1e-8)


def test_select_batch_step_matches_oracle_step():
    """step! on one selected batch (scs_select_batch) == the oracle step on Matrix(As'), vec(ys');
    re-selecting another batch of the same size re-gathers; -1 returns to the full data."""
    N, m = 900, 96
    p, om = _pair("ggn", N, m)
    rows = [np.arange(0, 900, 3), np.arange(1, 900, 3), np.arange(5, 900, 7)]
    p.set_batches(rows)
    x = np.random.default_rng(8).standard_normal(m) * 0.2
    try:
        from scsopt.iterate import init_method, step
        p.configure("l1", scsopt.PHuberSmootherL1L2(1.0))
        init_method(scsopt.ProxGGNSCORE(), p)
        for bi, r in enumerate(rows):
            xn, pri = step(scsopt.ProxGGNSCORE(), p, "l1", None, x, x, 1, batch=bi)
            oxn, opri = O.step(O.ProxGGNSCORE(), O.batch_problem(om, r), "l1", O.PHuberSmootherL1L2(1.0), x, x,
                               None, 1)
            np.testing.assert_allclose(xn, oxn, rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(pri, opri, rtol=1e-9)
        xf, _ = step(scsopt.ProxGGNSCORE(), p, "l1", None, x, x, 1)
        oxf, _ = O.step(O.ProxGGNSCORE(), om, "l1", O.PHuberSmootherL1L2(1.0), x, x, None, 1)
        np.testing.assert_allclose(xf, oxf, rtol=1e-9, atol=1e-12)
    finally:
        p.set_batches(None)


def test_batch_errors():
    N, m = 64, 32
    p, _ = _pair("lqn", N, m)
    with pytest.raises(scsopt.ScsError, match="out of range"):
        p.set_batches([np.array([0, N])])
    with pytest.raises(scsopt.ScsError, match="empty"):
        p.set_batches([np.array([0, 1]), np.array([], dtype=np.int64)])
    with pytest.raises(scsopt.ScsError):
        p.select_batch(0)                      # nothing registered
    q = scsopt.Problem(np.eye(4) * 2.0, np.ones(4), np.zeros(4), losses.quadratic(), 1e-3)
    q.set_batches([np.array([0, 1])])
    with pytest.raises(scsopt.ScsError, match="quadratic"):
        q.select_batch(0)


@pytest.mark.parametrize("method", ["lqn", "ggn"])
def test_sparse_minibatches_gathered_dense(method):
    """Batches of a sparse A are the reference's Matrix(As') (iterate.jl:207): the CSR rows of each
    batch are gathered into a dense view on the device; trajectory vs the oracle on the dense A."""
    import scipy.sparse as sp
    N, m = 1500, 96
    rng = np.random.default_rng(17)
    A = sp.random(N, m, density=0.08, random_state=3, format="csr") * 3.0
    x0 = rng.standard_normal(m) * 0.3
    if method == "lqn":
        y = rng.standard_normal(N)
        f, out, of = losses.least_squares(1.0 / N), None, O.Loss("least_squares", 1.0 / N)
        meth, ometh, reg = scsopt.ProxLQNSCORE(m=5), O.ProxLQNSCORE(m=5), "l1"
    else:
        y = (rng.random(N) < 0.5).astype(float)
        f, out = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N)
        of = O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce")
        meth, ometh, reg = scsopt.ProxGGNSCORE(), O.ProxGGNSCORE(), "l1"
    p = scsopt.Problem(A, y, x0, f, 1e-3, out_fn=out)
    om = O.Problem(A.toarray(), y, x0, of, 1e-3)
    perm = np.random.default_rng(4).permutation(N)
    s = scsopt.iterate(meth, p, reg, scsopt.PHuberSmootherL1L2(1.0), batch_size=400, batch_perm=perm, max_epoch=5,
                       verbose=0)
    o = O.iterate(ometh, om, reg, O.PHuberSmootherL1L2(1.0), max_epoch=5,
                  batches=O.loader_batches(N, 400, perm=perm))
    assert s.epochs == o.epochs and len(s.obj) == len(o.obj)
    np.testing.assert_allclose(s.obj, o.obj, rtol=1e-8)
    np.testing.assert_allclose(s.x, o.x, rtol=1e-6, atol=1e-9)
