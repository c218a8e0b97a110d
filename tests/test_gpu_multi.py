"""GPU: the one-process multi-device context (scs_create_multi, SURVEY.md §8b/§5: "single process
driving 8 devices").  On a one-GPU box the group has one device; it must give the bits of a plain
scs_create context for every method, with and without the RCCL exchange forced at that one rank
(the same packed Gram -> ncclAllReduce -> unpack path an 8-device group takes), through the group
entry points (host threads, row plan, device-0 outputs).  The 2..8-device row split is checked
against the per-rank split on the CPU (tests/test_shard_plan.py); groups of 2-4 sub-contexts run on
the one GPU with the host-staged exchange (SCS_MULTI_HOST_EXCHANGE)."""
import ctypes as C

import numpy as np
import pytest

import scsopt
from scsopt import _lib, losses

pytestmark = pytest.mark.gpu

N, M = 3001, 192


def _run(method, devices=None, force=False, batches=False, exchange="rccl"):
    x0 = np.random.default_rng(1234).standard_normal(M)
    if method == "ggn":
        f, out, kind, meth = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N), 1, scsopt.ProxGGNSCORE()
    elif method == "nscore":
        f, out, kind, meth = losses.logistic_margin(1.0 / N), None, 2, scsopt.ProxNSCORE()
    else:
        f, out, kind, meth = losses.least_squares(1.0 / N), None, 3, scsopt.ProxLQNSCORE(m=5)
    p = scsopt.Problem.synthetic(N, M, x0, f, 2e-3, kind=kind, seed=11, out_fn=out, devices=devices,
                                 device_exchange=exchange)
    if force:
        p.ctx.check(_lib.lib.scs_set_comm_force(p.ctx.h, 1))
    kw = dict(batch_size=1000, batch_perm=np.random.default_rng(3).permutation(N)) if batches else {}
    sol = scsopt.iterate(meth, p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=5, verbose=0, **kw)
    fx = p.fx(sol.x)
    g = p.gradx(sol.x)
    A, y = p.get_data(1000, 1001)   # rows read back across the group's devices
    p.ctx.close()
    return sol, fx, g, A, y


@pytest.mark.parametrize("method", ["ggn", "nscore", "lqn"])
@pytest.mark.parametrize("force,batches", [(False, False), (True, False), (True, True)])
def test_multi_one_device_bit_identical(method, force, batches):
    ref = _run(method, batches=batches)
    got = _run(method, devices=[0], force=force, batches=batches)
    assert got[0].epochs == ref[0].epochs
    assert np.array_equal(np.asarray(got[0].obj), np.asarray(ref[0].obj))
    assert np.array_equal(got[0].x, ref[0].x)
    assert got[1] == ref[1] and np.array_equal(got[2], ref[2])
    assert np.array_equal(got[3], ref[3]) and np.array_equal(got[4], ref[4])


@pytest.mark.parametrize("method", ["ggn", "nscore", "lqn"])
def test_multi_host_exchange_one_device_bit_identical(method):
    """SCS_MULTI_HOST_EXCHANGE at one device with the exchange forced: the host-staged sum of one slot
    is the identity, so the bits are scs_create's."""
    ref = _run(method)
    got = _run(method, devices=[0], force=True, exchange="host")
    assert np.array_equal(np.asarray(got[0].obj), np.asarray(ref[0].obj)) and np.array_equal(got[0].x, ref[0].x)
    assert got[1] == ref[1] and np.array_equal(got[2], ref[2])


@pytest.mark.parametrize("method", ["ggn", "nscore", "lqn"])
@pytest.mark.parametrize("ndev,batches", [(2, False), (3, False), (4, True)])
def test_multi_host_exchange_several_subcontexts(method, ndev, batches):
    """A group of 2-4 sub-contexts on the box's one GPU (SCS_MULTI_HOST_EXCHANGE: devices may repeat):
    the group's persistent worker threads, its row split (the first N % ndev sub-contexts one row more),
    per-device data generation, the exchange (every sub-context's payload summed in device order) and
    device-0 outputs -- the code an 8-GPU group runs, less RCCL.  Against the one-device run: the same
    epochs, obj / x / f / ∇f within 1e-10 (the row split changes the order of the sums), the data rows
    read back across the sub-contexts bitwise."""
    ref = _run(method, batches=batches)
    got = _run(method, devices=[0] * ndev, exchange="host", batches=batches)
    assert got[0].epochs == ref[0].epochs and len(got[0].obj) == len(ref[0].obj)
    np.testing.assert_allclose(got[0].obj, ref[0].obj, rtol=1e-10, atol=0)
    np.testing.assert_allclose(got[0].x, ref[0].x, rtol=1e-8, atol=1e-10)
    assert got[1] == pytest.approx(ref[1], rel=1e-10)
    np.testing.assert_allclose(got[2], ref[2], rtol=1e-8, atol=1e-12)
    assert np.array_equal(got[3], ref[3]) and np.array_equal(got[4], ref[4])
    again = _run(method, devices=[0] * ndev, exchange="host", batches=batches)   # bitwise run to run
    assert np.array_equal(np.asarray(again[0].obj), np.asarray(got[0].obj)) and np.array_equal(again[0].x, got[0].x)


def test_multi_host_exchange_fault_aborts(monkeypatch):
    """The abort path of a group (group_run): one sub-context's exchange fails (SCS_FAULT_EXCHANGE_RANK)
    while the other waits in it; after the grace period the failing worker releases the waiter, the
    call returns an error instead of hanging, and the group refuses further calls (SCS_ERR_COMM)."""
    import time
    x0 = np.random.default_rng(1234).standard_normal(M)
    p = scsopt.Problem.synthetic(N, M, x0, losses.least_squares(1.0 / N), 2e-3, kind=3, seed=11, devices=[0, 0],
                                 device_exchange="host")
    monkeypatch.setenv("SCS_FAULT_EXCHANGE_RANK", "1")
    t0 = time.time()
    with pytest.raises(_lib.ScsError):
        scsopt.iterate(scsopt.ProxLQNSCORE(m=5), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=3, verbose=0)
    assert time.time() - t0 < 60
    monkeypatch.delenv("SCS_FAULT_EXCHANGE_RANK")
    with pytest.raises(_lib.ScsError) as ei:   # the group is broken: destroy it
        p.fx(x0)
    assert ei.value.code == _lib.SCS_ERR_COMM
    p.ctx.close()


def test_multi_context_contract():
    ctx = _lib.Context(devices=[0])
    n = C.c_int()
    ctx.check(_lib.lib.scs_group_size(ctx.h, C.byref(n)))
    assert n.value == 1
    # the kernel-level entry points take a single-device context
    out = np.zeros(4)
    rc = _lib.lib.scs_gemv_n_eval(ctx.h, out.ctypes.data_as(_lib.c_dp), out.ctypes.data_as(_lib.c_dp))
    assert rc == _lib.SCS_ERR_ARG and b"single-device" in _lib.lib.scs_last_error(ctx.h)
    ctx.close()
    with pytest.raises(_lib.ScsError):   # one RCCL rank per GPU
        _lib.Context(devices=[0, 0])
    g = _lib.Context(devices=[0, 0], device_exchange="host")   # the host exchange takes a repeated GPU
    ctx.check(_lib.lib.scs_group_size(g.h, C.byref(n)))
    assert n.value == 2
    g.close()
