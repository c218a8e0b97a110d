"""GPU: the fallbacks that replace a failure when a co-resident or dependency-waiting launch cannot
complete (r06).  Each is driven on purpose and must give the bits of the mode it falls back to, with
a clean iterate!, and be counted (scs_fallback_counts):

  * the cooperative one-launch LU panel (lu.hip): SCS_LU_COOP_SPIN=0 makes every workgroup give up at
    once, as one that never became resident would (info = -1, the abort word); the factorization is
    redone with the column-step panels -- bitwise SCS_LU_PANEL=1 -- for Julia's `A \\ b`
    (scs_lu_eval), ProxNSCORE's reference-solver LU (prox-N-SCORE.jl:70) and the GGN sample-space
    system (prox-GGN-SCORE.jl:124-127);
  * the opt-in cooperative one-launch QR panel (qr.hip, SCS_QR_COOP=1): SCS_QR_COOP_SPIN=0 likewise; the
    solve is redone from the saved system with the per-column launches -- bitwise the default;
  * the ~30 s dependency waits that are never expected (a block waits only on blocks dispatched before
    it): SCS_FAULT_LATE reports them as timed out at the host check, and the one-launch Cholesky
    solves redo by per-block launches (bitwise SCS_SOLVE_PERSIST=0), the QR's backward solve likewise,
    the dependency-driven chain (SCS_CHOL_DAG=1) redoes the factor with one launch per operation
    (bitwise the default), the pipelined factor (SCS_CHOL_PIPE) redoes the step unpipelined (bitwise
    the default)."""
import numpy as np
import pytest

import scsopt
from scsopt import losses

pytestmark = pytest.mark.gpu


@pytest.fixture
def clean_env(monkeypatch):
    import os
    for k in list(os.environ):
        if k.startswith("SCS_"):
            monkeypatch.delenv(k)
    return monkeypatch


def _bits(v):
    return np.asarray(v, dtype=np.float64).view(np.uint64)


@pytest.mark.parametrize("n", [1000, 4100])
def test_lu_coop_timeout_redone_by_column_steps(n, clean_env):
    mp = clean_env
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    mp.setenv("SCS_LU_PANEL", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    mp.delenv("SCS_LU_PANEL")
    ctx = scsopt._lib.Context(0)
    mp.setenv("SCS_LU_COOP_SPIN", "0")
    x0, ipiv0, info0 = scsopt.lu_solve(A, b, ctx=ctx)
    assert info0 == info1 == 0
    assert np.array_equal(ipiv0, ipiv1) and np.array_equal(_bits(x0), _bits(x1))
    fb = ctx.fallback_counts()
    assert fb["lu_coop_redo"] == 1, fb
    mp.delenv("SCS_LU_COOP_SPIN")
    x2, ipiv2, info2 = scsopt.lu_solve(A, b, ctx=ctx)   # the cooperative panel itself: no redo
    assert np.array_equal(_bits(x2), _bits(x1)) and ctx.fallback_counts()["lu_coop_redo"] == 1


def test_lu_coop_timeout_in_iterate(clean_env):
    """ProxNSCORE with the reference's solver (`\\` = LU, prox-N-SCORE.jl:70) and ProxGGNSCORE's
    sample-space branch (N + 1 <= m: the (N+1)² system by LU): every factorization's panel gives up,
    every one is redone -- the trajectory bitwise the column-step run's."""
    mp = clean_env
    rng = np.random.default_rng(3)
    runs = {}
    for name, (N, m) in {"nscore": (600, 300), "ggn_sample": (200, 700)}.items():
        A = rng.standard_normal((N, m)) / np.sqrt(m)
        x0 = rng.standard_normal(m) * 0.2
        if name == "nscore":
            y = np.sign(rng.standard_normal(N))
            mk = lambda: scsopt.Problem(A, y, x0, losses.logistic_margin(1.0 / N), 2e-3)  # noqa: E731
            M = scsopt.ProxNSCORE
        else:
            y = (rng.random(N) < 0.5).astype(np.float64)
            mk = lambda: scsopt.Problem(A, y, x0, losses.logistic_ce(1.0 / N), 2e-3,  # noqa: E731
                                        out_fn=losses.sigmoid_ce(1.0 / N))
            M = scsopt.ProxGGNSCORE
        hm = scsopt.PHuberSmootherL1L2(1.0)
        out = {}
        for arm, env in (("steps", {"SCS_LU_PANEL": "1"}), ("giveup", {"SCS_LU_COOP_SPIN": "0"})):
            for k, v in env.items():
                mp.setenv(k, v)
            p = mk()
            if name == "nscore":
                p.set_solver("reference")
            sol = scsopt.iterate(M(), p, "l1", hm, max_epoch=4, verbose=0)
            out[arm] = (sol, p.ctx.fallback_counts())
            for k in env:
                mp.delenv(k)
        (a, fa), (b, fb) = out["steps"], out["giveup"]
        assert a.epochs == b.epochs == 4
        assert np.array_equal(_bits(a.x), _bits(b.x)) and np.array_equal(_bits(a.obj), _bits(b.obj))
        assert fa["lu_coop_redo"] == 0 and fb["lu_coop_redo"] == 4, (name, fa, fb)
        runs[name] = fb
    assert runs


def _ggn_problem(N, m, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((N, m)) / np.sqrt(m)
    y = (rng.random(N) < 1.0 / (1.0 + np.exp(-A @ rng.standard_normal(m)))).astype(np.float64)
    x0 = rng.standard_normal(m) * 0.2
    return lambda: scsopt.Problem(A, y, x0, losses.logistic_ce(1.0 / N), 2e-3, out_fn=losses.sigmoid_ce(1.0 / N))


def _run(mp, mk, env, solver=None, epochs=4):
    for k, v in env.items():
        mp.setenv(k, v)
    try:
        p = mk()
        if solver:
            p.set_solver(solver)
        sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=epochs,
                             verbose=0)
        return sol, p.ctx.fallback_counts()
    finally:
        for k in env:
            mp.delenv(k)


@pytest.mark.parametrize("m", [640, 2304])
def test_persistent_solve_timeout_redone_per_block(m, clean_env):
    mk = _ggn_problem(3000, m, m)
    a, fa = _run(clean_env, mk, {"SCS_SOLVE_PERSIST": "0"})
    b, fb = _run(clean_env, mk, {"SCS_FAULT_LATE": "1"})
    assert np.array_equal(_bits(a.x), _bits(b.x)) and np.array_equal(_bits(a.obj), _bits(b.obj))
    assert fa["solve_blocks"] == 0 and fb["solve_blocks"] == 4, (fa, fb)


@pytest.mark.parametrize("m", [640, 2304])
def test_qr_backward_solve_timeout_redone_per_block(m, clean_env):
    """Reference-solver mode (qr(JQJ) \\ Je, prox-GGN-SCORE.jl:131): R complete, Qᵀb kept; the
    backward solve again by per-block launches -- bitwise SCS_SOLVE_PERSIST=0."""
    mk = _ggn_problem(3000, m, m + 1)
    a, fa = _run(clean_env, mk, {"SCS_SOLVE_PERSIST": "0"}, solver="reference")
    b, fb = _run(clean_env, mk, {"SCS_FAULT_LATE": "2"}, solver="reference")
    assert np.array_equal(_bits(a.x), _bits(b.x)) and np.array_equal(_bits(a.obj), _bits(b.obj))
    assert fb["qr_blocks"] == 4, fb


def test_chain_wait_timeout_refactored(clean_env):
    """SCS_CHOL_DAG=1 (dependency-driven chain, opt-in): a chain wait that gave up leaves the factor
    incomplete; the system is restored from Gc and factored with one launch per operation -- bitwise
    the default run (the DAG form is itself bit-identical to it)."""
    mk = _ggn_problem(3000, 2304, 7)
    a, _ = _run(clean_env, mk, {})
    b, fb = _run(clean_env, mk, {"SCS_CHOL_DAG": "1", "SCS_FAULT_LATE": "4"})
    assert np.array_equal(_bits(a.x), _bits(b.x)) and np.array_equal(_bits(a.obj), _bits(b.obj))
    assert fb["chain_redo"] == 4, fb


@pytest.mark.parametrize("mode", ["1", "2"])
def test_pipeline_strip_wait_timeout_redone_unpipelined(mode, clean_env):
    """SCS_CHOL_PIPE (the factor hidden under the Gram, opt-in): a strip wait that gave up means a
    strip was factored incomplete; the step's Gram, factor and solve are redone unpipelined --
    bitwise the default run."""
    mk = _ggn_problem(5000, 3200, 11)
    a, _ = _run(clean_env, mk, {})
    b, fb = _run(clean_env, mk, {"SCS_CHOL_PIPE": mode, "SCS_FAULT_LATE": "8"})
    assert np.array_equal(_bits(a.x), _bits(b.x)) and np.array_equal(_bits(a.obj), _bits(b.obj))
    assert fb["pipe_redo"] == 4, fb


@pytest.mark.parametrize("m", [640, 2304])
def test_qr_coop_timeout_redone_by_column_steps(m, clean_env):
    """Reference-solver mode (qr(JQJ) \\ Je, prox-GGN-SCORE.jl:131) with the opt-in cooperative QR panel
    (SCS_QR_COOP=1): every panel gives up at once (SCS_QR_COOP_SPIN=0); each solve is redone from the
    saved system by the per-column launches -- the trajectory bitwise the default's, one redo per step."""
    mk = _ggn_problem(3000, m, m + 3)
    a, fa = _run(clean_env, mk, {}, solver="reference")
    b, fb = _run(clean_env, mk, {"SCS_QR_COOP": "1", "SCS_QR_COOP_SPIN": "0"}, solver="reference")
    c, fc = _run(clean_env, mk, {"SCS_QR_COOP": "1"}, solver="reference")
    assert np.array_equal(_bits(a.x), _bits(b.x)) and np.array_equal(_bits(a.obj), _bits(b.obj))
    assert fa["qr_coop_redo"] == 0 and fb["qr_coop_redo"] == 4 and fc["qr_coop_redo"] == 0, (fa, fb, fc)
    assert fc["qr_coop_refused"] == 0, fc
    # the cooperative panels themselves: the same trajectory to rounding (other summation order)
    np.testing.assert_allclose(c.obj, a.obj, rtol=1e-10, atol=0)
