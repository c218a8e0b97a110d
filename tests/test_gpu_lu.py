"""GPU parity of the hand-written blocked LU with partial pivoting (csrc/lu.hip).

The reference's `\\` on a dense Matrix is LAPACK getrf + getrs (prox-N-SCORE.jl:70; the NSCORE
/ GGN non-SPD fallback) and its sample-space `qr(...) \\ b` (prox-GGN-SCORE.jl:126) solves the
same non-symmetric system.  Pins:
  * pivot rows equal to LAPACK dgetrf's (scipy.linalg.lapack.dgetrf, 0-based) on matrices
    without near-ties, ties broken towards the first row as getf2's idamax does;
  * info = the first exactly-zero pivot (1-based), as dgetrf reports it;
  * the solution against LAPACK's getrs to 1e-14·cond(A) (max norm, relative to max |x|), and a
    backward error ||Ax - b|| / (||A|| ||x||) <= 1e-13 at every size.
"""
import time

import numpy as np
import pytest
import scipy.linalg as sla
from scipy.linalg import lapack

import scsopt
from scsopt import losses

pytestmark = pytest.mark.gpu


def _bwd(A, x, b):
    return float(np.linalg.norm(A @ x - b, np.inf) / (np.linalg.norm(A, np.inf) * np.linalg.norm(x, np.inf)))


@pytest.mark.parametrize("n", [1, 2, 5, 127, 128, 129, 300, 1000, 2176])
def test_lu_matches_lapack_getrf(n):
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    x, ipiv, info = scsopt.lu_solve(A, b)
    lu, piv, linfo = lapack.dgetrf(A)
    assert info == linfo == 0
    assert np.array_equal(ipiv, piv), np.nonzero(ipiv != piv)[0][:10]
    xr = sla.lu_solve((lu, piv), b)
    # forward error: both are backward stable, so they agree to ~ cond(A)·eps
    kappa = float(np.linalg.cond(A, np.inf)) if n > 1 else 1.0
    assert np.max(np.abs(x - xr)) <= 1e-14 * kappa * float(np.abs(xr).max())
    assert _bwd(A, x, b) <= 1e-13


def test_lu_pivoting_cases():
    """Zero diagonal (a swap is forced), equal magnitudes (first row wins), and a permutation."""
    cases = [np.array([[0.0, 1.0], [1.0, 0.0]]),
             np.array([[1.0, 2.0], [-1.0, 3.0]]),
             np.array([[2.0, 1.0, 1.0], [-2.0, 3.0, 1.0], [2.0, 0.0, 5.0]]),
             np.eye(200)[np.random.default_rng(1).permutation(200)] * 3.0]
    for A in cases:
        b = np.arange(1.0, A.shape[0] + 1.0)
        x, ipiv, info = scsopt.lu_solve(A, b)
        _, piv, linfo = lapack.dgetrf(A)
        assert info == linfo == 0
        assert np.array_equal(ipiv, piv)
        np.testing.assert_allclose(A @ x, b, rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize("n,zcol", [(6, 3), (300, 0), (300, 299), (700, 150)])
def test_lu_singular_info(n, zcol):
    """A zero column: dgetrf's info is the 1-based index of the first zero pivot."""
    rng = np.random.default_rng(n + zcol)
    A = rng.standard_normal((n, n))
    A[:, zcol] = 0.0
    _, ipiv, info = scsopt.lu_solve(A, np.ones(n))
    _, piv, linfo = lapack.dgetrf(A)
    assert info == linfo == zcol + 1
    assert np.array_equal(ipiv[:zcol], piv[:zcol])


@pytest.mark.parametrize("n", [4096, 8192])
def test_lu_large_backward_error(n, capsys):
    """Full-size factorization (64 blocks at n = 8192, the C2 m): backward error and time."""
    rng = np.random.default_rng(7)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    ctx = scsopt._lib.Context(0)
    scsopt.lu_solve(A[:256, :256], b[:256], ctx=ctx)   # warm-up (code objects, aux buffers)
    t0 = time.perf_counter()
    x, ipiv, info = scsopt.lu_solve(A, b, ctx=ctx)
    dt = time.perf_counter() - t0
    assert info == 0
    assert _bwd(A, x, b) <= 1e-13
    with capsys.disabled():
        print(f"\n[lu] n={n}: factor+solve+transfers {dt * 1e3:.1f} ms, backward error {_bwd(A, x, b):.2e}")


def test_solve_eval_lu_vs_cholesky():
    """The step's m x m system, (Aᵀ diag(w) A + diag(d)) x = rhs: Cholesky path vs forced LU vs host."""
    N, m = 1500, 1000
    p = scsopt.Problem.synthetic(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1.0, kind=3, seed=3)
    A, _ = p.get_data()
    rng = np.random.default_rng(2)
    w = rng.random(N) + 0.1
    d = rng.random(m) + 0.5
    rhs = rng.standard_normal(m)
    xc, used_c = p.solve_eval(w, d, rhs, mode=0)
    xl, used_l = p.solve_eval(w, d, rhs, mode=1)
    assert not used_c and used_l
    G = A.T @ (w[:, None] * A) + np.diag(d)
    xr = np.linalg.solve(G, rhs)
    np.testing.assert_allclose(xc, xr, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(xl, xr, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("mode", ["2", "3"])
@pytest.mark.parametrize("n", [300, 2176, 8320])
def test_lu_panel_variants_bit_identical(n, mode, monkeypatch):
    """Every panel form does the r02 column step's arithmetic (SCS_LU_PANEL=1): the same pivots and the
    same solution bit for bit.  2: the column step with its rows prefetched beside the candidate reads
    (lu_panel_step2_kernel); 3 (default): the cooperative one-launch panel, rows in registers, the
    candidates exchanged as tagged granules (lu_panel_coop_kernel).  n = 8320: 65 workgroups in the
    first panel (two 32-row passes per workgroup for mode 2)."""
    rng = np.random.default_rng(n + 7)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    monkeypatch.setenv("SCS_LU_PANEL", mode)
    x2, ipiv2, info2 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_PANEL", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info2 == 0
    assert np.array_equal(ipiv1, ipiv2)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))


def test_lu_coop_panel_largest_grid(monkeypatch):
    """n = 16384: the cooperative panel at its largest grid (128 workgroups, one per CU) -- bitwise the
    column steps, backward error <= 1e-13."""
    n = 16384
    rng = np.random.default_rng(5)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    x3, ipiv3, info3 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_PANEL", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info3 == 0
    assert np.array_equal(ipiv1, ipiv3)
    assert np.array_equal(x1.view(np.uint64), x3.view(np.uint64))
    assert _bwd(A, x3, b) <= 1e-13


@pytest.mark.parametrize("n", [300, 2176])
def test_lu_doubling_inverse_matches_elimination(n, monkeypatch):
    """The diagonal block's L11⁻¹ / U11⁻¹ by 16 x 16 inverses + MFMA doubling (lu_tri_inv_kernel, r05)
    against the r02 row-by-row elimination (SCS_LU_INV=1): different rounding of the same inverses, so
    the same pivots (no near-ties here) and solutions within a few ulps of cond(A)."""
    rng = np.random.default_rng(n + 11)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    x2, ipiv2, info2 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_INV", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info2 == 0
    assert np.array_equal(ipiv1, ipiv2)
    kappa = float(np.linalg.cond(A, np.inf))
    assert np.max(np.abs(x1 - x2)) <= 1e-14 * kappa * float(np.abs(x1).max())
    assert _bwd(A, x2, b) <= 1e-13


def test_lu_coop_publish_forms_bit_identical(monkeypatch):
    """The cooperative panel's two publication forms (rows stored by the eight lanes that hold them, the
    default, vs by a whole wave through LDS, SCS_LU_COOP_WIDE=1): the same factor bit for bit."""
    n = 2176
    rng = np.random.default_rng(n + 13)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    x2, ipiv2, info2 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_COOP_WIDE", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info2 == 0
    assert np.array_equal(ipiv1, ipiv2)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))


@pytest.mark.parametrize("n", [300, 2176, 8320])
def test_lu_coop_512_threads_bit_identical(n, monkeypatch):
    """The cooperative panel with 512-thread workgroups (256 rows each, SCS_LU_COOP_NT=512; the last
    workgroup holds 128 rows where h is an odd multiple of 128) against the r02 column steps: bit for bit."""
    rng = np.random.default_rng(n + 17)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    monkeypatch.setenv("SCS_LU_COOP_NT", "512")
    x2, ipiv2, info2 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_PANEL", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info2 == 0
    assert np.array_equal(ipiv1, ipiv2)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))


@pytest.mark.parametrize("nt", ["256", "512"])
@pytest.mark.parametrize("n", [5, 300, 2176, 8320])
def test_lu_coop_block_deferred_bit_identical(n, nt, monkeypatch):
    """The block-deferred cooperative panel (default, SCS_LU_COOP_BLK; lu_panel_blk_kernel): each column step
    updates its 16-column block only, the columns right of it take the block's 16 updates at its end in
    step order -- the column steps' operations per element, so the same pivots and bits as SCS_LU_PANEL=1,
    with 256- and 512-thread workgroups."""
    rng = np.random.default_rng(n + 29)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    monkeypatch.setenv("SCS_LU_COOP_NT", nt)
    x2, ipiv2, info2 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_PANEL", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info2 == 0
    assert np.array_equal(ipiv1, ipiv2)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))


@pytest.mark.parametrize("n", [300, 8320])
def test_lu_coop_record_first_panel_bit_identical(n, monkeypatch):
    """The r05/r06 cooperative panel without the block deferral (SCS_LU_COOP_BLK=0, the record-first
    lu_panel_coop_kernel) stays bitwise the column steps'."""
    rng = np.random.default_rng(n + 37)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    monkeypatch.setenv("SCS_LU_COOP_BLK", "0")
    x2, ipiv2, info2 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_PANEL", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info1 == info2 == 0
    assert np.array_equal(ipiv1, ipiv2)
    assert np.array_equal(x1.view(np.uint64), x2.view(np.uint64))


@pytest.mark.parametrize("n,zcol", [(300, 0), (300, 15), (300, 16), (700, 150), (700, 255)])
def test_lu_coop_block_deferred_zero_pivot(n, zcol, monkeypatch):
    """A zero column at a block's first / last step and inside one: info and the pivots (every column,
    the zero one kept in place as getf2 does) equal the column steps'."""
    rng = np.random.default_rng(n + zcol + 31)
    A = rng.standard_normal((n, n))
    A[:, zcol] = 0.0
    _, ipiv2, info2 = scsopt.lu_solve(A, np.ones(n))
    monkeypatch.setenv("SCS_LU_PANEL", "1")
    _, ipiv1, info1 = scsopt.lu_solve(A, np.ones(n))
    _, piv, linfo = lapack.dgetrf(A)
    assert info1 == info2 == linfo == zcol + 1
    assert np.array_equal(ipiv1, ipiv2) and np.array_equal(ipiv2[:zcol], piv[:zcol])


@pytest.mark.parametrize("n", [300, 1000, 2176, 8320])
def test_lu_outer_blocked_update(n, monkeypatch):
    """Outer blocks of four panels (SCS_LU_OB=4): inside a block each panel's moves reach the block's
    other columns (its earlier L columns too) and its update only the block's later columns; the trailing
    matrix takes the block's moves, a block forward substitution for its U rows and ONE K = 512 update;
    lu_solve applies a block's moves before its first forward step.  Pivots equal LAPACK dgetrf's (and
    the per-panel factor's), the solution within 1e-14·cond of LAPACK's, backward error <= 1e-13.
    n = 300: one partial outer block; 2176: 17 panels (the last outer block a single panel)."""
    rng = np.random.default_rng(n + 23)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    monkeypatch.setenv("SCS_LU_OB", "4")
    x4, ipiv4, info4 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_OB", "1")
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    _, piv, linfo = lapack.dgetrf(A)
    assert info4 == info1 == linfo == 0
    assert np.array_equal(ipiv4, piv) and np.array_equal(ipiv1, piv)
    kappa = float(np.linalg.cond(A, np.inf))
    xr = sla.lu_solve(lapack.dgetrf(A)[:2], b)
    assert np.max(np.abs(x4 - xr)) <= 1e-14 * kappa * float(np.abs(xr).max())
    assert _bwd(A, x4, b) <= 1e-13


def test_lu_smaller_system_after_larger_on_one_context():
    """The LU's work buffers and tile lists are sized for the largest system a context has seen; a
    smaller system afterwards (outer blocks of four panels, rectangle tile lists at the capacity's
    offsets) still gets LAPACK's pivots and a backward-stable solution."""
    ctx = scsopt._lib.Context(0)
    rng = np.random.default_rng(29)
    for n in (2176, 1000, 300):
        A = rng.standard_normal((n, n))
        b = rng.standard_normal(n)
        x, ipiv, info = scsopt.lu_solve(A, b, ctx=ctx)
        _, piv, linfo = lapack.dgetrf(A)
        assert info == linfo == 0
        assert np.array_equal(ipiv, piv)
        assert _bwd(A, x, b) <= 1e-13


@pytest.mark.parametrize("skip", ["0", "0x30", "auto"])
@pytest.mark.parametrize("n", [1100, 2176, 8320])
def test_lu_lookahead_bit_identical(n, skip, monkeypatch):
    """The lookahead outer step (SCS_LU_LA, the default since r06) against the one-stream step
    (SCS_LU_LA=0): the columns beyond the next outer block updated on a bulk stream beside the next
    block's panels, as full-grid (skip 0) or CU-bounded launches (a fixed skip set, or the default: full
    grid above 8192 trailing columns, then sized to the next panel) -- the same tiles, kernels and K
    order as the one-stream step, so the same pivots and solution bit for bit.  n = 1100: 9 blocks, one
    bulk update of a single block column; 8320: 65 blocks (15 bulk updates, both default forms)."""
    rng = np.random.default_rng(n + 19)
    A = rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    monkeypatch.setenv("SCS_LU_LA", "0")
    x0, ipiv0, info0 = scsopt.lu_solve(A, b)
    monkeypatch.setenv("SCS_LU_LA", "1")
    if skip != "auto":
        monkeypatch.setenv("SCS_LU_LA_SKIP", skip)
    x1, ipiv1, info1 = scsopt.lu_solve(A, b)
    assert info0 == info1 == 0
    assert np.array_equal(ipiv0, ipiv1)
    assert np.array_equal(x0.view(np.uint64), x1.view(np.uint64))
    assert _bwd(A, x1, b) <= 1e-13
