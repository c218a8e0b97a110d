"""GPU parity of the sparse-A path (BASELINE configs[4]: box-constrained least squares with
ProxLQNSCORE, the README's `sprandn(N, m, ρ)` problem class) against the oracle.

The device holds A as CSR (A·x) plus a CSC copy (Aᵀ·v); both products are per-row / per-column
gathers with a fixed summation order.  The oracle runs on the same matrix densified (sizes here
are small), so the comparison isolates the summation order:
  * A·x, Aᵀ·v: |err| <= 1e-13 · Σ|terms|;
  * LQN trajectories: objective history rtol 1e-8, same length/termination, x rtol 1e-6;
  * fp32-value arm: the device's fp32 values (read back widened) through the oracle -> the same
    fp64 bars; fp32 vs fp64 arm on the same problem -> objective within 1e-5 relative (the
    "tolerance study" row of SURVEY.md §8d C5).
"""
import numpy as np
import pytest

import scsopt
import scsopt_oracle as O
from scsopt import losses

pytestmark = pytest.mark.gpu


def _check_products(p, A):
    rng = np.random.default_rng(11)
    x = rng.standard_normal(A.shape[1])
    v = rng.standard_normal(A.shape[0])
    Ad = A.toarray() if hasattr(A, "toarray") else A
    z = p.gemv_n(x)
    np.testing.assert_allclose(z, Ad @ x, rtol=0, atol=1e-13 * float(np.max(np.abs(Ad) @ np.abs(x))) + 1e-300)
    t = p.gemv_t(v)
    np.testing.assert_allclose(t, Ad.T @ v, rtol=0, atol=1e-13 * float(np.max(np.abs(Ad).T @ np.abs(v))) + 1e-300)


@pytest.mark.parametrize("f32", [False, True])
def test_generated_pattern_and_products(f32):
    N, m, rho = 8192, 256, 0.05
    k = round(rho * m)
    p = scsopt.Problem.synthetic_sparse(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1e-4, density=rho,
                                        seed=7, f32=f32)
    assert p.nnz == N * k
    A, y = p.get_sparse()
    # every row holds k entries, every column k N / m (the layered-bijection construction)
    assert np.all(np.diff(A.indptr) == k)
    assert np.all(np.bincount(A.indices, minlength=m) == k * N // m)
    vals = A.data
    if f32:
        assert np.array_equal(vals, vals.astype(np.float32).astype(np.float64))
    # values N(0,1)/sqrt(k): loose moment check
    assert abs(np.mean(vals)) < 0.02 / np.sqrt(k) * 10
    assert abs(np.std(vals) * np.sqrt(k) - 1.0) < 0.02
    _check_products(p, A)
    # y = A x_true + 0.1 eps with x_true in [-1.5, 1.5]
    assert np.all(np.isfinite(y)) and np.std(y) > 0.1


def test_user_csr_input_and_edges():
    """Problem(A::SparseMatrixCSC, ...) from host CSR/CSC, with empty rows/columns and duplicates summed."""
    import scipy.sparse as sp
    rng = np.random.default_rng(3)
    N, m = 1000, 300
    A = sp.random(N, m, density=0.03, random_state=4, format="coo", data_rvs=rng.standard_normal)
    A = sp.coo_matrix((np.concatenate([A.data, [0.5, 0.25]]),
                       (np.concatenate([A.row, [3, 3]]), np.concatenate([A.col, [7, 7]]))), shape=(N, m))
    A = A.tocsr()
    A[10, :] = 0.0          # an empty row
    A[:, 20] = 0.0          # an empty column
    A.eliminate_zeros()
    y = rng.standard_normal(N)
    x0 = rng.standard_normal(m)
    ps = scsopt.Problem(A, y, x0, losses.least_squares(1.0 / N), 0.1)
    pd = scsopt.Problem(A.toarray(), y, x0, losses.least_squares(1.0 / N), 0.1)
    _check_products(ps, A)
    assert ps.fx(x0) == pytest.approx(pd.fx(x0), rel=1e-13)
    np.testing.assert_allclose(ps.gradx(x0), pd.gradx(x0), rtol=1e-12, atol=1e-15)
    om = O.Problem(A.toarray(), y, x0, O.Loss("least_squares", 1.0 / N), 0.1)
    assert ps.fx(x0) == pytest.approx(om.fx(x0), rel=1e-13)
    # all-zero matrix
    Z = sp.csr_matrix((N, m))
    pz = scsopt.Problem(Z, y, x0, losses.least_squares(1.0 / N), 0.1)
    np.testing.assert_array_equal(pz.gemv_n(x0), np.zeros(N))
    assert pz.fx(x0) == pytest.approx(0.5 * np.dot(y, y) / N, rel=1e-13)


def test_ragged_segments():
    """Segment shapes the flat fp64 product walks specially: a row far longer than one 64-slot
    window (dense row), runs of one-entry rows (many rows starting in one window), long runs of
    empty rows, a dense column (a long CSC segment), and a row whose end meets a window boundary."""
    import scipy.sparse as sp
    rng = np.random.default_rng(41)
    N, m = 5000, 20000
    rows, cols = [], []
    rows += [5] * m; cols += list(range(m))                                   # dense row: 5000 slots
    rows += list(range(100, 1300)); cols += list(rng.integers(0, m, 1200))     # one entry per row
    rows += list(range(N)); cols += [17000] * N                                # dense column
    for r in range(2000, 3000, 3):                                            # 256 entries = 64 slots
        rows += [r] * 256; cols += list(rng.choice(m, 256, replace=False))
    # rows 3000..4000 stay empty but for the dense column; the rest random
    C = sp.random(N, m, density=2e-3, random_state=42, format="coo")
    keep = (C.row < 3000) | (C.row >= 4000)
    rows += list(C.row[keep]); cols += list(C.col[keep])
    A = sp.coo_matrix((rng.standard_normal(len(rows)), (rows, cols)), shape=(N, m)).tocsr()
    A.sum_duplicates()
    p = scsopt.Problem(A, rng.standard_normal(N), np.zeros(m), losses.least_squares(1.0 / N), 0.1)
    _check_products(p, A)
    # deterministic: the same product twice is bit-identical
    x = rng.standard_normal(m)
    np.testing.assert_array_equal(p.gemv_n(x), p.gemv_n(x))


@pytest.mark.parametrize("N,m,rho", [(40000, 20000, 2e-4), (65536, 256, 0.05)])
def test_multiblock_products(N, m, rho):
    """Index ranges above one 16384-wide LDS block in either direction (several blocked partials,
    summed in fixed order): generated (power-of-two N) and user-provided unsorted CSR."""
    import scipy.sparse as sp
    if N & (N - 1) == 0:
        p = scsopt.Problem.synthetic_sparse(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1e-4, density=rho)
        A, _ = p.get_sparse()
    else:
        rng = np.random.default_rng(21)
        C = sp.random(N, m, density=rho, random_state=22, format="coo", data_rvs=rng.standard_normal)
        perm = rng.permutation(C.nnz)          # scrambled entry order (unsorted rows): the device sorts
        A = sp.coo_matrix((C.data[perm], (C.row[perm], C.col[perm])), shape=C.shape)
        p = scsopt.Problem(A, rng.standard_normal(N), np.zeros(m), losses.least_squares(1.0 / N), 0.1)
    _check_products(p, A)


@pytest.mark.parametrize("gram", ["auto", "0"])
@pytest.mark.parametrize("case", ["nscore_ls_f32", "ggn_logistic", "ggn_sample_space", "nscore_logistic"])
def test_gram_methods_on_sparse(case, gram, monkeypatch):
    """ProxNSCORE / ProxGGNSCORE on a sparse A (Jt*Q*Jt' of a SparseMatrixCSC): the Gram priced by nnz
    (sparse_gram_kernel, the default at these densities) or (SCS_SPARSE_GRAM=0) the dense MFMA tiles
    on a mirror built on the device from the CSR (duplicates summed); the products on the sparse
    copies; trajectories vs the oracle on the densified matrix at the trajectory bar."""
    import scipy.sparse as sp
    if gram != "auto":
        monkeypatch.setenv("SCS_SPARSE_GRAM", gram)
    rng = np.random.default_rng(41)
    if case == "nscore_ls_f32":
        N, m = 4096, 128
        x0 = rng.standard_normal(m) * 0.5
        p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), 1e-3, density=0.05, seed=5,
                                            f32=True)
        A, y = p.get_sparse()
        of = O.Loss("least_squares", 1.0 / N)
        meth, ometh = scsopt.ProxNSCORE(), O.ProxNSCORE()
    else:
        N, m = (96, 256) if case == "ggn_sample_space" else (3000, 160)
        C = sp.random(N, m, density=0.05, random_state=7, format="coo")
        rows = np.concatenate([C.row, C.row[:50]])             # duplicates (summed) + unsorted entries
        cols = np.concatenate([C.col, C.col[:50]])
        vals = np.concatenate([C.data, rng.standard_normal(50)]) * 2.0
        perm = rng.permutation(rows.size)
        A = sp.coo_matrix((vals[perm], (rows[perm], cols[perm])), shape=(N, m))
        y = (rng.random(N) < 0.5).astype(float)
        x0 = rng.standard_normal(m) * 0.3
        if case == "nscore_logistic":
            y = 2 * y - 1
            f, out, of = losses.logistic_margin(1.0 / N), None, O.Loss("logistic_margin", 1.0 / N)
            meth, ometh = scsopt.ProxNSCORE(), O.ProxNSCORE()
        else:
            f, out = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N)
            of = O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce")
            meth, ometh = scsopt.ProxGGNSCORE(), O.ProxGGNSCORE()
        p = scsopt.Problem(A, y, x0, f, 1e-3, out_fn=out)
    Ad = A.toarray() if hasattr(A, "toarray") else A
    om = O.Problem(Ad, y, x0, of, 1e-3)
    sol = scsopt.iterate(meth, p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=8, verbose=0)
    osol = O.iterate(ometh, om, "l1", O.PHuberSmootherL1L2(1.0), max_epoch=8)
    assert sol.epochs == osol.epochs and len(sol.obj) == len(osol.obj)
    np.testing.assert_allclose(sol.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.x, osol.x, rtol=1e-6, atol=1e-9)


def _c5_pair(N=8192, m=512, rho=0.02, f32=False, max_epoch=25, mem=20):
    x0 = np.random.default_rng(1234).standard_normal(m) * 0.5
    lam, mu = 1e-4, 0.6
    p = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), lam, density=rho, seed=2026,
                                        f32=f32, C_set=[-1.0, 1.0])
    A, y = p.get_sparse()
    om = O.Problem(A.toarray(), y, x0, O.Loss("least_squares", 1.0 / N), lam, C_set=[-1.0, 1.0])
    sol = scsopt.iterate(scsopt.ProxLQNSCORE(m=mem), p, "indbox", scsopt.PHuberSmootherIndBox(-1.0, 1.0, mu),
                         max_epoch=max_epoch, verbose=0)
    osol = O.iterate(O.ProxLQNSCORE(m=mem), om, "indbox", O.PHuberSmootherIndBox(-1.0, 1.0, mu),
                     max_epoch=max_epoch)
    return p, sol, osol


@pytest.mark.parametrize("f32", [False, True])
def test_c5_lqn_box_ls_trajectory(f32):
    """C5 in miniature: ProxLQNSCORE(mem = 20) + indbox + PHuberSmootherIndBox(μ = 0.6), λ = 1e-4."""
    p, sol, osol = _c5_pair(f32=f32)
    assert sol.epochs == osol.epochs
    assert len(sol.obj) == len(osol.obj)
    np.testing.assert_allclose(sol.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(sol.x, osol.x, rtol=1e-6, atol=1e-9)
    assert np.all(sol.x >= -1.0) and np.all(sol.x <= 1.0)
    assert sol.obj[-1] < sol.obj[0]


def test_c5_fp32_vs_fp64_arm():
    """The tolerance study: the same problem with fp32-stored values stays within 1e-5 (relative) in
    objective of the fp64 arm over the run."""
    _, s64, _ = _c5_pair(f32=False, max_epoch=20)
    _, s32, _ = _c5_pair(f32=True, max_epoch=20)
    n = min(len(s64.obj), len(s32.obj))
    np.testing.assert_allclose(s32.obj[:n], s64.obj[:n], rtol=1e-5)
    np.testing.assert_allclose(s32.x, s64.x, atol=1e-3)


@pytest.mark.parametrize("case,tall", [("ggn_logistic", "0"), ("nscore_logistic", "0"), ("ggn_logistic", "1")])
def test_streaming_sparse_gram(case, tall, monkeypatch):
    """§8f rank 3: a sparse A whose dense mirror is refused (SCS_SPARSE_MIRROR_MAX_GB=0) -- the Gram
    streams the CSR through a ring of two 1024-row dense slots (SCS_SPARSE_CHUNK_ROWS), accumulating
    N / 1024 chunk launches of the production kernel (scheduled K-split tail + combine included).
    Trajectory vs the oracle (rtol 1e-8) and vs the mirror path (rtol 1e-12)."""
    import scipy.sparse as sp
    monkeypatch.setenv("SCS_GRAM_TALL", tall)
    rng = np.random.default_rng(43)
    N, m = 3000 + 37, (256 if tall == "1" else 160)
    A = sp.random(N, m, density=0.04, random_state=9, format="csr", data_rvs=rng.standard_normal)
    y = (rng.random(N) < 0.5).astype(float)
    x0 = rng.standard_normal(m) * 0.3
    if case == "nscore_logistic":
        y = 2 * y - 1
        f, out, of = losses.logistic_margin(1.0 / N), None, O.Loss("logistic_margin", 1.0 / N)
        mk, omk = scsopt.ProxNSCORE, O.ProxNSCORE
    else:
        f, out = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N)
        of = O.Loss("logistic_ce", 1.0 / N, ggn="sigmoid_ce")
        mk, omk = scsopt.ProxGGNSCORE, O.ProxGGNSCORE
    runs = {}
    for mode, cap, sg in (("stream", "0", "0"), ("mirror", "1000", "0"), ("sparse", "0", "1")):
        monkeypatch.setenv("SCS_SPARSE_MIRROR_MAX_GB", cap)
        monkeypatch.setenv("SCS_SPARSE_CHUNK_ROWS", "1024")
        monkeypatch.setenv("SCS_SPARSE_GRAM", sg)
        p = scsopt.Problem(A, y, x0, f, 1e-3, out_fn=out)
        runs[mode] = scsopt.iterate(mk(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=6, verbose=0)
    osol = O.iterate(omk(), O.Problem(A.toarray(), y, x0, of, 1e-3), "l1", O.PHuberSmootherL1L2(1.0), max_epoch=6)
    st, mi = runs["stream"], runs["mirror"]
    assert st.epochs == osol.epochs == mi.epochs and len(st.obj) == len(osol.obj)
    np.testing.assert_allclose(st.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(st.x, osol.x, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(st.obj, mi.obj, rtol=1e-12, atol=0)
    spg = runs["sparse"]   # the Gram priced by nnz: other summation order, the same trajectory
    assert spg.epochs == osol.epochs and len(spg.obj) == len(osol.obj)
    np.testing.assert_allclose(spg.obj, osol.obj, rtol=1e-8, atol=0)
    np.testing.assert_allclose(spg.obj, mi.obj, rtol=1e-10, atol=0)



@pytest.mark.parametrize("f32", [False, True])
def test_sparse_gram_priced_by_nnz(f32, monkeypatch):
    """§8f rank 3 (VERDICT r02 Missing #1): G = Aᵀ diag(w) A of a sparse A in Σ_r nnz_r² work
    (sparse_gram_kernel) -- three 4096-column blocks of G (m = 9037, padded to 9088), rows whose
    block segments are longer than one wave (the overflow loop), empty rows and columns, user CSR
    with unsorted entries; vs the dense fp64 product entry by entry (|err| <= 1e-13·Σ|terms|),
    bitwise equal run to run (fixed row order per entry, no cross-wave atomics) and between the two
    kernel variants."""
    import scipy.sparse as sp
    monkeypatch.setenv("SCS_SPARSE_GRAM", "1")
    rng = np.random.default_rng(47)
    N, m = 2000, 9037
    A = sp.random(N, m, density=0.006, random_state=11, format="lil", data_rvs=rng.standard_normal)
    for r in range(4):                                       # long rows: ~450 entries per block
        cols = rng.choice(m, 1400, replace=False)
        A[r, cols] = rng.standard_normal(1400)
    A[10:14, :] = 0.0                                        # empty rows
    A[:, 4096:4100] = 0.0                                    # empty columns
    A = A.tocoo()
    perm = rng.permutation(A.nnz)
    A = sp.coo_matrix((A.data[perm], (A.row[perm], A.col[perm])), shape=(N, m))
    p = scsopt.Problem(A, rng.standard_normal(N), np.zeros(m), losses.least_squares(1.0 / N), 0.1, sparse_f32=f32)
    Ad = A.toarray()
    if f32:
        Ad = Ad.astype(np.float32).astype(np.float64)
    w = rng.random(N) + 0.5
    G = p.gram(w)
    ref = Ad.T @ (w[:, None] * Ad)
    bound = 1e-13 * (np.abs(Ad).T @ (w[:, None] * np.abs(Ad)))
    err = np.abs(G - ref)
    assert np.all(err <= bound), float(np.max(err - bound))
    assert np.array_equal(p.gram(w), G)
    g, p2 = p.ctx.kernel_names()
    assert g.startswith("sparse_gram_seg_kernel<")
    # every variant (the one-round-trip-per-8-rows kernel, the pipelined one at 32 / 64 rows per
    # batch, j- or b-major items, r03's default 5, the flat-issue walk 6 on the Gram-blocked copy)
    # accumulates the same products in the same row order as the table-driven walk on the segment
    # records (8, r04 default): bitwise G
    for var in ("6", "5", "2", "3", "4", "1"):
        monkeypatch.setenv("SCS_SPARSE_GRAM_KERNEL", var)
        assert np.array_equal(p.gram(w), G), var
    assert p.ctx.kernel_names()[0].startswith("sparse_gram_kernel<")
