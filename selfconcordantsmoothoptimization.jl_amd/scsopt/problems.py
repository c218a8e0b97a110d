"""Problem containers (src/problems.jl) backed by a device context.

``Problem(A, y, x0, f, λ; ...)`` uploads A (column-major, the Julia Matrix
layout) and y to HBM once; ``Problem(x0, f, λ; ...)`` is the data-free
ProblemGeneric (problems.jl:44-59).  ``Problem.synthetic(...)`` generates A
and y on the device (counter-based RNG, any row shard in place), which is how
the BASELINE configurations are built without ever materialising A on the
host.  Row sharding: pass ``comm=shard.Comm(...)`` and the local rows.
"""
from __future__ import annotations

import ctypes as C
import logging
from dataclasses import dataclass
from typing import Any, Optional

import numpy as np

from . import _lib
from ._lib import LOSS, GGN, REG, SMOOTH, dptr
from .losses import Loss, OutFn, ggn_kind
from .smoothers import Smoother, bounds_array

log = logging.getLogger("scsopt")


def _accepts_one_arg(fn):
    """Whether fn(x) binds: the Python reading of Julia's `applicable(grad_fx, x)` (a callable
    whose signature cannot be inspected is taken at its word and called)."""
    import inspect
    try:
        inspect.signature(fn).bind(None)
    except TypeError:
        return False
    except ValueError:
        return True
    return True


@dataclass
class GetP:
    """get_P(n, G, ind) (prox-reg-utils.jl:9-62): group structure for "gl".
    ind is 3 x grpNUM (1-based start, end; Int weight), its ranges partitioning
    1..n; G (1-based) maps the entries of P.matrix*x to variables -- a
    permutation of 1..n, read by get_reg only (the prox and the GL smoothers
    index x directly, as in the reference)."""
    n: int
    G: np.ndarray
    ind: np.ndarray

    def __post_init__(self):
        self.ind = np.asarray(self.ind, dtype=np.int64)
        self.G = np.asarray(self.G, dtype=np.int64)
        if self.ind.ndim != 2 or self.ind.shape[0] != 3:
            raise ValueError("ind must be a 3 x grpNUM integer matrix")
        self.grpNUM = int(self.ind.shape[1])
        self.grpSIZES = self.ind[1] - self.ind[0] + 1
        self.ntotal = int(self.grpSIZES.sum())
        if self.ntotal != self.n or self.G.shape != (self.n,) or \
                not np.array_equal(np.sort(self.G), np.arange(1, self.n + 1)):
            # get_Cmat / the GL smoothers raise DimensionMismatch for ntotal != n in the reference
            raise ValueError("gl groups must partition 1..n and G must be a permutation of 1..n")


def get_P(n, G, ind):
    return GetP(int(n), np.asarray(G), np.asarray(ind))


def _lam_tuple(lam):
    if isinstance(lam, (list, tuple, np.ndarray)):
        v = [float(t) for t in lam]
    else:
        v = [float(lam)]
    if len(v) not in (1, 2):
        raise ValueError("λ must be a scalar or a pair")
    return v


def _is_sparse(A):
    return hasattr(A, "tocsr") and hasattr(A, "tocsc") and hasattr(A, "nnz")


class Problem:
    """problems.jl:21-40 (data) / :5-19 (generic)."""

    def __init__(self, *args, Atest=None, ytest=None, L=None, sol=None, C_set=None, P=None,
                 out_fn: Optional[OutFn] = None, name=None, device=0, comm=None, N_global=None, row0=0,
                 sparse_f32=False, devices=None, device_exchange="rccl", Ntest_global=None, test_row0=0,
                 _ctx=None):
        if len(args) == 5:
            A, y, x0, f, lam = args
        elif len(args) == 3:
            A, y = None, None
            x0, f, lam = args
        else:
            raise TypeError("Problem(A, y, x0, f, λ; ...) or Problem(x0, f, λ; ...)")
        if not isinstance(f, Loss):
            raise TypeError("f must be a scsopt.losses kind (device losses replace Julia closures)")
        self.x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64))
        self.m = int(self.x0.shape[0])
        self.f = f
        self.λ = lam
        self.L = L
        self.x = np.zeros(self.m) if sol is None else np.ascontiguousarray(np.asarray(sol, dtype=np.float64))
        self.C_set = C_set
        self.P = P
        self.out_fn = out_fn
        self.name = name
        self.comm = comm
        self.generic = A is None and _ctx is None
        if f.kind == "callback":   # the data stays with the caller's closures; the device holds none
            if _ctx is not None or comm is not None:
                raise ValueError("a callback loss runs on one rank with host-side data")
            # y keeps its shape: an N x ny target is a multi-output problem (iterate.jl:105-107)
            self._cb_data = None if A is None else (A, np.asarray(y, dtype=np.float64))
            A, y, self.generic = None, None, True
        if devices is not None and (comm is not None or _is_sparse(A)):
            raise ValueError("devices=[...] (one process, several GPUs) takes a dense A and no comm")
        self.ctx = _ctx if _ctx is not None else _lib.Context(device, devices=devices, device_exchange=device_exchange)
        if comm is not None and comm.active and _ctx is None:
            comm.attach(self.ctx)
        if _ctx is None:
            if self.generic:
                self.N = 0
                self.ctx.check(_lib.lib.scs_set_data(self.ctx.h, 0, self.m, None, 0, None, 0, 0))
            elif _is_sparse(A):
                self._set_sparse(A, y, N_global, row0, f32=bool(sparse_f32))
            else:
                A = np.asarray(A, dtype=np.float64)
                if A.ndim != 2 or A.shape[1] != self.m:
                    raise ValueError(f"A must be N x m with m = length(x0) = {self.m}")
                Af = np.asfortranarray(A)  # Julia layout: column-major, lda = N
                yv = np.ascontiguousarray(np.asarray(y, dtype=np.float64).reshape(-1))
                self.N = int(A.shape[0])
                Ng = self.N if N_global is None else int(N_global)
                self.ctx.check(_lib.lib.scs_set_data(self.ctx.h, self.N, self.m,
                                                     Af.ctypes.data_as(_lib.c_dp), self.N, dptr(yv), Ng,
                                                     int(row0)))
        else:
            N = C.c_int64()
            self.ctx.check(_lib.lib.scs_get_dims(self.ctx.h, C.byref(N), None, None, None))
            self.N = int(N.value)
        Ng, r0 = C.c_int64(), C.c_int64()
        self.ctx.check(_lib.lib.scs_get_dims(self.ctx.h, None, None, C.byref(Ng), C.byref(r0)))
        self.N_global = int(Ng.value)   # the rows of all ranks (the minibatch loader's N)
        self.row0 = int(r0.value)       # this rank's first global row
        if comm is not None and comm.active:
            comm.bind_buffer(self.ctx)
        ggn = ggn_kind(out_fn)
        if out_fn is not None and f.kind in ("quadratic", "rosenbrock"):
            raise ValueError("out_fn needs a data loss")
        if out_fn is not None and out_fn.scale != f.scale:
            raise ValueError("f and out_fn must use the same scale (one device loss scale)")
        scale = f.scale
        self.ctx.check(_lib.lib.scs_set_loss(self.ctx.h, LOSS[f.kind], GGN[ggn], scale))
        self._cb_test = None
        if f.kind == "callback":
            self._bind_callback(f)
        self.set_test(Atest, ytest, Ntest_global=Ntest_global, row0=test_row0)

    # held-out data (problems.jl:27-28,67-68; iterate.jl:169-175) --------------------------
    def set_test(self, Atest=None, ytest=None, *, Ntest_global=None, row0=0, sparse_f32=False):
        """Atest / ytest: ftest(x) = f(Atest, ytest, x) -- the problem's own f, scale literal
        included -- is pushed into Solution.fvaltest at every stats push.  Both are required; one
        alone is the reference's xor case (iterate.jl:170-171): optim_loop! logs "Will skip
        testing..." and then, since `ftest` is never assigned, its first show_stat! (:201) raises
        UndefVarError -- iterate() does the same (scs_iterate_ex / the host loop).  Sharded: this
        rank's rows of the held-out set (Ntest_global rows in all); a devices=[...] problem takes
        the whole set."""
        self.ctx.check(_lib.lib.scs_set_test_data(self.ctx.h, 0, None, 0, None, 0, 0))   # clear
        self._cb_test = None
        self.test_model = False
        self.test_xor = False
        if Atest is None and ytest is None:
            return
        if self.generic and getattr(self.f, "kind", None) != "callback":
            raise ValueError("a ProblemGeneric has no test data (problems.jl:5-19)")
        if Atest is None or ytest is None:    # iterate.jl:170-171: recorded; the loop raises (:201)
            one = np.zeros(1)
            self.ctx.check(_lib.lib.scs_set_test_data(self.ctx.h, 0, None if Atest is None else dptr(one), 0,
                                                      None if ytest is None else dptr(one), 0, 0))
            self.test_xor = True
            return
        if self.f.kind == "quadratic":   # 1/2*(x'*(Atest*x)) + ytest'*x: Julia's DimensionMismatch otherwise
            shp = Atest.shape if hasattr(Atest, "shape") else np.shape(Atest)
            nglob = int(Ntest_global) if Ntest_global is not None else int(shp[0])
            if nglob != self.m or np.size(ytest) != shp[0]:
                raise ValueError(f"DimensionMismatch: the quadratic loss needs an m x m Atest (m = {self.m}) and "
                                 f"len(ytest) = m, got Atest {tuple(shp)}")
        if self.f.kind == "callback":
            if self._cb_data is None:
                raise ValueError("Atest / ytest need a data problem: Problem(A, y, x0, f, λ; Atest, ytest)")
            self._cb_test = (Atest, np.asarray(ytest, dtype=np.float64))
            self.ctx.check(_lib.lib.scs_set_test_callback(self.ctx.h, 1))
            self.test_model = True
            return
        yv = np.ascontiguousarray(np.asarray(ytest, dtype=np.float64).reshape(-1))
        Ng = int(Ntest_global) if Ntest_global is not None else 0
        if _is_sparse(Atest):
            csr = Atest.tocsr()
            if csr.shape[1] != self.m or csr.shape[0] != yv.shape[0]:
                raise ValueError(f"Atest must be Ntest x m (m = {self.m}) with len(ytest) = Ntest")
            rowptr = np.ascontiguousarray(csr.indptr, dtype=np.int64)
            colidx = np.ascontiguousarray(csr.indices, dtype=np.int32)
            val = np.ascontiguousarray(csr.data, dtype=np.float64)
            self.ctx.check(_lib.lib.scs_set_test_sparse(
                self.ctx.h, int(csr.shape[0]), int(val.shape[0]), rowptr.ctypes.data_as(_lib.c_i64p),
                colidx.ctypes.data_as(_lib.c_i32p), dptr(val), 1 if sparse_f32 else 0, dptr(yv), Ng, int(row0)))
        else:
            At = np.asarray(Atest, dtype=np.float64)
            if At.ndim != 2 or At.shape[1] != self.m or At.shape[0] != yv.shape[0]:
                raise ValueError(f"Atest must be Ntest x m (m = {self.m}) with len(ytest) = Ntest")
            Af = np.asfortranarray(At)
            self.ctx.check(_lib.lib.scs_set_test_data(self.ctx.h, int(At.shape[0]), Af.ctypes.data_as(_lib.c_dp),
                                                      int(At.shape[0]), dptr(yv), Ng, int(row0)))
        self.test_model = True

    def gen_test(self, Ntest, *, row0=None, seed=1234, kind=1, density=0.1):
        """Held-out rows of the synthetic generator: rows [row0, row0 + Ntest) with row0 = N_global
        by default (samples the training rows never saw, same x_true).  Sharded: this rank
        generates its contiguous block of the Ntest rows."""
        from .shard import row_range
        r0 = self.N_global if row0 is None else int(row0)
        comm = self.comm
        # one process per GPU: this rank's block; one process (one or several devices): all rows
        # (a devices=[...] context splits them itself)
        a, b = row_range(Ntest, comm.world, comm.rank) if comm is not None else (0, int(Ntest))
        spec = _lib.Synth(N_global=int(Ntest), row0=r0 + a, N=b - a, m=self.m, seed=seed, kind=kind, density=density)
        self.ctx.check(_lib.lib.scs_gen_test_data(self.ctx.h, C.byref(spec)))
        self._cb_test = None
        self.test_xor = False
        self.test_model = True

    def ftest(self, x):
        """f(Atest, ytest, x) (iterate.jl:173) on the device (a callback loss: on the host)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = C.c_double()
        self.ctx.check(_lib.lib.scs_eval_ftest(self.ctx.h, dptr(x), C.byref(out)))
        return out.value

    def _bind_callback(self, f):
        """Register f / grad_fx / hess_fx with scs_set_loss_callback; a Python exception inside a
        call is kept and re-raised by Context.check."""
        data = self._cb_data
        args = (lambda x: (x,)) if data is None else (lambda x: (data[0], data[1], x))
        ctx = self.ctx
        nout = 0
        if f.has_ggn:
            if data is None:
                raise ValueError("ProxGGNSCORE callbacks take the data: Problem(A, y, x0, callback(...), λ)")
            nout = int(np.asarray(f.out_fn(data[0], self.x0)).size)

        def ggn_pieces(x, m, outp):
            """prox-GGN-SCORE.jl:44-49 on the host; a non-diagonal Q is eigen-rotated (J̃ = VᵀJ,
            r̃ = Vᵀr, q = eigenvalues), which leaves JᵀQJ, Jᵀr and the sample-space system exact."""
            A, y = data
            yhat = f.out_fn(A, x)
            J = np.asarray(f.jac_yx(A, y, yhat, x), dtype=np.float64).reshape(nout, m)
            r = np.asarray(f.grad_fy(A, y, yhat), dtype=np.float64).ravel(order="F")
            Q = np.asarray(f.hess_fy(A, y, yhat), dtype=np.float64)
            if Q.ndim == 2 and np.count_nonzero(Q - np.diag(np.diagonal(Q))) == 0:
                Q = np.diagonal(Q).copy()
            if Q.ndim == 2:
                lam, V = np.linalg.eigh(0.5 * (Q + Q.T))
                J, r, q = V.T @ J, V.T @ r, lam
            else:
                q = Q.reshape(nout)
            out = np.ctypeslib.as_array(outp, shape=(nout * (m + 2),))
            out[:nout * m] = J.ravel(order="F")
            out[nout * m:nout * (m + 1)] = r
            out[nout * (m + 1):] = q

        def call(user, what, xp, m, outp):
            try:
                x = np.ctypeslib.as_array(xp, shape=(m,)).copy()
                if what == _lib.SCS_CB_F:
                    outp[0] = float(f.f(*args(x)))
                elif what == _lib.SCS_CB_GRAD:
                    if f.grad_fx is None:
                        raise ValueError("this method needs grad_fx: the device path has no automatic "
                                         "differentiation (the reference's ForwardDiff default)")
                    g = np.asarray(f.grad_fx(*args(x)), dtype=np.float64).reshape(m)
                    np.ctypeslib.as_array(outp, shape=(m,))[:] = g
                elif what == _lib.SCS_CB_GRAD_X:
                    # ProxGGNSCORE: grad_f = x -> model.grad_fx(x), ONE argument (prox-GGN-SCORE.jl:58-59),
                    # reached from its ss_type 3 line search (:83-84): Julia's MethodError when the
                    # user's grad_fx has no one-argument method (a data problem's grad_fx(A, y, x))
                    if f.grad_fx is None:
                        raise ValueError("this method needs grad_fx: the device path has no automatic "
                                         "differentiation (the reference's ForwardDiff default)")
                    if not _accepts_one_arg(f.grad_fx):
                        return _lib.SCS_CB_NO_METHOD
                    g = np.asarray(f.grad_fx(x), dtype=np.float64).reshape(m)
                    np.ctypeslib.as_array(outp, shape=(m,))[:] = g
                elif what == _lib.SCS_CB_HESS:
                    if f.hess_fx is None:
                        raise ValueError("ProxNSCORE needs hess_fx: the device path has no automatic "
                                         "differentiation (the reference's ForwardDiff default)")
                    H = np.asarray(f.hess_fx(*args(x)), dtype=np.float64).reshape(m, m)
                    np.ctypeslib.as_array(outp, shape=(m * m,))[:] = H.ravel(order="F")   # column-major
                elif what == _lib.SCS_CB_GGN:
                    ggn_pieces(x, m, outp)
                elif what == _lib.SCS_CB_FTEST:   # iterate.jl:173: the same closure on the held-out data
                    At, yt = self._cb_test
                    outp[0] = float(f.f(At, yt, x))
                else:
                    raise ValueError(f"unknown callback request {what}")
                return 0
            except BaseException as e:   # noqa: BLE001 -- handed back to the caller by Context.check
                ctx._cb_exc = e
                return 1

        cb = _lib.LOSS_FN(call)
        self.ctx._keep.append(cb)
        self.ctx.check(_lib.lib.scs_set_loss_callback(self.ctx.h, cb, None, nout))

    @classmethod
    def synthetic(cls, N, m, x0, f, lam, *, kind=1, seed=1234, density=0.1, out_fn=None, device=0,
                  comm=None, devices=None, device_exchange="rccl", test_N=None, **kw):
        """A ~ N(0,1)/sqrt(m) (kind 1, 2) or N(0,1) (kind 3) generated on the device, y from a
        sparse x_true (kind 1: Bernoulli(σ(A x_true)) ∈ {0,1}; kind 2: ±1; kind 3: A x_true + 0.1ε).
        With comm, this rank generates its contiguous row shard in place; with devices=[...] one
        process drives those GPUs and the library generates each one's row block."""
        from .shard import row_range
        if devices is not None and comm is not None:
            raise ValueError("devices=[...] (one process, several GPUs) and comm (one process per GPU) exclude "
                             "each other")
        rank, world = (comm.rank, comm.world) if comm is not None else (0, 1)
        r0, r1 = row_range(N, world, rank)
        ctx = _lib.Context(device, devices=devices, device_exchange=device_exchange)
        if comm is not None and comm.active:
            comm.attach(ctx)
        spec = _lib.Synth(N_global=N, row0=r0, N=r1 - r0, m=m, seed=seed, kind=kind, density=density)
        ctx.check(_lib.lib.scs_gen_data(ctx.h, C.byref(spec)))
        p = cls(x0, f, lam, out_fn=out_fn, device=device, comm=comm, _ctx=ctx, **kw)
        if test_N:   # held-out rows [N, N + test_N) of the same generator (same x_true)
            p.gen_test(int(test_N), row0=N, seed=seed, kind=kind, density=density)
        return p

    @classmethod
    def synthetic_sparse(cls, N, m, x0, f, lam, *, density=0.01, seed=1234, f32=False, device=0, **kw):
        """Sparse A (the README's sprandn(N, m, ρ) problem class, BASELINE configs[4]) generated on
        the device: k = round(ρ m) nonzeros per row, N(0,1)/sqrt(k) values, CSR + CSC copies;
        x_true ~ U(-1.5, 1.5), y = A x_true + 0.1ε.  N must be a power of two and a multiple of m."""
        ctx = _lib.Context(device)
        spec = _lib.Synth(N_global=N, row0=0, N=N, m=m, seed=seed, kind=4, density=density)
        ctx.check(_lib.lib.scs_gen_sparse(ctx.h, C.byref(spec), 1 if f32 else 0))
        return cls(x0, f, lam, device=device, _ctx=ctx, **kw)

    def _set_sparse(self, A, y, N_global, row0, f32):
        csr = A.tocsr()
        csc = A.tocsc()
        if csr.shape[1] != self.m:
            raise ValueError(f"A must be N x m with m = length(x0) = {self.m}")
        self.N = int(csr.shape[0])
        rowptr = np.ascontiguousarray(csr.indptr, dtype=np.int64)
        colidx = np.ascontiguousarray(csr.indices, dtype=np.int32)
        val = np.ascontiguousarray(csr.data, dtype=np.float64)
        colptr = np.ascontiguousarray(csc.indptr, dtype=np.int64)
        rowidx = np.ascontiguousarray(csc.indices, dtype=np.int32)
        valT = np.ascontiguousarray(csc.data, dtype=np.float64)
        yv = np.ascontiguousarray(np.asarray(y, dtype=np.float64).reshape(-1))
        Ng = self.N if N_global is None else int(N_global)
        i64, i32 = _lib.c_i64p, _lib.c_i32p
        self.ctx.check(_lib.lib.scs_set_sparse(
            self.ctx.h, self.N, self.m, int(val.shape[0]), rowptr.ctypes.data_as(i64), colidx.ctypes.data_as(i32),
            dptr(val), colptr.ctypes.data_as(i64), rowidx.ctypes.data_as(i32), dptr(valT), 1 if f32 else 0,
            dptr(yv), Ng, int(row0)))

    @property
    def nnz(self):
        n = C.c_int64()
        self.ctx.check(_lib.lib.scs_get_nnz(self.ctx.h, C.byref(n)))
        return int(n.value)

    def get_sparse(self):
        """The device CSR copy of A as a scipy.sparse.csr_matrix (values widened to fp64), and y."""
        import scipy.sparse as sp
        nnz = self.nnz
        rowptr = np.zeros(self.N + 1, dtype=np.int64)
        colidx = np.zeros(max(nnz, 1), dtype=np.int32)
        val = np.zeros(max(nnz, 1), dtype=np.float64)
        self.ctx.check(_lib.lib.scs_get_sparse(self.ctx.h, rowptr.ctypes.data_as(_lib.c_i64p),
                                               colidx.ctypes.data_as(_lib.c_i32p), dptr(val)))
        y = np.zeros(self.N, dtype=np.float64)
        self.ctx.check(_lib.lib.scs_get_data(self.ctx.h, 0, self.N, None, self.N, dptr(y)))
        return sp.csr_matrix((val[:nnz], colidx[:nnz], rowptr), shape=(self.N, self.m)), y

    # device evaluation helpers ------------------------------------------------
    def fx(self, x):
        """f(A, y, x) on the device (iterate.jl:168)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = C.c_double()
        self.ctx.check(_lib.lib.scs_eval_f(self.ctx.h, dptr(x), C.byref(out)))
        return out.value

    def gradx(self, x):
        """∇f(A, y, x) on the device (grad_fx)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        g = np.empty(self.m)
        self.ctx.check(_lib.lib.scs_eval_grad(self.ctx.h, dptr(x), dptr(g)))
        return g

    def get_data(self, r0=0, nr=None):
        nr = self.N - r0 if nr is None else nr
        A = np.zeros((self.m, nr), dtype=np.float64)   # column-major view: A.T is N x m
        y = np.zeros(nr, dtype=np.float64)
        self.ctx.check(_lib.lib.scs_get_data(self.ctx.h, r0, nr, dptr(A), nr, dptr(y)))
        return np.ascontiguousarray(A.T), y

    def configure(self, reg_name, hmu: Smoother):
        """Push reg_name / λ / C_set / P and the smoother to the device context."""
        if reg_name not in REG:
            raise _lib.ScsReferenceError(_lib.SCS_ERR_REF, "reg_name not valid.")
        lam = np.ascontiguousarray(_lam_tuple(self.λ), dtype=np.float64)
        lb = ub = None
        nb = 0
        ind = None
        ng = 0
        if reg_name == "indbox":
            if self.C_set is None:
                raise ValueError("indbox needs C_set")
            lo, hi = self.C_set[0], self.C_set[1]
            lb, ub = bounds_array(lo, self.m), bounds_array(hi, self.m)
            if lb.size != ub.size:
                lb = np.broadcast_to(lb, (self.m,)).copy()
                ub = np.broadcast_to(ub, (self.m,)).copy()
            nb = lb.size
        if reg_name == "gl":
            if self.P is None:
                raise ValueError("gl needs P = get_P(n, G, ind)")
            ind = np.ascontiguousarray(self.P.ind.T.reshape(-1), dtype=np.int64)  # column-major 3 x G
            ng = self.P.grpNUM
        self.ctx.check(_lib.lib.scs_set_reg(self.ctx.h, REG[reg_name], dptr(lam), lam.size, dptr(lb), dptr(ub),
                                            nb, ind.ctypes.data_as(_lib.c_i64p) if ind is not None else None,
                                            ng))
        if reg_name == "gl":
            G = np.ascontiguousarray(self.P.G, dtype=np.int64)
            self.ctx.check(_lib.lib.scs_set_group_map(self.ctx.h, G.ctypes.data_as(_lib.c_i64p), int(G.size)))
        slb = sub = None
        snb = 0
        if hmu.kind in ("phuber_indbox", "exp_indbox", "logexp_indbox"):
            slb, sub = bounds_array(hmu.lb, self.m), bounds_array(hmu.ub, self.m)
            if slb.size != sub.size:
                slb = np.broadcast_to(slb, (self.m,)).copy()
                sub = np.broadcast_to(sub, (self.m,)).copy()
            snb = slb.size
        self.ctx.check(_lib.lib.scs_set_smoother(self.ctx.h, SMOOTH[hmu.kind], hmu.mu, hmu.Mh, hmu.nu, dptr(slb),
                                                 dptr(sub), snb))
        self.ctx.check(_lib.lib.scs_set_L(self.ctx.h, int(self.L is not None),
                                          float(self.L) if self.L is not None else 0.0))

    def get_reg(self, x):
        """get_reg(model, x, reg_name) for the configured reg_name (regularizers.jl:4-31)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = C.c_double()
        self.ctx.check(_lib.lib.scs_eval_reg(self.ctx.h, dptr(x), C.byref(out)))
        return out.value

    def set_gram_cache(self, on=True):
        """Opt-in reuse of AᵀQA across steps when it is x-independent (least squares under
        ProxNSCORE, or ProxGGNSCORE with the linear out_fn); the reference recomputes it every
        step (prox-GGN-SCORE.jl:129), which stays the default.  Results are bit-identical."""
        self.ctx.check(_lib.lib.scs_set_gram_cache(self.ctx.h, int(bool(on))))

    def set_compute_f32(self, on=True):
        """The compute arm of the fp32-vs-fp64 study (BASELINE configs[4]): the sparse products of
        fp32-stored values (sparse_f32 / f32=True) and the L-BFGS two-loop in fp32 arithmetic;
        f, η, the step, the prox and the solves stay fp64.  Off (fp64) by default."""
        self.ctx.check(_lib.lib.scs_set_compute_f32(self.ctx.h, int(bool(on))))

    def set_solver(self, kind="default"):
        """"default": Cholesky (LU fallback) / LU; "reference": the reference's factorizations --
        Householder QR for ProxGGNSCORE's systems (prox-GGN-SCORE.jl:126,131), LU for ProxNSCORE's
        (prox-N-SCORE.jl:70).  scs_set_solver."""
        self.ctx.check(_lib.lib.scs_set_solver(self.ctx.h, _lib.SOLVER[kind]))

    def set_batches(self, batches=None):
        """Register the collected loader batches (iterate.jl:141-146): a list of row-index arrays
        (0-based, GLOBAL rows: on several ranks every rank passes the same list and keeps the rows
        it owns), gathered on the device as the As, ys of their step! calls (iterate.jl:205-207).
        None / [] clears the list.  f / get_reg stay on the full data."""
        if not batches:
            self.ctx.check(_lib.lib.scs_set_batches(self.ctx.h, None, None, 0))
            return
        rs = [np.asarray(b, dtype=np.int64).reshape(-1) for b in batches]
        rows = np.ascontiguousarray(np.concatenate(rs))
        off = np.zeros(len(rs) + 1, dtype=np.int64)
        off[1:] = np.cumsum([r.size for r in rs])
        self.ctx.check(_lib.lib.scs_set_batches(self.ctx.h, rows.ctypes.data_as(_lib.c_i64p),
                                                off.ctypes.data_as(_lib.c_i64p), len(rs)))
        if self.comm is not None and self.comm.active:   # the exchange payload may have grown
            self.comm.bind_buffer(self.ctx)

    def select_batch(self, b=-1):
        """The registered batch the following step! calls see as As, ys (-1: the full data)."""
        self.ctx.check(_lib.lib.scs_select_batch(self.ctx.h, int(b)))

    def _smoother_eval(self, hmu, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        gr = np.empty(self.m)
        Hr = np.empty(self.m)
        self.ctx.check(_lib.lib.scs_smoother_eval(self.ctx.h, dptr(x), dptr(gr), dptr(Hr)))
        return gr, Hr

    # kernel-level entry points used by the parity tests -----------------------
    def prox(self, z, Hr, lam, alpha):
        z = np.ascontiguousarray(z, dtype=np.float64)
        Hr = np.ascontiguousarray(Hr, dtype=np.float64)
        out = np.empty(self.m)
        self.ctx.check(_lib.lib.scs_prox_eval(self.ctx.h, dptr(z), dptr(Hr), float(lam), float(alpha), dptr(out)))
        return out

    def gram(self, w):
        w = np.ascontiguousarray(w, dtype=np.float64)
        G = np.zeros((self.m, self.m))
        self.ctx.check(_lib.lib.scs_gram_eval(self.ctx.h, dptr(w), dptr(G), self.m))
        return G.T.copy()  # column-major -> row-major (lower triangle valid)

    def gemv_t(self, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        out = np.empty(self.m)
        self.ctx.check(_lib.lib.scs_gemv_t_eval(self.ctx.h, dptr(v), dptr(out)))
        return out

    def gemv_n(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty(self.N)
        self.ctx.check(_lib.lib.scs_gemv_n_eval(self.ctx.h, dptr(x), dptr(out)))
        return out

    def solve_eval(self, w, dvec, rhs, mode=0):
        """(Aᵀ diag(w) A + diag(dvec)) \\ rhs through the step's solve path (mode 0: Cholesky with
        the LU fallback; 1: the LU).  Returns (x, used_lu)."""
        w = np.ascontiguousarray(w, dtype=np.float64)
        dvec = np.ascontiguousarray(dvec, dtype=np.float64)
        rhs = np.ascontiguousarray(rhs, dtype=np.float64)
        x = np.empty(self.m)
        used = C.c_int()
        self.ctx.check(_lib.lib.scs_solve_eval(self.ctx.h, dptr(w), dptr(dvec), dptr(rhs), int(mode), dptr(x),
                                               C.byref(used)))
        return x, bool(used.value)

    def get_columns(self, cols):
        """Columns of the local A (N x len(cols), float64)."""
        cols = np.ascontiguousarray(cols, dtype=np.int64)
        out = np.empty((cols.size, self.N))
        self.ctx.check(_lib.lib.scs_get_columns(self.ctx.h, cols.ctypes.data_as(_lib.c_i64p), cols.size, dptr(out)))
        return out.T

    def gram_atv_sample(self, w, v, pairs):
        """The production Gram launch (Aᵀv fused where a step fuses it): G entries at pairs (k x 2),
        Aᵀv, and whether the pass was fused."""
        w = np.ascontiguousarray(w, dtype=np.float64)
        v = np.ascontiguousarray(v, dtype=np.float64)
        ij = np.ascontiguousarray(np.asarray(pairs, dtype=np.int64).reshape(-1, 2))
        g = np.empty(ij.shape[0])
        atv = np.empty(self.m)
        fused = C.c_int()
        self.ctx.check(_lib.lib.scs_gram_atv_eval(self.ctx.h, dptr(w), dptr(v), ij.ctypes.data_as(_lib.c_i64p),
                                                  ij.shape[0], dptr(g), dptr(atv), C.byref(fused)))
        return g, atv, bool(fused.value)


def lu_solve(A, b, device=0, ctx=None):
    """Julia's `A \\ b` for a dense square matrix (getrf + getrs) on the device: the hand-written
    blocked LU with partial pivoting (lu.hip).  Returns (x, ipiv (0-based), info); with info > 0 (a
    zero pivot, dgetrf's info) x is None and ipiv holds dgetrf's pivots."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    n = A.shape[0]
    if A.shape != (n, n) or b.shape != (n,):
        raise ValueError("A must be n x n and b of length n")
    ctx = ctx or _lib.Context(device)
    x = np.zeros(n)
    ipiv = np.zeros(n, dtype=np.int32)
    info = C.c_int()
    ctx.check(_lib.lib.scs_lu_eval(ctx.h, n, dptr(A), dptr(b), dptr(x), ipiv.ctypes.data_as(_lib.c_i32p),
                                   C.byref(info)))
    return (x if info.value == 0 else None), ipiv, int(info.value)

