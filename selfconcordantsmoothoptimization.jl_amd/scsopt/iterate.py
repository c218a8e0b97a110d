"""iterate! / optim_loop! / Solution (src/algorithms/iterate.jl) over the device step.

The loop logic -- history pushes, the duplicated last-epoch entry, the
termination tests on the pre-step f_rel_error, the α -> L = 1/α mutation --
restates iterate.jl:56-76,100-267 line by line; every f(x), get_reg(x) and
step! runs in libscsopt on the GPU.
"""
from __future__ import annotations

import ctypes as C
import logging
import math
import sys
import time
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from . import _lib
from ._lib import dptr
from .methods import ProximalMethod, ProxLQNSCORE

log = logging.getLogger("scsopt")


@dataclass
class Solution:
    """iterate.jl:3-32."""
    x: np.ndarray
    obj: list
    fval: list
    pri_res_norm: list
    fvaltest: list
    rel: list
    objrel: list
    metricvals: dict
    times: list
    epochs: int
    model: Any


def _jl_max(a, b):
    """Julia max(::Float64, ::Float64): NaN propagates, -0.0 < +0.0."""
    a = float(a)
    b = float(b)
    if math.isnan(a):
        return a
    if math.isnan(b):
        return b
    if b < a or (math.copysign(1.0, b) < 0 < math.copysign(1.0, a)):
        return a
    return b


def _norm(v):
    return float(np.linalg.norm(v))


def step(method, model, reg_name, hmu, x, x_prev, iter_, return_dx=False, batch=None, grad_fx=None):
    """step!(method, model, reg_name, hμ, As, x, x_prev, ys, Cmat, iter; ∇fx, return_dx).

    As, ys: the full data, or registered batch `batch` (Problem.set_batches).  grad_fx: the
    reference's ∇fx keyword -- the step uses it as grad_f at every point (scs_step_grad)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    x_prev = np.ascontiguousarray(x_prev, dtype=np.float64)
    x_new = np.empty_like(x)
    dx = np.empty_like(x) if return_dx else None
    g = None
    if grad_fx is not None:
        g = np.ascontiguousarray(np.asarray(grad_fx, dtype=np.float64).reshape(-1))
        if g.shape != x.shape:
            raise ValueError(f"∇fx must have length m = {x.shape[0]}")
    pri = C.c_double()
    if batch is not None:
        model.select_batch(batch)
    try:
        model.ctx.check(_lib.lib.scs_step_grad(model.ctx.h, dptr(x), dptr(x_prev), int(iter_), dptr(g), dptr(x_new),
                                               dptr(dx), C.byref(pri)))
    finally:
        if batch is not None:
            model.select_batch(-1)
    if return_dx:
        return x_new, dx, pri.value
    return x_new, pri.value


def init_method(method, model):
    """init!(method, x) on the device (resets the L-BFGS memory)."""
    mem = method.m if isinstance(method, ProxLQNSCORE) else 0
    model.ctx.check(_lib.lib.scs_method_init(model.ctx.h, method.code, int(method.ss_type), int(bool(method.use_prox)),
                                             int(mem)))


def loader_batches(N, batch_size=None, slice_samples=False, shuffle_batch=True, local_max_iter=None, perm=None,
                   rng=None):
    """The collected batch list of optim_loop! (iterate.jl:124-146; utils.jl:14-25) as
    0-based row-index arrays, or None for the single full batch.

    * batch_size b: DataLoader(batchsize=b, shuffle=shuffle_batch) -> ceil(N/b) batches of
      consecutive rows of the (shuffled) order, the last one partial; collected once, so the
      same batches run every epoch.  The shuffle permutation is `perm` when given, else drawn
      from `rng` (numpy; Julia's global RNG stream is not reproducible here).
    * slice_samples (ignored when batch_size is set, :131-134): one-sample batches -- and since
      max_iter stays 1 (:127), only the first sample is ever used.
    * local_max_iter: only the first min(floor(local_max_iter), max_iter) batches (:124,128).
    """
    if batch_size is not None and slice_samples:
        log.info("Cannot use both batch_size and slice_samples=true... Now setting slice_samples=false...")
        slice_samples = False
    max_iter = int(math.ceil(N / batch_size)) if batch_size is not None else 1
    iend = max_iter
    if local_max_iter is not None and int(math.floor(local_max_iter)) > 0:
        iend = min(int(math.floor(local_max_iter)), max_iter)
    if slice_samples:
        return [np.arange(i, i + 1, dtype=np.int64) for i in range(min(iend, N))]
    if batch_size is None:
        return None
    b = int(batch_size)
    if b < 1:
        raise ValueError("batch_size must be >= 1")
    if shuffle_batch:
        order = np.asarray(perm, dtype=np.int64) if perm is not None else \
            (rng if rng is not None else np.random.default_rng()).permutation(N).astype(np.int64)
        if sorted(order.tolist()) != list(range(N)):
            raise ValueError("perm must be a permutation of 0..N-1")
    else:
        order = np.arange(N, dtype=np.int64)
    return [order[i * b:min((i + 1) * b, N)] for i in range(iend)]


def iterate(method: ProximalMethod, model, reg_name, hmu, *, metrics=None, alpha=None, batch_size=None,
            slice_samples=False, shuffle_batch=True, max_epoch=1000, comm_rounds=100, local_max_iter=None,
            x_tol=1e-10, f_tol=1e-10, verbose=1, device_loop=None, batch_perm=None, rng=None):
    """iterate!(method, model, reg_name, hμ; kwargs...) (iterate.jl:56-76).

    device_loop: run optim_loop! inside libscsopt (scs_iterate: one ABI call per solve);
    the default (None) does so whenever nothing needs the host per epoch (no metrics,
    verbose <= 1).  False forces the host restatement below (same device calls).
    batch_perm / rng: the shuffled loader's permutation (see loader_batches)."""
    if local_max_iter is not None:
        max_epoch = 1
    batches = None
    if (batch_size is not None or slice_samples) and getattr(model.f, "kind", None) == "callback":
        raise ValueError("minibatches need a device loss kind (a callback loss keeps its data on the host)")
    N = getattr(model, "N_global", getattr(model, "N", 0))
    if N and (batch_size is not None or slice_samples):
        batches = loader_batches(N, batch_size, slice_samples, shuffle_batch, local_max_iter, batch_perm, rng)
        comm = getattr(model, "comm", None)
        if comm is not None and comm.active:   # one batch list (one shuffle) for every rank
            batches = comm.broadcast_object(batches)
    if device_loop is None:
        device_loop = not metrics and verbose <= 1
    if device_loop and (metrics or verbose > 1):
        raise ValueError("device_loop runs without per-epoch metrics / printing")
    model.set_batches(batches)
    try:
        if device_loop:
            return device_optim_loop(method, model, reg_name, hmu, alpha=alpha, max_epoch=max_epoch, x_tol=x_tol,
                                     f_tol=f_tol, verbose=verbose)
        return optim_loop(method, model, reg_name, hmu, metrics=metrics, alpha=alpha, max_epoch=max_epoch,
                          x_tol=x_tol, f_tol=f_tol, verbose=verbose, nbatch=len(batches) if batches else 0)
    finally:
        if batches:
            model.set_batches(None)


def device_optim_loop(method, model, reg_name, hmu, *, alpha=None, max_epoch=1000, x_tol=1e-10, f_tol=1e-10,
                      verbose=1):
    """optim_loop! (iterate.jl:100-267) as one scs_iterate call; same Solution as optim_loop."""
    implemented = []
    method.set_name(implemented)
    if alpha is not None:
        model.L = 1 / alpha                                   # iterate.jl:113-115
    if method.name in implemented and method.ss_type == 1 and model.L is None and verbose > 0:
        print("[ Info: Neither L nor α is set for the problem... Now fixing α = 0.5...", file=sys.stderr)
    model.configure(reg_name, hmu)
    _xor_info(model)                                   # the library raises at the first push
    init_method(method, model)
    m = model.m
    cap = 2 * int(max_epoch) + 1                       # scsopt.h: up to two pushes per epoch
    keys = ("obj", "fval", "pri_res_norm", "rel", "objrel", "times", "fvaltest")
    hist = {k: np.empty(cap) for k in keys}
    test_model = bool(getattr(model, "test_model", False))
    h = _lib.History(*(dptr(hist[k]) if (k != "fvaltest" or test_model) else None for k in keys))
    x0 = np.ascontiguousarray(model.x0, dtype=np.float64)
    xs = np.ascontiguousarray(model.x, dtype=np.float64)
    x_out = np.empty(m)
    nh, ep = C.c_int64(), C.c_int64()
    model.ctx.check(_lib.lib.scs_iterate_ex(model.ctx.h, dptr(x0), dptr(xs), int(max_epoch), float(x_tol),
                                            float(f_tol), 1 if reg_name == "gl" else 0, dptr(x_out), C.byref(h),
                                            C.sizeof(_lib.History), C.byref(nh), C.byref(ep)))
    n = int(nh.value)
    pris = [None if (i == 0 and math.isnan(v)) else float(v) for i, v in enumerate(hist["pri_res_norm"][:n])]
    as_list = lambda k: [float(v) for v in hist[k][:n]]   # noqa: E731
    fvaltest = as_list("fvaltest") if test_model else []
    return Solution(x_out, as_list("obj"), as_list("fval"), pris, fvaltest, as_list("rel"), as_list("objrel"), {},
                    as_list("times"), int(ep.value), model)


XOR_INFO = ("Both input (Atest) and target (ytest) data are required for testing the model, but only one of these "
            "has been provided.\nWill skip testing...")
XOR_ERROR = ("UndefVarError: `ftest` not defined (only one of Atest / ytest was given: iterate.jl:170-171 leave ftest "
             "unassigned, show_stat! at :201 reads it)")


def _xor_info(model):
    """iterate.jl:170-171: optim_loop! logs this when exactly one of Atest / ytest is given; its first
    show_stat! (:201) then raises, since `ftest` was never assigned (the loops below do the same)."""
    xor = bool(getattr(model, "test_xor", False))
    if xor:
        log.info(XOR_INFO)
    return xor


def _show(opt_verbose, label, tag, epoch, obj, fval, pri, rel, dt, ftest=None):
    if opt_verbose > 1:
        print("\n" + "=" * 30)
        print(f"Optimizer:\t{label}")
        ft = "" if ftest is None else f"fvaltest = {ftest}\n"
        print(f"{tag} = {epoch}\nobj = {obj}\nfval = {fval}\npri_res_norm = {pri}\n{ft}rel_error = {rel}\n"
              f"Δtime = {dt}")


def optim_loop(method, model, reg_name, hmu, *, metrics=None, alpha=None, max_epoch=1000, x_tol=1e-10,
               f_tol=1e-10, verbose=1, nbatch=0):
    """optim_loop! (iterate.jl:100-267); nbatch > 0: the registered batches in order
    (Problem.set_batches), else the one full batch."""
    implemented = []
    method.set_name(implemented)
    if alpha is not None:
        model.L = 1 / alpha                                   # iterate.jl:113-115
    if method.name in implemented and method.ss_type == 1 and model.L is None and verbose > 0:
        print("[ Info: Neither L nor α is set for the problem... Now fixing α = 0.5...", file=sys.stderr)
    model.configure(reg_name, hmu)
    f = model.fx
    greg = model.get_reg
    fvals, pris, objs, rels, frels, times = [], [], [], [], [], []
    fvaltests = []
    test_model = bool(getattr(model, "test_model", False))   # iterate.jl:169-175
    test_xor = _xor_info(model)
    metric_vals = {k: [] for k in (metrics or {})}
    epochs = 0
    x_star = model.x
    pri = None
    obj_star = f(x_star) + greg(x_star)
    x = model.x0.copy()
    x_prev = x.copy()
    init_method(method, model)
    t0 = time.monotonic()

    def now():
        return int((time.monotonic() - t0) * 1000) / 1000   # Dates.now() has ms resolution

    def rel_of(xx):
        if reg_name == "gl":
            d = x_star - xx
            return float(np.mean(d * d))                       # mean_square_error (utils.jl:3-5)
        return _jl_max(_norm(xx - x_star) / _jl_max(_norm(x_star), 1.0), x_tol)

    def frel_of(ob):
        with np.errstate(divide="ignore", invalid="ignore"):
            q = np.float64(abs(ob - obj_star)) / np.float64(abs(obj_star))
        return _jl_max(q, f_tol)

    def push(ob, fv, pr, rl, fr, dt, xx, ft):
        # show_stat! (utils.jl:50-57: ftest, metrics) + update_stat! (utils.jl:106-113)
        if test_model:
            fvaltests.append(ft)
        objs.append(ob); fvals.append(fv); pris.append(pr); rels.append(rl); frels.append(fr); times.append(dt)
        for k in metric_vals:
            metric_vals[k].append(metrics[k](model, xx))

    def ftest(xx):   # evaluated as show_stat!'s argument, before anything is printed or pushed
        if test_xor:                                  # iterate.jl:201 with ftest unassigned
            raise _lib.ScsReferenceError(_lib.SCS_ERR_REF, XOR_ERROR)
        return model.ftest(xx) if test_model else None

    iend = max(nbatch, 1)
    for epoch_t in range(1, max_epoch + 1):
        dt = now()
        fval = f(x)
        obj = fval + greg(x)
        rel_error = rel_of(x)
        f_rel_error = frel_of(obj)
        ft = ftest(x)
        _show(verbose, method.label, "epoch", epoch_t - 1, obj, fval, pri, rel_error, dt, ft)
        push(obj, fval, pri, rel_error, f_rel_error, dt, x, ft)
        for i in range(1, iend + 1):                          # iterate.jl:204-255
            if epoch_t == max_epoch and i == iend:            # iterate.jl:219-231
                dt = now()
                fval = f(x)
                obj = fval + greg(x)
                rel_error = rel_of(x)
                ft = ftest(x)
                _show(verbose, method.label, "max_epoch", epoch_t, obj, fval, pri, rel_error, dt, ft)
                f_rel_error = frel_of(obj)
                push(obj, fval, pri, rel_error, f_rel_error, dt, x, ft)
            x_new, pri = step(method, model, reg_name, hmu, x, x_prev, epoch_t, batch=(i - 1) if nbatch else None)
            if _norm(x_new - x) < x_tol * max(_norm(x), 1.0) or f_rel_error <= f_tol or pri < x_tol:
                if epoch_t != max_epoch:                      # iterate.jl:235-247
                    dt = now()
                    fval = f(x_new)
                    obj = fval + greg(x_new)
                    rel_error = rel_of(x_new)
                    ft = ftest(x_new)
                    _show(verbose, method.label, "terminate_epoch", epoch_t, obj, fval, pri, rel_error, dt, ft)
                    f_rel_error = frel_of(obj)
                    push(obj, fval, pri, rel_error, f_rel_error, dt, x_new, ft)
                x_prev = x
                x = x_new
                epochs += 1
                break
            x_prev = x
            x = x_new
        if _norm(x - x_prev) < x_tol * max(_norm(x_prev), 1.0) or f_rel_error <= f_tol or pri < x_tol:
            break                                             # iterate.jl:257-259
        epochs += 1
    return Solution(x, objs, fvals, pris, fvaltests, rels, frels, metric_vals, times, epochs, model)
