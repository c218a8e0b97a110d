"""ctypes binding of libscsopt (include/scsopt.h).

The library is built in-tree (``make -C selfconcordantsmoothoptimization.jl_amd/csrc``)
and is the only compute path: nothing here falls back to a CPU
implementation.  If the shared object is missing, importing this module
raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCSOPT_LIB", os.path.join(_HERE, "libscsopt.so"))

SCS_OK, SCS_ERR_ARG, SCS_ERR_HIP, SCS_ERR_SOLVE, SCS_ERR_STATE, SCS_ERR_REF, SCS_ERR_COMM, SCS_ERR_CALLBACK = range(8)
SCS_MULTI_HOST_EXCHANGE = 1   # scs_create_multi_ex flag
SCS_CB_F, SCS_CB_GRAD, SCS_CB_HESS, SCS_CB_GGN, SCS_CB_FTEST, SCS_CB_GRAD_X = range(6)
SCS_CB_NO_METHOD = 2   # a callback's answer to SCS_CB_GRAD_X when grad_fx takes no single argument

LOSS = {"logistic_margin": 1, "logistic_ce": 2, "least_squares": 3, "quadratic": 4, "rosenbrock": 5, "callback": 6}
GGN = {None: 0, "sigmoid_ce": 1, "linear_ls": 2}
REG = {"l1": 1, "l2": 2, "indbox": 3, "gl": 4}
SMOOTH = {"phuber_l1l2": 1, "phuber_indbox": 2, "phuber_gl": 3, "exp_indbox": 4, "logexp_indbox": 5, "osba_l1l2": 6,
          "osba_gl": 7}
METHOD = {"nscore": 1, "ggnscore": 2, "lqnscore": 3}
SOLVER = {"default": 0, "reference": 1}

# One HIP runtime per process.  The product needs no torch: without it, libscsopt binds
# /opt/rocm's HIP runtime and RCCL (preloaded RTLD_GLOBAL below).  torch's wheel bundles its own
# copies, whose NEEDED names ("libamdhip64.so") differ from their SONAMEs ("libamdhip64.so.7"):
# a torch imported AFTER /opt/rocm's runtime is bound would load a second runtime.  So when torch
# is already imported (the tests, torch.distributed users), libscsopt's NEEDED entries resolve to
# torch's loaded copies (same SONAMEs) instead, and scsopt.shard refuses to import torch late.
if "torch" in sys.modules:
    RUNTIME = "torch"
else:
    _ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
    for _so in ("libamdhip64.so.7", "librccl.so.1"):
        _p = os.path.join(_ROCM, "lib", _so)
        if os.path.exists(_p):
            C.CDLL(_p, mode=C.RTLD_GLOBAL)
    RUNTIME = "rocm"


def require_torch_runtime(what):
    """torch may join the process only when libscsopt is bound to torch's runtime.  With RUNTIME ==
    "rocm" /opt/rocm's HIP runtime is already bound, and a torch imported since (or imported by the
    caller of `what`) brings its own second copy -- refused either way."""
    if RUNTIME == "rocm":
        late = "torch" in sys.modules
        raise ImportError(f"{what} needs torch, but scsopt was imported first and bound /opt/rocm's HIP runtime"
                          + (" (torch was imported after scsopt: the process now holds two HIP runtimes)"
                             if late else "") + "; import torch before scsopt in a process that uses torch")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libscsopt.so not found at {LIB_PATH}: build it with "
        "`make -C selfconcordantsmoothoptimization.jl_amd/csrc` (there is no CPU fallback)")

lib = C.CDLL(LIB_PATH)

c_dp = C.POINTER(C.c_double)
c_i64p = C.POINTER(C.c_int64)
c_i32p = C.POINTER(C.c_int32)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p)
LOSS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, c_dp, C.c_int64, c_dp)


class Synth(C.Structure):
    _fields_ = [("N_global", C.c_int64), ("row0", C.c_int64), ("N", C.c_int64), ("m", C.c_int64),
                ("seed", C.c_uint64), ("kind", C.c_int), ("density", C.c_double)]


class Timing(C.Structure):
    _fields_ = [("gram_ms", C.c_double), ("gram_calls", C.c_int64),
                ("gemv_ms", C.c_double), ("gemv_calls", C.c_int64),
                ("solve_ms", C.c_double), ("solve_calls", C.c_int64),
                ("step_ms", C.c_double), ("step_calls", C.c_int64),
                ("reduce_ms", C.c_double), ("reduce_calls", C.c_int64)]


class History(C.Structure):
    _fields_ = [("obj", C.POINTER(C.c_double)), ("fval", C.POINTER(C.c_double)),
                ("pri_res_norm", C.POINTER(C.c_double)), ("rel", C.POINTER(C.c_double)),
                ("objrel", C.POINTER(C.c_double)), ("times", C.POINTER(C.c_double)),
                ("fvaltest", C.POINTER(C.c_double))]


_SIGS = {
    "scs_version": (C.c_char_p, []),
    "scs_create": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
    "scs_destroy": (C.c_int, [C.c_void_p]),
    "scs_create_multi": (C.c_int, [c_i32p, C.c_int, C.POINTER(C.c_void_p)]),
    "scs_create_multi_ex": (C.c_int, [c_i32p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "scs_group_size": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "scs_last_error": (C.c_char_p, [C.c_void_p]),
    "scs_get_stream": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "scs_set_comm": (C.c_int, [C.c_void_p, C.c_int, C.c_int, ALLREDUCE_FN, C.c_void_p]),
    "scs_rccl_unique_id": (C.c_int, [C.c_void_p]),
    "scs_set_comm_rccl": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "scs_set_comm_force": (C.c_int, [C.c_void_p, C.c_int]),
    "scs_reduce_buffer_size": (C.c_int, [C.c_void_p, c_i64p]),
    "scs_set_reduce_buffer": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    "scs_comm_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                C.POINTER(C.c_int), C.c_char_p, C.c_int64]),
    "scs_set_data": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, c_dp, C.c_int64, c_dp, C.c_int64, C.c_int64]),
    "scs_gen_data": (C.c_int, [C.c_void_p, C.POINTER(Synth)]),
    "scs_get_data": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, c_dp, C.c_int64, c_dp]),
    "scs_get_dims": (C.c_int, [C.c_void_p, c_i64p, c_i64p, c_i64p, c_i64p]),
    "scs_set_test_data": (C.c_int, [C.c_void_p, C.c_int64, c_dp, C.c_int64, c_dp, C.c_int64, C.c_int64]),
    "scs_set_test_sparse": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, c_i64p, c_i32p, c_dp, C.c_int, c_dp,
                                      C.c_int64, C.c_int64]),
    "scs_gen_test_data": (C.c_int, [C.c_void_p, C.POINTER(Synth)]),
    "scs_set_test_callback": (C.c_int, [C.c_void_p, C.c_int]),
    "scs_eval_ftest": (C.c_int, [C.c_void_p, c_dp, c_dp]),
    "scs_has_test": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "scs_set_sparse": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, c_i64p, c_i32p, c_dp, c_i64p, c_i32p,
                                 c_dp, C.c_int, c_dp, C.c_int64, C.c_int64]),
    "scs_gen_sparse": (C.c_int, [C.c_void_p, C.POINTER(Synth), C.c_int]),
    "scs_get_nnz": (C.c_int, [C.c_void_p, c_i64p]),
    "scs_get_sparse": (C.c_int, [C.c_void_p, c_i64p, c_i32p, c_dp]),
    "scs_set_loss": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double]),
    "scs_set_loss_callback": (C.c_int, [C.c_void_p, LOSS_FN, C.c_void_p, C.c_int64]),
    "scs_set_reg": (C.c_int, [C.c_void_p, C.c_int, c_dp, C.c_int, c_dp, c_dp, C.c_int64, c_i64p, C.c_int64]),
    "scs_set_smoother": (C.c_int, [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_double, c_dp, c_dp,
                                   C.c_int64]),
    "scs_set_L": (C.c_int, [C.c_void_p, C.c_int, C.c_double]),
    "scs_method_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]),
    "scs_eval_f": (C.c_int, [C.c_void_p, c_dp, c_dp]),
    "scs_eval_grad": (C.c_int, [C.c_void_p, c_dp, c_dp]),
    "scs_eval_reg": (C.c_int, [C.c_void_p, c_dp, c_dp]),
    "scs_set_gram_cache": (C.c_int, [C.c_void_p, C.c_int]),
    "scs_set_solver": (C.c_int, [C.c_void_p, C.c_int]),
    "scs_set_compute_f32": (C.c_int, [C.c_void_p, C.c_int]),
    "scs_set_group_map": (C.c_int, [C.c_void_p, c_i64p, C.c_int64]),
    "scs_set_batches": (C.c_int, [C.c_void_p, c_i64p, c_i64p, C.c_int64]),
    "scs_select_batch": (C.c_int, [C.c_void_p, C.c_int64]),
    "scs_step": (C.c_int, [C.c_void_p, c_dp, c_dp, C.c_int64, c_dp, c_dp, c_dp]),
    "scs_step_grad": (C.c_int, [C.c_void_p, c_dp, c_dp, C.c_int64, c_dp, c_dp, c_dp, c_dp]),
    "scs_iterate": (C.c_int, [C.c_void_p, c_dp, c_dp, C.c_int64, C.c_double, C.c_double, C.c_int, c_dp,
                              C.POINTER(History), c_i64p, c_i64p]),
    "scs_iterate_ex": (C.c_int, [C.c_void_p, c_dp, c_dp, C.c_int64, C.c_double, C.c_double, C.c_int, c_dp,
                                 C.POINTER(History), C.c_size_t, c_i64p, c_i64p]),
    "scs_smoother_eval": (C.c_int, [C.c_void_p, c_dp, c_dp, c_dp]),
    "scs_prox_eval": (C.c_int, [C.c_void_p, c_dp, c_dp, C.c_double, C.c_double, c_dp]),
    "scs_gram_eval": (C.c_int, [C.c_void_p, c_dp, c_dp, C.c_int64]),
    "scs_gemv_t_eval": (C.c_int, [C.c_void_p, c_dp, c_dp]),
    "scs_gemv_n_eval": (C.c_int, [C.c_void_p, c_dp, c_dp]),
    "scs_solve_eval": (C.c_int, [C.c_void_p, c_dp, c_dp, c_dp, C.c_int, c_dp, C.POINTER(C.c_int)]),
    "scs_lu_eval": (C.c_int, [C.c_void_p, C.c_int64, c_dp, c_dp, c_dp, c_i32p, C.POINTER(C.c_int)]),
    "scs_get_columns": (C.c_int, [C.c_void_p, c_i64p, C.c_int64, c_dp]),
    "scs_gram_atv_eval": (C.c_int, [C.c_void_p, c_dp, c_dp, c_i64p, C.c_int64, c_dp, c_dp, C.POINTER(C.c_int)]),
    "scs_timing_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "scs_timing_get": (C.c_int, [C.c_void_p, C.POINTER(Timing)]),
    "scs_timing_reset": (C.c_int, [C.c_void_p]),
    "scs_fallback_counts": (C.c_int, [C.c_void_p, c_i64p, C.c_int]),
    "scs_kernel_names": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int64, C.c_char_p, C.c_int64]),
    "scs_sync": (C.c_int, [C.c_void_p]),
}

for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)  # AttributeError here = the .so does not export the header's symbol
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)


class ScsError(RuntimeError):
    """A non-reference failure (HIP, argument, state, communication)."""

    def __init__(self, code, msg):
        super().__init__(f"[scsopt rc={code}] {msg}")
        self.code = code


class ScsReferenceError(ScsError):
    """An error the reference itself raises via Base.error (same message text)."""


def version():
    return lib.scs_version().decode()


def dptr(a):
    """Pointer to a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"], "expected a contiguous float64 array"
    return a.ctypes.data_as(c_dp)


class Context:
    """Owns one scs_ctx: one device and stream (scs_create), or -- devices=[d0, d1, ...] -- one
    process driving several GPUs (scs_create_multi: the library splits the rows across them).
    device_exchange="host": the group's exchange through host memory instead of RCCL
    (SCS_MULTI_HOST_EXCHANGE; devices may repeat a GPU)."""

    def __init__(self, device=0, stream=None, devices=None, device_exchange="rccl"):
        h = C.c_void_p()
        if device_exchange not in ("rccl", "host"):
            raise ValueError("device_exchange is 'rccl' or 'host'")
        if devices is not None:
            devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            flags = SCS_MULTI_HOST_EXCHANGE if device_exchange == "host" else 0
            rc = lib.scs_create_multi_ex(devs, len(devices), flags, C.byref(h))
            if rc != SCS_OK:
                raise ScsError(rc, f"scs_create_multi_ex(devices={list(devices)}, {device_exchange}) failed")
            device = int(devices[0])
        else:
            rc = lib.scs_create(int(device), stream, C.byref(h))
            if rc != SCS_OK:
                raise ScsError(rc, f"scs_create(device={device}) failed")
        self.h = h
        self.device = device
        self.devices = list(devices) if devices is not None else [device]
        self._keep = []  # ctypes callbacks / buffers that must outlive the context
        self._cb_exc = None  # the exception a Python loss callback raised (re-raised by check)

    def check(self, rc):
        if rc != SCS_OK:
            if rc == SCS_ERR_CALLBACK and self._cb_exc is not None:
                exc, self._cb_exc = self._cb_exc, None
                raise exc
            msg = lib.scs_last_error(self.h).decode(errors="replace")
            if rc == SCS_ERR_REF:
                raise ScsReferenceError(rc, msg)
            raise ScsError(rc, msg)

    def close(self):
        if getattr(self, "h", None):
            lib.scs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self):
        s = C.c_void_p()
        self.check(lib.scs_get_stream(self.h, C.byref(s)))
        return s.value

    FALLBACKS = ("lu_coop_refused", "lu_coop_redo", "solve_blocks", "qr_blocks", "chain_redo", "pipe_redo",
                 "qr_coop_refused", "qr_coop_redo")

    def fallback_counts(self):
        """The fallbacks taken instead of failing since the context was created (scs_fallback_counts;
        SCS_FB_* in include/scsopt.h), as {name: count}."""
        n = len(self.FALLBACKS)
        out = (C.c_int64 * n)()
        self.check(lib.scs_fallback_counts(self.h, out, n))
        return dict(zip(self.FALLBACKS, (int(v) for v in out)))

    def kernel_names(self):
        """(main Gram kernel, sparse product kernel) of the latest launches, rocprofv3's names."""
        g, p = C.create_string_buffer(128), C.create_string_buffer(128)
        self.check(lib.scs_kernel_names(self.h, g, 128, p, 128))
        return g.value.decode(), p.value.decode()

    def comm_info(self):
        """What the exchange runs on, read back from the library (scs_comm_info): kind, the
        communicator's own rank count and rank (ncclCommCount / ncclCommUserRank for RCCL), the
        RCCL version and the path of the RCCL library the process resolved."""
        k, n, r, v = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        path = C.create_string_buffer(4096)
        self.check(lib.scs_comm_info(self.h, C.byref(k), C.byref(n), C.byref(r), C.byref(v), path, 4096))
        kinds = {0: "none", 1: "rccl", 2: "callback", 3: "group_rccl", 4: "group_host"}
        return {"kind": kinds.get(k.value, str(k.value)), "nranks": n.value, "rank": r.value,
                "rccl_version": v.value, "rccl_lib": path.value.decode(errors="replace")}

    def timing(self):
        t = Timing()
        self.check(lib.scs_timing_get(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in Timing._fields_}
