"""Smoother types (src/regularizers/{phuber,exponential,log-exp,ostrovskii-bach}-smooth.jl).

Each smoother carries the fields the algorithms read -- ``μ``, ``Mh``, ``ν``
(get_Mg, smoothing.jl:12-25) -- and a kind tag; its grad/hess run on the
device (csrc/vec.hip).  ``grad(problem, x)`` / ``hess(problem, x)`` evaluate
them through the C ABI for inspection and tests.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Optional

import numpy as np

HUBER_MH = 2.0   # phuber-smooth.jl:3  (huber_smooth_Mh)
HUBER_NU = 2.6   # phuber-smooth.jl:4  (huber_smooth_ν)
EXP_MH = 1.0     # exponential-smooth.jl:25
EXP_NU = 2.0     # exponential-smooth.jl:26
LOGEXP_MH = 1.0  # log-exp-smooth.jl:25
LOGEXP_NU = 2.0  # log-exp-smooth.jl:26
OSBA_MH = 2 * np.sqrt(2)   # ostrovskii-bach-smooth.jl:3
OSBA_NU = 3.0              # ostrovskii-bach-smooth.jl:4


@dataclass
class Smoother:
    kind: str
    mu: float
    Mh: float
    nu: float
    lb: Any = None
    ub: Any = None
    problem: Any = None

    # Julia field spellings
    @property
    def μ(self):
        return self.mu

    @property
    def ν(self):
        return self.nu

    def grad(self, problem, x):
        return problem._smoother_eval(self, x)[0]

    def hess(self, problem, x):
        return problem._smoother_eval(self, x)[1]


def PHuberSmootherL1L2(mu) -> Smoother:
    """phuber-smooth.jl:27."""
    return Smoother("phuber_l1l2", float(mu), HUBER_MH, HUBER_NU)


def PHuberSmootherIndBox(lb, ub, mu) -> Smoother:
    """phuber-smooth.jl:59-65."""
    return Smoother("phuber_indbox", float(mu), HUBER_MH, HUBER_NU, lb=lb, ub=ub)


def ExponentialSmootherIndBox(lb, ub, mu) -> Smoother:
    """exponential-smooth.jl:28-34."""
    return Smoother("exp_indbox", float(mu), EXP_MH, EXP_NU, lb=lb, ub=ub)


def PHuberSmootherGL(mu, problem) -> Smoother:
    """phuber-smooth.jl:137-148 (reads problem.λ and problem.P; λ1/λ2 unused by grad/hess)."""
    if problem.P is None:
        raise ValueError("PHuberSmootherGL needs a problem with group structure P (get_P)")
    return Smoother("phuber_gl", float(mu), HUBER_MH, HUBER_NU, problem=problem)


def LogExpSmootherIndBox(lb, ub, mu) -> Smoother:
    """log-exp-smooth.jl:28-34."""
    return Smoother("logexp_indbox", float(mu), LOGEXP_MH, LOGEXP_NU, lb=lb, ub=ub)


def OsBaSmootherL1L2(mu) -> Smoother:
    """ostrovskii-bach-smooth.jl:27 (grad/hess are 0/0 = NaN at x = 0, propagated as the reference does)."""
    return Smoother("osba_l1l2", float(mu), OSBA_MH, OSBA_NU)


def OsBaSmootherGL(mu, problem) -> Smoother:
    """ostrovskii-bach-smooth.jl:59-71 (reads problem.λ and problem.P)."""
    if problem.P is None:
        raise ValueError("OsBaSmootherGL needs a problem with group structure P (get_P)")
    return Smoother("osba_gl", float(mu), OSBA_MH, OSBA_NU, problem=problem)


def bounds_array(b, m):
    a = np.atleast_1d(np.asarray(b, dtype=np.float64))
    if a.size not in (1, m):
        raise ValueError("Lengths of the bounds do not match that of the variable.")
    return np.ascontiguousarray(a)
