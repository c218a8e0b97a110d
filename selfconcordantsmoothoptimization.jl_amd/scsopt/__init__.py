"""scsopt -- MI355X-native SCORE inner iteration with the API of
SelfConcordantSmoothOptimization.jl (Problem / iterate! / smoothers / methods).

    from scsopt import *
    model = Problem(A, y, x0, losses.logistic_margin(1/5), 1.0, out_fn=losses.sigmoid_ce(1/5))
    sol = iterate(ProxGGNSCORE(), model, "l1", PHuberSmootherL1L2(1.0))

All compute runs in libscsopt.so (HIP, gfx950); importing the package fails if
the library has not been built.
"""
from . import _lib, losses, shard
from ._lib import ScsError, ScsReferenceError, version
from .iterate import Solution, iterate, optim_loop, step
from .methods import ProximalMethod, ProxGGNSCORE, ProxLQNSCORE, ProxNSCORE
from .problems import Problem, get_P, lu_solve
from .smoothers import (ExponentialSmootherIndBox, LogExpSmootherIndBox, OsBaSmootherGL, OsBaSmootherL1L2,
                        PHuberSmootherGL, PHuberSmootherIndBox, PHuberSmootherL1L2, Smoother)

__all__ = ["Problem", "get_P", "iterate", "optim_loop", "step", "Solution", "ProximalMethod", "ProxNSCORE",
           "ProxGGNSCORE", "ProxLQNSCORE", "PHuberSmootherL1L2", "PHuberSmootherIndBox", "PHuberSmootherGL",
           "ExponentialSmootherIndBox", "LogExpSmootherIndBox", "OsBaSmootherL1L2", "OsBaSmootherGL", "Smoother",
           "losses", "shard", "ScsError", "ScsReferenceError", "version"]
