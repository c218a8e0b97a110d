"""Loss kinds: the closed-form stand-ins for the reference's user callbacks.

In the reference a problem carries Julia closures ``f(A, y, x)`` (and, for
ProxGGNSCORE, ``out_fn(A, x)`` plus a second method ``f(y, ŷ)``) whose
derivatives come from ForwardDiff or from user-supplied ``grad_fx``/
``hess_fx``/``jac_yx``/``grad_fy``/``hess_fy`` (problems.jl:21-40,61-81).
On the device the callbacks become a fixed menu of loss kinds evaluated by
HIP kernels; each kind states the reference expression it reproduces.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional


@dataclass(frozen=True)
class Loss:
    """x-form objective f(A, y, x)."""
    kind: str
    scale: float = 1.0

    def __repr__(self):
        return f"{self.kind}(scale={self.scale!r})"


@dataclass(frozen=True)
class OutFn:
    """out_fn(A, x) paired with its ŷ-form loss f(y, ŷ) (ProxGGNSCORE)."""
    kind: str
    scale: float = 1.0


def logistic_margin(scale: float = 1.0) -> Loss:
    """f(A,y,x) = scale*sum(log.(1 .+ exp.(-y .* (A*x))))   (test/test_algs.jl:9, README.md:113)."""
    return Loss("logistic_margin", float(scale))


def logistic_ce(scale: float = 1.0) -> Loss:
    """f(A,y,x) = f(y, σ(A*x)) with the cross-entropy f(y,ŷ) of test/test_algs.jl:10."""
    return Loss("logistic_ce", float(scale))


def least_squares(scale: float = 1.0) -> Loss:
    """f(A,y,x) = 0.5*sum((A*x .- y).^2)*scale   (README.md:212-214 with scale = 1/m)."""
    return Loss("least_squares", float(scale))


def quadratic() -> Loss:
    """f(A,y,x) = 1/2*(x'*(A*x)) + (y'*x)   (test/test_algs.jl:90; A is m x m)."""
    return Loss("quadratic", 1.0)


def rosenbrock() -> Loss:
    """f(x) = Σ 100(x[i+1]-x[i]^2)^2 + (1-x[i])^2   (README.md:49; ProblemGeneric, no data)."""
    return Loss("rosenbrock", 1.0)


@dataclass(frozen=True, eq=False)
class CallbackLoss(Loss):
    """The caller's own closures, evaluated on the host (SCS_LOSS_CALLBACK)."""
    f: Optional[Callable] = field(default=None, repr=False)
    grad_fx: Optional[Callable] = field(default=None, repr=False)
    hess_fx: Optional[Callable] = field(default=None, repr=False)
    out_fn: Optional[Callable] = field(default=None, repr=False)
    jac_yx: Optional[Callable] = field(default=None, repr=False)
    grad_fy: Optional[Callable] = field(default=None, repr=False)
    hess_fy: Optional[Callable] = field(default=None, repr=False)

    @property
    def has_ggn(self):
        return None not in (self.out_fn, self.jac_yx, self.grad_fy, self.hess_fy)


def callback(f, grad_fx=None, hess_fx=None, *, out_fn=None, jac_yx=None, grad_fy=None,
             hess_fy=None) -> CallbackLoss:
    """A user loss outside the menu: Problem(x0, f, λ; grad_fx, hess_fx) (problems.jl:44-59, f(x))
    or Problem(A, y, x0, f, λ; grad_fx, hess_fx, out_fn, jac_yx, grad_fy, hess_fy) (:61-81,
    f(A, y, x)), the reference's own keyword callbacks (prox-N-SCORE.jl:49-56,
    prox-L-BFGS-SCORE.jl:85-91, prox-GGN-SCORE.jl:44-49).  They run on the host with NumPy
    arrays; the smoother, the Gram / m x m solve or the sample-space system, damping, prox and the
    loop stay on the device.  There is no automatic differentiation here (the reference falls
    back to ForwardDiff): ProxLQNSCORE needs grad_fx, ProxNSCORE grad_fx and hess_fx,
    ProxGGNSCORE out_fn(A, x), jac_yx(A, y, ŷ, x) (rows = vec(ŷ), column-major for a
    multi-output ŷ), grad_fy(A, y, ŷ) and hess_fy(A, y, ŷ) (a vector = diagonal Q, or a
    symmetric matrix) plus grad_fx for the line search."""
    return CallbackLoss("callback", 1.0, f, grad_fx, hess_fx, out_fn, jac_yx, grad_fy, hess_fy)


def sigmoid_ce(scale: float = 1.0) -> OutFn:
    """Mfunc(A,x) = 1 ./ (1 .+ exp.(-A*x)) with f(y,ŷ) = -scale*sum(y.*log.(ŷ) .+ (1 .- y).*log.(1 .- ŷ))
    (test/test_algs.jl:10-11, README.md:135-139)."""
    return OutFn("sigmoid_ce", float(scale))


def linear_ls(scale: float = 1.0) -> OutFn:
    """out_fn(A,x) = A*x with f(y,ŷ) = 0.5*sum((ŷ .- y).^2)*scale   (README.md:233-239)."""
    return OutFn("linear_ls", float(scale))


def ggn_kind(out_fn: Optional[OutFn]):
    return None if out_fn is None else out_fn.kind
