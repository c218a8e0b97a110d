"""ProximalMethod types (src/algorithms/prox-*-SCORE.jl).

The structs keep the reference's fields and defaults; their ``step!`` runs
inside libscsopt (scs_step).  ``set_name`` / ``init`` mirror ``set_name!`` /
``init!``.
"""
from __future__ import annotations

from dataclasses import dataclass


class ProximalMethod:
    code = 0

    def set_name(self, implemented_algs):
        """set_name! (e.g. prox-GGN-SCORE.jl:24-33)."""
        if not self.use_prox:
            self.name = self._plain_name
            self.label = self._plain_label
        implemented_algs.append(self.name)
        return self


@dataclass
class ProxNSCORE(ProximalMethod):
    """prox-N-SCORE.jl:6-22."""
    ss_type: int = 1
    use_prox: bool = True
    name: str = "prox-newtonscore"
    label: str = "Prox-N-SCORE"
    code = 1
    _plain_name = "newtonscore"
    _plain_label = "Newton-SCORE"


@dataclass
class ProxGGNSCORE(ProximalMethod):
    """prox-GGN-SCORE.jl:6-22."""
    ss_type: int = 1
    use_prox: bool = True
    name: str = "prox-ggnscore"
    label: str = "Prox-GGN-SCORE"
    code = 2
    _plain_name = "ggnscore"
    _plain_label = "GGN-SCORE"


@dataclass
class ProxLQNSCORE(ProximalMethod):
    """prox-L-BFGS-SCORE.jl:6-30 (m = memory size; s_list/y_list/H0 live on the device)."""
    ss_type: int = 1
    use_prox: bool = True
    m: int = 10
    H0: float = 1.0
    name: str = "prox-lbfgsscore"
    label: str = "Prox-LBFGS-SCORE"
    code = 3
    _plain_name = "lbfgsscore"
    _plain_label = "LBFGS-SCORE"
