"""Generate tests/golden/*.json from the oracle (oracle/scsopt_oracle.py).

Provenance: the reference (Julia) cannot run in this container or on the GPU
box, so these trajectories are produced by the NumPy restatement on the
reference's own test literals (test/test_algs.jl:2-11, 82-96) and the README
Rosenbrock quick start (README.md:43-66, x0 = the test literal).  They are
"restatement of file:line, not reference-executed"; the oracle itself is
pinned by the reference's assertions in tests/test_oracle.py.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import scsopt_oracle as O  # noqa: E402

# ---- literals of test/test_algs.jl ------------------------------------------
LOGI_A = [[-0.560501, 0.0], [0.0, 1.85278], [-0.0192918, -0.827763], [0.128064, 0.110096], [0.0, -0.251176]]
LOGI_Y = [-1, -1, -1, 1, -1]
X0 = [0.5908446386657102, 0.7667970365022592]
HELDOUT_A = [[0.3, -1.1], [-0.7, 0.45], [1.2, 0.05]]   # held-out rows (not from the reference)
HELDOUT_Y = [1, -1, 1]
QP_A = [[1.53976, 0.201833, 0.433995, 0.156497, 0.180124],
        [0.201833, 2.37257, -0.0594941, -0.671533, 0.0739676],
        [0.433995, -0.0594941, 3.15025, 0.808797, 0.954656],
        [0.156497, -0.671533, 0.808797, 2.74361, 0.5621],
        [0.180124, 0.0739676, 0.954656, 0.5621, 1.76141]]
QP_Y = [0.8673472019512456, -0.9017438158568171, -0.4944787535042339, -0.9029142938652416, 0.8644013132535154]
QP_X0 = [-2.07754990163271, -2.311005948690538, -0.25157276401631606, -0.8858618022602884, 1.3116613046047525]
QP_XS = [-0.7139006111210786, 0.642716661564418, 0.3684773651494535, 0.5890487798472874, -0.8324174178513779]


def sol_dict(sol):
    return {"x": [float(v) for v in sol.x], "obj": sol.obj, "fval": sol.fval, "fvaltest": sol.fvaltest,
            "pri_res_norm": sol.pri_res_norm, "rel": sol.rel, "objrel": sol.objrel, "epochs": sol.epochs}


def cases():
    out = {}
    A = np.array(LOGI_A)
    y = np.array(LOGI_Y, dtype=float)
    for mname, mk in (("nscore", O.ProxNSCORE), ("ggnscore", O.ProxGGNSCORE), ("lqnscore", O.ProxLQNSCORE)):
        for reg in ("l1", "l2"):
            model = O.Problem(A, y, X0, O.Loss("logistic_margin", 1 / 5, ggn="sigmoid_ce"), 1)
            sol = O.iterate(mk(), model, reg, O.PHuberSmootherL1L2(1))
            out[f"logistic_{mname}_{reg}"] = sol_dict(sol)
        # the held-out set (problems.jl:27-28,67-68; ftest iterate.jl:169-175, pushed by show_stat!
        # utils.jl:55-57): the reference's tests never pass Atest / ytest, so the held-out rows here are
        # HELDOUT_A / HELDOUT_Y below -- a restatement case, not a reference literal
        model = O.Problem(A, y, X0, O.Loss("logistic_margin", 1 / 5, ggn="sigmoid_ce"), 1,
                          Atest=np.array(HELDOUT_A), ytest=np.array(HELDOUT_Y, dtype=float))
        sol = O.iterate(mk(), model, "l1", O.PHuberSmootherL1L2(1))
        out[f"logistic_{mname}_l1_heldout"] = sol_dict(sol)
    Aq = np.array(QP_A)
    for sname, sm, alpha in (("phuber", O.PHuberSmootherIndBox(-1.0, 1.0, 0.6), 0.8),
                             ("exp", O.ExponentialSmootherIndBox(-1.0, 1.0, 0.6), 1.0)):
        model = O.Problem(Aq, np.array(QP_Y), QP_X0, O.Loss("quadratic"), 1.0e-4, C_set=[-1.0, 1.0],
                          sol=np.array(QP_XS))
        sol = O.iterate(O.ProxNSCORE(), model, "indbox", sm, alpha=alpha)
        out[f"boxqp_nscore_{sname}"] = sol_dict(sol)
    model = O.Problem(None, None, X0, O.Loss("rosenbrock"), 1e-8)
    sol = O.iterate(O.ProxLQNSCORE(m=10), model, "l1", O.PHuberSmootherL1L2(1.0))
    out["rosenbrock_lqnscore_l1"] = sol_dict(sol)
    return out


def kernels():
    """Per-kernel vectors: smoother and prox on fixed inputs (x, z, Hr chosen to hit the branches)."""
    rng = np.random.default_rng(20240917)
    x = np.concatenate([[-2.0, -1.0, 0.0, -0.0, 1.0, 2.0, 1e-300, -1e-300, 0.5, -0.5],
                        rng.standard_normal(54)])
    k = {"x": x.tolist()}
    k["phuber_l1l2_mu1"] = {"grad": O.huber_grad(x, 1.0).tolist(), "hess": O.huber_hess(x, 1.0).tolist()}
    k["phuber_l1l2_mu0.3"] = {"grad": O.huber_grad(x, 0.3).tolist(), "hess": O.huber_hess(x, 0.3).tolist()}
    k["phuber_indbox_mu0.6"] = {"grad": O.huber_grad_indbox(x, 0.6, -1.0, 1.0).tolist(),
                                "hess": O.huber_hess_indbox(x, 0.6, -1.0, 1.0).tolist()}
    k["exp_indbox_mu0.6"] = {"grad": (-np.exp((-x + -1.0) / 0.6)).tolist(),
                             "hess": (1.0 / 0.6 * np.exp((-x + -1.0) / 0.6)).tolist()}
    Hr = np.abs(rng.standard_normal(x.size)) + 0.1
    z = x * 0.7
    k["prox_in"] = {"z": z.tolist(), "Hr": Hr.tolist(), "lam": 0.3, "alpha": 0.5}
    hinv = 1.0 / Hr
    k["prox_l1"] = O.prox_l1(z, hinv, 0.3, 0.5).tolist()
    k["prox_l2"] = O.prox_l2(z, hinv, 0.3, 0.5).tolist()
    k["get_Mg"] = {str(n): O.get_Mg(2.0, 2.6, 1.0, n) for n in (2, 8192, 16384, 65536)}
    return k


def hexify(o):
    """Exact float round-trip: store floats as repr strings (json floats are repr already)."""
    return o


if __name__ == "__main__":
    data = {"provenance": "oracle/scsopt_oracle.py restatement of the reference (Julia absent); "
                          "inputs are the literals of test/test_algs.jl and README.md",
            "cases": cases(), "kernels": kernels()}
    with open(os.path.join(HERE, "reference_tests.json"), "w") as f:
        json.dump(data, f, indent=1, allow_nan=True)
    print("wrote", os.path.join(HERE, "reference_tests.json"))
