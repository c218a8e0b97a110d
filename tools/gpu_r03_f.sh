#!/bin/bash
# r03: the reference solver mode (Householder QR) -- kernel-level vs LAPACK, trajectories vs the
# oracle's literal QR, the ill-conditioned C4-like system; then the QR solve's time at m = 8192.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity.py::test_householder_qr_solve" "tests/test_gpu_parity.py::test_reference_solver_trajectory" \
  "tests/test_gpu_parity.py::test_reference_solver_ill_conditioned" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^\[qr\]|passed|failed|Error" $O/pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 - > $O/qr_time.log 2>&1 <<'PY'
import sys, time, numpy as np
sys.path.insert(0, "selfconcordantsmoothoptimization.jl_amd")
import scsopt
from scsopt import losses
for m in (2048, 8192):
    N = m + 512
    p = scsopt.Problem.synthetic(N, m, np.zeros(m), losses.least_squares(1.0 / N), 1.0, kind=3, seed=5)
    rng = np.random.default_rng(6)
    w = (rng.random(N) + 0.5) / N; d = (rng.random(m) + 0.5) * 1e-2; rhs = rng.standard_normal(m)
    for mode in (0, 2, 2):
        t0 = time.perf_counter(); x, _ = p.solve_eval(w, d, rhs, mode=mode); t = time.perf_counter() - t0
        r = p.gemv_t(w * p.gemv_n(x)) + d * x - rhs
        print(f"m={m} mode={mode} wall={t*1e3:.1f} ms  |r|/|b| = {np.linalg.norm(r)/np.linalg.norm(rhs):.2e}")
    p.ctx.close()
PY
rc=$?; echo "qr timing rc=$rc"; cat $O/qr_time.log | grep "m="
