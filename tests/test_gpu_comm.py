"""GPU: the row-shard exchange on the real communicator stack, at world size 1.

A one-GPU box cannot run two RCCL ranks (RCCL refuses two ranks on one device), so the
exchange path is forced at one rank (scs_set_comm_force): packed Gram tiles -> all-reduce ->
unpack (for a sparse A: the nnz-priced Gram packed into the slots), the scalar loss and m-vector
sums, and the sample-space row all-gather all go through
(a) libscsopt's own RCCL communicator (ncclAllReduce on the context stream; the unique id
travels over torch.distributed) and (b) the torch.distributed "nccl" callback.  A one-rank sum
is the identity, so every trajectory must be BIT-identical to the unsharded run.  Each case
runs in a child process (its own process group).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch, torch.distributed as dist
import scsopt
from scsopt import losses, shard
mode, method = sys.argv[2], sys.argv[3]
torch.cuda.set_device(0)
# one rank: a FileStore rendezvous (no TCP port to race other jobs on the host for)
store = dist.FileStore(sys.argv[4], 1)
dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
N, m = {"ggn_sample": (151, 192), "ggn_sparse": (4096, 256)}.get(method, (3001, 256))
x0 = np.random.default_rng(1234).standard_normal(m)
if method in ("ggn", "ggn_sample"):
    f, out, kind, M = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N), 1, scsopt.ProxGGNSCORE
elif method == "ggn_sparse":   # the nnz-priced sparse Gram, packed into the exchange (gram_pack_launch)
    f, out, kind, M = losses.least_squares(1.0 / N), losses.linear_ls(1.0 / N), None, scsopt.ProxGGNSCORE
elif method == "nscore":
    f, out, kind, M = losses.logistic_margin(1.0 / N), None, 2, scsopt.ProxNSCORE
else:
    f, out, kind, M = losses.least_squares(1.0 / N), None, 3, scsopt.ProxLQNSCORE
res = {}
for tag in ("plain", "exchange"):
    comm = None
    if tag == "exchange":
        comm = shard.Comm(device=torch.device("cuda", 0), native=(mode == "rccl"), force=True)
    if kind is None:
        p = scsopt.Problem.synthetic_sparse(N, m, x0, f, 2e-3, density=0.05, seed=5, out_fn=out, comm=comm)
    else:
        p = scsopt.Problem.synthetic(N, m, x0, f, 2e-3, kind=kind, seed=5, out_fn=out, comm=comm)
    sol = scsopt.iterate(M(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=5, x_tol=0.0, f_tol=0.0,
                         verbose=0)
    tm = p.ctx.timing()
    res[tag] = {"obj": sol.obj, "x": sol.x.tolist(), "epochs": sol.epochs, "gram": p.ctx.kernel_names()[0]}
dist.destroy_process_group()
print("RESULT " + json.dumps(res))
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["rccl", "torch"])
@pytest.mark.parametrize("method", ["ggn", "nscore", "lqn", "ggn_sample", "ggn_sparse"])
def test_forced_exchange_bit_identical(mode, method, tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    pkg = os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd")
    store = str(tmp_path / "store")
    out = subprocess.run([sys.executable, "-c", _CHILD, pkg, mode, method, store], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    import json
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[7:])
    a, b = res["plain"], res["exchange"]
    assert a["epochs"] == b["epochs"]
    assert a["obj"] == b["obj"]
    assert np.array_equal(np.array(a["x"]).view(np.int64), np.array(b["x"]).view(np.int64))
    if method == "ggn_sparse":
        assert b["gram"].startswith("sparse_gram_seg_kernel<"), b["gram"]
