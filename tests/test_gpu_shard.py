"""GPU: the row-sharded path end to end on one device.

Two processes share cuda:0; each holds its row block of A (generated in place),
and libscsopt's all-reduce callback runs torch.distributed.all_reduce (gloo
backend here, which reduces device tensors; RCCL/"nccl" on a multi-GPU node).
The sharded trajectories must equal the single-process trajectory of the full
problem to fp64 tolerance (only the reduction order differs) and be identical
on both ranks.
"""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, M = 3001, 192
NS = 151          # sample-space case: N + 1 <= M
METHODS = ("ggn", "nscore", "lqn", "ggn_ls_cached", "ggn_sample", "ggn_batch", "nscore_batch_ordered",
           "ggn_sample_batch", "ggn_ls_gl", "ggn_sample_rebatch")
GS = 32           # ggn_ls_gl: C4's sparse-group lasso (groups of 32) on the row shards


def _run(method, comm=None):
    import scsopt
    from scsopt import losses
    x0 = np.random.default_rng(1234).standard_normal(M)
    if method == "ggn":
        f, out, kind = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N), 1
        meth = scsopt.ProxGGNSCORE()
    elif method == "nscore":
        f, out, kind = losses.logistic_margin(1.0 / N), None, 2
        meth = scsopt.ProxNSCORE()
    elif method == "ggn_sample":   # N + 1 <= m: the sharded sample-space branch (row all-gather)
        f, out, kind = losses.logistic_ce(1.0 / NS), losses.sigmoid_ce(1.0 / NS), 1
        meth = scsopt.ProxGGNSCORE()
        p = scsopt.Problem.synthetic(NS, M, x0, f, 2e-3, kind=kind, seed=13, out_fn=out, comm=comm)
        sol = scsopt.iterate(meth, p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=6, verbose=0)
        return {"obj": list(sol.obj), "x": sol.x.copy(), "epochs": sol.epochs}
    elif method in ("ggn_batch", "nscore_batch_ordered", "ggn_sample_batch"):
        # minibatches over the row shards (iterate.jl:125-146): global batch rows, each rank keeps
        # its own; the unshuffled 1000-row batches leave some ranks with no rows of a batch, and the
        # 48-row batches of the 151-row problem take the sample-space branch (per-batch row gather)
        n = NS if method == "ggn_sample_batch" else N
        if method == "nscore_batch_ordered":
            f, out, kind, meth = losses.logistic_margin(1.0 / n), None, 2, scsopt.ProxNSCORE()
        else:
            f, out, kind, meth = losses.logistic_ce(1.0 / n), losses.sigmoid_ce(1.0 / n), 1, scsopt.ProxGGNSCORE()
        p = scsopt.Problem.synthetic(n, M, x0, f, 2e-3, kind=kind, seed=19, out_fn=out, comm=comm)
        bs = 48 if method == "ggn_sample_batch" else 1000
        sol = scsopt.iterate(meth, p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=4, verbose=0, batch_size=bs,
                             shuffle_batch=method != "nscore_batch_ordered",
                             batch_perm=np.random.default_rng(3).permutation(n))
        return {"obj": list(sol.obj), "x": sol.x.copy(), "epochs": sol.epochs}
    elif method == "ggn_sample_rebatch":
        # two iterate! calls, each registering ONE batch (local_max_iter = 1) of another shuffle:
        # batch index 0 names different rows in the second list, so the all-gathered rows of the
        # first (the sharded sample-space view) must not be reused
        f, out = losses.logistic_ce(1.0 / NS), losses.sigmoid_ce(1.0 / NS)
        p = scsopt.Problem.synthetic(NS, M, x0, f, 2e-3, kind=1, seed=29, out_fn=out, comm=comm)
        objs, xs = [], []
        for seed in (3, 4):
            sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "l1", scsopt.PHuberSmootherL1L2(1.0), verbose=0,
                                 batch_size=48, local_max_iter=1,
                                 batch_perm=np.random.default_rng(seed).permutation(NS))
            objs += list(sol.obj)
            xs.append(sol.x.copy())
        return {"obj": objs, "x": np.concatenate(xs), "epochs": sol.epochs}
    elif method == "ggn_ls_gl":
        # C4 (BASELINE configs[3]) in miniature: least squares + l1/group lasso, PHuberSmootherGL(1e-2)
        # -- the GL smoother's global dot(Dg, Dg) and the group prox run redundantly on every rank
        f, out = losses.least_squares(1.0 / N), losses.linear_ls(1.0 / N)
        ng = M // GS
        p = scsopt.Problem.synthetic(N, M, x0, f, 1.0, kind=3, seed=23, out_fn=out, comm=comm)
        ind = np.array([[1 + GS * g for g in range(ng)], [GS * (g + 1) for g in range(ng)], [1] * ng])
        p.P = scsopt.get_P(M, np.arange(1, M + 1), ind)
        p.λ = [1e-8, 0.02]
        sol = scsopt.iterate(scsopt.ProxGGNSCORE(), p, "gl", scsopt.PHuberSmootherGL(1e-2, p), max_epoch=6,
                             verbose=0)
        return {"obj": list(sol.obj), "x": sol.x.copy(), "epochs": sol.epochs}
    elif method == "ggn_ls_cached":
        f, out, kind = losses.least_squares(1.0 / N), losses.linear_ls(1.0 / N), 3
        meth = scsopt.ProxGGNSCORE()
    else:
        f, out, kind = losses.least_squares(1.0 / N), None, 3
        meth = scsopt.ProxLQNSCORE(m=5)
    p = scsopt.Problem.synthetic(N, M, x0, f, 2e-3, kind=kind, seed=11, out_fn=out, comm=comm)
    if method == "ggn_ls_cached" and comm is not None:   # sharded: Gram reused, only ∇f all-reduced
        p.set_gram_cache(True)
    sol = scsopt.iterate(meth, p, "l1", scsopt.PHuberSmootherL1L2(1.0), max_epoch=6, verbose=0)
    return {"obj": list(sol.obj), "x": sol.x.copy(), "epochs": sol.epochs}


def _worker(rank, world, store_path, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "selfconcordantsmoothoptimization.jl_amd"))
    import torch
    import torch.distributed as dist
    from scsopt import shard
    # a FileStore rendezvous: no TCP port to race the host's other jobs for (a free port picked
    # and released can be taken before rank 0 listens on it: EADDRINUSE)
    dist.init_process_group("gloo", store=dist.FileStore(store_path, world), rank=rank, world_size=world)
    res = {}
    for method in METHODS:
        comm = shard.Comm(device=torch.device("cuda", 0))
        res[method] = _run(method, comm)
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tall", [(2, "0"), (2, "1"), (4, "1")])
def test_two_rank_shard_matches_single_process(world, tall, monkeypatch, tmp_path):
    """tall = "1" forces the 256 x 128 Gram kernel (the C3 kernel) at this small m, so the packed
    multi-rank slots of its tile halves (gram_unpack) are exercised too; world = 4 splits the 3001
    rows unevenly (751/750/750/750) and the 151-row sample-space case into 38/38/38/37.  The
    *_batch cases run minibatches over the shards (global batch rows; ranks without rows of a
    batch contribute zero) against the one-process run of the same batch list."""
    monkeypatch.setenv("SCS_GRAM_TALL", tall)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, str(tmp_path / "store"), out), nprocs=world, join=True)
    for method in METHODS:
        full = _run(method)
        r0 = out[0][method]
        for r in range(1, world):
            rr = out[r][method]
            assert rr["epochs"] == r0["epochs"] == full["epochs"], method
            assert rr["obj"] == r0["obj"], (method, r, rr["obj"], r0["obj"], full["obj"])   # identical bits
            assert np.array_equal(rr["x"], r0["x"]), method
        np.testing.assert_allclose(r0["obj"], full["obj"], rtol=1e-10, err_msg=method)
        np.testing.assert_allclose(r0["x"], full["x"], rtol=1e-8, atol=1e-12, err_msg=method)
