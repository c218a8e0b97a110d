"""bench.py -- iterate!() iterations/s on the BASELINE configurations.

Default (the driver's line): BASELINE.json configs[2] -- ProxGGNSCORE sparse
logistic regression, N = 2^20 samples x m = 2^14 features, fp64, A ~ N(0,1)/sqrt(m)
generated on the device (synthetic; no dataset), y ~ Bernoulli(σ(A x_true)) ∈ {0,1},
x_true 10 % dense, l1 with λ = 0.1·‖∇f(0)‖∞, PHuberSmootherL1L2(μ = 1),
ProxGGNSCORE(ss_type = 1), f(A,y,x) = CE(y, σ(Ax)) with scale 1/N.

One "step" = one iterate! epoch: f(x) + get_reg(x) + step! (for GGN: J/residual/Q
from σ(Ax), the MFMA Gram JᵀQJ = Aᵀ diag(s²q) A, Jᵀr, λ·diag(Hr), the m x m
Cholesky solve, SCORE damping and the prox).  N GPUs: A is row-sharded (strong
scaling: the global problem is fixed), one all-reduce per step.  The timed region
is ONE iterate!(max_epoch = K) call run inside libscsopt (scs_iterate: init!,
f(x*) + get_reg(x*) once, K epochs with the history bookkeeping), after a
separate warm-up call of W epochs; value = K / its wall time.

Other configs (--config): c1 Rosenbrock ProxLQNSCORE (configs[0]), c2 ProxNSCORE
logistic N=100k m=8k (configs[1]), c4 ProxGGNSCORE sparse-group lasso N=4M m=32k
(configs[3]; needs >= 4 GPUs at full size).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
    torchrun --nproc-per-node N bench.py --gpus N ...

Multi-GPU: under torchrun / torch.distributed.run (WORLD_SIZE set) every process is
one rank and WORLD_SIZE must equal --gpus.  Without WORLD_SIZE, --gpus N > 1 starts
the N rank processes itself (launch_ranks) before anything touches a GPU and exits
with the worst rank's status.  --comm picks the exchange and the process group:
rccl -> libscsopt's own RCCL communicator, "nccl" group (one GPU per rank);
torch -> torch.distributed.all_reduce over a "gloo" group, which also runs with
--share-device (ranks round-robin over fewer GPUs, to exercise the launcher on a
one-GPU box; the line then says so in "devices").
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix, AMD spec; 64 cycles/MFMA confirmed by PMC
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "t_iter_s", "reps", "stat", "threads_note")
METRIC = "iterate!() iterations/sec + achieved HBM GB/s, ProxGGNSCORE n=1M m=16k"

CONFIGS = {
    "c1": dict(method="lqn", loss="rosenbrock", N=0, m=2, reg="l1", lam=1e-8, mu=1.0, mem=10,
               workload="ProxLQNSCORE Rosenbrock + l1, BASELINE configs[0]"),
    "c2": dict(method="nscore", loss="logistic_margin", kind=2, N=100_000, m=8192, reg="l1", lam_frac=0.1, mu=1.0,
               workload="ProxNSCORE sparse-logistic (margin form) l1, BASELINE configs[1]"),
    "c3": dict(method="ggn", loss="logistic_ce", kind=1, N=1 << 20, m=1 << 14, reg="l1", lam_frac=0.1, mu=1.0,
               workload="ProxGGNSCORE sparse-logistic l1, BASELINE configs[2]"),
    "c4": dict(method="ggn", loss="least_squares", kind=3, N=1 << 22, m=1 << 15, reg="gl", lam1=1e-8, lam_frac=0.1,
               mu=1e-2, group=32, workload="ProxGGNSCORE sparse-group lasso (l1 + gl), BASELINE configs[3]"),
    "c5": dict(method="lqn", loss="least_squares", sparse=True, N=1 << 20, m=1 << 16, rho=0.01, reg="indbox",
               lam=1e-4, mu=0.6, mem=20,
               workload="ProxLQNSCORE(mem=20) box-constrained least squares, sparse A (CSR+CSC, rho=0.01), "
                        "indbox + PHuberSmootherIndBox, BASELINE configs[4]"),
    # the C5-shaped sparse A under ProxGGNSCORE (README.md:105's sprandn problem class with the GGN step):
    # the Gram priced by nnz (sparse_gram_kernel) + the m = 65536 Cholesky
    "c5ggn": dict(method="ggn", loss="least_squares", sparse=True, N=1 << 20, m=1 << 16, rho=0.01, reg="indbox",
                  lam=1e-4, mu=0.6,
                  workload="ProxGGNSCORE box-constrained least squares on the C5 sparse A (rho=0.01): sparse Gram "
                           "Jt*Q*Jt' priced by nnz + m=65536 Cholesky"),
}


def build_problem(cfg, N, m, comm, local, f32=False, devices=None, device_exchange="rccl"):
    import numpy as np
    import scsopt
    from scsopt import losses
    x0 = np.random.default_rng(1234).standard_normal(m)
    if cfg["loss"] == "rosenbrock":
        x0 = np.array([0.5908446386657102, 0.7667970365022592])
        model = scsopt.Problem(x0, losses.rosenbrock(), cfg["lam"], device=local)
        return model, scsopt.PHuberSmootherL1L2(cfg["mu"]), scsopt.ProxLQNSCORE(m=cfg["mem"])
    out = None
    if cfg.get("sparse"):
        ggn = cfg["method"] == "ggn"
        model = scsopt.Problem.synthetic_sparse(N, m, x0, losses.least_squares(1.0 / N), cfg["lam"],
                                                density=cfg["rho"], seed=2026, f32=f32, device=local,
                                                C_set=[-1.0, 1.0],
                                                out_fn=losses.linear_ls(1.0 / N) if ggn else None)
        meth = scsopt.ProxGGNSCORE() if ggn else scsopt.ProxLQNSCORE(m=cfg["mem"])
        return model, scsopt.PHuberSmootherIndBox(-1.0, 1.0, cfg["mu"]), meth
    if cfg["loss"] == "logistic_ce":
        f, out = losses.logistic_ce(1.0 / N), losses.sigmoid_ce(1.0 / N)
    elif cfg["loss"] == "logistic_margin":
        f = losses.logistic_margin(1.0 / N)
    else:
        f, out = losses.least_squares(1.0 / N), losses.linear_ls(1.0 / N)
    model = scsopt.Problem.synthetic(N, m, x0, f, 1.0, kind=cfg["kind"], seed=2026, density=0.1, out_fn=out,
                                     device=local, comm=comm, devices=devices, device_exchange=device_exchange)
    g0 = model.gradx(np.zeros(m))
    if cfg["reg"] == "gl":
        gs = cfg["group"]
        ng = m // gs
        ind = np.array([[1 + gs * g for g in range(ng)], [gs * (g + 1) for g in range(ng)], [1] * ng])
        model.P = scsopt.get_P(m, np.arange(1, m + 1), ind)
        gmax = float(np.max(np.linalg.norm(g0.reshape(ng, gs), axis=1)))
        model.λ = [cfg["lam1"], cfg["lam_frac"] * gmax]
        hmu = scsopt.PHuberSmootherGL(cfg["mu"], model)
    else:
        model.λ = cfg["lam_frac"] * float(np.max(np.abs(g0)))
        hmu = scsopt.PHuberSmootherL1L2(cfg["mu"])
    meth = {"ggn": scsopt.ProxGGNSCORE, "nscore": scsopt.ProxNSCORE, "lqn": scsopt.ProxLQNSCORE}[cfg["method"]]()
    return model, hmu, meth


def sampled_gram_check(model, m, seed=7, ncols=8):
    """Full-size parity property of the dominant kernel: the production Gram launch (with the Aᵀv
    fused where a step fuses it) against host fp64 dot products of columns read back from the
    device, for all pairs of `ncols` random columns and their Aᵀv entries; bound 1e-11·Σ|terms|
    (summation order differs; a wrong tile / weight / panel is an O(1) error)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    N = model.N
    cols = np.sort(rng.choice(m, ncols, replace=False))
    w = rng.random(N) + 0.5
    v = rng.standard_normal(N)
    pairs = [(int(i), int(j)) for a, i in enumerate(cols) for j in cols[a:]]
    g, atv, fused = model.gram_atv_sample(w, v, pairs)
    Ac = model.get_columns(cols)
    col = {int(c): k for k, c in enumerate(cols)}
    worst = 0.0
    for (i, j), gv in zip(pairs, g):
        a, b = Ac[:, col[i]], Ac[:, col[j]]
        ref = float((a * w) @ b)
        worst = max(worst, abs(gv - ref) / (1e-11 * float(np.abs(a * w * b).sum()) + 1e-300))
    ref_atv = Ac.T @ v
    bound = 1e-11 * (np.abs(Ac).T @ np.abs(v))
    worst_v = float(np.max(np.abs(atv[cols] - ref_atv) / (bound + 1e-300)))
    return {"gram_entries": len(pairs), "atv_entries": int(ncols), "fused_atv": fused,
            "max_err_over_bound": max(worst, worst_v), "bound": "1e-11 * sum|terms| (host fp64 dots)",
            "pass": bool(worst <= 1.0 and worst_v <= 1.0)}


def sparse_check(model, x, seed=7, f32_compute=False):
    """Full-size C5 check: f(x) and ∇f(x) of the run's final x on the device (the same CSR / CSC
    SpMV kernels the timed epochs use) against a host SciPy evaluation of the downloaded CSR copy
    of A -- least squares, f = 0.5·scale·Σ(Ax − y)², ∇f = scale·Aᵀ(Ax − y) (problems.py / losses.py).
    Bounds: 1e-11·Σ|terms| per gradient entry, 1e-11 relative on f (different summation orders); the
    fp32-arithmetic arm: 1e-4·Σ|terms| and 1e-4 relative (fp32 sums of ~655-term rows / ~640-term
    columns: n·2⁻²⁴ ≈ 4e-5 worst case)."""
    import numpy as np
    tol = 1e-4 if f32_compute else 1e-11
    A, y = model.get_sparse()
    scale = 1.0 / model.N
    z = A @ x
    r = z - y
    f_ref = 0.5 * scale * float(r @ r)
    g_ref = scale * (A.T @ r)
    g_bound = tol * scale * (abs(A).T @ np.abs(r)) + 1e-300
    f_dev = model.fx(x)
    g_dev = model.gradx(x)
    err_g = float(np.max(np.abs(g_dev - g_ref) / g_bound))
    err_f = abs(f_dev - f_ref) / (tol * abs(f_ref) + 1e-300)
    del A
    return {"f_rel_err_over_bound": err_f, "grad_max_err_over_bound": err_g, "nnz_checked": int(model.nnz),
            "bound": "%g * sum|terms| per entry (host SciPy CSR, fp64)%s" % (
                tol, "; fp32-arithmetic arm" if f32_compute else ""),
            "pass": bool(err_f <= 1.0 and err_g <= 1.0)}


def host_info():
    """The GPU box's host as the CPU baseline saw it."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    info["model"] = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return info


def cpu_threads():
    """Threads for the CPU baseline: the process's CPU share on the GPU box (OMP_NUM_THREADS, set to
    16 per GPU there; nproc / os.cpu_count() report the whole machine), capped by the affinity mask."""
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    return max(1, n)


GIB = float(1 << 30)


def memory_plan(cfg, N, m, world, gram_cache=False):
    """Per-rank device bytes of the row-sharded dense Gram methods: the local
    panel-blocked A (N_pad x m_pad fp64) + y and the sample vectors, G and its LU-fallback copy Gc
    (m_pad² each), W (m_pad x 128), the cached AᵀQA (--gram-cache) and, at world > 1, the packed
    128 x 128 tile exchange buffer [tiles ‖ Aᵀv].  The largest rank (row_range: first N % world
    ranks hold one more row) sets the plan."""
    rows = -(-int(N) // int(world))
    npad = -(-rows // 16) * 16
    mpad = -(-int(m) // 128) * 128
    nb = mpad // 128
    plan = {"rows_per_rank": rows, "A": 8.0 * npad * mpad, "sample_vectors": 8.0 * npad * 12}
    if cfg.get("method") != "lqn":
        plan["G"] = 8.0 * mpad * mpad
        plan["Gc"] = 8.0 * mpad * mpad
        plan["W"] = 8.0 * mpad * 128
        if gram_cache:
            plan["Gk"] = 8.0 * mpad * mpad
        if world > 1:
            plan["exchange"] = 8.0 * (nb * (nb + 1) // 2 * 128 * 128 + mpad + 64)
    plan["total"] = sum(v for k, v in plan.items() if k != "rows_per_rank")
    return plan


def plan_text(plan):
    return ", ".join(f"{k} {v / GIB:.1f} GiB" for k, v in plan.items() if k != "rows_per_rank")


def world_from_env(args, env):
    """(world, rank, local_rank) of this process and whether it must launch the ranks itself.
    Raises SystemExit with the reason when the launch does not match --gpus."""
    if args.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        rank = int(env.get("RANK", "0"))
        local = int(env.get("LOCAL_RANK", str(rank)))
        if world != args.gpus:
            raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                             f"(torchrun --nproc-per-node {args.gpus}) or drop WORLD_SIZE")
        return world, rank, local, False
    return args.gpus, 0, 0, args.gpus > 1


def check_devices(args, ndev):
    """Fail fast (before any rank starts) when the node has fewer GPUs than ranks, unless
    --share-device was asked for (only with --comm torch: RCCL refuses two ranks on one GPU)."""
    if getattr(args, "single_process", False) and getattr(args, "device_exchange", "rccl") == "host":
        if ndev < 1:
            raise SystemExit("--device-exchange host: no HIP device visible")
        return   # the host-staged group exchange takes repeated GPUs
    if args.share_device:
        if args.comm != "torch":
            raise SystemExit("--share-device needs --comm torch (RCCL takes one GPU per rank)")
        if ndev < 1:
            raise SystemExit("--share-device: no HIP device visible")
        return
    if ndev < args.gpus:
        raise SystemExit(f"--gpus {args.gpus} needs {args.gpus} visible GPUs, this node shows {ndev} "
                         f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', 'unset')}); "
                         "use --share-device --comm torch to rehearse the launcher on fewer GPUs")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_envs(n, port, base):
    """The environment of each of the n rank processes (torch.distributed.run's variables)."""
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append(e)
    return out


def launch_ranks(n, argv):
    """Start n rank processes of this script (one per GPU) and wait; if one fails the others are
    ended (their exact PIDs) and the worst status is returned.  The parent never touches a GPU."""
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=e)
             for e in rank_envs(n, free_port(), os.environ)]
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in pending:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def gather_rank_rows(row, world, dist):
    """Every rank's record (rows held, its own timed seconds, its timers, what its exchange runs on)
    on rank 0, in rank order -- the per-rank rows of the JSON line."""
    if world == 1 or dist is None:
        return [row]
    rows = [None] * world
    dist.all_gather_object(rows, row)
    return rows


def verify_ranks(rows, world, N):
    """The scaling run checks itself: one row per rank in rank order, the row blocks of
    shard.row_range tiling [0, N) exactly, and every RCCL communicator counting `world` ranks with
    its own rank equal to the process's.  Returns the list of problems (empty = consistent)."""
    bad = []
    if [r["rank"] for r in rows] != list(range(world)):
        bad.append(f"rank rows {[r['rank'] for r in rows]} != 0..{world - 1}")
    edges = [(r["row0"], r["row1"]) for r in rows]
    if edges and (edges[0][0] != 0 or edges[-1][1] != N or any(a[1] != b[0] for a, b in zip(edges, edges[1:]))):
        bad.append(f"row blocks {edges} do not tile [0, {N})")
    for r in rows:
        c = r.get("comm") or {}
        if c.get("kind") == "rccl" and (c.get("nranks") != world or c.get("rank") != r["rank"]):
            bad.append(f"rank {r['rank']}: RCCL communicator reports rank {c.get('rank')} of {c.get('nranks')}, "
                       f"the launch has {world}")
    return bad


def plumbing_check(world, rank, local, args):
    """--plumbing-check: the rank processes' wiring without a GPU (gloo), through the same helpers
    the measured run uses: world and rank, this rank's row block of the config's N (shard.row_range),
    an in-place SUM all-reduce of a per-rank payload (the exchange's shape, scaled down) checked
    against its closed form, the MAX-over-ranks of the timed seconds, and the gathered per-rank rows
    (gather_rank_rows + verify_ranks).  Rank 0 prints one JSON line; any mismatch exits non-zero."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd"))
    from scsopt.shard import row_range     # pure Python: no HIP runtime is bound
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world and dist.get_rank() == rank
    t = torch.tensor([float(rank), float(local), float(world)])
    got = [torch.zeros(3) for _ in range(world)]
    dist.all_gather(got, t)
    cfg = CONFIGS[args.config]
    N = args.N or cfg["N"]
    r0, r1 = row_range(N, world, rank)
    n = 4099                                       # payload doubles (odd: no alignment luck)
    pay = torch.arange(n, dtype=torch.float64) * (rank + 1) + rank
    dist.all_reduce(pay, op=dist.ReduceOp.SUM)
    s1 = world * (world + 1) / 2.0
    want = torch.arange(n, dtype=torch.float64) * s1 + (s1 - world)
    ok_sum = bool(torch.equal(pay, want))
    dt = torch.tensor([0.5 + 0.01 * rank], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    row = {"rank": rank, "local_rank": local, "row0": r0, "row1": r1, "rows": r1 - r0,
           "comm": {"kind": "callback", "nranks": world, "rank": rank}}
    rows = gather_rank_rows(row, world, dist)
    dist.barrier()
    if rank == 0:
        bad = verify_ranks(rows, world, N)
        if not ok_sum:
            bad.append("all-reduce SUM mismatch")
        if abs(float(dt.item()) - (0.5 + 0.01 * (world - 1))) > 1e-12:
            bad.append("MAX over ranks mismatch")
        print(json.dumps({"plumbing": [[int(v) for v in g.tolist()] for g in got], "gpus": args.gpus,
                          "comm": args.comm, "backend": "gloo", "config": args.config, "N": N,
                          "ranks": rows, "allreduce_ok": ok_sum, "max_s": float(dt.item()), "problems": bad}))
        if bad:
            dist.destroy_process_group()
            raise SystemExit("plumbing check FAILED: " + "; ".join(bad))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--N", type=int, default=0, help="override the config's N")
    ap.add_argument("--m", type=int, default=0, help="override the config's m")
    ap.add_argument("--f32", action="store_true", help="c5: fp32-stored sparse values (fp64 accumulation)")
    ap.add_argument("--f32-compute", action="store_true",
                    help="c5: fp32-stored values AND fp32 arithmetic in the sparse products and the L-BFGS two-loop "
                         "(scs_set_compute_f32; the compute arm of the BASELINE configs[4] study)")
    ap.add_argument("--gram-cache", action="store_true",
                    help="c4: reuse the x-independent AᵀQA of least squares across steps (scs_set_gram_cache; "
                         "reported separately -- the reference recomputes it every step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the sampled full-size Gram / Aᵀv check")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "torch"],
                    help="row-shard exchange: libscsopt's own RCCL communicator or a torch.distributed callback")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the exchange path (packed Gram -> all-reduce -> unpack) at one rank too")
    ap.add_argument("--cpu-Ns", type=int, default=2048)
    ap.add_argument("--cpu-ms", type=int, default=4096)
    ap.add_argument("--share-device", action="store_true",
                    help="let ranks share GPUs round-robin (launcher rehearsal on a small box; --comm torch)")
    ap.add_argument("--single-process", action="store_true",
                    help="--gpus N from ONE process: a multi-device context (scs_create_multi) splits the rows "
                         "across GPUs 0..N-1 and runs one host thread per device (the Julia drop-in's mode)")
    ap.add_argument("--device-exchange", choices=("rccl", "host"), default="rccl",
                    help="--single-process: the group's exchange over RCCL (one GPU per device) or host-staged "
                         "(SCS_MULTI_HOST_EXCHANGE: --gpus N sub-contexts round-robin over the visible GPUs -- a "
                         "rehearsal of the group on fewer GPUs, not a scaling number)")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="launch the ranks and check their world wiring over gloo, no GPU work")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]

    world, rank, local, spawn = world_from_env(args, os.environ)
    single = args.single_process and args.gpus > 1
    if single:
        if "WORLD_SIZE" in os.environ:
            raise SystemExit("--single-process runs without a launcher (one process drives the GPUs)")
        world, spawn = 1, False
    if spawn:
        # --gpus N without a launcher: the N rank processes are started here, before any GPU call
        # (counting devices does not initialise the GPU)
        if not args.plumbing_check:
            import torch
            check_devices(args, torch.cuda.device_count())
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.plumbing_check:
        plumbing_check(world, rank, local, args)
        return
    N = args.N or cfg["N"]
    m = args.m or cfg["m"]
    if cfg.get("sparse") and world > 1:
        raise SystemExit("c5 runs on one GPU (BASELINE configs[4]); the sparse generator is single-context")
    if cfg["loss"] == "rosenbrock" and world > 1:
        raise SystemExit("c1 (Rosenbrock, no data) has nothing to shard")

    import numpy as np
    import torch
    import torch.distributed as dist
    import scsopt
    from scsopt import shard
    from scsopt.iterate import device_optim_loop, init_method

    comm = None
    ndev = torch.cuda.device_count()
    if world > 1 or single:
        check_devices(args, ndev)
    host_x = single and args.device_exchange == "host"
    devices = ([i % max(1, ndev) for i in range(args.gpus)] if host_x else list(range(args.gpus))) if single else None
    if single and (cfg.get("sparse") or cfg["loss"] == "rosenbrock"):
        raise SystemExit("--single-process shards a dense A (c2, c3, c4)")
    dev = local % max(1, ndev) if args.share_device else local
    gloo = args.comm == "torch"
    if world > 1 or args.force_comm:
        # one process per GPU; the row-sharded exchange runs on libscsopt's own RCCL communicator
        # (--comm rccl, "nccl" group) or through torch.distributed.all_reduce (--comm torch, "gloo"
        # group); torch.distributed otherwise carries only the communicator's unique id and the
        # timing barrier / max
        torch.cuda.set_device(dev)
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(free_port())), ("RANK", "0"),
                     ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        comm = shard.Comm(device=torch.device("cuda", dev), native=not gloo, force=args.force_comm)
    if not cfg.get("sparse") and cfg["loss"] != "rosenbrock":
        # fail fast, before generating anything, when the local shard does not fit this GPU
        plan = memory_plan(cfg, N, m, args.gpus if single else world, gram_cache=args.gram_cache)
        sharing = (-(-world // max(1, ndev)) if args.share_device
                   else -(-args.gpus // max(1, ndev)) if host_x else 1)
        free, _total = torch.cuda.mem_get_info(dev)
        if plan["total"] * sharing > 0.97 * free:
            raise SystemExit(f"rank {rank}: {cfg['workload']} N={N} m={m} on {world} rank(s) needs "
                             f"{plan['total'] * sharing / GIB:.1f} GiB on GPU {dev} ({plan_text(plan)}; "
                             f"{plan['rows_per_rank']} rows per rank), {free / GIB:.1f} GiB free: "
                             f"use more GPUs (--gpus) or a smaller --N")
    if args.f32_compute:
        if not cfg.get("sparse") or cfg["method"] != "lqn":
            raise SystemExit("--f32-compute applies to the sparse ProxLQNSCORE config (c5)")
        args.f32 = True
    model, hmu, method = build_problem(cfg, N, m, comm, dev, f32=args.f32, devices=devices,
                                       device_exchange=args.device_exchange)
    if args.f32_compute:
        model.set_compute_f32(True)
    reg = cfg["reg"]
    if args.gram_cache:
        if cfg["loss"] != "least_squares" or cfg["method"] == "lqn":
            raise SystemExit("--gram-cache applies to the least-squares Gram methods (c4)")
        model.set_gram_cache(True)
    model.configure(reg, hmu)
    init_method(method, model)
    ctx = model.ctx

    def barrier():
        if comm is not None:
            dist.barrier()
        torch.cuda.synchronize()
        ctx.check(scsopt._lib.lib.scs_sync(ctx.h))

    def run_iterate(k):
        # one iterate!() call (iterate.jl:56-267) with max_epoch = k, entirely inside libscsopt
        # (scs_iterate): init!, f(x*) + get_reg(x*) once, then per epoch f(x) + get_reg(x) + step!
        # and the history bookkeeping.  x_tol = f_tol = 0 so every call runs exactly k epochs.
        return device_optim_loop(method, model, reg, hmu, max_epoch=k, x_tol=0.0, f_tol=0.0, verbose=0)

    steps, warmup = args.steps, args.warmup
    if cfg["loss"] == "rosenbrock" and steps < 50:
        steps = 50                               # microsecond-scale steps: time a meaningful batch
    lqn_sparse = cfg.get("sparse") and cfg["method"] == "lqn"
    if lqn_sparse:
        steps = max(steps, 50)                   # millisecond-scale steps: amortize iterate!'s f(x*) once
        warmup = max(warmup, 5)                  # and let the clocks settle (1 warm-up step: +-5 % box to box)
    # kernel timing: HIP events around the dominant launches inside the timed region.  Each event record
    # costs a dispatch gap (~5 us) of its own, so the millisecond-scale sparse epochs time the launches of
    # every TEVERY-th epoch (scs_iterate's pipelined loop; the setup passes are always timed)
    tevery = int(os.environ.get("SCS_BENCH_TIMING_EVERY", "10")) if lqn_sparse else 1
    ctx.check(scsopt._lib.lib.scs_timing_enable(ctx.h, tevery))
    if warmup > 0:
        run_iterate(warmup)
    barrier()
    ctx.check(scsopt._lib.lib.scs_timing_reset(ctx.h))
    t0 = time.perf_counter()
    sol = run_iterate(steps)
    barrier()
    dt = time.perf_counter() - t0
    objs = sol.obj
    tm = ctx.timing()
    gram_kname, prod_kname = ctx.kernel_names()
    cinfo = ctx.comm_info()   # read back from libscsopt: ncclCommCount / ncclCommUserRank, the RCCL loaded
    r0 = model.row0 if not single else 0
    my_row = {"rank": rank, "local_rank": local, "device": dev, "row0": int(r0),
              "row1": int(r0) + int(model.N), "rows": int(model.N), "time_s": dt,
              "ms_per_step_local": 1e3 * dt / steps,
              "breakdown_ms_per_step": ({k.replace("_ms", ""): tm[k] / steps for k in tm if k.endswith("_ms")}
                                        if tevery == 1 else None),
              "launch_counts": {k.replace("_calls", ""): int(tm[k]) for k in tm if k.endswith("_calls")},
              "comm": {k: cinfo[k] for k in ("kind", "nranks", "rank")}}
    rank_rows = gather_rank_rows(my_row, world, dist if comm is not None else None)
    if comm is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cpu" if gloo else torch.device("cuda", dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    check = None
    if rank == 0 and not cfg.get("sparse") and cfg["loss"] != "rosenbrock" and not args.no_check and not single:
        check = sampled_gram_check(model, m)   # kernel-level entry points: single-device contexts
    if rank == 0 and cfg.get("sparse") and not args.no_check:
        check = sparse_check(model, np.asarray(sol.x, dtype=np.float64), f32_compute=args.f32_compute)

    if rank == 0:
        ms_step = 1e3 * dt / steps
        value = steps / dt
        N_local = -(-model.N // args.gpus) if single else model.N   # device 0's rows (row_range)
        line = {
            "metric": METRIC if args.config == "c3" else f"iterate!() iterations/sec, {cfg['workload']}",
            "value": value, "unit": "iterations/s", "n_gpus": args.gpus if single else world, "steps": steps,
            "warmup": warmup,
            "ms_per_step": ms_step, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": ("f32 (fp32-stored A values; fp32 arithmetic in the sparse products and the two-loop, "
                      "f / eta / step / prox in f64)" if args.f32_compute else
                      "f64 (fp32-stored A values)" if args.f32 else "f64"), "data": "synthetic (on-device counter RNG: A ~ N(0,1)/sqrt(m), y from a sparse x_true)",
            "config": {"workload": cfg["workload"], "N": N, "m": m, "lambda": model.λ, "mu": hmu.mu,
                       "method": type(method).__name__, "ss_type": method.ss_type,
                       "parallelism": (f"row-shard x{args.gpus} (one process, scs_create_multi"
                                       + (", host-staged exchange)" if host_x else ")") if single
                                       else f"row-shard x{world}"),
                       "devices": (len(set(devices)) if single else min(world, ndev) if args.share_device
                                   else world),
                       "exchange": (("rccl (libscsopt)" if args.comm == "rccl"
                                     else "torch.distributed callback (gloo)")
                                    + (" forced at one rank" if world == 1 else "")) if comm is not None else None},
        }
        line["comm"] = {"kind": cinfo["kind"], "nranks": cinfo["nranks"], "rccl_version": cinfo["rccl_version"],
                        "rccl_lib": cinfo["rccl_lib"]}
        if not single:
            line["ranks"] = rank_rows
            problems = verify_ranks(rank_rows, world, model.N_global)
        else:
            problems = ([] if cinfo["nranks"] == args.gpus or host_x else
                        [f"the group's RCCL communicator counts {cinfo['nranks']} devices, --gpus {args.gpus}"])
        line["ranks_consistent"] = not problems
        if problems:
            line["ranks_problems"] = problems
        if args.share_device and world > ndev:
            line["config"]["shared_device"] = (f"{world} ranks on {ndev} GPU(s): a launcher rehearsal, "
                                               "not a scaling number")
        if host_x and args.gpus > ndev:
            line["config"]["shared_device"] = (f"{args.gpus} sub-contexts on {ndev} GPU(s) with the host-staged "
                                               "exchange: a rehearsal of the multi-device group, not a scaling number")
        if tm["gram_calls"]:
            main_calls = steps                      # one Gram per GGN/NSCORE step; the solver's own
            gram_avg_ms = tm["gram_ms"] / max(1, tm["gram_calls"])   # launches are timed under "solve"
            gram_flops = float(N_local) * m * (m + 1)   # algorithmic symmetric Gram per launch
            if gram_kname.startswith("sparse_gram"):
                # priced by nnz: every row of the generated pattern has k = round(rho·m) entries and
                # contributes k(k+1)/2 multiply-adds to the upper triangle
                k = int(round(cfg["rho"] * m))
                gram_flops = float(N_local) * k * (k + 1)
            achieved = gram_flops / (gram_avg_ms * 1e-3) / 1e12
            traffic = None
            kname = gram_kname or "unknown"   # the library reports the kernel it launched
            # PMC summaries (tools/gpu_gram_pmc.sh, tools/gpu_pmc_c2.sh + tools/pmc_summary.py), one per (N, m):
            # their bytes are used only when they were measured on the kernel this run launched
            for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*_gram_pmc*.json")), reverse=True):
                if world != 1 or args.gram_cache:
                    break
                with open(pmc) as f:
                    pm = json.load(f)
                if pm.get("N") == N and pm.get("m") == m and pm.get("kernel", "").split("::")[-1] == kname:
                    traffic = pm.get("hbm_bytes_per_launch")
                    line["roofline_traffic_source"] = os.path.relpath(pmc, ROOT)
                    break
            line["roofline"] = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                                "kernel": kname, "avg_ms": gram_avg_ms, "launches": main_calls,
                                "flops_per_launch": gram_flops}
            if gram_kname.startswith("sparse_gram"):
                # the Gram of a sparse A is a gather, not an MFMA contraction: its roofline is HBM on the
                # ALGORITHMIC bytes -- the CSR and CSC copies once (value + 4-B index per entry, the row /
                # column pointers) plus the upper-triangle G write -- with the MFMA fraction kept beside it;
                # walk_bytes_est is what Gustavson-by-column moves (every (column, 4096-row block) item
                # reads the block segment of each row of the column, ~k/16 entries, plus ~36 B of row
                # metadata): the traffic the kernel's design implies, ~100x the algorithmic bytes
                nnz_a = model.nnz
                vbytes = 4 if args.f32 else 8
                alg = 2.0 * nnz_a * (vbytes + 4) + 8.0 * (N_local + 1) + 8.0 * (m + 1) + 8.0 * m * (m + 1) / 2
                nblk_g = -(-m // 4096)
                items = 4096.0 * nblk_g * (nblk_g + 1) / 2
                walk = items * (nnz_a / m) * ((nnz_a / N_local) / nblk_g * (vbytes + 2) + 36.0)
                gbs = alg / (gram_avg_ms * 1e-3) / 1e9
                # PMC bytes of the sparse Gram (tools/gpu_pmc_sgram.sh + tools/pmc_summary_sgram.py) when the
                # summary names the kernel launched here at this shape
                for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "pmc_sgram", "summary_*.json")),
                                  reverse=True):
                    with open(pmc) as f:
                        pm = json.load(f)
                    if (world == 1 and pm.get("N") == N and pm.get("m") == m and not args.f32
                            and pm.get("kernel", "").split("::")[-1] == kname):
                        traffic = pm.get("hbm_bytes_per_launch")
                        line["roofline_traffic_source"] = os.path.relpath(pmc, ROOT)
                        break
                line["roofline"] = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                                    "avg_ms": gram_avg_ms, "launches": main_calls, "bytes_per_launch": alg,
                                    "walk_bytes_est": walk, "walk_over_algorithmic": walk / alg,
                                    "walk_gbs": walk / (gram_avg_ms * 1e-3) / 1e9,
                                    "mfma_tflops": achieved, "mfma_frac": achieved / FP64_MFMA_PEAK_TFLOPS,
                                    "flops_per_launch": gram_flops}
        if tm["gemv_calls"] and lqn_sparse:
            # LDS-blocked CSR (A·x) and CSC (Aᵀ·v) passes, launched equally often.  Bytes each launch must
            # move: nnz·(value + 2 B local index) + the per-block row pointers (8 B per row and block)
            # + one partial per row and block + the gathered vector once (mean of the two launches)
            nnz = model.nnz
            vb = 4 if args.f32 else 8
            nb_csr = -(-m // 16384)
            nb_csc = -(-N // 16384)
            csr = nnz * (vb + 2) + 8 * nb_csr * (N + 1) + 8 * nb_csr * N + 8 * m
            csc = nnz * (vb + 2) + 8 * nb_csc * (m + 1) + 8 * nb_csc * m + 8 * N
            per_launch = 0.5 * (csr + csc)
            avg_ms = tm["gemv_ms"] / tm["gemv_calls"]
            achieved = per_launch / (avg_ms * 1e-3) / 1e9
            traffic = None
            kname = prod_kname or "unknown"
            # PMC bytes (tools/pmc_summary_spmv.py) only when the file names the kernel launched here
            pmc = os.path.join(ROOT, "profiles", "r02_c5_spmv_pmc_%s.json" % ("f32" if args.f32 else "f64"))
            if os.path.exists(pmc) and world == 1 and N == 1 << 20 and m == 1 << 16:
                with open(pmc) as f:
                    pm = json.load(f)
                if pm.get("kernel") == kname:
                    traffic = pm.get("hbm_bytes_per_launch")
                    line["roofline_traffic_source"] = os.path.relpath(pmc, ROOT)
            line["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                                "avg_ms": avg_ms, "launches_per_step": 2, "timed_launches": tm["gemv_calls"],
                                "timing_sample": "every %d-th epoch's launches + the call's setup passes" % tevery,
                                "bytes_per_launch": per_launch}
            line["config"]["nnz"] = nnz
            if args.f32:
                # the full-size fp32-vs-fp64 studies of this configuration (tools/c5_tolerance.py): the storage
                # arm (r03) stores A's values in fp32 and computes in fp64; the compute arm (r04) also runs
                # the sparse products and the two-loop in fp32 arithmetic
                tol = os.path.join(ROOT, "profiles", *(("r04", "c5", "tolerance_f32compute.json")
                                                       if args.f32_compute else ("r03", "c5", "tolerance.json")))
                if os.path.exists(tol) and N == 1 << 20 and m == 1 << 16:
                    with open(tol) as f:
                        ts = json.load(f)
                    line["tolerance_study"] = {k: ts[k] for k in ("max_rel_dobj", "max_dx_inf", "max_active_diff")}
                    line["tolerance_study"].update(epochs=ts["config"]["epochs"], source=os.path.relpath(tol, ROOT),
                                                   arms=ts["arms"])
        elif tm["gemv_calls"] and not cfg.get("sparse"):
            # streaming passes (A·x in f(x), Aᵀv in step!): each reads the local A once
            line["hbm_gbs_streaming"] = (tm["gemv_calls"] * 8.0 * N_local * m) / (tm["gemv_ms"] * 1e-3) / 1e9
            line["hbm_frac_streaming"] = line["hbm_gbs_streaming"] / HBM_PEAK_GBS
        if args.gram_cache and tm["solve_calls"]:
            # cached AᵀQA: the step's dominant kernel is the m x m Cholesky factor + solves
            solve_avg_ms = tm["solve_ms"] / tm["solve_calls"]
            solve_flops = m ** 3 / 3.0 + 2.0 * m * m
            achieved = solve_flops / (solve_avg_ms * 1e-3) / 1e12
            line["roofline"] = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": None,
                                "kernel": "chol_factor + chol_solve (cached Gram)", "avg_ms": solve_avg_ms,
                                "launches": tm["solve_calls"], "flops_per_launch": solve_flops}
            line["config"]["gram_cache"] = True
        if tevery == 1:
            line["breakdown_ms_per_step"] = {k.replace("_ms", ""): tm[k] / steps for k in tm if k.endswith("_ms")}
        line["objective_last"] = objs[-1]
        if check is not None:
            line["parity_check"] = check
        do_cpu = not args.no_cpu_baseline and world == 1 and not single   # the CPU baseline: rank 0 at N = 1 only
        if do_cpu and args.config == "c1":
            try:
                out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline_c1.py")],
                                     capture_output=True, text=True, timeout=120, check=True)
                cb = json.loads(out.stdout.strip().splitlines()[-1])
                line["cpu_baseline"] = {k: cb[k] for k in CPU_KEYS if k in cb}
            except Exception as e:  # the baseline is reported, never the target
                line["cpu_baseline"] = {"value": None, "error": repr(e)[:300]}
        if do_cpu and args.config == "c5":
            try:
                out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline_lqn.py"), "--N", str(N),
                                      "--m", str(m), "--rho", str(cfg["rho"]), "--mem", str(cfg["mem"])],
                                     capture_output=True, text=True, timeout=300, check=True)
                cb = json.loads(out.stdout.strip().splitlines()[-1])
                line["cpu_baseline"] = {k: cb[k] for k in CPU_KEYS if k in cb}
            except Exception as e:  # the baseline is reported, never the target
                line["cpu_baseline"] = {"value": None, "error": repr(e)[:300]}
        if do_cpu and args.config in ("c2", "c3", "c4"):
            env = dict(os.environ)
            cores = cpu_threads()
            env["OPENBLAS_NUM_THREADS"] = str(cores)
            env["OMP_NUM_THREADS"] = str(cores)
            try:
                meth = {"c2": "nscore", "c3": "ggn", "c4": "ggn_ls"}[args.config]
                Ns = args.cpu_Ns if m <= 16384 else 256   # bounded sample (the dgemm is Ns·m² flops)
                out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--N", str(N),
                                      "--m", str(m), "--Ns", str(Ns), "--ms", str(min(args.cpu_ms, m)),
                                      "--method", meth, "--reps", "3"],
                                     capture_output=True, text=True, env=env, timeout=300, check=True)
                cb = json.loads(out.stdout.strip().splitlines()[-1])
                line["cpu_baseline"] = {k: cb[k] for k in CPU_KEYS if k in cb}
            except Exception as e:  # the baseline is reported, never the target
                line["cpu_baseline"] = {"value": None, "error": repr(e)[:300]}
        if isinstance(line.get("cpu_baseline"), dict):
            line["cpu_baseline"]["host"] = host_info()
        print(json.dumps(line))
        if problems:
            raise SystemExit("scaling run inconsistent: " + "; ".join(problems))
        if check is not None and not check["pass"]:
            raise SystemExit("full-size parity check FAILED: " + json.dumps(check))
    # release the library context (its streams, a CU-masked one included) before the runtime and
    # any profiler tear down, instead of leaving it to interpreter-exit finalizers
    ctx.close()
    if comm is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
