"""bench.py -- iterate!() iterations/s of ProxGGNSCORE on the BASELINE headline config.

Workload (BASELINE.json metric, configs[2]): sparse logistic regression,
N = 2^20 samples x m = 2^14 features, fp64, A ~ N(0,1)/sqrt(m) generated on
the device (synthetic; no dataset), y ~ Bernoulli(σ(A x_true)) ∈ {0,1},
x_true 10 % dense, l1 with λ = 0.1·‖∇f(0)‖∞, PHuberSmootherL1L2(μ = 1),
ProxGGNSCORE(ss_type = 1), f(A,y,x) = CE(y, σ(Ax)) with scale 1/N.

One "step" = one iterate! epoch: f(x) + get_reg(x) + step!(ProxGGNSCORE)
(J/residual/Q from σ(Ax), the MFMA Gram JᵀQJ = Aᵀ diag(s²q) A, Jᵀr, λ·diag(Hr),
the m x m solve, SCORE damping and the prox).  N GPUs: A is row-sharded
(strong scaling: the global problem is fixed), one all-reduce per step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix, AMD spec (not in the local guide)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--m", type=int, default=1 << 14)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-Ns", type=int, default=2048)
    ap.add_argument("--cpu-ms", type=int, default=4096)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import scsopt
    from scsopt import losses, shard
    from scsopt.iterate import init_method, step

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    comm = None
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        comm = shard.Comm(device=torch.device("cuda", local))
    N, m = args.N, args.m
    x0 = np.random.default_rng(1234).standard_normal(m)
    model = scsopt.Problem.synthetic(N, m, x0, losses.logistic_ce(1.0 / N), 1.0, kind=1, seed=2026, density=0.1,
                                     out_fn=losses.sigmoid_ce(1.0 / N), device=local, comm=comm)
    g0 = model.gradx(np.zeros(m))
    model.λ = 0.1 * float(np.max(np.abs(g0)))
    hmu = scsopt.PHuberSmootherL1L2(1.0)
    method = scsopt.ProxGGNSCORE()
    model.configure("l1", hmu)
    init_method(method, model)
    ctx = model.ctx

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ctx.check(scsopt._lib.lib.scs_sync(ctx.h))

    x = x0.copy()
    x_prev = x.copy()
    it = 0

    def one_epoch():
        nonlocal x, x_prev, it
        it += 1
        fval = model.fx(x)                       # iterate.jl:189-190
        obj = fval + model.get_reg(x)
        x_new, pri = step(method, model, "l1", hmu, x, x_prev, it)   # iterate.jl:233
        x_prev, x = x, x_new
        return obj, pri

    ctx.check(scsopt._lib.lib.scs_timing_enable(ctx.h, 1))
    for _ in range(args.warmup):
        one_epoch()
    barrier()
    ctx.check(scsopt._lib.lib.scs_timing_reset(ctx.h))
    t0 = time.perf_counter()
    objs = []
    for _ in range(args.steps):
        objs.append(one_epoch()[0])
    barrier()
    dt = time.perf_counter() - t0
    tm = ctx.timing()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=torch.device("cuda", local))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    if rank == 0:
        ms_step = 1e3 * dt / args.steps
        value = args.steps / dt
        N_local = model.N
        gram_avg_ms = tm["gram_ms"] / max(1, tm["gram_calls"])
        gram_flops = float(N_local) * m * (m + 1)   # algorithmic symmetric Gram per launch
        achieved = gram_flops / (gram_avg_ms * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "r01_gram_pmc.json")
        if os.path.exists(pmc) and world == 1:
            with open(pmc) as f:
                pm = json.load(f)
            if pm.get("N") == N and pm.get("m") == m:
                traffic = pm.get("hbm_bytes_per_launch")
        line = {
            "metric": "iterate!() iterations/sec + achieved HBM GB/s, ProxGGNSCORE n=1M m=16k",
            "value": value, "unit": "iterations/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_step, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (on-device counter RNG: A ~ N(0,1)/sqrt(m), y ~ Bernoulli)",
            "config": {"workload": "ProxGGNSCORE sparse-logistic l1, BASELINE configs[2]", "N": N, "m": m,
                       "lambda": model.λ, "mu": 1.0, "ss_type": 1, "parallelism": f"row-shard x{world}"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                         "kernel": "gram_f64_kernel", "avg_ms": gram_avg_ms,
                         "flops_per_launch": gram_flops},
            "breakdown_ms_per_step": {k.replace("_ms", ""): tm[k] / args.steps for k in tm if k.endswith("_ms")},
            # streaming passes (A·x in f(x), Aᵀv in step!): each reads the local A once
            "hbm_gbs_streaming": (tm["gemv_calls"] * 8.0 * N_local * m) / (tm["gemv_ms"] * 1e-3) / 1e9
            if tm["gemv_calls"] else None,
            "objective_last": objs[-1],
        }
        if not args.no_cpu_baseline:
            env = dict(os.environ)
            cores = int(env.get("OMP_NUM_THREADS", "16"))
            env["OPENBLAS_NUM_THREADS"] = str(cores)
            try:
                out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--N", str(N),
                                      "--m", str(m), "--Ns", str(args.cpu_Ns), "--ms", str(args.cpu_ms)],
                                     capture_output=True, text=True, env=env, timeout=300, check=True)
                cb = json.loads(out.stdout.strip().splitlines()[-1])
                line["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
                line["cpu_baseline"]["t_iter_s"] = cb["t_iter_s"]
            except Exception as e:  # the baseline is reported, never the target
                line["cpu_baseline"] = {"value": None, "error": repr(e)[:300]}
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
