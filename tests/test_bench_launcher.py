"""CPU: bench.py's multi-GPU launcher -- argument and world plumbing, the device check and the
per-rank memory plan (BASELINE north_star: iterations/s at 1, 2, 4, 8 GPUs for the row-sharded
path; the driver's SCALE run starts bench.py under torch.distributed.run, a user may start it
with --gpus N alone)."""
import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

HBM_GIB = 288e9 / (1 << 30)   # MI355X: 288 GB of HBM3E per GPU


def _args(**kw):
    a = dict(gpus=1, comm="rccl", share_device=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_world_from_env():
    assert bench.world_from_env(_args(gpus=1), {}) == (1, 0, 0, False)
    assert bench.world_from_env(_args(gpus=4), {}) == (4, 0, 0, True)          # self-launch
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    assert bench.world_from_env(_args(gpus=4), env) == (4, 2, 2, False)        # under torchrun
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 4"):
        bench.world_from_env(_args(gpus=4), {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.world_from_env(_args(gpus=0), {})


def test_check_devices():
    bench.check_devices(_args(gpus=8), 8)
    with pytest.raises(SystemExit, match="needs 8 visible GPUs, this node shows 1"):
        bench.check_devices(_args(gpus=8), 1)
    bench.check_devices(_args(gpus=2, comm="torch", share_device=True), 1)
    with pytest.raises(SystemExit, match="needs --comm torch"):
        bench.check_devices(_args(gpus=2, comm="rccl", share_device=True), 1)


def test_rank_envs():
    envs = bench.rank_envs(3, 29555, {"KEEP": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
               and e["KEEP"] == "1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]


def test_memory_plan_c3_c4():
    c3, c4 = bench.CONFIGS["c3"], bench.CONFIGS["c4"]
    p1 = bench.memory_plan(c3, c3["N"], c3["m"], 1)
    assert p1["A"] == 8.0 * (1 << 20) * (1 << 14) and "exchange" not in p1
    assert p1["total"] / (1 << 30) < HBM_GIB
    p8 = bench.memory_plan(c3, c3["N"], c3["m"], 8)
    assert p8["rows_per_rank"] == (1 << 17) and p8["A"] == p1["A"] / 8 and p8["exchange"] > 0
    # C4 (N = 2^22, m = 2^15): 1 TiB of A -- fits on 8 GPUs, not on 4
    assert bench.memory_plan(c4, c4["N"], c4["m"], 8)["total"] / (1 << 30) < 0.9 * HBM_GIB
    assert bench.memory_plan(c4, c4["N"], c4["m"], 4)["total"] / (1 << 30) > HBM_GIB
    assert "plan" not in bench.plan_text(p8) and "GiB" in bench.plan_text(p8)


def _bench(*argv, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                          env=e, timeout=timeout)


def test_self_launch_world_plumbing():
    """--gpus 2 without a launcher starts two rank processes that form one world of size 2."""
    r = _bench("--gpus", "2", "--comm", "torch", "--plumbing-check")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["plumbing"] == [[0, 0, 2], [1, 1, 2]] and line["gpus"] == 2


def test_too_few_gpus_exits_nonzero():
    """--gpus 8 where fewer GPUs are visible fails before starting anything (here: none)."""
    r = _bench("--gpus", "8")
    assert r.returncode != 0
    assert "needs 8 visible GPUs" in r.stderr


def test_world_mismatch_exits_nonzero():
    r = _bench("--gpus", "4", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_verify_ranks():
    rows = [{"rank": r, "row0": a, "row1": b, "comm": {"kind": "rccl", "nranks": 4, "rank": r}}
            for r, (a, b) in enumerate([(0, 3), (3, 6), (6, 8), (8, 10)])]
    assert bench.verify_ranks(rows, 4, 10) == []
    bad = [dict(r) for r in rows]
    bad[2] = dict(bad[2], comm={"kind": "rccl", "nranks": 1, "rank": 0})   # a communicator of one
    assert any("RCCL communicator reports rank 0 of 1" in p for p in bench.verify_ranks(bad, 4, 10))
    gap = [dict(r) for r in rows]
    gap[1] = dict(gap[1], row1=5)
    assert any("do not tile" in p for p in bench.verify_ranks(gap, 4, 10))
    assert bench.verify_ranks(rows[:3], 4, 10)   # a missing rank


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_eight_rank_plumbing(launcher):
    """The driver's N=8 SCALE run, rehearsed on CPU with gloo: 8 rank processes (self-launched or
    under torch.distributed.run, as the driver starts it) form one world, take the C3 row blocks of
    shard.row_range, sum a payload in place, take the MAX of the timed seconds and gather the
    per-rank rows through the same helpers the measured run uses (gather_rank_rows / verify_ranks)."""
    if launcher == "self":
        r = _bench("--gpus", "8", "--comm", "torch", "--plumbing-check", timeout=400)
    else:
        e = dict(os.environ)
        e.pop("WORLD_SIZE", None)
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                            "--master-addr", "127.0.0.1", "--master-port", str(bench.free_port()),
                            os.path.join(ROOT, "bench.py"), "--gpus", "8", "--comm", "torch", "--plumbing-check"],
                           capture_output=True, text=True, env=e, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["plumbing"] == [[i, i, 8] for i in range(8)]
    assert line["allreduce_ok"] and line["problems"] == [] and line["max_s"] == pytest.approx(0.57)
    assert [x["rows"] for x in line["ranks"]] == [(1 << 20) // 8] * 8
