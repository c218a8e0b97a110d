"""CPU: the row bookkeeping of a multi-device context (csrc/shard_plan.h, used by scs_create_multi),
compiled with the host sanitizers (-fsanitize=address,undefined) and checked against
scsopt.shard.row_range -- one process driving several GPUs must give each device the rows one
process per GPU gives each rank."""
import os
import shutil
import subprocess

import pytest

from scsopt.shard import row_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "shard_plan_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_shard_plan_matches_row_range_under_sanitizers(tmp_path):
    exe = tmp_path / "shard_plan_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    SRC, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) > 50
    for ln in lines:
        parts = ln.split()
        N, nd = int(parts[0]), int(parts[1])
        got = [tuple(int(v) for v in b.split(":")) for b in parts[2:]]
        assert got == [row_range(N, nd, d) for d in range(nd)], (N, nd)
