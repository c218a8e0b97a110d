"""Test configuration.

`-m "not gpu"`: oracle vs the reference's own assertions and the committed
golden fixtures, host logic, gloo world-size-2 sharding, and the C-ABI
library loading / exporting every symbol of include/scsopt.h.
`-m gpu`: parity of the HIP path (called through the C ABI) against the
oracle -- run on an MI355X.
"""
import os
import subprocess
import sys

import pytest
# the tests use torch (streams, torch.distributed): import it before scsopt so libscsopt binds
# torch's HIP runtime (scsopt/_lib.py); the torch-free import is covered by test_abi.py
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd")
LIB = os.path.join(PKG, "scsopt", "libscsopt.so")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "reference_tests.json")) as f:
        return json.load(f)
