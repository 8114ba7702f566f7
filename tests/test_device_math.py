"""The product's device math, executed on the host (gp_device.hpp is __host__ __device__).

Exact fast division for every lattice divisor g and g^2 (g <= 1625) and the
product's Philox / U(m) draws against the C oracle.  CPU-only: compiles a tiny
host program with hipcc.
"""
import os
import shutil
import subprocess

import pytest

from tests.oracle_ctypes import lib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def output(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("dm") / "device_math_check")
    subprocess.check_call([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "helpers", "device_math_check.cpp")])
    return subprocess.run([exe], check=True, capture_output=True, text=True).stdout.splitlines()


def test_fastdiv_exact(output):
    assert output[0].startswith("fastdiv ok")


def test_product_philox_matches_oracle(output):
    assert "KAT0 6627e8d5 e169c58d" in output
    n = 0
    for line in output:
        if line.startswith("U "):
            seed, stream, node, rnd, m, u = map(int, line.split()[1:])
            assert lib().or_uniform(seed, stream, node, rnd, m) == u
            n += 1
    assert n == 200


def test_ratio_moved_matches_exact_test(output):
    """gp_device.hpp ratio_moved: the division-free shortcut never changes the
    push-sum stability decision (Program.fs:114-123, SRS v1) -- 4e6 cases, ratios
    < 2^32, moves from 0 to the whole range and around the 1e-10 edge."""
    line = [l for l in output if l.startswith("ratio_moved")][0].split()
    cases, fast, bad = int(line[1]), int(line[3]), int(line[5])
    assert cases == 4000000 and bad == 0
    assert fast > cases // 4  # the shortcut does decide a large share
