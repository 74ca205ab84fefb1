"""Host build of the register networks and tree sums of csrc/sortnet.hpp (tests/host/sortnet_check.cpp):
the selection networks against std::sort, and the NZ tree sum (padding adds skipped, one final +0.0;
DESIGN.md §5.11) against the spec's stride-halving tree, bit for bit, with signed zeros and denormals."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "approximate-consensus-simulation_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sortnet_and_nz_tree_on_host(tmp_path):
    exe = tmp_path / "sortnet_check"
    subprocess.run(["g++", "-O2", "-fopenmp", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(HERE, "host", "sortnet_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "networks: 0 mismatches" in r.stdout and ", 0 mismatches" in r.stdout.split(";")[1]
