"""The round-3 fault's geometry through the debug-bounds build, once per
round: zero out-of-range reports from
the kernels' own range checks, outputs exact against the oracle.  The build
itself is compiled by tests/test_abi.py::test_debug_bounds_build_compiles."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT, has_gpu_device

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu_device(), reason="needs a HIP device")]

DEBUG_LIB = os.path.join(ROOT, "nkfs_amd", "lib", "debug", "libnkfs_crt.so")


@pytest.mark.timeout(240)
def test_round3_fault_geometry_under_debug_bounds():
    assert os.path.exists(DEBUG_LIB), "build() makes the debug-bounds library (make DEBUG_BOUNDS=1)"
    env = dict(os.environ, NKFS_LIB=DEBUG_LIB)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "helpers", "debug_bounds_probe.py")], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=220)
    reports = [ln for ln in r.stdout.splitlines() if "nkfs bounds" in ln]
    assert not reports, "\n".join(reports[:20])
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "debug-bounds ok" in r.stdout
