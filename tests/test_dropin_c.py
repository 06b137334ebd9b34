"""A plain-C caller, written the way the reference's own code calls crt/
(crt/nk8.c:601-723, client/lib/client.c:137-148), compiled against
include/nkfs_crt.h and linked to libnkfs_crt.so -- the drop-in boundary as a
maintainer would use it."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "dropin_client.c")
LIBDIR = os.path.join(ROOT, "nkfs_amd", "lib")


def build(tmp_path):
    exe = str(tmp_path / "dropin_client")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-std=gnu11", "-I", os.path.join(ROOT, "include"), SRC,
                    "-L", LIBDIR, "-lnkfs_crt", "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def test_compiles_and_links_against_headers(tmp_path):
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
def test_runs_on_gpu(tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin_client: ok" in r.stdout
