"""The multi-rank bench path on the GPU box (SURVEY.md
§8(e)).  The driver's 8-GPU scaling run has never had a node, so these keep
the N > 1 code path exercised on every round's one-GPU box:

* bench.py at world size 2 under torch.distributed.run, control
  collectives over gloo, both ranks' kernels on the box's GPU (each rank a
  fresh process): both ranks' digests all-gathered and checked against the
  oracle (`verified_ranks == 2`) and the line's keys as the driver reads
  them.  Two processes share one GPU, so its rates are not a measurement.
* bench.py's control collectives on RCCL (backend "nccl") at world size 1
  on the box's GPU (tools/rccl_smoke.py).

Stripes are independent (crt/nk8.c:344-444): no data-path collective."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT, has_gpu_device

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu_device(), reason="needs a HIP device")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _last_json(text):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            return json.loads(line)
    return None


@pytest.mark.timeout(300)
def test_bench_two_ranks_gloo_on_one_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--config", "c2",
           "--stripes", "4096", "--steps", "3", "--warmup", "1", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = _last_json(r.stdout)
    assert line is not None, r.stdout[-3000:]
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["warmup"] == 1
    assert line["verified_ranks"] == 2 and line["verified"] is True
    assert len(line["digest_xor_per_rank"]) == 2
    assert line["digest_xor_per_rank"][0] != line["digest_xor_per_rank"][1]  # distinct stripe ranges
    assert line["scaling"] == "weak" and line["config"]["stripes_all_gpus"] == 2 * 4096
    assert line["config"]["parallelism"] == "stripe-partition x2"
    pr = line["per_rank"]
    assert len(pr["encode_us"]) == 2 and len(pr["decode_us"]) == 2 and min(pr["encode_us"]) > 0
    roof = line["roofline"]
    assert {"achieved", "peak", "frac", "bound", "unit", "bytes_per_launch"} <= set(roof)
    assert roof["bytes_per_launch"] == 4096 * (4096 + 4 * 2048 + 32)
    assert line["value"] > 0 and line["ms_per_step"] > 0


@pytest.mark.timeout(200)
def test_rccl_control_collectives_world1():
    env = dict(os.environ, NKFS_SMOKE_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_smoke.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert "rccl smoke ok" in r.stdout
