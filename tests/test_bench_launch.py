"""bench.py --gpus N started without a launcher spawns N fresh rank processes
itself (torch.distributed.run, rendezvous on 127.0.0.1) before any GPU call,
and every rank checks world == --gpus.  CPU only: --launch-check makes the
ranks meet over gloo and rank 0 report what it saw (the reference's one
worker per chain, main_inversion.jl:15)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=220, cwd=ROOT)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    lines = [x for x in p.stdout.decode().splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n


@pytest.mark.timeout(120)
def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-check"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=100, cwd=ROOT)
    assert p.returncode != 0 and b"--gpus 3" in p.stderr


def test_host_cores_read_from_os():
    sys.path.insert(0, ROOT)
    import bench

    used, facts = bench.host_cores()
    assert facts["sched_getaffinity"] == len(os.sched_getaffinity(0))
    assert facts["os_cpu_count"] == os.cpu_count()
    assert 1 <= used <= facts["sched_getaffinity"]
