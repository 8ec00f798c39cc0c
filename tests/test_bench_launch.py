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
    assert out["leg_check"] == {"ranks": n}  # a multi-rank leg under run_leg's deadline


@pytest.mark.timeout(240)
def test_stalled_leg_still_prints_the_line():
    """A rank that never joins a multi-rank leg's collective: rank 0 prints
    the line (everything measured before the leg) with that leg as a deadline
    error when the ranks' agreed deadline passes, and the run exits non-zero
    instead of hanging until the driver's limit (bench.run_leg)."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["TD_BENCH_STALL_LEG"] = "leg_check:1"
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check",
                        "--leg-deadline", "8"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=220,
                       cwd=ROOT)
    el = time.time() - t0
    assert p.returncode != 0, p.stderr.decode(errors="replace")[-3000:]
    lines = [x for x in p.stdout.decode().splitlines() if x.startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr.decode(errors="replace")[-3000:])
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2
    assert out["leg_check"]["error"] == "deadline"
    assert el < 8 + 100  # the deadline, not the process group's 120 s timeout


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
