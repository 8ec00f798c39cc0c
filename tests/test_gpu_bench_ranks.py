"""bench.py's N > 1 path, as the driver launches it (torch.distributed.run,
one process per rank), rehearsed on one GPU: two ranks over gloo, both on
device 0 (TD_BENCH_BACKEND=gloo TD_BENCH_DEVICE=0), reduced sizes.  The
JSON line must carry the config-4 ranks block with a swap trace equal to the
one-process ladder's, its per-round split and roofline, and the config-5
stress chains block with its roofline (BASELINE configs 4 and 5;
main_inversion.jl:15, define_TDstructure.jl:56)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(420)
@pytest.mark.parametrize("launcher", ["torchrun", "none"])
def test_bench_two_ranks_gloo(launcher):
    """launcher "none": plain `bench.py --gpus 2`, which starts its two ranks
    itself before any GPU call (bench.spawn_ranks)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(TD_BENCH_BACKEND="gloo", TD_BENCH_DEVICE="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    pre = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
            "127.0.0.1", "--master-port", str(port)] if launcher == "torchrun" else [sys.executable])
    cmd = pre + [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--iters-per-step", "500", "--no-cpu-baseline", "--no-full-evaluate", "--no-dropin",
           "--batch-chains", "0", "--config4-rounds", "40", "--stress-iters", "100", "--no-phases"]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=400, cwd=ROOT)
    text = p.stdout.decode(errors="replace")
    assert p.returncode == 0, text[-4000:]
    lines = [x for x in text.splitlines() if x.startswith("{")]
    assert len(lines) == 1, text[-4000:]  # rank 0 alone prints
    line = lines[0]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["roofline"]["bound"] == "latency"
    c4 = out["config4_ranks"]
    assert c4["replicas"] == 2 and c4["trace_matches_single_process"] is True, c4
    assert c4["proposals_per_s"] > 0
    hl = c4["modes"]["host_loop"]  # (gloo: no device_swaps mode, which needs RCCL)
    assert set(hl["split_us_per_round"]) == {"compute", "gather", "decide"} and hl["split_us_per_round"]["gather"] > 0
    for roof in (c4["roofline"], hl["roofline"]):
        assert roof["bound"] == "latency" and roof["achieved"] > 0 and roof["unit"] == "GB/s"
        assert roof["latency"]["cycles_per_proposal"] > 0
    sc = out["stress_chains"]
    assert sc["chains"] == 2 and sc["proposals_per_s"] > 0
    assert sc["roofline"]["bound"] == "latency" and sc["roofline"]["achieved"] > 0
    assert "stress_sharded" in out


@pytest.mark.timeout(300)
def test_bench_stalled_leg_prints_headline():
    """The driver's N-GPU run must not hang silently on a multi-rank leg: rank 1
    stalls in the config-4 leg (TD_BENCH_STALL_LEG) before its first collective;
    when the ranks' agreed deadline passes, rank 0 prints ONE line with the
    headline already measured, config4_ranks as a deadline error and the later
    legs as skipped, and the run exits non-zero (bench.run_leg)."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(TD_BENCH_BACKEND="gloo", TD_BENCH_DEVICE="0", TD_BENCH_STALL_LEG="config4_ranks:1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--iters-per-step", "500", "--no-cpu-baseline", "--no-full-evaluate", "--no-dropin", "--batch-chains", "0",
           "--config4-rounds", "40", "--stress-iters", "100", "--no-phases", "--leg-deadline", "20"]
    t0 = time.time()
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=280, cwd=ROOT)
    el = time.time() - t0
    text = p.stdout.decode(errors="replace")
    assert p.returncode != 0, text[-4000:]
    lines = [x for x in text.splitlines() if x.startswith("{")]
    assert len(lines) == 1, text[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["roofline"]["frac"] <= 1.0
    assert out["config4_ranks"]["error"] == "deadline", out["config4_ranks"]
    assert out["stress_chains"]["error"].startswith("skipped") and out["stress_sharded"]["error"].startswith("skipped")
    assert el < 250
