"""Ray-sharded evaluate on the GPU (mcmc-in-tonga_amd/sharded.py, SURVEY 8e's
intra-chain split): two fresh child processes (gloo, both on device 0), each
owning half the rays of a stress-shaped geometry, gather their ptS and compute
phi with td_misfit; both ranks must end with (ptS, phi, likelihood)
bit-identical to one context's td_evaluate of all rays -- for unrelated
models and for a chain-like walk of one edit per call (each shard's
incremental path)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from sharded_worker import models  # noqa: E402

NRAYS = 3000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_single_process_sharded_is_plain_evaluate(tt):
    ds = tt.synthetic_rays(500, seed=5)
    sc = tt.RayShardedContext(ds, tt.Exchange())
    ctx = tt.TdContext.from_datastruct(ds)
    tt.lib().tdt_set_incremental(ctx.h, 0)
    for cells in models(tt)[:6]:
        ptS, phi, lk = sc.evaluate(cells)
        p2, f2, l2, _ = ctx.evaluate(cells)
        assert np.array_equal(ptS, p2) and phi == f2 and lk == l2
    sc.close()
    ctx.close()


@pytest.mark.timeout(400)
def test_two_processes_sharded_equals_whole(tt, tmp_path):
    import torch.distributed  # noqa: F401  (warm the import before two children load it at once)

    world, port = 2, _free_port()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "sharded_worker.py"), str(r), str(world),
                               str(port), str(tmp_path / ("r%d.json" % r)), str(NRAYS)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode(errors="replace"))
    assert all(p.returncode == 0 for p in procs), outs
    r = [json.load(open(tmp_path / ("r%d.json" % k))) for k in range(world)]
    assert r[0]["res"] == r[1]["res"]
    assert r[0]["bounds"][0][1] == r[1]["bounds"][1][0] and 0 < r[0]["P_local"] and 0 < r[1]["P_local"]
    ds = tt.synthetic_rays(NRAYS, seed=5)
    ctx = tt.TdContext.from_datastruct(ds)
    tt.lib().tdt_set_incremental(ctx.h, 0)
    for cells, got in zip(models(tt), r[0]["res"]):
        ptS, phi, lk, _ = ctx.evaluate(cells)
        assert bytes.fromhex(got["ptS"]) == ptS.tobytes()
        assert got["phi"] == phi and got["lk"] == lk
    ctx.close()
