"""BASELINE config 4 on the GPU: 8 tempered replicas x 2000 cells, geometric
T in [1, 8], a temperature swap every 10 proposals.

* one process: the 8 DEVICE replicas (one td_chain_run_batch launch per
  round) make exactly the moves and swaps of 8 HOST replicas, which evaluate
  every proposal in full as the reference does (TD_inversion_function.jl:93,
  141,191,238);
* two fresh child processes (subprocess, gloo, both on device 0, 4 replicas
  each) exchanging phi through torch.distributed: every rank sees the same
  gathered vector and the ladder's trace equals the one-process ladder;
* RCCL on the one GPU: a rank under `torch.distributed.run --nproc-per-node 1`
  with process group "nccl", the 8 replicas (tests/rccl_worker.py), once with
  Exchange.allgather forced through all_gather_into_tensor (the host loop)
  and once with the swaps decided in the kernel over the library's own RCCL
  communicator (td_rounds_exchange): both traces equal the one-process ladder;
* the device-decided ladder on one rank (no collective) and through a lone
  RCCL communicator, against the same.
"""
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
from tempering_worker import ladder_chains  # noqa: E402

NREP, NCELLS, SWAP_EVERY, ROUNDS = 8, 2000, 10, 320  # bench.py config4_tempering: 20 + 300 rounds


def trace_of(tt, chains):
    lad = tt.TemperingLadder(chains, tmax=8.0, seed=4242)
    assert lad.batch or chains[0].params.engine == tt.TD_ENGINE_HOST
    trace = []
    for _ in range(ROUNDS):
        phis = lad.step(SWAP_EVERY)
        trace.append([[float(x) for x in phis], [int(x) for x in lad.levels]])
    return trace, lad


@pytest.fixture(scope="module")
def ctx(tt, ds):
    c = tt.TdContext.from_datastruct(ds)
    yield c
    c.close()


@pytest.fixture(scope="module")
def device_run(tt, ctx):
    prm = tt.define_TDstructrure().replace(max_cells=2 * NCELLS)
    chains = ladder_chains(tt, ctx, prm, 0, NREP, NCELLS, tt.TD_ENGINE_DEVICE)
    trace, lad = trace_of(tt, chains)
    models = [c.model() for c in chains]
    out = dict(trace=trace, models=models, rates=lad.swap_rates(), stats=[c.stats() for c in chains],
               digest=lad.trace_digest(), levels=[int(x) for x in lad.levels])
    for c in chains:
        c.close()
    return out


def test_config4_ladder_device_matches_host(tt, ctx, device_run):
    prm = tt.define_TDstructrure().replace(max_cells=2 * NCELLS)
    chains = ladder_chains(tt, ctx, prm, 0, NREP, NCELLS, tt.TD_ENGINE_HOST)
    trace, lad = trace_of(tt, chains)
    assert trace == device_run["trace"]
    for c, m, st in zip(chains, device_run["models"], device_run["stats"]):
        h = c.model()
        assert np.array_equal(h.xCell, m.xCell) and np.array_equal(h.zeta, m.zeta)
        assert c.stats()["accepted"] == st["accepted"] and c.stats()["proposed"] == st["proposed"]
        c.close()
    assert lad.swap_rates() == device_run["rates"]
    assert sum(sum(st["accepted"]) for st in device_run["stats"]) > 0
    assert any(r > 0 for r in device_run["rates"])  # temperatures actually moved
    assert sorted(device_run["trace"][-1][1]) == list(range(NREP))


def test_config4_end_states_match_oracle(orc, ds, device_run):
    """The 8 replicas' end states after the bench's 320 rounds (3200
    proposals each, at their ladder temperatures): (ptS, phi) of each final
    model == the C oracle's evaluate of it, bit for bit (MCsub.jl:123-185)."""
    for m, st in zip(device_run["models"], device_run["stats"]):
        ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, m.cells())
        assert ref["rc"] == 0
        assert ref["phi"] == m.phi == st["phi"]
        assert np.array_equal(ref["ptS"], m.ptS)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(400)
def test_config4_two_processes_gloo_match_one_process(tt, device_run, tmp_path):
    import torch.distributed  # noqa: F401  (warm the import before two children load it at once)

    world, local, port = 2, NREP // 2, _free_port()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "tempering_worker.py"), str(r), str(world),
                               str(port), str(tmp_path / ("r%d.json" % r)), str(local), str(ROUNDS),
                               str(SWAP_EVERY), str(NCELLS)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT)
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
    assert r[0]["trace"] == r[1]["trace"]  # every rank gathered the same phis and made the same swaps
    assert r[0]["trace"] == device_run["trace"]  # ... and they are the one-process ladder's
    ms = device_run["models"]
    assert r[0]["ncells"] + r[1]["ncells"] == [len(m.xCell) for m in ms]
    assert r[0]["zeta_sum"] + r[1]["zeta_sum"] == [float(sum(m.zeta)) for m in ms]


def device_swap_ladder(tt, ctx, comm=None):
    """The same 8 replicas, all on this GPU, the swaps decided in the kernel
    (td_rounds_exchange): one rank with no collective, or through `comm`."""
    prm = tt.define_TDstructrure().replace(max_cells=2 * NCELLS)
    chains = ladder_chains(tt, ctx, prm, 0, NREP, NCELLS, tt.TD_ENGINE_DEVICE)
    ex = tt.Exchange()
    ex.comm = comm
    lad = tt.TemperingLadder(chains, ex, tmax=8.0, seed=4242, device_swaps=True)
    assert lad.device_swaps
    lad.run(20, SWAP_EVERY)
    lad.run(ROUNDS - 20, SWAP_EVERY)
    lad.close()
    out = dict(digest=lad.trace_digest(), levels=[int(x) for x in lad.levels], models=[c.model() for c in chains],
               stats=[c.stats() for c in chains], rates=lad.swap_rates(), timing=lad.timing)
    for c in chains:
        c.close()
    return out


def same_as_device_run(out, device_run):
    assert out["digest"] == device_run["digest"]
    assert out["levels"] == device_run["levels"]
    for m, dm, st, ds_ in zip(out["models"], device_run["models"], out["stats"], device_run["stats"]):
        assert np.array_equal(m.xCell, dm.xCell) and np.array_equal(m.zeta, dm.zeta)
        assert st["accepted"] == ds_["accepted"] and st["phi"] == ds_["phi"] and st["iterations"] == ds_["iterations"]


def test_config4_device_swaps_one_rank(tt, ctx, device_run):
    """td_rounds_exchange with no collective: the replicas' phis meet in device
    memory and every workgroup decides the swaps; the trace, levels, models
    and counts equal the host-decided ladder's."""
    out = device_swap_ladder(tt, ctx)
    same_as_device_run(out, device_run)
    assert out["rates"] == device_run["rates"]


def test_config4_device_swaps_lone_rccl_comm(tt, ctx, device_run):
    """The same through a one-rank RCCL communicator of the library: every
    round an ncclAllGather on the exchange stream, which waits on the flag
    the kernel raises (hipStreamWaitValue64) and then writes the round's
    gdone; same trace."""
    comm = tt.NativeComm(0)
    try:
        assert np.array_equal(comm.allgather(np.array([1.5, -2.0])), [1.5, -2.0])
        out = device_swap_ladder(tt, ctx, comm)
    finally:
        comm.close()
    same_as_device_run(out, device_run)
    assert out["timing"]["exchange_us_per_round"] > 0.0


@pytest.mark.timeout(400)
def test_config4_rccl_world1_matches_one_process(tt, device_run, tmp_path):
    """One rank under torch.distributed.run with process group "nccl": the
    host loop (allgather forced through RCCL's all_gather_into_tensor, the
    rounds resident on their own hardware queue) and the device-decided
    ladder (the library's RCCL communicator) both reproduce the one-process
    ladder -- the first RCCL runs of the exchange step on an MI355X."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "rccl_worker.py"),
           str(tmp_path / "rccl"), str(ROUNDS), str(SWAP_EVERY), str(NCELLS), str(NREP)]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=380)
    log = p.stdout.decode(errors="replace")
    assert p.returncode == 0, log[-4000:]
    r = json.load(open(str(tmp_path / "rccl") + ".0.json"))
    assert r["world"] == 1
    assert r["host_loop"]["trace"] == device_run["trace"]
    assert r["host_loop"]["digest"] == r["device_swaps"]["digest"] == device_run["digest"]
    assert r["device_swaps"]["levels"] == device_run["levels"]
    for a, b, c in zip(r["host_loop"]["stats"], r["device_swaps"]["stats"], device_run["stats"]):
        assert a["phi"] == b["phi"] == c["phi"] and a["accepted"] == b["accepted"] == c["accepted"]
    print("rccl world 1:", json.dumps({k: {x: y for x, y in v.items() if x not in ("trace", "stats")}
                                       for k, v in r.items() if isinstance(v, dict)}))
