"""BASELINE config 4 through RCCL on ONE GPU: a rank started by
`torch.distributed.run --nproc-per-node N` (tests/test_gpu_config4.py), every
rank holding 8/N replicas on its device, process group "nccl" (= RCCL).

usage: rccl_worker.py OUT_PREFIX ROUNDS SWAP_EVERY NCELLS NREP

Two ladders over the same replicas, each written to OUT_PREFIX.<rank>.json:

* host loop: TemperingLadder.step per round -- the resident round, then
  Exchange.allgather FORCED through torch.distributed's
  all_gather_into_tensor even at world 1 (no identity shortcut), then the
  swap decision in Python; compute / gather / decide seconds per round;
* device swaps: TemperingLadder.run with the library's own RCCL communicator
  (NativeComm, its id shipped through torch.distributed): td_rounds_exchange,
  the allgathers issued on an exchange stream that waits on the kernel's
  flag, the swaps decided inside the kernel -- no host in the loop.

Replica g = rank * local + j: seed 100 + g, chain id 1 + g, model
random_model(NCELLS, 100 + g).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    out, rounds, swap_every, ncells, nrep = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5])
    import torch
    import torch.distributed as dist

    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local_rank)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    rank, world = dist.get_rank(), dist.get_world_size()
    assert dist.get_backend() == "nccl"
    import tonga
    from tempering_worker import ladder_chains

    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds, device=local_rank)
    prm = tt.define_TDstructrure().replace(max_cells=2 * ncells)
    local = nrep // world
    res = {"rank": rank, "world": world}

    # 1. the host loop, the allgather forced through RCCL
    chains = ladder_chains(tt, ctx, prm, rank, local, ncells, tt.TD_ENGINE_DEVICE)
    ex = tt.Exchange(dist, "cuda", force=True)
    lad = tt.TemperingLadder(chains, ex, tmax=8.0, seed=4242)
    assert lad.resident
    trace = []
    t0 = time.perf_counter()
    for _ in range(rounds):
        phis = lad.step(swap_every)
        trace.append([[float(x) for x in phis], [int(x) for x in lad.levels]])
    el = time.perf_counter() - t0
    lad.close()
    res["host_loop"] = {"trace": trace, "digest": lad.trace_digest(), "ms_per_round": el / rounds * 1e3,
                        "compute_us_per_round": lad.compute_s / rounds * 1e6,
                        "gather_us_per_round": lad.gather_s / rounds * 1e6,
                        "decide_us_per_round": lad.decide_s / rounds * 1e6,
                        "stats": [c.stats() for c in chains]}
    for c in chains:
        c.close()

    # 2. device swaps through the library's RCCL communicator
    chains = ladder_chains(tt, ctx, prm, rank, local, ncells, tt.TD_ENGINE_DEVICE)
    ex = tt.Exchange(dist, "cuda", native=local_rank)
    lad = tt.TemperingLadder(chains, ex, tmax=8.0, seed=4242, device_swaps=True)
    assert lad.device_swaps
    warm = min(20, rounds)
    lad.run(warm, swap_every)
    t0 = time.perf_counter()
    lad.run(rounds - warm, swap_every)
    el = time.perf_counter() - t0
    lad.close()
    res["device_swaps"] = {"digest": lad.trace_digest(), "ms_per_round": el / max(rounds - warm, 1) * 1e3,
                           "timing": lad.timing, "levels": [int(x) for x in lad.levels],
                           "stats": [c.stats() for c in chains]}
    for c in chains:
        c.close()
    ex.comm.close()
    ctx.close()
    with open("%s.%d.json" % (out, rank), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
