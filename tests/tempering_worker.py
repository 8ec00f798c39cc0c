"""One rank of a multi-process tempering ladder of real td_chain replicas
(BASELINE config 4 shape), started by tests/test_gpu_config4.py as a FRESH
child process (subprocess), never by exec of a GPU process.

usage: tempering_worker.py RANK WORLD PORT OUT.json LOCAL ROUNDS SWAP_EVERY NCELLS

Every rank holds LOCAL replicas on device 0 (rehearsal of one rank per GPU),
exchanges phi through torch.distributed gloo (Exchange.allgather; the GPU
runs use RCCL, the same code with backend "nccl") and writes its swap trace.
Replica g = rank * LOCAL + j: seed 100 + g, chain id 1 + g, model
random_model(NCELLS, 100 + g) -- SURVEY 8d config 4 (seeds 100 + rank).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ladder_chains(tt, ctx, prm, rank, local, ncells, engine):
    out = []
    for j in range(local):
        g = rank * local + j
        p = tt.chain_params(prm, None, seed=100 + g, chain=1 + g, engine=engine)
        out.append(tt.Chain(ctx, p, tt.random_model(ncells, 100 + g)))
    return out


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    local, rounds, swap_every, ncells = (int(x) for x in sys.argv[5:9])
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    import tonga

    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds, device=0)
    prm = tt.define_TDstructrure().replace(max_cells=2 * ncells)
    chains = ladder_chains(tt, ctx, prm, rank, local, ncells, tt.TD_ENGINE_DEVICE)
    lad = tt.TemperingLadder(chains, tt.Exchange(dist, "cpu"), tmax=8.0, seed=4242)
    trace = []
    for _ in range(rounds):
        phis = lad.step(swap_every)
        trace.append([[float(x) for x in phis], [int(x) for x in lad.levels]])
    models = [c.model() for c in chains]
    with open(out, "w") as f:
        json.dump({"trace": trace, "ncells": [len(m.xCell) for m in models],
                   "zeta_sum": [float(sum(m.zeta)) for m in models],
                   "phi": [c.stats()["phi"] for c in chains]}, f)
    for c in chains:
        c.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
