"""One rank of a ray-sharded evaluate (mcmc-in-tonga_amd/sharded.py), started
by tests/test_gpu_sharded.py as a FRESH child process (subprocess), never by
exec of a GPU process.  Every rank owns its ray range on device 0 (rehearsal
of one rank per GPU), gathers ptS over torch.distributed gloo (RCCL on the
GPU box: the same code with backend "nccl") and writes what it got.

usage: sharded_worker.py RANK WORLD PORT OUT.json NRAYS
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def models(tt):
    """Unrelated models, then a chain-like walk of one edit per call (the
    shards' incremental paths): birth, change, move, death."""
    import numpy as np

    out = [tt.random_model(n, s).cells() for n, s in ((3000, 1), (200, 2), (1, 3))]
    x, y, z, v = (np.array(a) for a in tt.random_model(2000, 4).cells())
    out.append((x, y, z, v))
    rng = np.random.default_rng(9)
    for k in range(12):
        x, y, z, v = x.copy(), y.copy(), z.copy(), v.copy()
        a = k % 4
        if a == 0:
            x, y, z, v = (np.append(q, q[7] + 1.5) for q in (x, y, z, v))
        elif a == 1:
            v[int(rng.integers(len(v)))] = float(rng.uniform(0, 50))
        elif a == 2:
            i = int(rng.integers(len(x)))
            x[i] += 3.0
            z[i] -= 2.0
        else:
            i = int(rng.integers(len(x)))
            x, y, z, v = (np.delete(q, i) for q in (x, y, z, v))
        out.append((x, y, z, v))
    return out


def main():
    rank, world, port, out, nrays = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    import tonga

    tt = tonga.load()
    ds = tt.synthetic_rays(nrays, seed=5)
    sc = tt.RayShardedContext(ds, tt.Exchange(dist, "cpu"), device=0)
    res = []
    for cells in models(tt):
        ptS, phi, lk = sc.evaluate(cells)
        res.append({"ptS": ptS.tobytes().hex(), "phi": phi, "lk": lk})
    with open(out, "w") as f:
        json.dump({"bounds": sc.bounds, "P_local": sc.P_local, "res": res}, f)
    sc.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
