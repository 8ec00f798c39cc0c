"""Ray-sharded evaluate (mcmc-in-tonga_amd/sharded.py), CPU side: the ray
partition, the sub-DataStruct, and the world-2 gloo exchange (every rank's
shard gathered in ray order, phi over all rays) with a host stand-in for the
per-rank context -- the C oracle, as test infrastructure -- so that the N > 1
path is covered without a GPU.  The HIP path is tests/test_gpu_sharded.py."""
import json
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_rays_partition():
    import tonga

    tt = tonga.load()
    rng = np.random.default_rng(3)
    for n, world in ((381, 1), (381, 2), (381, 8), (7, 8), (10000, 8), (1, 3)):
        pts = rng.integers(1, 131, n)
        b = tt.shard_rays(pts, world)
        assert len(b) == world and b[0][0] == 0 and b[-1][1] == n
        assert all(b[k][1] == b[k + 1][0] and b[k][0] <= b[k][1] for k in range(world - 1))
        loads = [int(pts[a:c].sum()) for a, c in b]
        if n >= world:  # balanced to within one ray's points of the ideal share
            assert max(loads) - pts.sum() / world <= pts.max()
    ds = tt.load_data_Tonga()
    rp = tt.ray_points(ds)
    assert int(rp.sum()) == int((~np.isnan(ds.rayX)).sum())


def test_sub_datastruct_slices_rays():
    import tonga

    tt = tonga.load()
    ds = tt.load_data_Tonga()
    s = tt.sub_datastruct(ds, 100, 200)
    assert s.rayX.shape == (ds.rayX.shape[0], 100) and s.rayL.shape == (ds.rayL.shape[0], 100)
    assert np.array_equal(s.tS, ds.tS[100:200]) and np.array_equal(s.allSig, ds.allSig[100:200])
    assert np.array_equal(s.rayZ, ds.rayZ[:, 100:200], equal_nan=True)


class HostContext:
    """Stand-in for TdContext in the CPU suite: the C oracle (checker code)."""

    def __init__(self, ds, device=-1):
        import oracle

        self.o = oracle
        self.ds = ds
        self.P = int((~np.isnan(ds.rayX)).sum())

    def evaluate(self, cells):
        d = self.ds
        r = self.o.evaluate(d.rayX, d.rayY, d.rayZ, d.rayL, d.rayU, d.tS, d.allSig, cells)
        return r["ptS"], r["phi"], r["likelihood"], None

    def misfit(self, ptS, tS, allSig):
        from oracle import oracle_np

        return oracle_np.chi2(ptS, tS, allSig), oracle_np.likelihood(allSig)

    def close(self):
        pass


def _worker(rank, world, port, outdir):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    import tonga

    tt = tonga.load()
    ds = tt.synthetic_rays(300, seed=5)
    sc = tt.RayShardedContext(ds, tt.Exchange(dist, "cpu"), make_context=HostContext)
    res = []
    for nc, seed in ((50, 1), (400, 2), (1, 3)):
        ptS, phi, lk = sc.evaluate(tt.random_model(nc, seed).cells())
        res.append({"ptS": [float(x) for x in ptS], "phi": phi, "lk": lk})
    with open(os.path.join(outdir, "r%d.json" % rank), "w") as f:
        json.dump({"bounds": sc.bounds, "res": res}, f)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_gloo_world2_sharded_evaluate_equals_whole(tmp_path, orc):
    import torch.multiprocessing as mp

    import tonga

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [json.load(open(tmp_path / ("r%d.json" % k))) for k in range(2)]
    assert r[0] == r[1]  # every rank ends with the same (ptS, phi, likelihood)
    b = r[0]["bounds"]
    assert b[0][0] == 0 and b[0][1] == b[1][0] and 0 < b[0][1] < 300
    tt = tonga.load()
    ds = tt.synthetic_rays(300, seed=5)
    for (nc, seed), got in zip(((50, 1), (400, 2), (1, 3)), r[0]["res"]):
        ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig,
                           tt.random_model(nc, seed).cells())
        assert np.array_equal(np.array(got["ptS"]), ref["ptS"])
        assert got["phi"] == ref["phi"] and got["lk"] == ref["likelihood"]
