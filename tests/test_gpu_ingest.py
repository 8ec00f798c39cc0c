"""GPU: td_trilinear (ingest.hip) -- the slowness of every ray point,
pre_process_data.jl:34 with load_3Dvel.jl:32's Gridded(Linear()) -- equals
the numpy oracle (oracle_np.trilinear, the same association) bit for bit;
points outside the grid are a BoundsError as in Interpolations.jl; and the
whole ingest (lau.vel + raypaths.p + p_tstar.dat + stations.lst ->
DataStruct -> evaluate) runs on synthetic files of those formats."""
import importlib

import numpy as np
import pytest

from ingest_files import write_all
from oracle import oracle_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ing(tt):
    return importlib.import_module(tt.__name__ + ".ingest")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_trilinear_bit_exact(ing, seed):
    rng = np.random.default_rng(seed)
    nx, ny, nz = [(9, 7, 11), (2, 2, 2), (40, 33, 60)][seed]
    xs, ys, zs = (np.sort(rng.uniform(a, b, n)) for (a, b), n in zip(((0, 10), (-5, 5), (0, 700)), (nx, ny, nz)))
    v = rng.uniform(0.1, 0.3, (nx, ny, nz))
    npts = 20000
    p = [rng.uniform(a[0], a[-1], npts) for a in (xs, ys, zs)]
    for c, a in enumerate((xs, ys, zs)):  # knots, faces, corners
        p[c][:200] = a[rng.integers(0, len(a), 200)]
        p[c][200:210] = a[0]
        p[c][210:220] = a[-1]
    got = ing.Gridded(xs, ys, zs, v)(p[0], p[1], p[2])
    want = oracle_np.trilinear(xs, ys, zs, v, p[0], p[1], p[2])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_bounds_error(ing):
    xs, ys, zs = np.arange(3.0), np.arange(4.0), np.arange(5.0)
    g = ing.Gridded(xs, ys, zs, np.ones((3, 4, 5)))
    assert g([0.5], [0.5], [0.5])[0] == 1.0
    for bad in ([2.0000001], [-1e-12], [np.nan]):
        with pytest.raises(ValueError, match="BoundsError"):
            g(bad, [0.5], [0.5])


def test_ingest_end_to_end(tt, ing, tmp_path):
    write_all(str(tmp_path), seed=5, nrays=40)
    raypaths, traces = ing.pre_process_data(str(tmp_path))
    itp = ing.load_3Dvel(str(tmp_path / "lau.vel"))
    ok = ~np.isnan(raypaths["x"])
    want = oracle_np.trilinear(itp.xs, itp.ys, itp.zs, itp.values, raypaths["x"][ok], raypaths["y"][ok],
                               raypaths["z"][ok])
    assert np.array_equal(raypaths["u"][ok], want)
    assert np.isnan(raypaths["u"][~ok]).all()
    ds = ing.load_data_Tonga_from(raypaths, traces)
    assert ds.rayX.shape == raypaths["x"].shape and len(ds.tS) == 40
    model, ds, valid = tt.evaluate(tt.random_model(300, 9), ds, tt.define_TDstructrure())
    assert valid == 1 and np.isfinite(model.phi) and len(model.ptS) == 40
