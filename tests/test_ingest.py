"""Ray/slowness ingest: pre_process_data.jl and
load_3Dvel.jl on synthetic files of their formats (the real lau.vel,
raypaths.p, p_tstar.dat, stations.lst do not ship).  CPU: parsing, layout,
the reference's quirks, and the trilinear oracle against scipy's
RegularGridInterpolator.  Parity with Interpolations.jl itself is unpinned
(not in the reference tree): see oracle_np.trilinear."""
import importlib

import numpy as np
import pytest

from ingest_files import write_all


@pytest.fixture(scope="module")
def ing(tt):
    return importlib.import_module(tt.__name__ + ".ingest")


def test_load_3Dvel(ing, tmp_path):
    w = write_all(str(tmp_path))
    itp = ing.load_3Dvel(str(tmp_path / "lau.vel"))
    assert np.array_equal(itp.xs, w["xs"]) and np.array_equal(itp.ys, w["ys"]) and np.array_equal(itp.zs, w["zs"])
    vp = np.array([[[float("%.6f" % v) for v in row] for row in plane] for plane in w["vp"][0]])
    assert np.array_equal(itp.values, 1.0 / vp)  # sn[1,:,:,:] = 1 ./ vps (P)


@pytest.mark.parametrize("trailing", [False, True])
def test_load_raypath_layout(ing, tmp_path, trailing):
    w = write_all(str(tmp_path), seed=1, trailing_separator=trailing)
    r = ing.load_raypath(str(tmp_path / "raypaths.p"), itp=None)
    rays = w["rays"]
    n = len(rays) + (1 if trailing else 0)  # a file ending in a separator adds an empty ray (:37-40)
    m = max(len(a) for a in rays)
    assert r["x"].shape == (m, n)
    for i, a in enumerate(rays):
        c = len(a)
        got = np.column_stack([r["x"][:c, i], r["y"][:c, i], r["z"][:c, i]])
        assert np.array_equal(got, np.array([[float("%.6f" % v) for v in row] for row in a]))
        assert np.isnan(r["x"][c:, i]).all()
    if trailing:
        assert np.isnan(r["x"][:, -1]).all()


def test_load_traceinfo(ing, tmp_path):
    w = write_all(str(tmp_path), seed=2)
    t = ing.load_traceinfo(str(tmp_path / "p_tstar.dat"), str(tmp_path / "stations.lst"))
    assert list(t["station"]) == [row[0] for row in w["traces"]]
    assert np.allclose(t["tStar"], [row[4] for row in w["traces"]], rtol=0, atol=5e-5)
    assert np.allclose(t["aveatten"], [row[7] for row in w["traces"]], rtol=0, atol=5e-6)
    lat = [w["stations"][row[0]][0] for row in w["traces"]]
    assert np.allclose(t["latitude"], lat, atol=5e-5)


def test_trilinear_oracle_vs_scipy():
    from scipy.interpolate import RegularGridInterpolator

    from oracle import oracle_np
    rng = np.random.default_rng(4)
    xs, ys, zs = np.sort(rng.uniform(0, 10, 9)), np.sort(rng.uniform(-5, 5, 7)), np.sort(rng.uniform(0, 700, 11))
    v = rng.uniform(0.1, 0.3, (9, 7, 11))
    p = np.column_stack([rng.uniform(xs[0], xs[-1], 500), rng.uniform(ys[0], ys[-1], 500),
                         rng.uniform(zs[0], zs[-1], 500)])
    p[:20] = np.column_stack([xs[rng.integers(0, 9, 20)], ys[rng.integers(0, 7, 20)], zs[rng.integers(0, 11, 20)]])
    got = oracle_np.trilinear(xs, ys, zs, v, p[:, 0], p[:, 1], p[:, 2])
    want = RegularGridInterpolator((xs, ys, zs), v, method="linear")(p)
    assert np.allclose(got, want, rtol=1e-13, atol=0)
    i, j, k = (np.searchsorted(a, p[:20, c]) for c, a in enumerate((xs, ys, zs)))
    assert np.array_equal(got[:20], v[i, j, k])  # at the knots: the grid values exactly
    out = oracle_np.trilinear(xs, ys, zs, v, [xs[0] - 1e-9], [ys[0]], [zs[0]])
    assert np.isnan(out).all()
