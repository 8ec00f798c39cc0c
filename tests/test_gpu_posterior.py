"""GPU: posterior cross-sections (plot_model_hist, MCsub.jl:753-825) against the
numpy oracle -- the v_nearest value of every model at every node, and the mean
/ std over models in Julia's association for a Vector of matrices -- bit for
bit, including the pairwise split beyond 1024 models and the 1-model NaN std."""
import numpy as np
import pytest

from oracle import oracle_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(tt, ds):
    return tt.TdContext.from_datastruct(ds)


def models_of(tt, sizes, seed0):
    return [tt.random_model(n, seed0 + k).cells() for k, n in enumerate(sizes)]


def check(ctx, models, qx, qy, qz):
    mean, std, vals = ctx.rasterize(models, qx, qy, qz, want_values=True)
    m2, s2, v2 = oracle_np.rasterize(models, qx, qy, qz)
    assert np.array_equal(vals, v2)
    assert np.array_equal(mean, m2)
    assert np.array_equal(std, s2, equal_nan=True)
    return mean, std


def test_small_and_mixed_model_sizes(tt, ctx):
    rng = np.random.default_rng(0)
    qx, qy, qz = rng.uniform(-100, 1100, 700), rng.uniform(-200, 500, 700), rng.uniform(-10, 700, 700)
    check(ctx, models_of(tt, [5, 40, 300, 1200, 7, 2000, 90, 600, 12, 100], 100), qx, qy, qz)  # n < 16
    check(ctx, models_of(tt, list(rng.integers(5, 400, 40)), 200), qx, qy, qz)  # sequential block
    _, std = check(ctx, models_of(tt, [300], 300), qx, qy, qz)  # one model: std = 0/0 = NaN
    assert np.all(np.isnan(std))


def test_more_than_1024_models(tt, ctx):
    """The pairwise split of Julia's mapreduce (blocks of <= 1024)."""
    rng = np.random.default_rng(1)
    qx, qy, qz = rng.uniform(0, 1000, 64), rng.uniform(-200, 400, 64), rng.uniform(0, 600, 64)
    models = [tuple(rng.uniform([0, -200, 0, 0], [1000, 400, 600, 50], (6, 4)).T) for _ in range(1100)]
    check(ctx, models, qx, qy, qz)


def test_plot_model_hist_sections(tt, ds):
    prm = tt.define_TDstructrure().replace(xzMap=True, ySlice=[0, 150], xyMap=True, zSlice=[100])
    hist = [[tt.random_model(80 + 10 * j, 10 * c + j) for j in range(6)] for c in range(2)]
    maps = tt.plot_model_hist(hist, ds, prm)
    assert set(maps) == {("xz", 0), ("xz", 150), ("xy", 100)}
    xv, yv, zv = (np.asarray(v) for v in (ds.xVec, ds.yVec, ds.zVec))
    flat = [m.cells() for chain in hist for m in chain]
    # the reference's comprehension order: m[i, j] = v_nearest(xVec[i], l0, zVec[j])
    i, j = 7, 11
    vals = [oracle_np.rasterize([c], [xv[i]], [150.0], [zv[j]])[0][0] for c in flat]
    m_ref = oracle_np.julia_mapreduce_arrays([np.array([v]) for v in vals])[0] / len(vals)
    assert maps[("xz", 150)]["mean"].shape == (len(xv), len(zv))
    assert maps[("xz", 150)]["mean"][i, j] == m_ref
    mk = maps[("xy", 100)]
    assert mk["mean"].shape == (len(xv), len(yv))
    assert np.array_equal(np.isnan(mk["masked"]), mk["std"] > 5)
