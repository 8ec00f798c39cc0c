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


def test_batched_search_ties_nan_and_chunks(tt, ctx):
    """A section's nodes take the all-models launch (k_raster_brute): a
    model's cells are split over 8 waves (slices of 625 at 5000 cells), so
    duplicated cells far apart in index (ties across slices: the lower index
    wins), NaN cells, an empty model, models of fewer cells than slices x 8,
    cells beyond the 1e9 sentinel distance and nodes on cell sites; 6 models,
    not a multiple of the 8 XCDs the models are dealt over."""
    rng = np.random.default_rng(5)
    base = tt.random_model(5000, 55).cells()
    x, y, z, ze = (a.copy() for a in base)
    x[4000:4600], y[4000:4600], z[4000:4600] = x[100:700], y[100:700], z[100:700]  # chunk 0 vs chunk 1
    ze[4000:4600] = ze[100:700] + 1.0
    x[::97] = np.nan
    far = (np.full(50, 4e4), np.full(50, 4e4), np.full(50, 4e4), np.arange(50.0))  # d >= 1e9: never counts
    empty = (np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0))
    qx = np.concatenate([rng.uniform(-100, 1100, 500), x[100:300]])
    qy = np.concatenate([rng.uniform(-200, 500, 500), y[100:300]])
    qz = np.concatenate([rng.uniform(-10, 700, 500), z[100:300]])
    qx[::50] = np.nan
    check(ctx, [(x, y, z, ze), far, empty, base, tt.random_model(2048, 9).cells(), tt.random_model(2049, 10).cells(),
               tt.random_model(3, 11).cells(), tt.random_model(37, 12).cells()],
          qx, qy, qz)


def test_many_nodes_take_the_per_model_search(tt, ctx):
    """Nodes x cells beyond the batched launch's budget: one search per model
    (the evaluate path's bucket grid), the same answer."""
    rng = np.random.default_rng(6)
    n = 60000
    qx, qy, qz = rng.uniform(-100, 1100, n), rng.uniform(-200, 500, n), rng.uniform(-10, 700, n)
    check(ctx, models_of(tt, [5000, 4500], 400), qx, qy, qz)
