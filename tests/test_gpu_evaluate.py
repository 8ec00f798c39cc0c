"""GPU parity of the forward model (td_evaluate / td_interpolate) against the
CPU oracle: nearest-cell indices, ptS, phi and likelihood must be BIT-EXACT
(the kernels reproduce the reference's FP64 rounding and Julia's sum order).
The north-star tolerance (1e-6 relative for t*/log-likelihood) is therefore
met with margin; every assertion below is exact equality."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def ref_eval(orc, ds, cells, debug_prior=0):
    return orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, cells, debug_prior)


def assert_same(ctx, orc, ds, cells):
    ptS, phi, lk, near = ctx.evaluate(cells, want_nearest=True)
    ref = ref_eval(orc, ds, cells)
    assert ref["rc"] == 0
    assert np.array_equal(near, ref["nearest"]), "nearest indices differ"
    assert np.array_equal(ptS, ref["ptS"]), np.max(np.abs(ptS - ref["ptS"]))
    assert phi == ref["phi"]
    assert lk == ref["likelihood"]
    return ptS, phi


@pytest.fixture(scope="module")
def ctx(tt, ds):
    return tt.TdContext.from_datastruct(ds)


@pytest.mark.parametrize("ncells,seed", [(200, 1), (1000, 2), (2000, 100), (5000, 3), (0, 1), (1, 7), (63, 5)])
def test_configs_381_rays(tt, orc, ds, ctx, ncells, seed):
    assert_same(ctx, orc, ds, tt.random_model(ncells, seed).cells())


def test_reference_evaluate_api(tt, orc, ds):
    prm = tt.define_TDstructrure()
    model = tt.random_model(1000, 2)
    m2, ds2, valid = tt.evaluate(model, ds, prm)
    assert m2 is model and ds2 is ds and valid == 1
    ref = ref_eval(orc, ds, model.cells())
    assert np.array_equal(model.ptS, ref["ptS"]) and model.phi == ref["phi"]
    assert model.tS is ds.tS and model.likelihood == ref["likelihood"]
    m3, _, _ = tt.evaluate(tt.random_model(5, 1), ds, prm.replace(debug_prior=1))
    assert m3.phi == 1 and m3.likelihood == 1


def test_ties_duplicates_and_sentinel(tt, orc, ds, ctx):
    base = tt.random_model(300, 11)
    # duplicate every 3rd cell later in the list (exact distance ties: first index must win)
    x, y, z, zeta = (np.concatenate([a, a[::3]]) for a in base.cells())
    zeta[300:] += 1.0  # duplicates carry different values, so a wrong tie-break changes ptS
    assert_same(ctx, orc, ds, (x, y, z, zeta))
    # cells placed exactly ON ray points (distance 0) and mirrored pairs equidistant to a point
    px = ds.rayX[~np.isnan(ds.rayX)]
    py = ds.rayY[~np.isnan(ds.rayY)]
    pz = ds.rayZ[~np.isnan(ds.rayZ)]
    sel = np.arange(0, len(px), 97)
    x2 = np.concatenate([px[sel], px[sel] + 3.0, px[sel] - 3.0])
    y2 = np.concatenate([py[sel], py[sel], py[sel]])
    z2 = np.concatenate([pz[sel], pz[sel], pz[sel]])
    zeta2 = np.arange(len(x2), dtype=np.float64) % 50
    assert_same(ctx, orc, ds, (x2, y2, z2, zeta2))
    # every cell farther than sqrt(1e9): nothing beats the sentinel, zeta0 = 0
    far = (np.full(4, 1e5), np.zeros(4), np.zeros(4), np.ones(4))
    ptS, _ = assert_same(ctx, orc, ds, far)
    assert np.all(ptS == 0.0)


def test_model_jld_cells_on_381_rays(tt, orc, ds, ctx, kat):
    # the reference's own saved models (frame-shifted vs these rays, still valid input)
    off = kat["cell_off"]
    for k in range(0, len(off) - 1, 9):
        sl = slice(off[k], off[k + 1])
        assert_same(ctx, orc, ds, (kat["xCell"][sl], kat["yCell"][sl], kat["zCell"][sl], kat["zeta"][sl]))


def test_edge_rays_and_long_rays(tt, orc):
    # rays of 0, 1, 2 points, full-length, NaN inside Y of a valid point, and a
    # 2100-point ray (exercises Julia's pairwise sum split above 1024 terms)
    m = 2100
    rays = [np.zeros((0, 3)), np.array([[1.0, 2.0, 3.0]]), np.array([[0, 0, 0], [10, 0, 5.0]])]
    t = np.linspace(0, 1, m)[:, None]
    rays.append(np.array([20.0, -100.0, 600.0]) + t * np.array([800.0, 300.0, -600.0]))
    r5 = np.array([[100.0, 10.0, 50.0], [110.0, np.nan, 60.0], [120.0, 12.0, 70.0]])
    rays.append(r5)
    n = len(rays)
    X, Y, Z = (np.full((m, n), np.nan) for _ in range(3))
    for i, r in enumerate(rays):
        X[:len(r), i], Y[:len(r), i], Z[:len(r), i] = r[:, 0], r[:, 1], r[:, 2]
    U = np.where(np.isnan(X), np.nan, 0.1 + 0.001 * np.nan_to_num(Z))
    L, Uu = tt.segments(X, Y, Z, U)
    # the NaN in Y makes two rayL entries NaN; keep the layout valid by giving
    # those segments a finite length (the reference would carry the NaN into ptS)
    L[0:2, 4] = [3.0, 4.0]
    tS = np.linspace(0.1, 0.5, n)
    sig = np.linspace(0.05, 0.3, n)
    ds2 = tt.DataStruct(tS, tS, tS, tS, sig, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, X, Y, Z, L, Uu, U)
    c2 = tt.TdContext.from_datastruct(ds2)
    for nc, seed in ((1, 1), (37, 2), (700, 3)):
        assert_same(c2, orc, ds2, tt.random_model(nc, seed).cells())
    c2.close()


def test_long_and_short_rays_on_the_grid(tt, orc):
    """Rays of 1, 2, 9, 17 and 2100 points (Julia's pairwise split above 1024
    terms) through the grid search (>= 256 cells) against the oracle."""
    m = 2100
    t = np.linspace(0, 1, m)[:, None]
    rays = [np.array([[1.0, 2.0, 3.0]]), np.array([[0, 0, 0], [10, 0, 5.0]]),
            np.array([300.0, 50.0, 100.0]) + np.linspace(0, 1, 9)[:, None] * np.array([50.0, 20.0, 30.0]),
            np.array([500.0, -50.0, 200.0]) + np.linspace(0, 1, 17)[:, None] * np.array([-80.0, 40.0, 60.0]),
            np.array([20.0, -100.0, 600.0]) + t * np.array([800.0, 300.0, -600.0])]
    n = len(rays)
    X, Y, Z = (np.full((m, n), np.nan) for _ in range(3))
    for i, r in enumerate(rays):
        X[:len(r), i], Y[:len(r), i], Z[:len(r), i] = r[:, 0], r[:, 1], r[:, 2]
    U = np.where(np.isnan(X), np.nan, 0.1 + 0.001 * np.nan_to_num(Z))
    L, Uu = tt.segments(X, Y, Z, U)
    tS = np.linspace(0.1, 0.5, n)
    sig = np.linspace(0.05, 0.3, n)
    ds2 = tt.DataStruct(tS, tS, tS, tS, sig, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, X, Y, Z, L, Uu, U)
    c2 = tt.TdContext.from_datastruct(ds2)
    for nc, seed in ((300, 4), (2000, 5)):
        assert_same(c2, orc, ds2, tt.random_model(nc, seed).cells())
    c2.close()


def test_layout_error_is_reported(tt, ds):
    L = ds.rayL.copy()
    L[3, 10] = np.nan
    with pytest.raises(tt.TdError) as e:
        tt.TdContext(ds.rayX, ds.rayY, ds.rayZ, L, ds.rayU, ds.tS, ds.allSig)
    assert e.value.code == 2 and "DimensionMismatch" in str(e.value)


def test_interpolate_matches_oracle(tt, orc, ctx):
    cells = tt.random_model(800, 12).cells()
    rng = np.random.default_rng(1)
    xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
    X = rng.uniform(xmin, xmax, 333)
    Y = rng.uniform(ymin, ymax, 333)
    Z = rng.uniform(zmin, zmax, 333)
    z, near = ctx.interpolate(cells, X, Y, Z, want_nearest=True)
    zr, ir = orc.interpolation(cells, X, Y, Z)
    assert np.array_equal(z, zr) and np.array_equal(near, ir)
    z_first = zr[0]
    # broadcast Y/Z of length 1 (the xzMap / xyMap cross sections, MCsub.jl:317-322)
    Xn = np.concatenate([X[:50], [np.nan], X[50:60]])
    z, near = ctx.interpolate(cells, Xn, [150.0], [300.0], want_nearest=True)
    zr, ir = orc.interpolation(cells, Xn, [150.0], [300.0])
    assert len(z) == 50 and np.array_equal(z, zr) and np.array_equal(near, ir)
    # single point (birth / death queries)
    assert tt.Interpolation(tt.define_TDstructrure(), tt.Model(800.0, *cells), [X[0]], [Y[0]], [Z[0]])[0] == z_first
    with pytest.raises(tt.TdError) as e:
        ctx.interpolate(cells, X[:5], Y[:2], Z[:5])
    assert e.value.code == 5


def test_evaluate_batch_equals_single(tt, ctx):
    models = [tt.random_model(n, s).cells() for n, s in ((10, 1), (500, 2), (0, 3), (1500, 4))]
    ptS, phi, lk = ctx.evaluate_batch(models)
    for k, c in enumerate(models):
        p1, f1, l1, _ = ctx.evaluate(c)
        assert np.array_equal(ptS[k], p1) and phi[k] == f1 and lk[k] == l1


def test_set_sigma_changes_phi_and_likelihood(tt, orc, ds):
    c = tt.TdContext.from_datastruct(ds)
    cells = tt.random_model(400, 8).cells()
    sig = np.full(ds.tS.shape, 0.2)
    c.set_sigma(sig)
    ptS, phi, lk, _ = c.evaluate(cells)
    ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, sig, cells)
    assert phi == ref["phi"] and lk == ref["likelihood"]
    c.close()


def test_stress_geometry_subset(tt, orc):
    # config-5 geometry at a size the oracle finishes in seconds: 1500 rays x 3000 cells
    s = tt.synthetic_rays(1500, seed=5)
    c = tt.TdContext.from_datastruct(s)
    assert_same(c, orc, s, tt.random_model(3000, 5).cells())
    c.close()


@pytest.mark.timeout(300)
def test_stress_full_size_matches_oracle(tt, orc):
    """Config 5 at its BASELINE size (10k rays x 20k cells, 584k points, 1.2e10
    point x cell distances) against the C oracle, the rays split over the host
    cores (oracle.evaluate_threaded, bit-identical to one whole evaluate):
    nearest indices, ptS, phi and likelihood bit for bit, through the default
    method (the 4-lane grid search at this size) and the brute force.  Also the
    size-independent property that phi is the sequential chi^2 of the ptS."""
    s = tt.synthetic_rays(10000, seed=5)
    c = tt.TdContext.from_datastruct(s)
    cells = tt.random_model(20000, 5).cells()
    ref = orc.evaluate_threaded(s.rayX, s.rayY, s.rayZ, s.rayL, s.rayU, s.tS, s.allSig, cells)
    assert ref["rc"] == 0 and len(ref["nearest"]) == c.P
    for m in (c.NN_AUTO, c.NN_BRUTE):
        c.set_nn_method(m)
        ptS, phi, lk, near = c.evaluate(cells, want_nearest=True)
        assert np.array_equal(near, ref["nearest"]), (m, int(np.sum(near != ref["nearest"])))
        assert np.array_equal(ptS, ref["ptS"]) and phi == ref["phi"] and lk == ref["likelihood"]
    C = 0.0
    for p, t, sg in zip(ptS, s.tS, s.allSig):
        d = p - t
        C = C + ((d * d) * 1.0) / (sg * sg)
    assert phi == C
    c.close()


def _both_methods(tt, ctx, orc, ds, cells):
    out = []
    for m in (ctx.NN_BRUTE, ctx.NN_GRID, ctx.NN_BRUTE_SPLIT):
        ctx.set_nn_method(m)
        out.append(ctx.evaluate(cells, want_nearest=True))
    ctx.set_nn_method(ctx.NN_AUTO)
    ref = ref_eval(orc, ds, cells)
    for ptS, phi, _, near in out:
        assert np.array_equal(near, ref["nearest"])
        assert np.array_equal(ptS, ref["ptS"]) and phi == ref["phi"]


def test_grid_search_adversarial(tt, orc, ds, ctx):
    """Bucket grid vs brute force vs oracle where a grid is most likely to go
    wrong: lattice cells (exact ties, points on bucket faces), one tight
    cluster (every point falls back), planar / collinear cells (degenerate
    axes), NaN cells, and cells far from every ray."""
    xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
    gx, gy, gz = np.meshgrid(np.linspace(xmin, xmax, 12), np.linspace(ymin, ymax, 8), np.linspace(zmin, zmax, 6),
                             indexing="ij")
    lat = (gx.ravel(), gy.ravel(), gz.ravel(), np.arange(gx.size, dtype=np.float64) % 47 + 1)
    _both_methods(tt, ctx, orc, ds, lat)
    # lattice with integer spacing: ray points land on faces and midpoints often
    ix, iy, iz = np.meshgrid(np.arange(0, 1000, 50.0), np.arange(-250, 400, 50.0), np.arange(0, 650, 50.0),
                             indexing="ij")
    _both_methods(tt, ctx, orc, ds, (ix.ravel(), iy.ravel(), iz.ravel(), np.ones(ix.size) * 3.0 + (ix.ravel() % 7)))
    rng = np.random.default_rng(4)
    n = 500
    clus = (400 + rng.uniform(0, 1, n), 100 + rng.uniform(0, 1, n), 300 + rng.uniform(0, 1, n), rng.uniform(1, 49, n))
    _both_methods(tt, ctx, orc, ds, clus)
    planar = (rng.uniform(0, 1000, n), rng.uniform(-250, 400, n), np.full(n, 200.0), rng.uniform(1, 49, n))
    _both_methods(tt, ctx, orc, ds, planar)
    line = (rng.uniform(0, 1000, n), np.full(n, 50.0), np.full(n, 100.0), rng.uniform(1, 49, n))
    _both_methods(tt, ctx, orc, ds, line)
    m = tt.random_model(600, 8)
    x, y, z, zeta = (a.copy() for a in m.cells())
    x[::50] = np.nan
    z[7::60] = np.nan
    _both_methods(tt, ctx, orc, ds, (x, y, z, zeta))
    far = (rng.uniform(5e4, 6e4, n), rng.uniform(5e4, 6e4, n), rng.uniform(0, 10, n), rng.uniform(1, 49, n))
    _both_methods(tt, ctx, orc, ds, far)
    mixed = tuple(np.concatenate([a, b]) for a, b in zip(m.cells(), far))
    _both_methods(tt, ctx, orc, ds, mixed)


def test_grid_interpolate_adversarial(tt, orc, ctx):
    """td_interpolate (grid rasterisation queries) against the oracle with
    queries on lattice faces, outside the box and NaN-terminated."""
    rng = np.random.default_rng(12)
    cells = tt.random_model(2000, 13).cells()
    X = np.concatenate([np.arange(-100, 1100, 25.0), rng.uniform(-500, 1500, 300), [np.nan, 5.0]])
    Y = np.concatenate([np.full(48, 50.0), rng.uniform(-500, 800, 300), [0.0, 0.0]])
    Z = np.concatenate([np.arange(0, 48 * 14, 14.0), rng.uniform(-100, 800, 300), [0.0, 0.0]])
    for m in (ctx.NN_BRUTE, ctx.NN_GRID, ctx.NN_BRUTE_SPLIT):
        ctx.set_nn_method(m)
        zr, near = ctx.interpolate(cells, X, Y, Z, want_nearest=True)
        ref, ref_ids = orc.interpolation(cells, X, Y, Z)
        assert np.array_equal(zr, ref) and np.array_equal(near, ref_ids)
    ctx.set_nn_method(ctx.NN_AUTO)


@pytest.mark.parametrize("ncells", [200, 2500])
def test_many_rays_exact_chi2(tt, orc, ncells):
    """10k synthetic rays: chi^2 over 10k terms takes the block-wide exact scan
    (exact_sum.h) -- phi must still equal the oracle's sequential loop."""
    ds = tt.synthetic_rays(10000, seed=5)
    ctx = tt.TdContext.from_datastruct(ds)
    cells = tt.random_model(ncells, 17).cells()
    ptS, phi, lk, near = ctx.evaluate(cells, want_nearest=True)
    ref = ref_eval(orc, ds, cells)
    assert np.array_equal(near, ref["nearest"])
    assert np.array_equal(ptS, ref["ptS"])
    assert phi == ref["phi"] and lk == ref["likelihood"]
    ctx.close()


@pytest.mark.parametrize("npts", [1, 5, 255, 257, 3001, 16845, 70000, 133000, 600000])
def test_tile_brute_force_plans(tt, orc, ctx, npts):
    """The one-launch brute force (k_nn_tile) over the shapes its plan takes:
    one point per CU (256 slices), a few points per CU, a full config-3 point
    set, and point sets of several tiles per CU (133k: 3 tiles of 174 points;
    600k, the stress geometry's size: 3 tiles of 782 points in 2 slices);
    cell counts below one group of 8, on and off slice / round boundaries,
    exact ties across slices (duplicated cells) and NaN cells.  Index and
    value must equal the oracle's v_nearest and the split search."""
    rng = np.random.default_rng(npts)
    xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
    X = rng.uniform(xmin, xmax, npts)
    Y = rng.uniform(ymin, ymax, npts)
    Z = rng.uniform(zmin, zmax, npts)
    for nc in ((1, 7, 8, 9, 333, 1023, 5000) if npts <= 16845 else (5000,) if npts < 500000 else (2000,)):
        x, y, z, zeta = (a.copy() for a in tt.random_model(nc, nc + 3).cells())
        if nc >= 9:  # duplicates far apart in index (different slices), different values
            k = nc // 3
            x[-k:], y[-k:], z[-k:] = x[:k], y[:k], z[:k]
            zeta[-k:] = zeta[:k] + 1.0
            x[1::37] = np.nan
        cells = (x, y, z, zeta)
        ref, ref_ids = orc.interpolation(cells, X, Y, Z)
        for m in (ctx.NN_BRUTE, ctx.NN_BRUTE_SPLIT):
            ctx.set_nn_method(m)
            zr, near = ctx.interpolate(cells, X, Y, Z, want_nearest=True)
            assert np.array_equal(near, ref_ids), (m, nc, np.flatnonzero(near != ref_ids)[:5])
            assert np.array_equal(zr, ref), (m, nc)
    ctx.set_nn_method(ctx.NN_AUTO)


def test_grid_large_query_sets(tt, orc, ctx):
    """Query sets of >= 65,536 points take the 4-lanes-per-point grid kernel
    (k_nn_grid4); it and its fallbacks (points outside the cells' box,
    unproven blocks, overfull buckets) against the oracle: lattice cells with
    queries on bucket faces,
    a tight cluster (every point falls back to the wave-wide passes), NaN
    cells, duplicated cells (ties across buckets), cells far from the
    queries."""
    rng = np.random.default_rng(21)
    xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
    n = 70000
    X = np.concatenate([rng.uniform(xmin, xmax, n - 2048), np.arange(0, 1024, 1.0) * 1.0, rng.uniform(-3e3, 3e3, 1024)])
    Y = np.concatenate([rng.uniform(ymin, ymax, n - 2048), np.full(1024, 50.0), rng.uniform(-3e3, 3e3, 1024)])
    Z = np.concatenate([rng.uniform(zmin, zmax, n - 2048), np.arange(0, 1024, 1.0) % 650, rng.uniform(-1e3, 1e3, 1024)])
    ix, iy, iz = np.meshgrid(np.arange(0, 1000, 50.0), np.arange(-250, 400, 50.0), np.arange(0, 650, 50.0),
                             indexing="ij")
    lattice = (ix.ravel(), iy.ravel(), iz.ravel(), 3.0 + (ix.ravel() % 7))
    m = tt.random_model(3000, 23)
    x, y, z, zeta = (a.copy() for a in m.cells())
    x[::50] = np.nan
    k = 600
    x[-k:], y[-k:], z[-k:] = x[:k], y[:k], z[:k]  # duplicates: the lower index must win
    zeta[-k:] = zeta[:k] + 1.0
    clus = (400 + rng.uniform(0, 1, 500), 100 + rng.uniform(0, 1, 500), 300 + rng.uniform(0, 1, 500),
            rng.uniform(1, 49, 500))
    far = (rng.uniform(5e4, 6e4, 500), rng.uniform(5e4, 6e4, 500), rng.uniform(0, 10, 500), rng.uniform(1, 49, 500))
    for cells in (lattice, (x, y, z, zeta), clus, far):
        ref, ref_ids = orc.interpolation(cells, X, Y, Z)
        ctx.set_nn_method(ctx.NN_GRID)
        zr, near = ctx.interpolate(cells, X, Y, Z, want_nearest=True)
        ctx.set_nn_method(ctx.NN_AUTO)
        assert np.array_equal(near, ref_ids), np.flatnonzero(near != ref_ids)[:5]
        assert np.array_equal(zr, ref)
