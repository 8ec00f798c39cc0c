"""The two CPU restatements (C and numpy) agree exactly, including on the
adversarial cases that exercise the tie / sentinel / NaN semantics of
v_nearest (MCsub.jl:249-257) and the NaN truncation of evaluate
(MCsub.jl:149-161).  No reference output covers these rows; agreement of two
independent restatements is what pins them (oracle/README.md)."""
import numpy as np
import pytest

from oracle import oracle_np


def csr(ds):
    m, n = ds.rayX.shape
    npts = (~np.isnan(ds.rayX)).sum(0)
    px = np.concatenate([ds.rayX[:c, i] for i, c in enumerate(npts)])
    py = np.concatenate([ds.rayY[:c, i] for i, c in enumerate(npts)])
    pz = np.concatenate([ds.rayZ[:c, i] for i, c in enumerate(npts)])
    w = np.concatenate([np.concatenate([ds.rayL[:c - 1, i] * ds.rayU[:c - 1, i], [0.0]]) if c > 0 else []
                        for i, c in enumerate(npts)])
    return npts, px, py, pz, w


@pytest.mark.parametrize("ncells,seed", [(0, 9), (1, 1), (7, 2), (200, 1), (1000, 2)])
def test_evaluate_c_vs_numpy_381(tt, orc, ds, ncells, seed):
    model = tt.random_model(ncells, seed)
    ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, model.cells())
    assert ref["rc"] == 0
    npts, px, py, pz, w = csr(ds)
    ptS, phi, lk, idx = oracle_np.evaluate_csr(npts, px, py, pz, w, ds.tS, ds.allSig, model.cells())
    assert np.array_equal(idx, ref["nearest"])
    assert np.array_equal(ptS, ref["ptS"])
    assert phi == ref["phi"] and lk == ref["likelihood"]


def test_v_nearest_ties_first_index_wins(orc):
    # two identical cells and one equidistant cell: the lowest index wins (strict <)
    mx, my, mz = np.array([5.0, 1.0, 1.0, -1.0]), np.array([0.0, 0.0, 0.0, 0.0]), np.zeros(4)
    mv = np.array([10.0, 20.0, 30.0, 40.0])
    v, i = orc.v_nearest(0.0, 0.0, 0.0, mx, my, mz, mv)
    assert (v, i) == (20.0, 1)
    assert oracle_np.nearest_index([0.0], [0.0], [0.0], mx, my, mz)[0] == 1


def test_v_nearest_sentinel_and_nan(orc):
    far = np.array([1e5]), np.array([0.0]), np.array([0.0])  # d = 1e10 >= 1e9: never taken
    v, i = orc.v_nearest(0.0, 0.0, 0.0, *far, np.array([3.0]))
    assert (v, i) == (0.0, -1)
    exactly = np.array([31622.776601683792]), np.zeros(1), np.zeros(1)
    d = exactly[0][0] ** 2
    v, i = orc.v_nearest(0.0, 0.0, 0.0, *exactly, np.array([3.0]))
    assert (i == 0) == (d < 1e9)
    nanc = np.array([np.nan, 2.0]), np.zeros(2), np.zeros(2)
    v, i = orc.v_nearest(0.0, 0.0, 0.0, *nanc, np.array([1.0, 2.0]))
    assert (v, i) == (2.0, 1)
    assert oracle_np.nearest_index([0.0], [0.0], [0.0], *nanc)[0] == 1
    assert oracle_np.nearest_index([0.0], [0.0], [0.0], *far)[0] == -1


def test_interpolation_broadcast_and_nan_truncation(orc):
    cells = (np.array([0.0, 10.0]), np.array([0.0, 0.0]), np.array([0.0, 0.0]), np.array([1.0, 2.0]))
    z, ids = orc.interpolation(cells, [1.0, 9.0, np.nan, 4.0], [0.0], [0.0])
    assert list(z) == [1.0, 2.0] and list(ids) == [0, 1]  # stops at the first NaN of X
    with pytest.raises(IndexError):
        orc.interpolation(cells, [1.0, 2.0, 3.0], [0.0, 0.0], [0.0])


def _rays_from_lists(rays, m):
    n = len(rays)
    X, Y, Z = (np.full((m, n), np.nan) for _ in range(3))
    for i, r in enumerate(rays):
        r = np.asarray(r, dtype=np.float64).reshape(-1, 3)
        X[:len(r), i], Y[:len(r), i], Z[:len(r), i] = r[:, 0], r[:, 1], r[:, 2]
    return X, Y, Z


def test_edge_rays_one_point_empty_full_length(tt, orc):
    m = 6
    rays = [
        [],                                                    # npoints = 0
        [[1, 2, 3]],                                           # npoints = 1: no segment
        [[0, 0, 0], [10, 0, 0]],                               # one segment
        [[k * 3.0, 1.0, 2.0 * k] for k in range(m)],           # full length, no NaN
    ]
    X, Y, Z = _rays_from_lists(rays, m)
    U = np.where(np.isnan(Z), np.nan, 0.125)
    L, Uu = tt.segments(X, Y, Z, U)
    cells = tt.random_model(5, 3).cells()
    tS, sig = np.array([0.1, 0.2, 0.3, 0.4]), np.array([0.05, 0.1, 0.2, 0.3])
    ref = orc.evaluate(X, Y, Z, L, Uu, tS, sig, cells)
    assert ref["rc"] == 0
    assert ref["ptS"][0] == 0.0 and ref["ptS"][1] == 0.0
    npts = np.array([0, 1, 2, m])
    P = int(npts.sum())
    px = np.concatenate([X[:c, i] for i, c in enumerate(npts)])
    py = np.concatenate([Y[:c, i] for i, c in enumerate(npts)])
    pz = np.concatenate([Z[:c, i] for i, c in enumerate(npts)])
    w = np.concatenate([np.concatenate([L[:c - 1, i] * Uu[:c - 1, i], [0.0]]) if c > 0 else [] for i, c in enumerate(npts)])
    assert len(px) == P
    ptS, phi, lk, idx = oracle_np.evaluate_csr(npts, px, py, pz, w, tS, sig, cells)
    assert np.array_equal(ptS, ref["ptS"]) and phi == ref["phi"] and np.array_equal(idx, ref["nearest"])


def test_layout_mismatch_is_an_error(tt, orc):
    X, Y, Z = _rays_from_lists([[[0, 0, 0], [1, 0, 0], [2, 0, 0]]], 4)
    U = np.full_like(X, 0.2)
    L, Uu = tt.segments(X, Y, Z, U)
    L[1, 0] = np.nan  # rayL truncated one segment early
    ref = orc.evaluate(X, Y, Z, L, Uu, np.zeros(1), np.ones(1), tt.random_model(3, 1).cells())
    assert ref["rc"] == -1


def test_debug_prior_returns_one(tt, orc, ds):
    ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig,
                       tt.random_model(10, 1).cells(), debug_prior=1)
    assert ref["phi"] == 1.0 and ref["likelihood"] == 1.0


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_threaded_oracle_equals_whole_evaluate(tt, orc, ds, threads):
    """oracle.evaluate_threaded (the checker of config 5 at full size) is the
    whole-geometry evaluate bit for bit: per-ray t* in ray ranges, then the
    sequential chi^2 over all rays (MCsub.jl:142-173)."""
    cells = tt.random_model(300, 11).cells()
    a = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, cells)
    b = orc.evaluate_threaded(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, cells, threads=threads)
    assert a["rc"] == b["rc"] == 0
    assert np.array_equal(a["nearest"], b["nearest"]) and np.array_equal(a["ptS"], b["ptS"])
    assert a["phi"] == b["phi"] and a["likelihood"] == b["likelihood"]
