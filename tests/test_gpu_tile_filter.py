"""The chain's phase-B tile filter (chain_kernels.hip tile_may_hit / tile_may_hit2, FP32) must never drop
a tile that holds a point within the tile's cached maximum distance: in FP64, dist2(q, p) <= maxd for some
point p of the tile => the tile passes.  Otherwise a proposal could miss a point whose nearest cell it
changes (MCsub.jl:247-263 through the chain's incremental search).  Checked on tiles of 16 real ray points
each (boxes rounded outward to FP32), queries on, near and far from them, and maxima set EXACTLY to a
query's FP64 minimum distance -- the boundary case -- for both filter forms."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def dist2(px, py, pz, qx, qy, qz):
    dx, dy, dz = px - qx, py - qy, pz - qz  # (mx-x)^2 + (my-y)^2 + (mz-z)^2 left to right, no FMA
    return (dx * dx + dy * dy) + dz * dz


def outward_box(v):
    lo, hi = np.float32(v.min()), np.float32(v.max())
    if float(lo) > v.min():
        lo = np.nextafter(lo, np.float32(-np.inf))
    if float(hi) < v.max():
        hi = np.nextafter(hi, np.float32(np.inf))
    return lo, hi


@pytest.mark.parametrize("mode", [0, 1])
def test_tile_filter_never_drops_a_tile_in_reach(tt, ds, mode):
    rng = np.random.default_rng(17 + mode)
    X, Y, Z = (np.asarray(a, dtype=np.float64).T.ravel() for a in (ds.rayX, ds.rayY, ds.rayZ))
    ok = ~np.isnan(X)
    X, Y, Z = X[ok], Y[ok], Z[ok]
    nt = 400
    starts = rng.integers(0, len(X) - 16, nt)
    pts = [np.stack([X[s:s + 16], Y[s:s + 16], Z[s:s + 16]], 1) for s in starts]
    pts[:50] = [p * 37.0 + 1000.0 * rng.standard_normal(3) for p in pts[:50]]  # large coordinates too
    lo = np.zeros((3, nt), dtype=np.float32)
    hi = np.zeros((3, nt), dtype=np.float32)
    for t, p in enumerate(pts):
        for a in range(3):
            lo[a, t], hi[a, t] = outward_box(p[:, a])
    nq = 300
    qs = np.empty((nq, 3))
    for k in range(nq):  # on a point, near a box, or anywhere in the cloud
        t = rng.integers(nt)
        kind = k % 3
        if kind == 0:
            qs[k] = pts[t][rng.integers(16)]
        elif kind == 1:
            qs[k] = pts[t][rng.integers(16)] + rng.standard_normal(3) * rng.choice([1e-9, 1e-4, 1.0, 30.0])
        else:
            qs[k] = pts[rng.integers(nt)].mean(0) + rng.standard_normal(3) * 200.0
    md = np.array([[dist2(p[:, 0], p[:, 1], p[:, 2], *q).min() for p in pts] for q in qs])  # [nq, nt]
    # each tile's maximum: exactly some query's minimum distance to it (the boundary), or a random one
    owner = rng.integers(0, nq, nt)
    maxd = md[owner, np.arange(nt)].copy()
    maxd[::7] *= rng.uniform(0.5, 2.0, len(maxd[::7]))
    hit = np.zeros(nq * nt, dtype=np.uint8)
    f32 = ctypes.POINTER(ctypes.c_float)
    L = tt.lib()
    lo_c, hi_c = np.ascontiguousarray(lo), np.ascontiguousarray(hi)
    qs_c = np.ascontiguousarray(qs)
    rc = L.tdt_tile_filter(lo_c.ctypes.data_as(f32), hi_c.ctypes.data_as(f32),
                           maxd.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), nt,
                           qs_c.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), nq, mode,
                           hit.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    assert rc == 0
    hit = hit.reshape(nq, nt).astype(bool)
    must = md <= maxd[None, :]
    missed = np.argwhere(must & ~hit)
    assert missed.size == 0, (missed[:5], [(md[q, t], maxd[t]) for q, t in missed[:5]])
    exact = np.setdiff1d(np.arange(nt), np.arange(0, nt, 7))
    assert must[owner[exact], exact].all()  # (the boundary pairs, maximum == the distance, are in the set)
    assert hit.mean() < 0.6  # (and it does prune)
