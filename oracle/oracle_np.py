"""Independent numpy restatement of the forward model -- TEST INFRASTRUCTURE ONLY.

Written separately from tstar_oracle.c (vectorised over cells, different code
path) so the two restatements can check each other where no reference output
exists (nearest-cell search, ray integral).  Cites the same Julia lines.
"""
import math

import numpy as np


def nearest_index(px, py, pz, xc, yc, zc):
    """MCsub.jl:247-263 vectorised: for each point, the first cell index at the
    minimum FP64 squared distance ((dx^2 + dy^2) + dz^2); -1 when no distance is
    strictly below the 1e9 sentinel.  NaN distances never win (NaN < m is false)."""
    px, py, pz = (np.asarray(a, dtype=np.float64).reshape(-1, 1) for a in (px, py, pz))
    xc, yc, zc = (np.asarray(a, dtype=np.float64).reshape(1, -1) for a in (xc, yc, zc))
    if xc.shape[1] == 0:
        return np.full(px.shape[0], -1, dtype=np.int64)
    dx, dy, dz = xc - px, yc - py, zc - pz
    d = (dx * dx + dy * dy) + dz * dz  # numpy evaluates left to right, no FMA
    d = np.where(np.isnan(d), np.inf, d)
    idx = np.argmin(d, axis=1)  # first occurrence of the minimum
    best = d[np.arange(d.shape[0]), idx]
    return np.where(best < 1e9, idx, -1).astype(np.int64)


def julia_sum(a, vf=8, ic=4):
    """Julia 1.5 Base.sum association (see tstar_oracle.c for the derivation)."""
    a = [float(v) for v in a]
    n = len(a)
    if n == 0:
        return 0.0
    if n == 1:
        return a[0]
    if n < 16:
        s = a[0] + a[1]
        for v in a[2:]:
            s = s + v
        return s

    def block(f, l):
        if f == l:
            return a[f]
        v = a[f] + a[f + 1]
        T = l - f - 1
        W = vf * ic
        Q = T // W if T >= W else 0
        i = f + 2
        if Q:
            acc = np.zeros((ic, vf))
            acc[0, 0] = v
            blk = np.asarray(a[i:i + Q * W]).reshape(Q, ic, vf)
            for q in range(Q):
                acc = acc + blk[q]
            r = acc[0].copy()
            for k in range(1, ic):
                r = acc[k] + r
            h = vf // 2
            while h >= 1:
                r = r[:h] + r[h:2 * h]
                h //= 2
            v = float(r[0])
            i += Q * W
        for j in range(i, l + 1):
            v = v + a[j]
        return v

    def impl(f, l):
        if l - f < 1024:
            return block(f, l)
        mid = f + ((l - f) >> 1)
        return impl(f, mid) + impl(mid + 1, l)

    return impl(0, n - 1)


def chi2(ptS, tS, allSig):
    """MCsub.jl:169-172 (sequential in k)."""
    C = 0.0
    for p, t, s in zip(ptS, tS, allSig):
        d = float(p) - float(t)
        C = C + ((d * d) * 1.0) / (float(s) * float(s))
    return C


def likelihood(allSig):
    """MCsub.jl:179."""
    n = len(allSig)
    c = math.sqrt(2 * math.pi)
    return julia_sum([(-math.log(float(s) * c)) * float(n) for s in allSig])


def evaluate_csr(npts, px, py, pz, w, tS, allSig, cells):
    """MCsub.jl:123-185 on the compact layout: npts[i] valid points of ray i
    stored consecutively; w[k] = rayL*rayU of the segment starting at point k
    (ignored for the last point of each ray).  Returns (ptS, phi, lik, nearest)."""
    xc, yc, zc, ze = (np.asarray(a, dtype=np.float64) for a in cells)
    idx = nearest_index(px, py, pz, xc, yc, zc)
    zeta0 = np.where(idx >= 0, ze[np.maximum(idx, 0)] if len(ze) else 0.0, 0.0)
    ptS = np.zeros(len(npts))
    off = 0
    for i, c in enumerate(npts):
        z = zeta0[off:off + c]
        rz = 0.5 * (z[:-1] + z[1:])
        terms = w[off:off + c - 1] * (rz / 1000.0) if c > 1 else np.zeros(0)
        ptS[i] = julia_sum(terms)
        off += c
    return ptS, chi2(ptS, tS, allSig), likelihood(allSig), idx


def julia_mapreduce_arrays(vals):
    """sum over a Vector of arrays (Base.mapreduce for non-bitstype elements):
    n < 16 left to right; else pairwise halves (mid = (lo+hi)>>1) down to
    blocks of <= 1024 elements, each added left to right (the @simd loop cannot
    reassociate array additions).  vals: list of float64 arrays (same shape)."""
    n = len(vals)
    if n == 1:
        return vals[0].copy()
    if n < 16:
        s = vals[0] + vals[1]
        for v in vals[2:]:
            s = s + v
        return s

    def impl(lo, hi):
        if hi - lo < 1024:
            s = vals[lo] + vals[lo + 1]
            for k in range(lo + 2, hi + 1):
                s = s + vals[k]
            return s
        mid = (lo + hi) >> 1
        return impl(lo, mid) + impl(mid + 1, hi)

    return impl(0, n - 1)


def rasterize(models, qx, qy, qz):
    """plot_model_hist (MCsub.jl:761-775): the v_nearest value of every model at
    every query point, then Statistics.mean and std (corrected) over the models
    -- mean = sum(A)/n, std = sqrt.(sum(abs2.(A .- mean)) / (n-1)), both sums
    in the association above.  models: list of (x, y, z, zeta) arrays."""
    vals = []
    for xc, yc, zc, ze in models:
        idx = nearest_index(qx, qy, qz, xc, yc, zc)
        ze = np.asarray(ze, dtype=np.float64)
        vals.append(np.where(idx >= 0, ze[np.maximum(idx, 0)] if len(ze) else 0.0, 0.0))
    n = len(vals)
    mean = julia_mapreduce_arrays(vals) / float(n)
    dev = [(v - mean) * (v - mean) for v in vals]
    with np.errstate(invalid="ignore", divide="ignore"):
        std = np.sqrt(julia_mapreduce_arrays(dev) / float(n - 1))
    return mean, std, np.array(vals)


def trilinear(xs, ys, zs, values, px, py, pz):
    """Gridded(Linear()) of Interpolations.jl as used at load_3Dvel.jl:32 and
    pre_process_data.jl:34 (restated: the package is not in the reference tree
    and its version is unpinned -- the 8-corner association below is this
    build's, shared with ingest.hip; parity unpinned for the last ulps).
    Per axis: i = searchsortedlast(knots, x) clamped to [1, n-1] (0-based
    [0, n-2]), t = (x - k_i) / (k_{i+1} - k_i); outside [k_1, k_n] -> NaN (the
    reference throws a BoundsError).  values[i, j, k]; lerp x, then y, then z."""
    xs, ys, zs = (np.asarray(a, dtype=np.float64) for a in (xs, ys, zs))
    v = np.asarray(values, dtype=np.float64)
    px, py, pz = (np.asarray(a, dtype=np.float64).ravel() for a in (px, py, pz))

    def axis(k, x):
        i = np.clip(np.searchsorted(k, x, side="right") - 1, 0, len(k) - 2)
        ok = (x >= k[0]) & (x <= k[-1])
        t = (x - k[i]) / (k[i + 1] - k[i])
        return i, t, ok

    i, tx, okx = axis(xs, px)
    j, ty, oky = axis(ys, py)
    k, tz, okz = axis(zs, pz)
    ux, uy, uz = 1.0 - tx, 1.0 - ty, 1.0 - tz
    c2 = []
    for dz in (0, 1):
        c1 = [ux * v[i, j + dy, k + dz] + tx * v[i + 1, j + dy, k + dz] for dy in (0, 1)]
        c2.append(uy * c1[0] + ty * c1[1])
    out = uz * c2[0] + tz * c2[1]
    return np.where(okx & oky & okz, out, np.nan)
