"""Independent numpy restatement of the rj-MCMC loop in prior-sampling mode --
TEST INFRASTRUCTURE ONLY (tests/test_gpu_prior_recovery.py).

With ``debug_prior = 1`` the reference's ``evaluate`` returns phi = 1 without
touching the data (MCsub.jl:134-136), so the chain samples the prior implied
by its proposal and acceptance rules.  This module runs K independent chains
of TD_inversion_function.jl:70-274 at once (vectorised over chains, numpy's
PCG64 -- NOT the build's Philox streams, and none of the build's code), so a
bias in the build's shared RNG / normal quantile / acceptance code
(chain_logic.h), which DEVICE-vs-HOST engine equality cannot see, shows up as
a difference in distribution.

Restated lines:
  start       MCsub.jl:86-87 (log-uniform nCells), :92-94 (cells uniform in the
              box), :97-108 (zeta per prior)
  action      TD_inversion_function.jl:72 rand(1:4)
  birth       :77-124 (Interpolation at the new site :81 = value of the nearest
              cell, :82 Normal(czeta, sig_zeta); validity and alpha per prior)
  death       :127-180 (kill = rand(1:nCells); zetanew = Interpolation of the
              reduced model at the killed site :146; alpha per prior)
  change      :184-218
  move        :221-250 (Normal(site, (sig/100)(max-min)) per axis, box check)
with phi_n - phi = 0 in every alpha.
"""
import math

import numpy as np


def run(K, iters, box, prior=1, seed=0, sig=10, zeta_scale=50, max_cells=100, min_cells=5):
    """K independent prior-sampling chains, `iters` iterations each.
    Returns (nCells[K], zeta list of arrays, x list of arrays)."""
    rng = np.random.default_rng(seed)
    xmin, xmax, ymin, ymax, zmin, zmax = box
    lo = np.array([xmin, ymin, zmin])
    hi = np.array([xmax, ymax, zmax])
    zs = float(zeta_scale)
    sz = zs * sig / 100  # TD_inversion_function.jl:22
    rr = (sig / 100) * (hi - lo)  # :30-32
    s2p = math.sqrt(2 * math.pi)
    M = max_cells + 1
    C = np.full((K, M, 3), np.nan)
    Z = np.zeros((K, M))
    # build_starting (MCsub.jl:86-108)
    N = np.floor(np.exp(rng.random(K) * math.log(max_cells / min_cells) + math.log(min_cells))).astype(np.int64)
    for k in range(K):
        n = N[k]
        C[k, :n] = lo + (hi - lo) * rng.random((n, 3))
        if prior == 1:
            Z[k, :n] = rng.random(n) * zs
        elif prior == 2:
            Z[k, :n] = rng.normal(0.0, zs, n)
        else:
            Z[k, :n] = -np.log(rng.random(n)) * zs
    cols = np.arange(M)[None, :]
    rows = np.arange(K)

    def nearest_value(pts, skip=None):
        """Interpolation (MCsub.jl:306-327 -> v_nearest :247-263) of each chain's
        current cells at pts[K,3]; `skip` = a killed position left out (the
        reduced model of :132-135)."""
        d = ((C - pts[:, None, :]) ** 2).sum(axis=2)
        live = cols < N[:, None]
        if skip is not None:
            live &= cols != skip[:, None]
        d = np.where(live & (d < 1e9), d, np.inf)
        j = np.argmin(d, axis=1)  # first index of the minimum
        v = Z[rows, j]
        return np.where(np.isfinite(d[rows, j]), v, 0.0)

    for _ in range(iters):
        action = rng.integers(1, 5, K)  # :72
        u = rng.random(K)
        # ---- birth :76-124
        b = (action == 1) & (N < max_cells)
        site = lo + (hi - lo) * rng.random((K, 3))
        czeta = nearest_value(site)
        zn = czeta + sz * rng.standard_normal(K)
        dz2 = (czeta - zn) ** 2 / (2 * sz ** 2)
        with np.errstate(over="ignore"):
            if prior == 1:
                valid = (zn > 0) & (zn < zs)
                a = (N / (N + 1)) * (sz * s2p / zs) * np.exp(dz2)
            elif prior == 2:
                valid = np.ones(K, dtype=bool)
                a = (N / (N + 1)) * (sz / zs) * np.exp(-zn ** 2 / zs ** 2 + dz2)
            else:
                valid = zn > 0
                a = (N / (N + 1)) * (s2p * sz / zs) * np.exp(-zn / zs + dz2)
        acc = b & valid & (u < np.minimum(1.0, a))
        idx = np.nonzero(acc)[0]
        C[idx, N[idx]] = site[idx]
        Z[idx, N[idx]] = zn[idx]
        N[idx] += 1
        # ---- death :126-180
        d = (action == 2) & (N > min_cells) & ~acc
        kill = np.minimum((rng.random(K) * N).astype(np.int64), N - 1)
        ks = C[rows, kill]
        zk = Z[rows, kill]
        zdn = nearest_value(ks, skip=kill)
        dz2 = (zk - zdn) ** 2 / (2 * sz ** 2)
        with np.errstate(over="ignore"):
            if prior == 1:
                valid = np.ones(K, dtype=bool)
                a = (N / np.maximum(N - 1, 1)) * (zs / (sz * s2p)) * np.exp(-dz2)
            elif prior == 2:
                valid = np.ones(K, dtype=bool)
                a = (N / np.maximum(N - 1, 1)) * (zs / sz) * np.exp(zk ** 2 / (2 * zs ** 2) - dz2)
            else:
                valid = zdn > 0
                a = (N / np.maximum(N - 1, 1)) * (zs / (s2p * sz)) * np.exp(zk / zs - dz2)
        accd = d & valid & (u < np.minimum(1.0, a))
        for k in np.nonzero(accd)[0]:  # deleteat! (:132-135): later cells shift down
            n, j = N[k], kill[k]
            C[k, j:n - 1] = C[k, j + 1:n]
            Z[k, j:n - 1] = Z[k, j + 1:n]
            C[k, n - 1] = np.nan
            N[k] -= 1
        # ---- change :183-218 (alpha = exp(0) = 1 for uniform)
        c = (action == 3) & (N > 0)
        ci = np.minimum((rng.random(K) * N).astype(np.int64), N - 1)
        zo = Z[rows, ci]
        zc = zo + sz * rng.standard_normal(K)
        with np.errstate(over="ignore"):
            if prior == 1:
                valid = (zc > 0) & (zc < zs)
                a = np.ones(K)
            elif prior == 2:
                valid = np.ones(K, dtype=bool)
                a = np.exp((zo ** 2 - zc ** 2) / (2 * zs ** 2))
            else:
                valid = zc > 0
                a = np.exp((zo - zc) / zs)
        accc = c & valid & (u < np.minimum(1.0, a))
        Z[rows[accc], ci[accc]] = zc[accc]
        # ---- move :220-250 (alpha = 1 inside the box)
        m = (action == 4) & (N > 0)
        mi = np.minimum((rng.random(K) * N).astype(np.int64), N - 1)
        ns = C[rows, mi] + rr * rng.standard_normal((K, 3))
        inside = np.all((ns >= lo) & (ns <= hi), axis=1)
        accm = m & inside & (u < 1.0)
        C[rows[accm], mi[accm]] = ns[accm]
    zetas = [Z[k, :N[k]].copy() for k in range(K)]
    xs = [C[k, :N[k], 0].copy() for k in range(K)]
    return N.copy(), zetas, xs
