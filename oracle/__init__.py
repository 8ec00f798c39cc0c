"""CPU parity oracle for the t* forward model -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker (or the
timed CPU baseline).  The product path (``mcmc-in-tonga_amd``) never imports
it and fails loudly when its HIP library is missing.

Two independent restatements of the reference (Julia, /root/reference):

* ``liboracle_tstar.so`` (``tstar_oracle.c``) -- scalar C, same loop order and
  FP64 rounding as the Julia source, wrapped here with ctypes;
* ``oracle_np`` -- a vectorised numpy restatement used to cross-check the C one.

Pinning: chi^2, likelihood and Julia's sum association are pinned bit-exactly
by ``/root/reference/model.jld`` (tests/golden/model_jld_kat.npz).  The
nearest-cell search and ray integral have no reference output (Julia is not
installed; no shipped output covers them), so they are pinned only by the
two restatements agreeing plus adversarial cases.  See oracle/README.md.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_tstar.so")

_d = ctypes.c_double
_i64 = ctypes.c_int64
_pd = ctypes.POINTER(ctypes.c_double)
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pi32 = ctypes.POINTER(ctypes.c_int32)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_v_nearest.restype = _d
        L.oracle_v_nearest.argtypes = [_d, _d, _d, _pd, _pd, _pd, _pd, _i64, _pi64]
        L.oracle_npoints.restype = _i64
        L.oracle_npoints.argtypes = [_pd, _i64]
        L.oracle_interpolation.restype = _i64
        L.oracle_interpolation.argtypes = [_pd, _pd, _pd, _pd, _i64, _pd, _i64, _pd, _i64, _pd, _i64, _pd, _pi64]
        L.oracle_julia_sum.restype = _d
        L.oracle_julia_sum.argtypes = [_pd, _i64]
        L.oracle_chi2.restype = _d
        L.oracle_chi2.argtypes = [_pd, _pd, _pd, _i64]
        L.oracle_likelihood.restype = _d
        L.oracle_likelihood.argtypes = [_pd, _i64]
        L.oracle_segments.restype = None
        L.oracle_segments.argtypes = [_pd, _pd, _pd, _pd, _i64, _i64, _pd, _pd]
        L.oracle_interp1.restype = None
        L.oracle_interp1.argtypes = [_pd, _pd, _i64, _pd, _i64, _pd]
        L.oracle_evaluate.restype = ctypes.c_int
        L.oracle_evaluate.argtypes = [_pd, _pd, _pd, _pd, _pd, _i64, _i64, _pd, _pd,
                                      _pd, _pd, _pd, _pd, _i64, ctypes.c_int, _pd, _pd, _pd, _pi32]
        _lib = L
    return _lib


def _p(a, t=_pd):
    return a.ctypes.data_as(t)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def v_nearest(x, y, z, mx, my, mz, mv):
    """MCsub.jl:247-263 -> (value, 0-based index or -1)."""
    mx, my, mz, mv = map(_f64, (mx, my, mz, mv))
    idx = ctypes.c_int64(0)
    v = lib().oracle_v_nearest(x, y, z, _p(mx), _p(my), _p(mz), _p(mv), len(mx), ctypes.byref(idx))
    return v, idx.value


def julia_sum(a):
    a = _f64(a)
    return lib().oracle_julia_sum(_p(a), len(a))


def chi2(ptS, tS, allSig):
    ptS, tS, allSig = map(_f64, (ptS, tS, allSig))
    return lib().oracle_chi2(_p(ptS), _p(tS), _p(allSig), len(ptS))


def likelihood(allSig):
    allSig = _f64(allSig)
    return lib().oracle_likelihood(_p(allSig), len(allSig))


def segments(x, y, z, U):
    """x/y/z/U are (m, n) arrays (points x rays, as DataStruct.rayX)."""
    m, n = x.shape
    f = lambda a: _f64(np.asarray(a).T)  # column-major == C-order of the transpose
    X, Y, Z, UU = f(x), f(y), f(z), f(U)
    L = np.empty((n, m - 1))
    Uo = np.empty((n, m - 1))
    lib().oracle_segments(_p(X), _p(Y), _p(Z), _p(UU), m, n, _p(L), _p(Uo))
    return L.T.copy(), Uo.T.copy()


def interp1(x, y, xx):
    x, y, xx = map(_f64, (x, y, xx))
    yy = np.empty_like(xx)
    lib().oracle_interp1(_p(x), _p(y), len(x), _p(xx), len(xx), _p(yy))
    return yy


def interpolation(cells, X, Y, Z):
    xc, yc, zc, ze = map(_f64, cells)
    X, Y, Z = map(_f64, (np.atleast_1d(X), np.atleast_1d(Y), np.atleast_1d(Z)))
    out = np.empty(max(len(X), 1))
    ids = np.empty(max(len(X), 1), dtype=np.int64)
    np_ = lib().oracle_interpolation(_p(xc), _p(yc), _p(zc), _p(ze), len(xc), _p(X), len(X), _p(Y), len(Y),
                                     _p(Z), len(Z), _p(out), _p(ids, _pi64))
    if np_ < 0:
        raise IndexError("Y/Z shorter than npoints (Julia BoundsError)")
    return out[:np_].copy(), ids[:np_].copy()


def evaluate(rayX, rayY, rayZ, rayL, rayU, tS, allSig, cells, debug_prior=0):
    """MCsub.jl:123-185.  ray arrays are (m, n) / (m-1, n) as in DataStruct.

    Returns dict(ptS, phi, likelihood, nearest[P], rc)."""
    m, n = rayX.shape
    f = lambda a: _f64(np.asarray(a).T)
    X, Y, Z, L, U = f(rayX), f(rayY), f(rayZ), f(rayL), f(rayU)
    tS, allSig = _f64(tS), _f64(allSig)
    xc, yc, zc, ze = map(_f64, cells)
    P = int((~np.isnan(rayX)).sum())
    ptS = np.zeros(n)
    nearest = np.full(max(P, 1), -2, dtype=np.int32)
    phi = ctypes.c_double(0)
    lk = ctypes.c_double(0)
    rc = lib().oracle_evaluate(_p(X), _p(Y), _p(Z), _p(L), _p(U), m, n, _p(tS), _p(allSig), _p(xc), _p(yc),
                               _p(zc), _p(ze), len(xc), int(debug_prior), _p(ptS), ctypes.byref(phi),
                               ctypes.byref(lk), _p(nearest, _pi32))
    return dict(ptS=ptS, phi=phi.value, likelihood=lk.value, nearest=nearest[:P], rc=rc)


def evaluate_threaded(rayX, rayY, rayZ, rayL, rayU, tS, allSig, cells, threads=None):
    """MCsub.jl:123-185 for geometries too large for one core (config 5:
    584k points x 20k cells): the rays are split into contiguous ranges, each
    range's ptS and nearest cells come from `evaluate` on that range in its own
    thread (ctypes releases the GIL), and phi / likelihood are the C oracle's
    chi2 / likelihood over all rays in k order.  Identical to `evaluate` on
    the whole geometry: a ray's t* depends on that ray alone (MCsub.jl:142-163)
    and the chi^2 is the same sequential sum (MCsub.jl:169-173)."""
    import threading

    n = rayX.shape[1]
    if threads is None:
        try:
            threads = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            threads = os.cpu_count() or 1
        threads = max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    threads = max(1, min(threads, n))
    bounds = [(n * k // threads, n * (k + 1) // threads) for k in range(threads)]
    parts = [None] * threads

    def work(k):
        a, b = bounds[k]
        parts[k] = evaluate(rayX[:, a:b], rayY[:, a:b], rayZ[:, a:b], rayL[:, a:b], rayU[:, a:b], tS[a:b],
                            allSig[a:b], cells)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ptS = np.concatenate([p["ptS"] for p in parts])
    nearest = np.concatenate([p["nearest"] for p in parts])
    rc = max(p["rc"] for p in parts)
    return dict(ptS=ptS, phi=chi2(ptS, tS, allSig), likelihood=likelihood(allSig), nearest=nearest, rc=rc)
