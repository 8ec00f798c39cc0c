"""Forward model -- drop-in mirror of MCsub.jl's ``evaluate`` / ``Interpolation``.

Same names, argument meaning and return values as the reference:

* ``evaluate(model, dataStruct, TD_parameters) -> (model, dataStruct, valid)``
  (MCsub.jl:123-185): mutates and returns the SAME model object, setting
  ``phi``, ``ptS`` (fresh array), ``tS`` (alias of dataStruct.tS) and
  ``likelihood``; honours ``debug_prior``.
* ``Interpolation(TD_parameters, model, X, Y, Z) -> ndarray`` (MCsub.jl:306-336).
* ``v_nearest(x, y, z, mx, my, mz, mv)`` (MCsub.jl:247-263).

All arithmetic runs in libtdstar's HIP kernels (``TdContext``); there is no
CPU path.  ``interp_style == 2`` (IDW) is broken in the reference (MCsub.jl:332
uses undefined names) and raises here too.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, f64, lib, ptr


class TdContext:
    """A td_ctx: the device-resident copy of a DataStruct's ray geometry."""

    def __init__(self, rayX, rayY, rayZ, rayL, rayU, tS, allSig, device=-1):
        self.m, self.n = np.asarray(rayX).shape
        # column-major m x n == C-order of the n x m transpose
        cm = lambda a: f64(np.asarray(a, dtype=np.float64).T)
        self._arrays = [cm(rayX), cm(rayY), cm(rayZ), cm(rayL), cm(rayU), f64(tS), f64(allSig)]
        X, Y, Z, L, U, t, s = self._arrays
        h = ctypes.c_void_p()
        check(lib().td_create(ctypes.byref(h), int(device), ptr(X), ptr(Y), ptr(Z), ptr(L), ptr(U), self.m, self.n,
                              ptr(t), ptr(s)))
        self.h = h
        info = _lib.TdInfo()
        check(lib().td_get_info(self.h, ctypes.byref(info)), self.h)
        self.P = int(info.npoints)
        self.S = int(info.nsegments)
        self.likelihood_const = float(info.likelihood)
        self.arch = info.arch.decode()
        self.device = int(info.device)
        self.num_cus = int(info.num_cus)

    @classmethod
    def from_datastruct(cls, ds, device=-1):
        return cls(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, device)

    def close(self):
        if getattr(self, "h", None):
            lib().td_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_sigma(self, allSig):
        s = f64(allSig)
        check(lib().td_set_sigma(self.h, ptr(s)), self.h)
        info = _lib.TdInfo()
        check(lib().td_get_info(self.h, ctypes.byref(info)), self.h)
        self.likelihood_const = float(info.likelihood)

    def misfit(self, ptS, tS, allSig):
        """(phi, likelihood) of a given ptS (MCsub.jl:169-182) on this device:
        the reduction step of a ray-sharded evaluate (td_misfit)."""
        p, t, s = f64(ptS), f64(tS), f64(allSig)
        if not (len(p) == len(t) == len(s)):
            raise ValueError("ptS, tS and allSig must have the same length")
        phi, lk = ctypes.c_double(), ctypes.c_double()
        check(lib().td_misfit(self.h, len(p), ptr(p), ptr(t), ptr(s), ctypes.byref(phi), ctypes.byref(lk)), self.h)
        return phi.value, lk.value

    INCR_FULL, INCR_LAUNCH, INCR_RESIDENT = 0, 1, 2

    def set_incremental(self, mode):
        """td_evaluate's incremental path: INCR_RESIDENT (default: a resident
        kernel answers every call), INCR_LAUNCH (one launch per call; use it when
        other GPU work, e.g. a collective, runs between evaluates) or INCR_FULL."""
        check(lib().td_set_incremental(self.h, int(mode)), self.h)

    NN_AUTO, NN_BRUTE, NN_GRID, NN_BRUTE_SPLIT = 0, 1, 2, 3

    def set_nn_method(self, method):
        """Nearest-cell search: NN_AUTO (bucket grid from 256 cells on), NN_BRUTE
        (every point x every cell, the reference's loop: one launch of k_nn_tile
        where it fits), NN_GRID, NN_BRUTE_SPLIT (brute force through k_nn_partial
        + k_nn_merge).  Same answer."""
        check(lib().tdt_set_nn_method(self.h, int(method)), self.h)

    def timing(self, enable=None, reset=False, kernel=None):
        """Per-kernel HIP-event timing: enable/reset, or read (launches, total_ms) of `kernel`."""
        if enable is not None:
            check(lib().td_timing_enable(self.h, int(bool(enable))), self.h)
        if reset:
            check(lib().td_timing_reset(self.h), self.h)
        if kernel is not None:
            n = ctypes.c_int64()
            ms = ctypes.c_double()
            check(lib().td_timing_get(self.h, kernel.encode(), ctypes.byref(n), ctypes.byref(ms)), self.h)
            return n.value, ms.value
        return None

    def evaluate(self, cells, debug_prior=0, want_nearest=False):
        """-> (ptS[n], phi, likelihood, nearest[P] or None)"""
        xc, yc, zc, ze = (f64(c) for c in cells)
        ptS = np.zeros(self.n)
        phi = ctypes.c_double()
        lk = ctypes.c_double()
        near = np.empty(max(self.P, 1), dtype=np.int32) if want_nearest else None
        check(lib().td_evaluate(self.h, ptr(xc), ptr(yc), ptr(zc), ptr(ze), len(xc), int(debug_prior), ptr(ptS),
                                ctypes.byref(phi), ctypes.byref(lk),
                                ptr(near, _lib._pi32) if near is not None else None), self.h)
        return ptS, phi.value, lk.value, (near[:self.P] if near is not None else None)

    def evaluate_batch(self, models):
        """Several cell sets -> (ptS[k, n], phi[k], likelihood[k])."""
        off = np.zeros(len(models) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(m[0]) for m in models])
        cat = [f64(np.concatenate([m[i] for m in models])) if len(models) else np.zeros(0) for i in range(4)]
        ptS = np.zeros((len(models), self.n))
        phi = np.zeros(len(models))
        lk = np.zeros(len(models))
        check(lib().td_evaluate_batch(self.h, len(models), ptr(off, _lib._pi64), *(ptr(c) for c in cat), ptr(ptS),
                                      ptr(phi), ptr(lk)), self.h)
        return ptS, phi, lk

    def rasterize(self, models, qx, qy, qz, want_values=False):
        """td_rasterize: -> (mean[nq], std[nq], values[nmodels, nq] or None).
        models: list of (x, y, z, zeta) cell arrays in model_hist order."""
        off = np.zeros(len(models) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(m[0]) for m in models])
        cat = [f64(np.concatenate([np.asarray(m[k], dtype=np.float64) for m in models])) for k in range(4)]
        qx, qy, qz = (f64(np.ravel(a)) for a in (qx, qy, qz))
        nq = len(qx)
        mean, std = np.empty(nq), np.empty(nq)
        vals = np.empty((len(models), nq)) if want_values else None
        check(lib().td_rasterize(self.h, len(models), ptr(off, _lib._pi64), *(ptr(c) for c in cat), ptr(qx), ptr(qy),
                                 ptr(qz), nq, ptr(mean), ptr(std), ptr(vals) if want_values else None), self.h)
        return mean, std, vals

    def interpolate(self, cells, X, Y, Z, want_nearest=False):
        """-> (zeta[npoints], nearest[npoints] or None)"""
        xc, yc, zc, ze = (f64(c) for c in cells)
        X, Y, Z = (f64(np.atleast_1d(a)) for a in (X, Y, Z))
        out = np.empty(max(len(X), 1))
        near = np.empty(max(len(X), 1), dtype=np.int32) if want_nearest else None
        npo = ctypes.c_int64()
        check(lib().td_interpolate(self.h, ptr(xc), ptr(yc), ptr(zc), ptr(ze), len(xc), ptr(X), len(X), ptr(Y),
                                   len(Y), ptr(Z), len(Z), ptr(out),
                                   ptr(near, _lib._pi32) if near is not None else None, ctypes.byref(npo)), self.h)
        k = npo.value
        return out[:k].copy(), (near[:k].copy() if near is not None else None)


def context_for(dataStruct):
    """The (cached) device context of a DataStruct; geometry never changes
    during a chain (deepcopy(dataStruct) only duplicates values)."""
    if dataStruct._td_ctx is None:
        dataStruct._td_ctx = TdContext.from_datastruct(dataStruct)
    return dataStruct._td_ctx


def evaluate(model, dataStruct, TD_parameters):
    """MCsub.jl:123-185."""
    valid = 1
    model.phi = 1
    model.likelihood = 1
    if TD_parameters.debug_prior == 1:  # :134-136
        return model, dataStruct, valid
    if TD_parameters.interp_style != 1:
        raise NotImplementedError("interp_style=2 (IDW) is broken in the reference (MCsub.jl:332)")
    ctx = context_for(dataStruct)
    ptS, phi, lk, _ = ctx.evaluate(model.cells())
    model.phi = phi
    model.ptS = ptS
    model.tS = dataStruct.tS
    model.likelihood = lk
    return model, dataStruct, valid


def Interpolation(TD_parameters, model, X, Y, Z, dataStruct=None):  # noqa: N802 -- reference name
    """MCsub.jl:306-336 (interp_style 1).  The reference needs no DataStruct here;
    any context works (geometry is not used), so one is created on demand."""
    if TD_parameters.interp_style != 1:
        raise NotImplementedError("interp_style=2 (IDW) is broken in the reference (MCsub.jl:332)")
    ctx = context_for(dataStruct) if dataStruct is not None else _scratch_context()
    z, _ = ctx.interpolate(model.cells(), X, Y, Z)
    return z


def v_nearest(x, y, z, mx, my, mz, mv, dataStruct=None):
    """MCsub.jl:247-263 for one point (value of the first nearest cell, 0.0 if none < 1e9)."""
    ctx = context_for(dataStruct) if dataStruct is not None else _scratch_context()
    v, _ = ctx.interpolate((mx, my, mz, mv), [x], [y], [z])
    return float(v[0])


_scratch = None


def _scratch_context():
    """A context with no rays, for Interpolation calls that carry no DataStruct."""
    global _scratch
    if _scratch is None:
        e = np.zeros((1, 0))
        _scratch = TdContext(e, e, e, np.zeros((0, 0)), np.zeros((0, 0)), np.zeros(0), np.zeros(0))
    return _scratch
