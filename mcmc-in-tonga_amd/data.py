"""Input data: the shipped 381-ray geometry, slowness, and synthetic configs.

Mirrors the parts of load_data_Tonga.jl that build the hot-path fields of
``DataStruct``.  The reference's loader cannot run on the shipped files (it
opens ``Data/raypaths.jld``/``traces.jld`` with keys ``x,y,z,u,aveatten``;
the repository ships ``381raypaths.jld`` with ``x_n,y_n,z_n`` and no slowness),
so:

* ray points come from ``data/rays381.npz`` (converted from
  ``Data/381raypaths.jld`` by tests/golden/make_fixtures.py);
* slowness U = 1/Vp(z) from ak135 (``Data/ak135f.txt``) with ``interp1``
  semantics (MCsub.jl:54-74) -- a documented SUBSTITUTE for the 3-D model the
  reference read from ``raypaths.jld["u"]``;
* the study box is the ray-frame grid of plot_distribution.jl:36-40
  (xVec -79.477:20:1060.52, yVec -164.40:20:495.60, zVec 0:20:660).
"""
import os

import numpy as np

from .config import define_TDstructrure
from .defstruct import DataStruct, Model

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")

# plot_distribution.jl:36-40 (the ray frame of Data/381raypaths.jld)
XVEC = (-79.47730270810919, 20.0, 1060.5226972918908)
YVEC = (-164.40158664642206, 20.0, 495.59841335357794)
ZVEC = (0.0, 20.0, 660.0)


def julia_range(a, step, b):
    """Elements of the Julia range a:step:b (a + k*step, k = 0..floor((b-a)/step))."""
    n = int(np.floor((b - a) / step + 1e-9)) + 1
    return a + step * np.arange(n)


def box():
    """(xmin, xmax, ymin, ymax, zmin, zmax) = min/max of xVec, yVec, zVec."""
    return (XVEC[0], XVEC[2], YVEC[0], YVEC[2], ZVEC[0], ZVEC[2])


def lonlat2xy(lon0, lat0, beta, lon1, lat1):
    """MCsub.jl:5-31."""
    re = 6371
    r2d = 180.0 / np.pi
    xx = (np.asarray(lon1) - lon0) * re / r2d
    yy = (np.asarray(lat1) - lat0) * re / r2d
    x1 = (xx - yy * np.tan(beta)) * np.cos(beta)
    y1 = x1 * np.tan(beta) + yy / np.cos(beta)
    return x1, y1


def interp1(x, y, xx):
    """MCsub.jl:54-74: linear interpolation on half-open intervals x[j] <= xx < x[j+1]
    (so at a repeated depth the deeper layer wins); NaN outside [x[0], x[-1])."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xx = np.asarray(xx, dtype=np.float64)
    j = np.searchsorted(x, xx, side="right") - 1  # largest j with x[j] <= xx
    ok = (j >= 0) & (j < len(x) - 1) & ~np.isnan(xx)
    jj = np.clip(j, 0, len(x) - 2)
    ok &= xx < x[jj + 1]
    yy = y[jj] + (xx - x[jj]) / (x[jj + 1] - x[jj]) * (y[jj + 1] - y[jj])
    return np.where(ok, yy, np.nan)


def ak135_slowness(z):
    """U = 1 / Vp(z) [s/km] from ak135 (substitute for the reference's 3-D model)."""
    t = np.load(os.path.join(DATA_DIR, "ak135f.npz"))
    return 1.0 / interp1(t["depth"], t["vp"], z)


def segments(x, y, z, U):
    """load_data_Tonga.jl:66-69: rayL, rayU from m x n point arrays."""
    dx = x[:-1, :] - x[1:, :]
    dy = y[:-1, :] - y[1:, :]
    dz = z[:-1, :] - z[1:, :]
    rayl = np.sqrt((dx * dx + dy * dy) + dz * dz)
    rayu = 0.5 * (U[:-1, :] + U[1:, :])
    return rayl, rayu


def pad_rays(npts, px, py, pz, m=None):
    """CSR points -> m x n NaN tail-padded arrays (DataStruct.rayX layout)."""
    npts = np.asarray(npts, dtype=np.int64)
    m = int(npts.max()) if m is None else int(m)
    n = len(npts)
    out = [np.full((m, n), np.nan) for _ in range(3)]
    off = 0
    for i, c in enumerate(npts):
        for a, src in zip(out, (px, py, pz)):
            a[:c, i] = src[off:off + c]
        off += c
    return out


def _datastruct(rayX, rayY, rayZ, tS, allSig, extra=None):
    return _datastruct_u(rayX, rayY, rayZ, ak135_slowness(rayZ), tS, allSig, extra)


def _datastruct_u(rayX, rayY, rayZ, U, tS, allSig, extra=None):
    """DataStruct from rays and their slowness (load_data_Tonga.jl:66-88)."""
    rayL, rayU = segments(rayX, rayY, rayZ, U)
    e = extra or {}
    nan = np.full(len(tS), np.nan)
    return DataStruct(
        tS=np.asarray(tS, dtype=np.float64), allaveatten=e.get("allaveatten", nan), allLats=e.get("allLats", nan),
        allLons=e.get("allLons", nan), allSig=np.asarray(allSig, dtype=np.float64), dataX=e.get("dataX", nan),
        dataY=e.get("dataY", nan), xVec=e.get("xVec", julia_range(*XVEC)), yVec=e.get("yVec", julia_range(*YVEC)),
        zVec=e.get("zVec", julia_range(*ZVEC)),
        elonsX=e.get("elonsX", nan), elatsY=e.get("elatsY", nan), elons=e.get("elons", nan),
        elats=e.get("elats", nan), edep=e.get("edep", nan), coastX=np.zeros(0), coastY=np.zeros(0),
        rayX=rayX, rayY=rayY, rayZ=rayZ, rayL=rayL, rayU=rayU, U=U)


def load_data_Tonga(TD_parameters=None):  # noqa: N802 -- reference name (load_data_Tonga.jl:4)
    """The 381-ray data set as a DataStruct (see module docstring for substitutions)."""
    TD_parameters = TD_parameters or define_TDstructrure()
    d = np.load(os.path.join(DATA_DIR, "rays381.npz"))
    rayX, rayY, rayZ = pad_rays(d["npts"], d["x"], d["y"], d["z"], m=int(d["m"]))
    lat0, lon0, beta = -23.1000, 174.6000, 0.463647609  # load_data_Tonga.jl:26-28
    dataX, dataY = lonlat2xy(lon0, lat0, beta, d["longitude"], d["latitude"])
    elonsX, elatsY = lonlat2xy(lon0, lat0, beta, d["EventLongitude"], d["EventLatitude"])
    extra = dict(allLats=d["latitude"], allLons=d["longitude"], dataX=dataX, dataY=dataY, elonsX=elonsX,
                 elatsY=elatsY, elons=d["EventLongitude"], elats=d["EventLatitude"], edep=d["EventDepth"])
    return _datastruct(rayX, rayY, rayZ, d["tStar"], d["error"], extra)


def synthetic_rays(nrays, seed=5, spacing=11.0, zrange=(50.0, 650.0)):
    """events uniform in the box (z in zrange), stations at
    z = 0, straight rays resampled every ~`spacing` km, NaN tail padding.
    t* "observations" are drawn U(0.05, 1.2) with sigma U(0.04, 0.6) (ranges of
    381traces)."""
    rng = np.random.default_rng(seed)
    xmin, xmax, ymin, ymax, _, _ = box()
    ev = np.stack([rng.uniform(xmin, xmax, nrays), rng.uniform(ymin, ymax, nrays),
                   rng.uniform(zrange[0], zrange[1], nrays)], 1)
    stn = np.stack([rng.uniform(xmin, xmax, nrays), rng.uniform(ymin, ymax, nrays), np.zeros(nrays)], 1)
    length = np.linalg.norm(stn - ev, axis=1)
    npts = np.maximum(2, np.ceil(length / spacing).astype(np.int64) + 1)
    P = int(npts.sum())
    px, py, pz = np.empty(P), np.empty(P), np.empty(P)
    off = 0
    for i in range(nrays):
        t = np.linspace(0.0, 1.0, npts[i])
        seg = ev[i][None, :] + t[:, None] * (stn[i] - ev[i])[None, :]
        px[off:off + npts[i]], py[off:off + npts[i]], pz[off:off + npts[i]] = seg[:, 0], seg[:, 1], seg[:, 2]
        off += npts[i]
    rayX, rayY, rayZ = pad_rays(npts, px, py, pz)
    tS = rng.uniform(0.05, 1.2, nrays)
    sig = rng.uniform(0.04, 0.6, nrays)
    return _datastruct(rayX, rayY, rayZ, tS, sig)


def random_model(ncells, seed, zeta_scale=50):
    """A fixed synthetic model for configs 1-4: cells uniform in the
    box, zeta ~ U(0, zeta_scale) -- the build_starting prior (MCsub.jl:92-100).
    numpy PCG64 (default_rng(seed))."""
    rng = np.random.default_rng(seed)
    xmin, xmax, ymin, ymax, zmin, zmax = box()
    x = xmin + (xmax - xmin) * rng.random(ncells)
    y = ymin + (ymax - ymin) * rng.random(ncells)
    z = zmin + (zmax - zmin) * rng.random(ncells)
    zeta = rng.random(ncells) * zeta_scale
    return Model(float(ncells), x, y, z, zeta)


# BASELINE.json configs: name -> (rays, cells, model seed)
CONFIGS = {
    "config1": ("rays381", 200, 1),
    "config2": ("rays381", 1000, 2),
    "config3": ("rays381", 5000, 3),
    "config4": ("rays381", 2000, 100),  # + rank
    "config5": ("synthetic10k", 20000, 5),
}
