"""Ray and slowness ingest: pre_process_data.jl:15-124
and load_3Dvel.jl:4-34, plus the DataStruct assembly of load_data_Tonga.jl
from their outputs.

The reference turns ``Data/raypaths.p`` (ray points), ``Data/lau.vel`` (a
3-D velocity model) and ``Data/p_tstar.dat`` + ``Data/stations.lst`` (t*
data) into ``raypaths.jld`` / ``traces.jld``, which load_data_Tonga.jl then
reads.  None of these inputs ship with the reference, so this
module is exercised on synthetic files of the same formats.  The one heavy
step -- the slowness of every ray point, ``itp.(ix, iy, iz)`` with
``Gridded(Linear())`` -- runs on the GPU (``td_trilinear``, ingest.hip);
parsing is host text work.
"""
import ctypes

import numpy as np

from . import _lib
from .config import define_TDstructrure
from .data import _datastruct_u, julia_range, lonlat2xy

SEPARATOR = "1234567"  # pre_process_data.jl:26: a line starting with it closes a ray


class Gridded:
    """``interpolate((x, y, z), sn, Gridded(Linear()))`` (load_3Dvel.jl:32)."""

    def __init__(self, xs, ys, zs, values, device=0):
        self.xs, self.ys, self.zs = (np.ascontiguousarray(a, dtype=np.float64) for a in (xs, ys, zs))
        self.values = np.asarray(values, dtype=np.float64)  # (nx, ny, nz)
        assert self.values.shape == (len(self.xs), len(self.ys), len(self.zs))
        self.device = device

    def __call__(self, x, y, z):
        """itp.(x, y, z) at many points, on the GPU; BoundsError outside the grid."""
        px, py, pz = (np.ascontiguousarray(np.ravel(a), dtype=np.float64) for a in (x, y, z))
        out = np.empty(len(px))
        nout = ctypes.c_int64()
        v = np.ascontiguousarray(self.values.ravel(order="F"))  # x fastest, as Julia stores sn[1,:,:,:]
        P = _lib.ptr
        _lib.check(_lib.lib().td_trilinear(self.device, P(self.xs), len(self.xs), P(self.ys), len(self.ys),
                                           P(self.zs), len(self.zs), P(v), P(px), P(py), P(pz), len(px), P(out),
                                           ctypes.byref(nout)))
        if nout.value:
            raise ValueError("BoundsError: %d points outside the velocity grid" % nout.value)
        return out.reshape(np.shape(x))


def load_3Dvel(path="./Data/lau.vel", TD_parameters=None, device=0):  # noqa: N802 -- reference name
    """load_3Dvel.jl:4-34: the P slowness grid of lau.vel in the ray frame."""
    with open(path) as fh:
        vel = fh.read().splitlines()
    nnx, nny, nnz = (int(v) for v in vel[0].split()[:3])
    lat0, lon0, beta = (float(v) for v in vel[1].split()[:3])
    lat = np.empty((nnx, nny))
    lon = np.empty((nnx, nny))
    for i in range(nnx):
        for j in range(nny):
            f = vel[i * nny + j + 2].split()  # vel[(i-1)*nny+j+2], 1-based
            lat[i, j], lon[i, j] = float(f[0]), float(f[1])
    dataX, dataY = lonlat2xy(lon0, lat0, beta, lon, lat)
    z = np.array([float(v) for v in vel[nnx * nny + 2].split()])  # vel[nnx*nny+3]
    vps = np.empty((2, nnx, nny, nnz))
    for p in (1, 2):
        for i in range(nnx):
            for j in range(nny):
                f = vel[(i + p * nnx) * nny + j + 3].split()  # vel[(i-1+p*nnx)*nny+j+3], 1-based
                vps[p - 1, i, j, :] = [float(v) for v in f[:nnz]]
    sn = 1.0 / vps
    # round.(dataX; digits=2)[:,1], round.(dataY; digits=2)[1,:]: Julia rounds x*100 half-to-even, as np.round
    return Gridded(np.round(dataX, 2)[:, 0], np.round(dataY, 2)[0, :], z, sn[0], device=device)


def load_raypath(path="./Data/raypaths.p", itp=None):
    """pre_process_data.jl:15-63: the rays of raypaths.p as NaN-padded m x n
    arrays x, y, z and their slowness u = itp.(x, y, z)."""
    with open(path) as fh:
        lines = fh.read().splitlines()
    X, Y, Z = [], [], []
    ix, iy, iz = [], [], []
    for i, line in enumerate(lines):
        tok = line.split()
        if tok[0] == SEPARATOR:
            if ix:  # :22-25: a separator before any point is skipped
                X.append(ix), Y.append(iy), Z.append(iz)
                ix, iy, iz = [], [], []
        else:
            ix.append(float(tok[0])), iy.append(float(tok[1])), iz.append(float(tok[2]))
        if i == len(lines) - 1:  # :37-40 (a file ending in a separator adds an empty ray, as there)
            X.append(ix), Y.append(iy), Z.append(iz)
    m = max(len(r) for r in X)
    out = {k: np.full((m, len(X)), np.nan) for k in ("x", "y", "z", "u")}
    for r, (a, b, c) in enumerate(zip(X, Y, Z)):
        out["x"][:len(a), r], out["y"][:len(a), r], out["z"][:len(a), r] = a, b, c
    if itp is not None:
        ok = ~np.isnan(out["x"])
        u = np.full(out["x"].shape, np.nan)
        u[ok] = itp(out["x"][ok], out["y"][ok], out["z"][ok])
        out["u"] = u
    return out


def load_traceinfo(p_tstar="./Data/p_tstar.dat", stations="./Data/stations.lst"):
    """pre_process_data.jl:68-120: the t* data with station coordinates."""
    stalat, stalon = {}, {}
    with open(stations) as fh:
        for line in fh.read().splitlines():
            f = line.split()
            stalat[f[0]], stalon[f[0]] = float(f[1]), float(f[2])
    cols = {k: [] for k in ("station", "EventLatitude", "EventLongitude", "EventDepth", "latitude", "longitude",
                            "tStar", "error", "aveatten")}
    with open(p_tstar) as fh:
        for line in fh.read().splitlines():
            f = line.split()
            cols["station"].append(f[0])
            for k, c in (("EventLatitude", 1), ("EventLongitude", 2), ("EventDepth", 3), ("tStar", 4),
                         ("error", 5), ("aveatten", 7)):
                cols[k].append(float(f[c]))
            cols["latitude"].append(stalat[f[0]])
            cols["longitude"].append(stalon[f[0]])
    return {k: (np.array(v) if k == "station" else np.array(v, dtype=np.float64)) for k, v in cols.items()}


def pre_process_data(data_dir="./Data", TD_parameters=None, device=0):
    """pre_process_data.jl: (raypaths, traces) -- what it saves as raypaths.jld / traces.jld."""
    import os
    itp = load_3Dvel(os.path.join(data_dir, "lau.vel"), TD_parameters, device)
    return (load_raypath(os.path.join(data_dir, "raypaths.p"), itp),
            load_traceinfo(os.path.join(data_dir, "p_tstar.dat"), os.path.join(data_dir, "stations.lst")))


def load_data_Tonga_from(raypaths, traces, TD_parameters=None):  # noqa: N802
    """load_data_Tonga.jl:4-88 on the pre-processed data: study area from the
    stations (:41-48), segments from the rays and their 3-D slowness (:66-69)."""
    TD_parameters = TD_parameters or define_TDstructrure()
    lat0, lon0, beta = -23.1000, 174.6000, 0.463647609  # load_data_Tonga.jl:26-28
    dataX, dataY = lonlat2xy(lon0, lat0, beta, traces["longitude"], traces["latitude"])
    elonsX, elatsY = lonlat2xy(lon0, lat0, beta, traces["EventLongitude"], traces["EventLatitude"])
    b, s = float(TD_parameters.buffer), float(TD_parameters.XYnodeSpacing)
    xVec = julia_range(np.min(dataX) - b, s, np.max(dataX) + b)
    yVec = julia_range(np.min(dataY) - b, s, np.max(dataY) + b)
    zVec = julia_range(float(TD_parameters.min_depth), float(TD_parameters.ZnodeSpacing), float(TD_parameters.max_depth))
    extra = dict(allaveatten=traces["aveatten"], allLats=traces["latitude"], allLons=traces["longitude"],
                 dataX=dataX, dataY=dataY, elonsX=elonsX, elatsY=elatsY, elons=traces["EventLongitude"],
                 elats=traces["EventLatitude"], edep=traces["EventDepth"], xVec=xVec, yVec=yVec, zVec=zVec)
    return _datastruct_u(raypaths["x"], raypaths["y"], raypaths["z"], raypaths["u"], traces["tStar"],
                         traces["error"], extra)
