#!/opt/conda/bin/python3.9
"""Convert the reference's shipped data files into small, loader-free fixtures.

Run ONCE in the build container (the only place where /root/reference and h5py
exist):

    /opt/conda/bin/python3.9 tests/golden/make_fixtures.py

Nothing here executes anything from the reference: the JLD files are HDF5 and
are read with h5py's plain dataset readers (no pickle, no Julia).  Outputs are
plain ``.npz`` (numpy, ``allow_pickle=False``-loadable) and are committed:

* ``mcmc-in-tonga_amd/data/rays381.npz`` -- the 381 ray paths of
  ``Data/381raypaths.jld`` (keys ``x_n,y_n,z_n``, shape (131, 381) in HDF5 =
  points x rays, NaN tail padding), stored compactly as per-ray point counts +
  the concatenated valid points; plus ``tStar``/``error``/station/event info
  from ``Data/381traces.jld`` (one object reference per datum).
* ``mcmc-in-tonga_amd/data/ak135f.npz`` -- depth / Vp columns of
  ``Data/ak135f.txt`` (used to synthesise slowness U).
* ``tests/golden/model_jld_kat.npz`` -- the known-answer records of
  ``model.jld`` (2 chains x 50 saved ``Model`` structs, DefStruct.jl:32-48):
  cells, zeta, phi, ptS, tS, likelihood, action, accept, zeta_xz, zeta_xy,
  and same_as (the saved position whose object a position aliases).  These pin the chi^2 reduction
  (MCsub.jl:169-173) and the likelihood expression (MCsub.jl:179-182), whose
  value also pins Julia's reassociated ``sum`` order (see oracle/README).
* ``tests/golden/model_jld_structure.json`` -- the HDF5 structure of
  ``model.jld`` (user block, objects, storage layouts, types, attributes):
  the JLD writer (mcmc-in-tonga_amd/jld_h5.py) must reproduce it.
"""
import os
import sys

import h5py
import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DATA_OUT = os.path.join(REPO, "mcmc-in-tonga_amd", "data")


def deref_scalars(f, ds):
    """JLD stores Vector{Any} of scalars as an array of object references."""
    return np.array([f[r][()] for r in ds[0, :]])


def rays():
    f = h5py.File(os.path.join(REF, "Data", "381raypaths.jld"), "r")
    x, y, z = (f[k][()] for k in ("x_n", "y_n", "z_n"))  # (131, 381)
    m, n = x.shape
    assert (np.isnan(x) == np.isnan(y)).all() and (np.isnan(x) == np.isnan(z)).all()
    npts = (~np.isnan(x)).sum(axis=0).astype(np.int32)
    for r in range(n):  # tail padding only
        assert not np.isnan(x[: npts[r], r]).any() and np.isnan(x[npts[r]:, r]).all()
    cat = lambda a: np.concatenate([a[: npts[r], r] for r in range(n)])
    t = h5py.File(os.path.join(REF, "Data", "381traces.jld"), "r")
    out = dict(
        m=np.int64(m), npts=npts, x=cat(x), y=cat(y), z=cat(z),
        tStar=deref_scalars(t, t["tStar"]).astype(np.float64),
        error=deref_scalars(t, t["error"]).astype(np.float64),
        latitude=deref_scalars(t, t["latitude"]).astype(np.float64),
        longitude=deref_scalars(t, t["longitude"]).astype(np.float64),
        EventLatitude=deref_scalars(t, t["EventLatitude"]).astype(np.float64),
        EventLongitude=deref_scalars(t, t["EventLongitude"]).astype(np.float64),
        EventDepth=deref_scalars(t, t["EventDepth"]).astype(np.float64),
    )
    np.savez_compressed(os.path.join(DATA_OUT, "rays381.npz"), **out)
    print("rays381: m=%d n=%d P=%d" % (m, n, int(npts.sum())))


def ak135():
    rows = []
    with open(os.path.join(REF, "Data", "ak135f.txt")) as fh:
        for line in fh:
            line = line.strip()
            if line:
                rows.append([float(v) for v in line.split(",")])
    a = np.array(rows)
    np.savez_compressed(os.path.join(DATA_OUT, "ak135f.npz"), depth=a[:, 0], vp=a[:, 1], vs=a[:, 2])
    print("ak135f: %d rows" % len(a))


MODEL_FIELDS = ["nCells_", "xCell_", "yCell_", "zCell_", "zeta_", "phi_", "ptS_", "tS_",
                "likelihood_", "action_", "accept_", "zeta_xz_", "zeta_xy_"]
MODEL_FMT = ["<f8", "R", "R", "R", "R", "<f8", "R", "R", "<f8", "<i8", "<i8", "<f8", "<f8"]


def model_kat():
    f = h5py.File(os.path.join(REF, "model.jld"), "r")
    dt = np.dtype([(n, (h5py.ref_dtype if t == "R" else t)) for n, t in zip(MODEL_FIELDS, MODEL_FMT)])
    mt = h5py.h5t.py_create(dt)
    recs = []
    first = {}  # a Model saved twice (model_hist aliasing) is one stored object
    top = f["model"]
    for c in range(top.shape[0]):
        chain = f[top[c]]
        for j in range(chain.shape[0]):
            d = f[chain[j]]
            addr = h5py.h5o.get_info(d.id).addr
            first.setdefault(addr, len(recs))
            a = np.empty((), dtype=dt)
            d.id.read(h5py.h5s.ALL, h5py.h5s.ALL, a, mtype=mt)
            g = lambda k: np.asarray(f[a[k][()]][()], dtype=np.float64)
            recs.append(dict(chain=c + 1, nCells=float(a["nCells_"]), x=g("xCell_"), y=g("yCell_"),
                             z=g("zCell_"), zeta=g("zeta_"), phi=float(a["phi_"]), ptS=g("ptS_"),
                             tS=g("tS_"), likelihood=float(a["likelihood_"]),
                             action=int(a["action_"]), accept=int(a["accept_"]),
                             zeta_xz=float(a["zeta_xz_"]), zeta_xy=float(a["zeta_xy_"]),
                             same_as=first[addr]))
    tS = recs[0]["tS"]
    assert all((r["tS"] == tS).all() for r in recs)
    ncell = np.array([len(r["x"]) for r in recs], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(ncell)]).astype(np.int64)
    np.savez_compressed(
        os.path.join(HERE, "model_jld_kat.npz"),
        chain=np.array([r["chain"] for r in recs], dtype=np.int64),
        nCells=np.array([r["nCells"] for r in recs]),
        cell_off=off,
        xCell=np.concatenate([r["x"] for r in recs]),
        yCell=np.concatenate([r["y"] for r in recs]),
        zCell=np.concatenate([r["z"] for r in recs]),
        zeta=np.concatenate([r["zeta"] for r in recs]),
        phi=np.array([r["phi"] for r in recs]),
        likelihood=np.array([r["likelihood"] for r in recs]),
        action=np.array([r["action"] for r in recs], dtype=np.int64),
        accept=np.array([r["accept"] for r in recs], dtype=np.int64),
        zeta_xz=np.array([r["zeta_xz"] for r in recs]),
        zeta_xy=np.array([r["zeta_xy"] for r in recs]),
        same_as=np.array([r["same_as"] for r in recs], dtype=np.int64),
        ptS=np.stack([r["ptS"] for r in recs]),
        tS=tS,
    )
    print("model.jld: %d models, %d data" % (len(recs), len(tS)))


def model_jld_structure():
    """The HDF5 structure of model.jld (jld_h5.fingerprint): what the JLD
    writer must reproduce for the same models (tests/test_jld.py)."""
    import json
    sys.path.insert(0, os.path.join(REPO, "mcmc-in-tonga_amd"))
    import jld_h5
    fp = jld_h5.fingerprint(os.path.join(REF, "model.jld"))
    with open(os.path.join(HERE, "model_jld_structure.json"), "w") as fh:
        json.dump(fp, fh)
    print("model.jld structure: %d entries" % len(fp))


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference not mounted; fixtures are already committed")
    os.makedirs(DATA_OUT, exist_ok=True)
    rays()
    ak135()
    model_kat()
    model_jld_structure()
