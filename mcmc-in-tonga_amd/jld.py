"""Saved models in JLD, the reference's output format.

main_inversion.jl:18 ends a run with ``save("model.jld", "model", models)``
(``models`` = one ``model_hist`` per chain); the Julia post-processing
(``loadnplot.jl``) reads it back with ``load``.  ``save``/``load`` here write
and read that file with the same HDF5 layout the reference's own
``model.jld`` has (jld_h5.py documents it; tests/test_jld.py compares the
structure with the reference file's and round-trips the reference's 100
models bit for bit).

HDF5 comes from h5py, which this image has only in ``/opt/conda/bin/python3.9``
(not in the package's interpreter): the models cross to it as a packed
``.npz``.  ``TONGA_H5PY_PYTHON`` names another interpreter; an interpreter
that can import h5py itself runs jld_h5 in-process.  Off the hot path.
"""
import importlib.util
import os
import subprocess
import sys
import tempfile

import numpy as np

from .defstruct import Model

_HERE = os.path.dirname(os.path.abspath(__file__))
_CONDA = "/opt/conda/bin/python3.9"
_ARRAYS = ("xCell", "yCell", "zCell", "zeta", "ptS", "tS")


def h5py_python():
    """The interpreter that runs jld_h5.py: None = this one (h5py importable)."""
    env = os.environ.get("TONGA_H5PY_PYTHON")
    if env:
        return env
    if importlib.util.find_spec("h5py") is not None:
        return None
    if os.path.exists(_CONDA):
        return _CONDA
    raise RuntimeError("JLD I/O needs h5py: none importable here and %s is absent "
                       "(set TONGA_H5PY_PYTHON to an interpreter with h5py)" % _CONDA)


def available():
    try:
        h5py_python()
        return True
    except RuntimeError:
        return False


def pack(models):
    """models: list of chains, each a list of Model -> flat arrays (jld_h5's format).
    A Model object saved more than once (model_hist aliases the current model
    when it did not change between saves, TD_inversion_function.jl:280) is
    stored once and referenced again, as JLD does: ``entry`` maps each saved
    position to its stored model."""
    flat, entry, seen = [], [], {}
    for chain in models:
        for m in chain:
            if id(m) not in seen:
                seen[id(m)] = len(flat)
                flat.append(m)
            entry.append(seen[id(m)])
    out = {"chain_off": np.concatenate([[0], np.cumsum([len(c) for c in models])]).astype(np.int64),
           "entry": np.array(entry, dtype=np.int64)}
    for k in ("nCells", "phi", "likelihood", "zeta_xz", "zeta_xy"):
        out[k] = np.array([float(getattr(m, k)) for m in flat], dtype=np.float64)
    for k in ("action", "accept"):
        out[k] = np.array([int(getattr(m, k)) for m in flat], dtype=np.int64)
    for k in _ARRAYS:
        arrs = [np.asarray(getattr(m, k), dtype=np.float64).ravel() for m in flat]
        out[k] = np.concatenate(arrs) if arrs else np.zeros(0)
        out[k + "_off"] = np.concatenate([[0], np.cumsum([len(a) for a in arrs])]).astype(np.int64)
    return out


def unpack(p):
    """Inverse of pack: list of chains of Model (a model stored once and
    referenced twice comes back as one object, twice)."""
    made = {}

    def model(j):
        if j not in made:
            a = {k: p[k][int(p[k + "_off"][j]):int(p[k + "_off"][j + 1])].copy() for k in _ARRAYS}
            made[j] = Model(float(p["nCells"][j]), a["xCell"], a["yCell"], a["zCell"], a["zeta"],
                            float(p["phi"][j]), a["ptS"], a["tS"], float(p["likelihood"][j]),
                            int(p["action"][j]), int(p["accept"][j]), float(p["zeta_xz"][j]),
                            float(p["zeta_xy"][j]))
        return made[j]

    co, entry = p["chain_off"], p["entry"]
    return [[model(int(entry[e])) for e in range(int(co[c]), int(co[c + 1]))] for c in range(len(co) - 1)]


def _module():
    """jld_h5 in this interpreter (h5py importable here)."""
    sys.path.insert(0, _HERE)
    try:
        import jld_h5  # noqa: WPS433
    finally:
        sys.path.remove(_HERE)
    return jld_h5


def _subprocess(py, args):
    r = subprocess.run([py, os.path.join(_HERE, "jld_h5.py")] + list(args), capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("jld_h5.py %s failed: %s" % (args[0], (r.stderr or r.stdout).strip()[-2000:]))
    return r.stdout


def save(path, models):
    """save(path, "model", models) as main_inversion.jl:18 (models: list of chains of Model)."""
    p, py, path = pack(models), h5py_python(), os.path.abspath(path)
    if py is None:
        _module().write(path, p)
        return
    with tempfile.TemporaryDirectory() as td:
        tmp = os.path.join(td, "models.npz")
        np.savez(tmp, **p)
        _subprocess(py, ["write", tmp, path])


def load(path):
    """load(path, "model"): list of chains of Model."""
    py, path = h5py_python(), os.path.abspath(path)
    if py is None:
        return unpack(_module().read(path))
    with tempfile.TemporaryDirectory() as td:
        tmp = os.path.join(td, "models.npz")
        _subprocess(py, ["read", path, tmp])
        with np.load(tmp, allow_pickle=False) as z:
            return unpack({k: z[k] for k in z.files})


# DataStruct fields in DefStruct.jl:5-30 order (jld_h5.py keeps the same list: it
# runs standalone under the h5py interpreter)
DS_FIELDS = ["tS", "allaveatten", "allLats", "allLons", "allSig", "dataX", "dataY", "xVec", "yVec", "zVec",
             "elonsX", "elatsY", "elons", "elats", "edep", "coastX", "coastY", "rayX", "rayY", "rayZ", "rayL",
             "rayU", "U"]
DS_RANGES = ("xVec", "yVec", "zVec")


def _range_triple(v):
    v = np.asarray(v, dtype=np.float64).ravel()
    step = float(v[1] - v[0]) if len(v) > 1 else 0.0
    return np.array([float(v[0]) if len(v) else 0.0, step, float(len(v))])


def save_checkpoint(path, model, dataStruct, it, burnin, model_hist=(), saved=0, model_num=0):  # noqa: N803
    """A chain checkpoint with the fields of TD_inversion_function.jl:285
    (burnin = True: model, dataStruct, iter, saved_#, model_num, model_hist)
    or :292 (burnin = False: model, dataStruct, iter)."""
    p = pack([[model], list(model_hist) if burnin else []])
    p["ck_iter"] = np.array(float(it))
    p["ck_iter_int"] = np.array(0 if burnin else 1)  # :285 iter (Float64 loop variable), :292 Int64(iter)
    p["ck_burnin"] = np.array(1 if burnin else 0)
    p["ck_saved"] = np.array(int(saved))
    p["ck_model_num"] = np.array(int(model_num))
    for fld in DS_FIELDS:
        v = getattr(dataStruct, fld)
        if fld in DS_RANGES:
            p["ds_" + fld + "_range"] = _range_triple(v)
        else:
            p["ds_" + fld] = np.asarray(v, dtype=np.float64)
    _write_packed(path, p, "write_checkpoint")


def load_checkpoint(path):
    """The checkpoint entries TD_inversion_function.jl:56-66 reads back:
    dict(model, iter, burnin, model_hist, saved, model_num, ds) -- model_hist,
    saved, model_num only when burnin (as the reference)."""
    p = _read_packed(path, "read_checkpoint")
    chains = unpack(p)
    out = {"model": chains[0][0], "iter": float(p["ck_iter"]), "iter_is_int": bool(int(p["ck_iter_int"])),
           "burnin": bool(int(p["ck_burnin"])), "model_hist": chains[1] if len(chains) > 1 else [],
           "ds": {k[3:]: p[k] for k in p if k.startswith("ds_")}}
    if out["burnin"]:
        out["saved"] = int(p["ck_saved"])
        out["model_num"] = int(p["ck_model_num"])
    return out


def _write_packed(path, p, cmd):
    py, path = h5py_python(), os.path.abspath(path)
    if py is None:
        getattr(_module(), cmd)(path, p)
        return
    with tempfile.TemporaryDirectory() as td:
        tmp = os.path.join(td, "packed.npz")
        np.savez(tmp, **p)
        _subprocess(py, [cmd, tmp, path])


def _read_packed(path, cmd):
    py, path = h5py_python(), os.path.abspath(path)
    if py is None:
        return getattr(_module(), cmd)(path)
    with tempfile.TemporaryDirectory() as td:
        tmp = os.path.join(td, "packed.npz")
        _subprocess(py, [cmd, path, tmp])
        with np.load(tmp, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}


def fingerprint(path):
    """jld_h5.fingerprint: the file's HDF5 structure as nested lists (JSON types)."""
    import json
    py, path = h5py_python(), os.path.abspath(path)
    if py is None:
        return json.loads(json.dumps(_module().fingerprint(path)))
    return json.loads(_subprocess(py, ["fingerprint", path]))
