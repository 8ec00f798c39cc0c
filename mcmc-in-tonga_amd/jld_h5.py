"""JLD (Julia's HDF5 format) for the saved models -- the h5py side.

main_inversion.jl:18 ends a run with ``save("model.jld", "model", models)``:
``models`` is one ``Vector{Any}`` of saved ``Model`` structs
(DefStruct.jl:32-48) per chain.  JLD (the version Julia 1.5 wrote, format
0.1.3) lays that out as:

* a 512-byte user block holding ``Julia data file (HDF5), version 0.1.3``;
* ``/_creator``: ENDIAN_BOM, JULIA_MAJOR/MINOR/PATCH (uint32), WORD_SIZE (int64);
* ``/_types/00000001``: the committed compound type of ``Model`` (field names
  with a trailing ``_``; arrays as object references), attribute
  ``julia type = "Model"``;
* ``/model``: one object reference per chain (``julia eltype =
  Core.Array{Core.Any,1}``), each to ``/_refs/NNNNNNNN``, a reference array
  (``julia eltype = Core.Any``) of that chain's models, each a scalar dataset
  of the committed type whose array fields point to further ``/_refs``
  entries -- numbered depth-first in writing order;
* every dataset in compact storage, string attributes fixed-length UTF-8,
  null-terminated, scalar; superblock version 0 (libver "earliest").

This module needs h5py and runs under an interpreter that has it (in this
image ``/opt/conda/bin/python3.9``); the package's Python calls it through
``jld.py``.  ``write``/``read`` exchange the models with the caller as a
packed ``.npz`` (no pickle).  It has no other dependency and executes nothing
from the files it reads.

usage: python jld_h5.py write PACKED.npz OUT.jld
       python jld_h5.py read IN.jld PACKED.npz
       python jld_h5.py write_checkpoint PACKED.npz OUT.jld
       python jld_h5.py read_checkpoint IN.jld PACKED.npz
"""
import sys

import h5py
import numpy as np
from h5py import h5a, h5d, h5g, h5o, h5p, h5s, h5t

HEADER = b"Julia data file (HDF5), version 0.1.3"
USERBLOCK = 512
MODEL_FIELDS = ["nCells_", "xCell_", "yCell_", "zCell_", "zeta_", "phi_", "ptS_", "tS_",
                "likelihood_", "action_", "accept_", "zeta_xz_", "zeta_xy_"]
MODEL_KINDS = ["<f8", "R", "R", "R", "R", "<f8", "R", "R", "<f8", "<i8", "<i8", "<f8", "<f8"]
ARRAY_FIELDS = ["xCell_", "yCell_", "zCell_", "zeta_", "ptS_", "tS_"]
COMPACT_MAX = 65000  # bytes: HDF5's compact storage limit is 64 KiB (larger arrays: contiguous)


def model_dtype():
    return np.dtype([(n, (h5py.ref_dtype if k == "R" else k)) for n, k in zip(MODEL_FIELDS, MODEL_KINDS)])


def model_raw_dtype():
    """The same record with each object reference as its 8-byte address (what
    an HDF5 object reference holds): written byte for byte, no conversion."""
    return np.dtype([(n, ("<u8" if k == "R" else k)) for n, k in zip(MODEL_FIELDS, MODEL_KINDS)])


def model_type():
    """Model's compound HDF5 type, built member by member (object references
    as H5T_STD_REF_OBJ, as in the reference file)."""
    raw = model_raw_dtype()
    tid = h5t.create(h5t.COMPOUND, raw.itemsize)
    for n, k in zip(MODEL_FIELDS, MODEL_KINDS):
        mt = {"<f8": h5t.IEEE_F64LE, "<i8": h5t.STD_I64LE, "R": h5t.STD_REF_OBJ}[k]
        tid.insert(n.encode(), raw.fields[n][1], mt)
    return tid


def _ref(fid, name):
    """The object reference to `name`: its object header address."""
    oid = h5o.open(fid, name.encode())
    return np.uint64(h5o.get_info(oid).addr)


def _str_attr(oid, name, value):
    b = value.encode()
    st = h5t.C_S1.copy()
    st.set_size(len(b))
    st.set_strpad(h5t.STR_NULLTERM)
    st.set_cset(h5t.CSET_UTF8)
    aid = h5a.create(oid, name.encode(), st, h5s.create(h5s.SCALAR))
    aid.write(np.array(b, dtype="S%d" % len(b)), mtype=st)


def _dataset(fid, name, data, ftype=None, mtype=None):
    data = np.asarray(data)
    space = h5s.create(h5s.SCALAR) if data.shape == () else h5s.create_simple(data.shape)
    dcpl = h5p.create(h5p.DATASET_CREATE)
    if data.nbytes <= COMPACT_MAX:
        dcpl.set_layout(h5d.COMPACT)
    ftype = ftype if ftype is not None else h5t.py_create(data.dtype)
    did = h5d.create(fid, name.encode(), ftype, space, dcpl=dcpl)
    did.write(h5s.ALL, h5s.ALL, data, mtype=mtype if mtype is not None else h5t.py_create(data.dtype))
    return did


class _Refs:
    """/_refs/NNNNNNNN names in JLD's depth-first writing order."""

    def __init__(self):
        self.n = 0

    def next(self):
        self.n += 1
        return "_refs/%08d" % self.n


def write(path, packed, julia_version=(1, 5, 2)):
    """Write the models of ``packed`` (see jld.py: pack) as ``save(path, "model", models)``."""
    chain_off = packed["chain_off"]
    f = h5py.File(path, "w", userblock_size=USERBLOCK, libver="earliest")
    fid = f.id
    for g in ("_creator", "_refs", "_types"):
        h5g.create(fid, g.encode())
    _dataset(fid, "_creator/ENDIAN_BOM", np.array(0x04030201, dtype="<u4"))
    for k, v in zip(("JULIA_MAJOR", "JULIA_MINOR", "JULIA_PATCH"), julia_version):
        _dataset(fid, "_creator/" + k, np.array(v, dtype="<u4"))
    _dataset(fid, "_creator/WORD_SIZE", np.array(64, dtype="<i8"))
    mtid = model_type()
    mtid.commit(fid, b"_types/00000001")
    _str_attr(mtid, "julia type", "Model")
    raw = model_raw_dtype()
    assert raw.itemsize == mtid.get_size()
    refs = _Refs()
    chain_refs = []
    entry = packed["entry"]
    written = {}  # stored model -> its reference (a model saved twice is written once)
    for c in range(len(chain_off) - 1):
        lo, hi = int(chain_off[c]), int(chain_off[c + 1])
        list_name = refs.next()
        model_refs = []
        for e in range(lo, hi):
            j = int(entry[e])
            if j in written:
                model_refs.append(written[j])
                continue
            rec_name = refs.next()
            arrays = {}
            for fld in ARRAY_FIELDS:
                key = fld[:-1]
                off = packed[key + "_off"]
                a = np.ascontiguousarray(packed[key][int(off[j]):int(off[j + 1])], dtype="<f8")
                nm = refs.next()
                _dataset(fid, nm, a)
                arrays[fld] = _ref(fid, nm)
            rec = np.zeros((), dtype=raw)
            rec["nCells_"] = packed["nCells"][j]
            rec["phi_"] = packed["phi"][j]
            rec["likelihood_"] = packed["likelihood"][j]
            rec["action_"] = packed["action"][j]
            rec["accept_"] = packed["accept"][j]
            rec["zeta_xz_"] = packed["zeta_xz"][j]
            rec["zeta_xy_"] = packed["zeta_xy"][j]
            for fld, r in arrays.items():
                rec[fld] = r
            _dataset(fid, rec_name, rec, ftype=mtid, mtype=mtid)  # raw bytes in the committed type
            written[j] = _ref(fid, rec_name)
            model_refs.append(written[j])
        arr = np.array(model_refs, dtype="<u8").reshape(hi - lo)
        did = _dataset(fid, list_name, arr, ftype=h5t.STD_REF_OBJ, mtype=h5t.STD_REF_OBJ)
        _str_attr(did, "julia eltype", "Core.Any")
        chain_refs.append(_ref(fid, list_name))
    top = np.array(chain_refs, dtype="<u8").reshape(len(chain_refs))
    did = _dataset(fid, "model", top, ftype=h5t.STD_REF_OBJ, mtype=h5t.STD_REF_OBJ)
    _str_attr(did, "julia eltype", "Core.Array{Core.Any,1}")
    f.close()
    with open(path, "r+b") as fh:  # the JLD user block
        fh.write(HEADER + b"\0" * (USERBLOCK - len(HEADER)))


# ---------------------------------------------------------------- checkpoints ----
# TD_inversion_function.jl:285 / :292 save(modelname, "model", m, "dataStruct", d, "iter", iter,
# ["saved_#", n, "model_num", k, "model_hist", hist,] "burnin", b).  Model records and the
# Vector{Any} of models follow model.jld's layout (pinned by the reference file); the rest
# (DataStruct's committed compound, StepRangeLen / TwicePrecision members, Bool) follows JLD
# 0.1.3's conventions without a reference file to pin it (no checkpoint ships).
DS_FIELDS = ["tS", "allaveatten", "allLats", "allLons", "allSig", "dataX", "dataY", "xVec", "yVec", "zVec",
             "elonsX", "elatsY", "elons", "elats", "edep", "coastX", "coastY", "rayX", "rayY", "rayZ", "rayL",
             "rayU", "U"]
DS_RANGES = ("xVec", "yVec", "zVec")
DS_MATRICES = ("elonsX", "elatsY", "elons", "elats", "edep", "coastX", "coastY", "rayX", "rayY", "rayZ", "rayL",
               "rayU", "U")


def _twice_type():
    t = h5t.create(h5t.COMPOUND, 16)
    t.insert(b"hi_", 0, h5t.IEEE_F64LE)
    t.insert(b"lo_", 8, h5t.IEEE_F64LE)
    return t


def _range_raw_dtype():
    tw = np.dtype([("hi_", "<f8"), ("lo_", "<f8")])
    return np.dtype([("ref_", tw), ("step_", tw), ("len_", "<i8"), ("offset_", "<i8")])


def write_checkpoint(path, packed, julia_version=(1, 5, 2)):
    """One chain checkpoint.  packed: jld.pack([[model], model_hist]) plus
    ck_* scalars and ds_* DataStruct arrays (see jld.save_checkpoint)."""
    f = h5py.File(path, "w", userblock_size=USERBLOCK, libver="earliest")
    fid = f.id
    for g in ("_creator", "_refs", "_types"):
        h5g.create(fid, g.encode())
    _dataset(fid, "_creator/ENDIAN_BOM", np.array(0x04030201, dtype="<u4"))
    for k, v in zip(("JULIA_MAJOR", "JULIA_MINOR", "JULIA_PATCH"), julia_version):
        _dataset(fid, "_creator/" + k, np.array(v, dtype="<u4"))
    _dataset(fid, "_creator/WORD_SIZE", np.array(64, dtype="<i8"))
    refs = _Refs()
    mtid = model_type()
    mtid.commit(fid, b"_types/00000001")
    _str_attr(mtid, "julia type", "Model")
    raw = model_raw_dtype()
    written = {}

    def model_record(j, name):
        arrays = {}
        for fld in ARRAY_FIELDS:
            key = fld[:-1]
            off = packed[key + "_off"]
            a = np.ascontiguousarray(packed[key][int(off[j]):int(off[j + 1])], dtype="<f8")
            nm = refs.next()
            _dataset(fid, nm, a)
            arrays[fld] = _ref(fid, nm)
        rec = np.zeros((), dtype=raw)
        for k in ("nCells", "phi", "likelihood", "action", "accept", "zeta_xz", "zeta_xy"):
            rec[k + "_"] = packed[k][j]
        for fld, r in arrays.items():
            rec[fld] = r
        _dataset(fid, name, rec, ftype=mtid, mtype=mtid)
        written[j] = _ref(fid, name)

    entry, co = packed["entry"], packed["chain_off"]
    model_record(int(entry[0]), "model")  # "model", CurrentModel
    # "dataStruct": committed compound; arrays by reference, ranges inline (isbits)
    tw = _twice_type()
    tw.commit(fid, b"_types/00000002")
    _str_attr(tw, "julia type", "Base.TwicePrecision{Core.Float64}")
    rr = _range_raw_dtype()
    rt = h5t.create(h5t.COMPOUND, rr.itemsize)
    rt.insert(b"ref_", 0, tw)
    rt.insert(b"step_", 16, tw)
    rt.insert(b"len_", 32, h5t.STD_I64LE)
    rt.insert(b"offset_", 40, h5t.STD_I64LE)
    rt.commit(fid, b"_types/00000003")
    _str_attr(rt, "julia type", "Base.StepRangeLen{Core.Float64,Base.TwicePrecision{Core.Float64},"
                                "Base.TwicePrecision{Core.Float64}}")
    members, off = [], 0
    for fld in DS_FIELDS:
        size = rr.itemsize if fld in DS_RANGES else 8
        members.append((fld, off, size))
        off += size
    dt = h5t.create(h5t.COMPOUND, off)
    for fld, o, _ in members:
        dt.insert((fld + "_").encode(), o, rt if fld in DS_RANGES else h5t.STD_REF_OBJ)
    dt.commit(fid, b"_types/00000004")
    _str_attr(dt, "julia type", "DataStruct")
    rec = np.zeros(off, dtype=np.uint8)
    for fld, o, size in members:
        if fld in DS_RANGES:
            first, step, n = packed["ds_" + fld + "_range"]
            r = np.zeros((), dtype=rr)
            r["ref_"]["hi_"], r["step_"]["hi_"], r["len_"], r["offset_"] = first, step, int(n), 1
            rec[o:o + size] = np.frombuffer(r.tobytes(), dtype=np.uint8)
        else:
            a = np.asarray(packed["ds_" + fld], dtype="<f8")
            if fld in DS_MATRICES:  # Julia m x n column-major == HDF5 (n, m)
                a = a.reshape(-1, 1) if a.ndim == 1 else a
                a = np.ascontiguousarray(a.T)
            nm = refs.next()
            _dataset(fid, nm, a)
            rec[o:o + 8] = np.frombuffer(np.array(_ref(fid, nm), dtype="<u8").tobytes(), dtype=np.uint8)
    space = h5s.create(h5s.SCALAR)
    dcpl = h5p.create(h5p.DATASET_CREATE)
    dcpl.set_layout(h5d.COMPACT)
    did = h5d.create(fid, b"dataStruct", dt, space, dcpl=dcpl)
    did.write(h5s.ALL, h5s.ALL, rec, mtype=dt)
    # "iter": Float64 after burn-in (the loop variable of 1:n_iter), Int64 before (:292 Int64(iter))
    if int(packed["ck_iter_int"]):
        _dataset(fid, "iter", np.array(int(packed["ck_iter"]), dtype="<i8"))
    else:
        _dataset(fid, "iter", np.array(float(packed["ck_iter"]), dtype="<f8"))
    burnin = bool(int(packed["ck_burnin"]))
    if burnin:
        _dataset(fid, "saved_#", np.array(int(packed["ck_saved"]), dtype="<i8"))
        _dataset(fid, "model_num", np.array(int(packed["ck_model_num"]), dtype="<i8"))
        model_refs = []
        for e in range(int(co[1]), int(co[2])):
            j = int(entry[e])
            if j not in written:
                model_record(j, refs.next())
            model_refs.append(written[j])
        arr = np.array(model_refs, dtype="<u8").reshape(len(model_refs))
        did = _dataset(fid, "model_hist", arr, ftype=h5t.STD_REF_OBJ, mtype=h5t.STD_REF_OBJ)
        _str_attr(did, "julia eltype", "Core.Any")
    did = _dataset(fid, "burnin", np.array(1 if burnin else 0, dtype="u1"))
    _str_attr(did, "julia type", "Core.Bool")
    f.close()
    with open(path, "r+b") as fh:
        fh.write(HEADER + b"\0" * (USERBLOCK - len(HEADER)))


def read_checkpoint(path):
    """The entries TD_inversion_function.jl:56-66 reads back, packed like
    write_checkpoint's input (model = chain 0, model_hist = chain 1)."""
    f = h5py.File(path, "r")
    mdt = model_dtype()
    mt = h5t.py_create(mdt)
    cols = {k: [] for k in ("nCells", "phi", "likelihood", "action", "accept", "zeta_xz", "zeta_xy")}
    arrays = {fld[:-1]: [] for fld in ARRAY_FIELDS}
    stored, entry = {}, []

    def take(d):
        key = h5o.get_info(d.id).addr
        if key not in stored:
            stored[key] = len(stored)
            a = np.empty((), dtype=mdt)
            d.id.read(h5s.ALL, h5s.ALL, a, mtype=mt)
            for k in cols:
                cols[k].append(a[k + "_"][()])
            for fld in ARRAY_FIELDS:
                arrays[fld[:-1]].append(np.asarray(f[a[fld][()]][()], dtype=np.float64).ravel())
        entry.append(stored[key])

    take(f["model"])
    chain_off = [0, 1]
    burnin = bool(f["burnin"][()])
    out = {}
    if burnin:
        hist = f["model_hist"]
        for j in range(hist.shape[0]):
            take(f[hist[j]])
        out["ck_saved"] = np.array(int(f["saved_#"][()]))
        out["ck_model_num"] = np.array(int(f["model_num"][()]))
    chain_off.append(len(entry))
    it = f["iter"]
    out["ck_iter"] = np.array(float(it[()]))
    out["ck_iter_int"] = np.array(1 if it.dtype.kind == "i" else 0)
    out["ck_burnin"] = np.array(1 if burnin else 0)
    out["chain_off"] = np.array(chain_off, dtype=np.int64)
    out["entry"] = np.array(entry, dtype=np.int64)
    for k, v in cols.items():
        out[k] = np.array(v, dtype=np.int64 if k in ("action", "accept") else np.float64)
    for k, v in arrays.items():
        out[k] = np.concatenate(v) if v else np.zeros(0)
        out[k + "_off"] = np.concatenate([[0], np.cumsum([len(a) for a in v])]).astype(np.int64)
    ds = f["dataStruct"]
    rr = _range_raw_dtype()
    ddt = np.dtype([(fld + "_", rr if fld in DS_RANGES else h5py.ref_dtype) for fld in DS_FIELDS])
    rec = np.empty((), dtype=ddt)
    ds.id.read(h5s.ALL, h5s.ALL, rec, mtype=h5t.py_create(ddt))
    for fld in DS_FIELDS:
        v = rec[fld + "_"][()]
        if fld in DS_RANGES:
            # Julia's StepRangeLen: r[i] = ref + (i - offset) * step in TwicePrecision (hi + lo);
            # the first element is ref + (1 - offset) * step
            ref = float(v["ref_"]["hi_"]) + float(v["ref_"]["lo_"])
            step = float(v["step_"]["hi_"]) + float(v["step_"]["lo_"])
            first = ref + (1 - int(v["offset_"])) * step
            out["ds_" + fld + "_range"] = np.array([first, step, v["len_"]], dtype=np.float64)
        else:
            a = np.asarray(f[v][()], dtype=np.float64)
            out["ds_" + fld] = np.ascontiguousarray(a.T) if fld in DS_MATRICES else a
    f.close()
    return out


def read(path):
    """The ``model`` entry of a JLD file (a vector of chains of Models), packed."""
    f = h5py.File(path, "r")
    mdt = model_dtype()
    mt = h5t.py_create(mdt)
    chain_off = [0]
    cols = {k: [] for k in ("nCells", "phi", "likelihood", "action", "accept", "zeta_xz", "zeta_xy")}
    arrays = {fld[:-1]: [] for fld in ARRAY_FIELDS}
    top = f["model"]
    entry, stored = [], {}
    for c in range(top.shape[0]):
        chain = f[top[c]]
        for j in range(chain.shape[0]):
            d = f[chain[j]]
            key = h5o.get_info(d.id).addr  # the same stored model, referenced again
            if key in stored:
                entry.append(stored[key])
                continue
            stored[key] = len(stored)
            entry.append(stored[key])
            a = np.empty((), dtype=mdt)
            d.id.read(h5s.ALL, h5s.ALL, a, mtype=mt)
            for k in cols:
                cols[k].append(a[k + "_"][()])
            for fld in ARRAY_FIELDS:
                arrays[fld[:-1]].append(np.asarray(f[a[fld][()]][()], dtype=np.float64).ravel())
        chain_off.append(chain_off[-1] + chain.shape[0])
    f.close()
    out = {"chain_off": np.array(chain_off, dtype=np.int64), "entry": np.array(entry, dtype=np.int64)}
    for k, v in cols.items():
        out[k] = np.array(v, dtype=np.int64 if k in ("action", "accept") else np.float64)
    for k, v in arrays.items():
        out[k] = np.concatenate(v) if v else np.zeros(0)
        out[k + "_off"] = np.concatenate([[0], np.cumsum([len(a) for a in v])]).astype(np.int64)
    return out


def fingerprint(path):
    """The file's structure, for comparing two JLD files: user block, every
    object (path, kind, shape, storage layout, type -- compound members with
    offsets, committed-type name), every attribute (string type and value)."""
    out = []
    with open(path, "rb") as fh:
        out.append(["userblock", fh.read(USERBLOCK).rstrip(b"\0").decode()])
    f = h5py.File(path, "r")

    def tdesc(t):
        cls = t.get_class()
        if cls == h5t.COMPOUND:
            return ["compound", t.get_size(), [[t.get_member_name(i).decode(), t.get_member_offset(i),
                                                tdesc(t.get_member_type(i))] for i in range(t.get_nmembers())]]
        if cls == h5t.STRING:
            return ["string", t.get_size(), t.get_strpad(), t.get_cset(), bool(t.is_variable_str())]
        if cls == h5t.REFERENCE:
            return ["reference", t.get_size()]
        return [int(cls), t.get_size(), int(t.get_order()) if cls in (h5t.INTEGER, h5t.FLOAT) else 0,
                int(t.get_sign()) if cls == h5t.INTEGER else -1]

    def attrs(obj):
        res = []
        for name in sorted(obj.attrs.keys()):
            aid = obj.attrs.get_id(name)
            v = obj.attrs[name]
            res.append([name, tdesc(aid.get_type()), v.decode() if isinstance(v, bytes) else repr(v)])
        return res

    def visit(name, obj):
        if isinstance(obj, h5py.Dataset):
            t = obj.id.get_type()
            committed = h5py.h5i.get_name(t).decode() if t.committed() else None
            out.append([name, "dataset", list(obj.shape), obj.id.get_create_plist().get_layout(), tdesc(t),
                        committed, attrs(obj)])
        elif isinstance(obj, h5py.Datatype):
            out.append([name, "datatype", tdesc(obj.id), attrs(obj)])
        else:
            out.append([name, "group", attrs(obj)])

    f.visititems(visit)
    out.append(["superblock", list(f.id.get_create_plist().get_version())])
    f.close()
    return out


def main(argv):
    if len(argv) == 4 and argv[1] == "write":
        with np.load(argv[2], allow_pickle=False) as z:
            write(argv[3], {k: z[k] for k in z.files})
    elif len(argv) == 4 and argv[1] == "read":
        np.savez(argv[3], **read(argv[2]))
    elif len(argv) == 4 and argv[1] == "write_checkpoint":
        with np.load(argv[2], allow_pickle=False) as z:
            write_checkpoint(argv[3], {k: z[k] for k in z.files})
    elif len(argv) == 4 and argv[1] == "read_checkpoint":
        np.savez(argv[3], **read_checkpoint(argv[2]))
    elif len(argv) == 3 and argv[1] == "fingerprint":
        import json
        print(json.dumps(fingerprint(argv[2])))
    else:
        sys.exit(__doc__)


if __name__ == "__main__":
    main(sys.argv)
