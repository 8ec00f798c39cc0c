"""Diagnostic: cycles per nearest-cell query through the device chain's bucket grid (one wave, back to
back; tdt_chain_query_lat) at 381 rays x 5000 cells -- the whole query, its loads alone, its arithmetic
alone -- for ray points (phase D's orphans) and points drawn in the prior box (phase B's births)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
prm = tt.define_TDstructrure().replace(max_cells=10000)
ctx = tt.TdContext.from_datastruct(ds)
model = tt.random_model(5000, 3)
ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=7, chain=1), model)
ch.run(1000)
rng = np.random.default_rng(3)
X, Y, Z = (np.asarray(a, dtype=np.float64).ravel() for a in (ds.rayX, ds.rayY, ds.rayZ))
ok = ~np.isnan(X)
X, Y, Z = X[ok], Y[ok], Z[ok]
nq = 2000
sel = rng.integers(0, len(X), nq)
ray_pts = np.stack([X[sel], Y[sel], Z[sel]], 1)
lo, hi = np.array([X.min(), Y.min(), Z.min()]), np.array([X.max(), Y.max(), Z.max()])  # (about the prior box)
box_pts = lo + (hi - lo) * rng.random((nq, 3))
L = tt.lib()
res = {}
print("chain ready", flush=True, file=sys.stderr)
for name, pts in (("ray points", ray_pts), ("prior box", box_pts)):
    p = np.ascontiguousarray(pts, dtype=np.float64)
    row = {}
    for mode, mname in ((0, "query"), (1, "loads only"), (2, "math only"), (3, "bucket indices"), (4, "face bound"),
                        (5, "wave min u64"), (6, "query, descriptor fields")):
        out = (ctypes.c_int64 * 4)()
        for _ in range(2):  # (the second run: warm caches)
            assert L.tdt_chain_query_lat(ch.h, p.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), nq, mode, out) == 0
        row[mname] = round(out[0] / nq, 1)
        print(name, mname, row[mname], flush=True, file=sys.stderr)
        if mode in (0, 6):
            row["unproven" + ("" if mode == 0 else " (6)")] = int(out[1])
            row["digest" + ("" if mode == 0 else " (6)")] = int(out[3])
    res[name] = row
print(json.dumps(res, indent=1))
ch.close()
ctx.close()
