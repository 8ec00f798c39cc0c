"""The nearest-cell search alone (tdt_nn_bench: back-to-back launches between
two HIP events) at the config-3 point set, over cell counts: the tile search,
the split search and the bucket grid.  TFLOP/s counts 8 per distance."""
import ctypes
import json
import sys

sys.path.insert(0, '.')
import numpy as np
import tonga

tt = tonga.load()
lib = tt.lib()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
P = ctx.P
pd = ctypes.POINTER(ctypes.c_double)
out = {}
variants = [("split", 3, {}), ("grid", 2, {}), ("tile", 1, {})]
for nc in (1000, 5000, 20000):
    cells = [np.ascontiguousarray(a) for a in tt.random_model(nc, 5).cells()]
    ptrs = [a.ctypes.data_as(pd) for a in cells]
    for name, meth, env in variants:
        us = ctypes.c_double(0)
        rc = lib.tdt_nn_bench(ctx.h, *ptrs, nc, meth, 20, ctypes.byref(us))
        assert rc == 0, rc
        out["%d/%s" % (nc, name)] = (round(us.value, 2), round(8.0 * P * nc / (us.value * 1e-6) / 1e12, 2))
print(json.dumps(out))
