"""k_nn_tile alone (tdt_nn_bench, back-to-back launches) at the config-3 point set for 200 / 1000 / 5000 /
20000 cells.  (profiles/r05/nn_tile/ holds the sweep over 2 / 3 / 4 points per lane taken with a TD_NN_PPL
knob of the library, removed after it: 2 per lane stays.)"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
lib = tt.lib()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
P = ctx.P
pd = ctypes.POINTER(ctypes.c_double)
out = {"ppl": os.environ.get("TD_NN_PPL", "2")}
import numpy as np  # noqa: E402
for nc in (200, 1000, 5000, 20000):
    cells = [np.ascontiguousarray(a) for a in tt.random_model(nc, 5).cells()]
    ptrs = [a.ctypes.data_as(pd) for a in cells]
    us = ctypes.c_double(0)
    assert lib.tdt_nn_bench(ctx.h, *ptrs, nc, 1, 50, ctypes.byref(us)) == 0
    out[nc] = {"us": round(us.value, 2), "tflops": round(8.0 * P * nc / (us.value * 1e-6) / 1e12, 2),
               "frac_no_fma": round(8.0 * P * nc / (us.value * 1e-6) / 39.3e12, 3)}
print(json.dumps(out))
