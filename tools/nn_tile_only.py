"""Diagnostic: the tile nearest search alone at the config-3 point set x N
cells (tdt_nn_bench, method 1), for counter passes (rocprofv3 --pmc)."""
import ctypes
import sys

sys.path.insert(0, '.')
import numpy as np
import tonga

tt = tonga.load()
lib = tt.lib()
ctx = tt.TdContext.from_datastruct(tt.load_data_Tonga())
nc = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
pd = ctypes.POINTER(ctypes.c_double)
cells = [np.ascontiguousarray(a) for a in tt.random_model(nc, 5).cells()]
us = ctypes.c_double(0)
assert lib.tdt_nn_bench(ctx.h, *[a.ctypes.data_as(pd) for a in cells], nc, 1, reps, ctypes.byref(us)) == 0
print("tile %d cells: %.2f us, %.2f TFLOP/s (8 per distance)" % (nc, us.value, 8.0 * ctx.P * nc / (us.value * 1e-6) / 1e12))
