"""Diagnostic: one nearest-cell search method alone (tdt_nn_bench) at the
config-3 rays x 5000 cells, or the stress rays (10k synthetic) x 20000 cells,
for counter passes (rocprofv3 --pmc).  usage: nn_grid_only.py [stress] [method]"""
import ctypes
import sys

sys.path.insert(0, '.')
import numpy as np
import tonga

tt = tonga.load()
lib = tt.lib()
stress = len(sys.argv) > 1 and sys.argv[1] == "stress"
meth = int(sys.argv[2]) if len(sys.argv) > 2 else 2  # 1 tile, 2 grid, 3 split
ds = tt.synthetic_rays(10000, seed=5) if stress else tt.load_data_Tonga()
nc = 20000 if stress else 5000
ctx = tt.TdContext.from_datastruct(ds)
pd = ctypes.POINTER(ctypes.c_double)
cells = [np.ascontiguousarray(a) for a in tt.random_model(nc, 5).cells()]
us = ctypes.c_double(0)
assert lib.tdt_nn_bench(ctx.h, *[a.ctypes.data_as(pd) for a in cells], nc, meth, 50, ctypes.byref(us)) == 0
print("method %d, P=%d x %d cells: %.2f us per search" % (meth, ctx.P, nc, us.value))
