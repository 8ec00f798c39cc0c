"""Brute-force nearest timing against the cell count at the config-3 point set
(16,845 points): the slope of time(N) is the per-distance cost, the intercept
the fixed cost of a launch.  FLOP/s counts 8 per distance (no FMA)."""
import json
import os
import sys

sys.path.insert(0, '.')
import tonga

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
tt.lib().tdt_set_incremental(ctx.h, 0)
out = {}
for nc in (500, 1000, 2500, 5000, 10000, 20000, 40000):
    cells = tt.random_model(nc, 5).cells()
    for meth, kname in ((ctx.NN_BRUTE, "nn_tile"), (ctx.NN_BRUTE_SPLIT, "nn_partial")):
        ctx.set_nn_method(meth)
        for _ in range(2):
            ctx.evaluate(cells)
        ctx.timing(enable=True, reset=True)
        for _ in range(10):
            ctx.evaluate(cells)
        n, ms = ctx.timing(kernel=kname)
        us = ms / max(n, 1) * 1e3
        out["%s/%d" % (kname, nc)] = (round(us, 2), round(8.0 * ctx.P * nc / (us * 1e-6) / 1e12, 2))
        ctx.timing(enable=False)
print(json.dumps(out))
