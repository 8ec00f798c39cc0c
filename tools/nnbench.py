"""Brute-force nearest search timing: the one-launch tile search (k_nn_tile)
against the split search (k_nn_partial + k_nn_merge) at config 3 and the
stress size; device time per evaluate from HIP events."""
import json
import os
import sys

sys.path.insert(0, '.')
import tonga

tt = tonga.load()
out = {}
for name, nr, nc in (("config3", None, 5000), ("stress", 10000, 20000)):
    ds = tt.load_data_Tonga() if nr is None else tt.synthetic_rays(nr, seed=5)
    ctx = tt.TdContext.from_datastruct(ds)
    tt.lib().tdt_set_incremental(ctx.h, 0)
    cells = tt.random_model(nc, 5).cells()
    variants = [(ctx.NN_BRUTE, "2", None), (ctx.NN_BRUTE, "1", None), (ctx.NN_BRUTE, "2", "1"),
                (ctx.NN_BRUTE, "1", "1"), (ctx.NN_BRUTE_SPLIT, "2", None)]
    for meth, ppl, nopad in variants:
        os.environ["TD_TILE_PPL"] = ppl
        if nopad:
            os.environ["TD_TILE_NOPAD"] = nopad
        else:
            os.environ.pop("TD_TILE_NOPAD", None)
        tag = "ppl%s%s" % (ppl, "_nopad" if nopad else "")
        ctx.set_nn_method(meth)
        for _ in range(2):
            ctx.evaluate(cells)
        ctx.timing(enable=True, reset=True)
        for _ in range(10):
            ctx.evaluate(cells)
        for k in ("nn_tile", "nn_partial", "nn_merge"):
            n, ms = ctx.timing(kernel=k)
            if n:
                out["%s/%s/%s" % (name, k, tag)] = round(ms / n * 1e3, 2)
        ctx.timing(enable=False)
    out["%s/P" % name] = ctx.P
    ctx.close()
print(json.dumps(out))
