import ctypes, json, os, sys, time
import numpy as np
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
import tonga
tt = tonga.load()
ds = tt.synthetic_rays(10000, seed=5)
ctx = tt.TdContext.from_datastruct(ds)
prm = tt.define_TDstructrure().replace(max_cells=40000)
ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=77, chain=1), tt.random_model(20000, 5))
ch.run(200)
L = tt.lib()
a, b = (ctypes.c_int64 * 80)(), (ctypes.c_int64 * 80)()
p0 = np.array(ch.stats()["proposed"], dtype=float)
L.tdt_chain_profile(ch.h, 1, a)
t0 = time.perf_counter(); ch.run(2000); el = time.perf_counter() - t0
L.tdt_chain_profile(ch.h, 0, b)
d = np.array(b[:], dtype=float) - np.array(a[:], dtype=float)
prop = np.array(ch.stats()["proposed"], dtype=float) - p0
n = 2000
cyc = d[:7].copy(); cyc[6] += d[12] + d[13]
names = ["top", "B", "C", "D", "E", "F", "G"]
out = {"us_per_prop": el / n * 1e6, "cycles": {k: round(v / n, 1) for k, v in zip(names, cyc)}, "total": round(cyc.sum() / n, 1),
       "by_action": {nm: {"share": round(prop[i] / max(prop.sum(), 1), 3), **{p: round(x, 1) for p, x in zip(("top", "B", "C", "D", "E", "F", "G12", "G13", "G"), d[16 + 10 * i: 16 + 10 * i + 9] / max(prop[i], 1))}} for i, nm in enumerate(("birth", "death", "change", "move"))},
       "diag": {k: round(d[k] / n, 3) for k in (14, 15, 64, 65, 66, 67, 68, 69, 70, 71)}}
print(json.dumps(out, indent=1))
