"""Diagnostic: phase stamps of the drop-in server's scripted proposals (TD_SHADOW_PROFILE=1), per
td_evaluate, from a DROPIN chain of `iters` proposals at 381 rays x N cells.  usage: shadow_phases.py [iters]"""
import ctypes
import json
import os
import sys

os.environ["TD_SHADOW_PROFILE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

PH = ["top", "B", "C", "D", "E", "F", "G12", "G13", "G"]
tt = tonga.load()
ds = tt.load_data_Tonga()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
model = tt.random_model(5000, 3)
prm = tt.define_TDstructrure().replace(max_cells=10000)
ctx = tt.TdContext.from_datastruct(ds)
ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000, chain=1, engine=tt.TD_ENGINE_DROPIN), model)
ch.run(iters)
out = (ctypes.c_int64 * 80)()
assert tt.lib().tdt_shadow_profile(ctx.h, out) == 0
o = list(out)
n_eval = ch.stats()["evaluations"]
cyc = [o[k] for k in range(7)]
cyc[6] += o[12] + o[13]
res = {"evaluates": n_eval, "cycles_per_evaluate": round(sum(cyc) / max(n_eval, 1), 1),
       "phases": {p: round(c / max(n_eval, 1), 1) for p, c in zip(["top", "B", "C", "D", "E", "F", "G"], cyc)},
       "by_action": {}}
for a, name in enumerate(("birth", "death", "change", "move")):
    row = o[16 + 10 * a: 16 + 10 * a + 9]
    tot = o[8 + a]
    res["by_action"][name] = {p: v for p, v in zip(PH, row)}
    res["by_action"][name]["total"] = tot
print(json.dumps(res, indent=1))
ch.close()
ctx.close()
