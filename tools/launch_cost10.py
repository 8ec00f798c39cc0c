"""Diagnostic: one config-4 replica (381 rays x 2000 cells) run as launches of
10 proposals (a tempering round's work on one GPU of the 8-GPU ladder): wall
time per launch, and the stamped launch preamble parts (mirrors, chi^2 terms,
draws + first proposal) and epilogue."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
prm = tt.define_TDstructrure().replace(max_cells=4000)
ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=100, chain=1), tt.random_model(2000, 4))
ch.run(100)
L = tt.lib()
for prof in (0, 1):
    o0 = (ctypes.c_int64 * 80)()
    L.tdt_chain_profile(ch.h, prof, o0)  # stamps off (wall time) / on (where the cycles go)
    n = 300
    t0 = time.perf_counter()
    for _ in range(n):
        ch.run(10)
    el = (time.perf_counter() - t0) / n
    o = (ctypes.c_int64 * 80)()
    L.tdt_chain_profile(ch.h, prof, o)
    d = [o[k] - o0[k] for k in range(80)]
    launches = max(d[78], 1)
    print(json.dumps({"stamped": prof == 1, "us_per_launch_wall": round(el * 1e6, 1),
                      "preamble_cycles": round(d[76] / launches, 1), "mirrors": round(d[72] / launches, 1),
                      "terms_init": round(d[73] / launches, 1), "draws_first_proposal": round(d[74] / launches, 1),
                      "epilogue_cycles": round(d[77] / launches, 1),
                      "loop_cycles_per_iter": round(sum(d[:7]) / max(10 * launches, 1), 1)}))
