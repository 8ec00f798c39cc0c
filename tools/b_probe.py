"""Phase B's inside (run with TD_LIB_PATH = a -DTD_B_PROBE build): tid 0's cycles from phase B's start to
the end of its tile pass, to its preload issued, and to its count / the barrier, per proposal, beside the
stamped B and the whole proposal (the headline config, 5000 proposals)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
prm = tt.define_TDstructrure().replace(max_cells=10000)
ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000, chain=1), tt.random_model(5000, 3))
ch.run(5000)
L = tt.lib()
a, b = (ctypes.c_int64 * 80)(), (ctypes.c_int64 * 80)()
L.tdt_chain_profile(ch.h, 1, a)
ch.run(5000)
L.tdt_chain_profile(ch.h, 0, b)
d = [b[k] - a[k] for k in range(80)]
n = 5000.0
print(json.dumps({"B_stamped": d[1] / n, "to_tile_pass_end": d[72] / n, "to_preload_issued": d[73] / n,
                  "to_count_or_barrier": d[74] / n, "total": sum(d[:7]) / n + (d[12] + d[13]) / n}))
