"""Where a short k_chain_run launch spends its cycles (diagnostic stamps)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
out = {}
for k in (1, 10):
    prm = tt.define_TDstructrure().replace(max_cells=10000)
    ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=5, chain=1), tt.random_model(5000, 3))
    if len(sys.argv) > 1:
        assert tt.lib().tdt_chain_set_lds_mode(ch.h, int(sys.argv[1])) == 0
    ch.run(50)
    buf = (ctypes.c_int64 * 80)()
    tt.lib().tdt_chain_profile(ch.h, 1, buf)
    base = list(buf)
    for _ in range(100):
        ch.run(k)
    tt.lib().tdt_chain_profile(ch.h, 0, buf)
    d = [a - b for a, b in zip(buf, base)]
    L = max(d[78], 1)
    out["k%d" % k] = {"launches": d[78], "preamble_cyc": d[76] // L, "epilogue_cyc": d[77] // L,
                      "phases_per_launch": [x // L for x in d[:14]], "pre_parts": [x // L for x in d[72:75]], "total_per_launch_cyc": (d[76] + d[77] + sum(d[:7])) // L}
    ch.close()
print(json.dumps(out))
