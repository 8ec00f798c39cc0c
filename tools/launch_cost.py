"""Per-launch cost of k_chain_run at few iterations (HIP events): the fixed
launch/preamble cost that td_evaluate's incremental path and tempering rounds pay."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
res = {}
for N in (200, 5000):
    prm = tt.define_TDstructrure().replace(max_cells=2 * N)
    ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=5, chain=1), tt.random_model(N, 3))
    ch.run(100)
    for k in (1, 2, 10, 100):
        reps = 200 if k < 100 else 50
        ctx.timing(enable=True, reset=True)
        t0 = time.perf_counter()
        for _ in range(reps):
            ch.run(k)
        el = time.perf_counter() - t0
        nl, ms = ctx.timing(kernel="chain_run")
        ctx.timing(enable=False)
        res["N%d_k%d" % (N, k)] = {"event_us": round(ms * 1e3 / nl, 2), "wall_us": round(el / reps * 1e6, 2)}
    ch.close()
print(json.dumps(res))
