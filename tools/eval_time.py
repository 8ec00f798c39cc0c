"""td_evaluate's full path (381 rays x 5000 cells, the bench's full_evaluate config): wall time per call
from Python, the host-side breakdown (tdt_dropin_timing slots 12-15) and the kernels (HIP events).
   python tools/eval_time.py [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import tonga  # noqa: E402

tt = tonga.load()


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    ds = tt.load_data_Tonga()
    cells = tt.random_model(5000, 3).cells()
    ctx = tt.TdContext.from_datastruct(ds)
    tt.lib().tdt_set_incremental(ctx.h, 0)
    for _ in range(50):
        ctx.evaluate(cells)
    runs = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.evaluate(cells)
        runs.append((time.perf_counter() - t0) / reps * 1e3)
    dt = np.zeros(18, dtype=np.int64)
    tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data)
    for _ in range(reps):
        ctx.evaluate(cells)
    tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data)
    host = {k: round(float(dt[i]) / 1e3 / reps, 3) for k, i in (("pack_cells", 12), ("issue", 13), ("wait", 14),
                                                                ("chi2_copy_out", 15))}
    ctx.timing(enable=True, reset=True)
    for _ in range(reps):
        ctx.evaluate(cells)
    km = {}
    for k in ("nn_grid_build", "nn_grid", "ray_sums"):
        nl, ms = ctx.timing(kernel=k)
        if nl:
            km[k] = round(ms / nl * 1e3, 3)
    ctx.timing(enable=False)
    print(json.dumps({"evaluate_ms_min": round(min(runs), 4), "runs": [round(r, 4) for r in runs], "host_us": host,
                      "kernel_us": km}))
    ctx.close()


if __name__ == "__main__":
    main()
