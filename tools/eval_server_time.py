"""td_evaluate's full path, resident launch vs the three launches: wall time per call from Python
(381 x 5000 cells, the bench's full_evaluate config) and the server's own device time per evaluate.
   python tools/eval_server_time.py [reps]"""
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
    out = {}
    for name, mode in (("server", 1), ("launches", 0), ("server_stamped", 2)):
        ctx = tt.TdContext.from_datastruct(ds)
        tt.lib().tdt_set_incremental(ctx.h, 0)
        tt.lib().tdt_eval_server_config(ctx.h, mode, 0, 0)
        for _ in range(20):
            ctx.evaluate(cells)
        best = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.evaluate(cells)
            best.append((time.perf_counter() - t0) / reps * 1e3)
        st = np.zeros(20, dtype=np.int64)
        tt.lib().tdt_eval_server_stats(ctx.h, st.ctypes.data)
        dt = np.zeros(18, dtype=np.int64)
        tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data)
        for _ in range(reps):
            ctx.evaluate(cells)
        tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data)
        host = {k: round(float(dt[i]) / 1e3 / reps, 3) for k, i in (("pack_cells", 12), ("issue", 13), ("wait", 14),
                                                                    ("chi2_copy_out", 15))}
        out[name] = {"evaluate_ms_min": round(min(best), 4), "evaluate_ms_runs": [round(b, 4) for b in best],
                     "host_us": host, "served": int(st[0]), "launches": int(st[1]), "failures": int(st[2]),
                     "device_us_per_evaluate": round(st[3] / 1e3 / max(st[0], 1), 3), "nwg": int(st[6]),
                     "lds_pts": int(st[7]),
                     "phase_us_from_take": {k: round(float(st[8 + j]) / 1e3 / max(st[18], 1), 3) for j, k in enumerate(
                         ("taken", "cells_loaded", "slot_returned", "fill_drained", "released", "barrier_passed",
                          "search_round1", "search_done", "sums_done", "acked"))}}
        if mode == 2:
            sd = np.zeros(6, dtype=np.int64)
            tt.lib().tdt_eval_server_search_diag(ctx.h, sd.ctypes.data)
            nw = max(int(st[18]) * int(st[6]), 1)  # workgroup-rounds stamped
            out[name]["search_round1_per_wg"] = {
                "barrier_to_loads_us": round(sd[0] / 1e3 / nw, 3), "to_reduced_us": round(sd[1] / 1e3 / nw, 3),
                "unproven_pts": round(sd[2] / nw, 3), "most_entries": round(sd[3] / nw, 3),
                "unproven_us": round(sd[4] / 1e3 / nw, 3), "zeta_rest_us": round(sd[5] / 1e3 / nw, 3)}
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
