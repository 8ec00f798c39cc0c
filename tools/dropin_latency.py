"""Latency of td_evaluate's incremental path per call (Python ctypes loop;
the chain-shaped edit sequence of tests/test_gpu_incremental.py) and of a
one-point query answered by the resident server."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_incremental import edit  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
out = {}
for mode in (2, 1, 0):
    ctx = tt.TdContext.from_datastruct(ds)
    tt.lib().tdt_set_incremental(ctx.h, mode)
    rng = np.random.default_rng(1)
    cur = tt.random_model(5000, 3).cells()
    ctx.evaluate(cur)
    props = []
    c = cur
    for _ in range(400):
        p = edit(rng, c, tt.box())
        props.append(p)
        if rng.random() < 0.55:
            c = p
    # replay: evaluate each proposal (the host accepted the same ones)
    t_eval = []
    c = cur
    rng = np.random.default_rng(1)
    for p in props:
        t0 = time.perf_counter()
        ctx.evaluate(p)
        t_eval.append(time.perf_counter() - t0)
    import ctypes
    dg = (ctypes.c_int64 * 4)()
    tt.lib().tdt_shadow_diag(ctx.h, dg)
    if mode == 2 and os.environ.get("TD_SHADOW_PROFILE"):
        pr = (ctypes.c_int64 * 80)()
        tt.lib().tdt_shadow_profile(ctx.h, pr)
        L = max(len(props), 1)
        out["server_phases_cyc_per_eval"] = [pr[k] // L for k in range(14)]
        out["server_preamble_cyc"] = pr[76]
    t_q = []
    for _ in range(300):
        t0 = time.perf_counter()
        ctx.interpolate(props[-1], [100.0], [50.0], [200.0])
        t_q.append(time.perf_counter() - t0)
    t_noop = []
    for _ in range(300):
        t0 = time.perf_counter()
        ctx.evaluate(props[-1])  # the same model again: cached, pure host + ctypes cost
        t_noop.append(time.perf_counter() - t0)
    out["mode%d" % mode] = {"evaluate_us_median": round(np.median(t_eval[50:]) * 1e6, 2),
                            "query_us_median": round(np.median(t_q) * 1e6, 2),
                            "cached_repeat_us_median": round(np.median(t_noop) * 1e6, 2),
                            "last_eval_busy_us": dg[1] / 100.0, "clock_mhz": round(dg[0] / max(dg[1], 1) * 100, 1),
                            "polls": dg[2]}
    ctx.close()
print(json.dumps(out))
