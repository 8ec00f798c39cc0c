"""Diagnostic: 200 td_evaluate calls at config 3 (381 rays x 5000 cells), for a
rocprofv3 timeline of one evaluation (kernels, copies, gaps)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
cells = tt.random_model(5000, 3).cells()
for _ in range(20):
    ctx.evaluate(cells)
t0 = time.perf_counter()
for _ in range(200):
    ctx.evaluate(cells)
print("evaluate_us", (time.perf_counter() - t0) / 200 * 1e6)
