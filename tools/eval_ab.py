"""bench.full_evaluate alone (config 3: 381 rays x 5000 cells), for same-box
A/B runs of td_evaluate variants (e.g. TD_FUSE_RAYS=0 / 1).
usage: python tools/eval_ab.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
out = bench.full_evaluate(tt, ctx, tt.random_model(5000, 3), 5000, reps=reps)
print(json.dumps({"fuse": os.environ.get("TD_FUSE_RAYS", "1"),
                  **{k: (v["evaluate_ms"], v["kernel_ms"], v["host_us"]) for k, v in out.items()}}))
