"""Run only bench.dropin (for rocprofv3 traces of td_evaluate's incremental path)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
print(json.dumps(bench.dropin(tt, ds, tt.random_model(N, 3), iters=1000, host_iters=100)))
