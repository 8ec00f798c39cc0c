"""Print the chain's LDS plan (tdt_chain_lds) for the bench and stress configs."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
for name, ds, N in (("config3", tt.load_data_Tonga(), 5000), ("stress", tt.synthetic_rays(10000, seed=5), 20000)):
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=2 * N)
    ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1, chain=1), tt.random_model(N, 3))
    out = (ctypes.c_int64 * 4)()
    assert tt.lib().tdt_chain_lds(ch.h, out) == 0
    print(name, "lds layout bytes", out[0], "hbm layout bytes", out[1], "super in lds", out[2], "takes lds layout", out[3])
    ch.close()
    ctx.close()
