#!/usr/bin/env python3
"""Two chains per CU: config-3 chains packed one per CU in the
8-wave LDS layout (the bench's many_chains) against two per CU in the 4-wave
rays-in-HBM kernel (lds_mode 2), and one per CU of the 8-wave HBM layout
(lds_mode 1).  Launches of `iters` proposals, timed after a warm-up launch.
usage: packed_chains.py [iters]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=10000)
    model = tt.random_model(5000, 3)
    out = {}
    for name, C, mode in (("lds_1perCU", 256, 0), ("hbm_1perCU", 256, 1), ("tiles4w_1perCU", 256, 2),
                          ("tiles4w_2perCU", 512, 2), ("hbm4w_2perCU", 512, 3)):
        chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model) for j in range(C)]
        for c in chains:
            assert tt.lib().tdt_chain_set_lds_mode(c.h, mode) == 0
        tt.run_batch(chains, iters)
        t0 = time.perf_counter()
        tt.run_batch(chains, iters)
        el = time.perf_counter() - t0
        out[name] = {"chains": C, "lds_mode": mode, "proposals_per_s": round(C * iters / el, 1),
                     "ms_per_launch": round(el * 1e3, 3)}
        print(name, out[name], flush=True)
        for c in chains:
            c.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
