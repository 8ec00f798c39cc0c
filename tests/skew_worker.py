"""Child process of tests/test_gpu_skew.py: run with TD_LIB_PATH = the wave-skew build
(mcmc-in-tonga_amd/libtdstar_skew.so, chain_kernels.hip SKEW).  The device chain against the host
engine on test_gpu_chain's shapes (the 8-cell model at max_cells 12 first: inactive proposals every few
iterations), printing one JSON line per launch: equal or not, and the skew build's spin-guard slot
(nonzero: a spin wait gave up).  Stops at the first mismatch or guard trip (the state is then broken)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
L = tt.lib()
for ncells, max_cells, iters, seed in [(8, 12, 600, 4), (200, 300, 400, 1), (1000, 1100, 250, 2),
                                       (5000, 5100, 120, 3)]:
    prm = tt.define_TDstructrure().replace(max_cells=max_cells)
    model = tt.random_model(ncells, seed)
    dev = tt.Chain(ctx, tt.chain_params(prm, None, seed=seed, chain=1, engine=tt.TD_ENGINE_DEVICE), model)
    host = tt.Chain(ctx, tt.chain_params(prm, None, seed=seed, chain=1, engine=tt.TD_ENGINE_HOST), model)
    prof = (ctypes.c_int64 * 80)()
    for k in range(4):
        dev.run(iters // 4)
        host.run(iters // 4)
        L.tdt_chain_profile(dev.h, 0, prof)
        sd, sh = dev.stats(), host.stats()
        same = sd["phi"] == sh["phi"] and sd["accepted"] == sh["accepted"] and sd["ncells"] == sh["ncells"]
        print(json.dumps({"cells": ncells, "launch": k, "same": same, "guard": int(prof[79]),
                          "sites": [int(prof[56 + w]) for w in range(8)] if prof[79] else None}), flush=True)
        if not same or prof[79]:
            sys.exit(1)
    dev.close()
    host.close()
