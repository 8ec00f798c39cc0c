#!/usr/bin/env python3
"""Batches of 256, 300 and 512 config-3 chains with the launcher's own layout choice (more chains
than CUs: two per CU), proposals/s of a 2000-proposal launch.  usage: auto_pack.py"""
import os, sys, time, json
sys.path.insert(0, os.getcwd())
import tonga
tt = tonga.load(); ds = tt.load_data_Tonga(); ctx = tt.TdContext.from_datastruct(ds)
prm = tt.define_TDstructrure().replace(max_cells=10000); model = tt.random_model(5000, 3)
out = {}
for C in (256, 300, 512):
    ch = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model) for j in range(C)]
    tt.run_batch(ch, 2000); t0 = time.perf_counter(); tt.run_batch(ch, 2000); el = time.perf_counter() - t0
    out[C] = round(C * 2000 / el / 1e6, 2); print(C, out[C], 'M/s', flush=True)
    for c in ch: c.close()
print(json.dumps(out))
