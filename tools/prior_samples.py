"""Dump device-chain prior samples (debug_prior = 1) for offline comparison
with oracle/chain_np.py.  usage: prior_samples.py PRIOR K ITERS SEED OUT.npz"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
prior, K, iters, seed, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
ds = tt.synthetic_rays(4, seed=1)
ctx = tt.TdContext.from_datastruct(ds)
prm = tt.define_TDstructrure().replace(debug_prior=1, prior=prior)
res = {}
for tag, engine in (("dev", tt.TD_ENGINE_DEVICE), ("host", tt.TD_ENGINE_HOST)):
    kk = K if engine == tt.TD_ENGINE_DEVICE else min(K, 256)
    chains = [tt.Chain(ctx, tt.chain_params(prm, None, seed=seed, chain=1 + k, engine=engine)) for k in range(kk)]
    tt.run_batch(chains, iters)
    ms = [c.model() for c in chains]
    for c in chains:
        c.close()
    res[tag + "_n"] = np.array([len(m.xCell) for m in ms])
    res[tag + "_zeta"] = np.concatenate([m.zeta for m in ms])
    res[tag + "_x"] = np.concatenate([m.xCell for m in ms])
    res[tag + "_y"] = np.concatenate([m.yCell for m in ms])
    res[tag + "_z"] = np.concatenate([m.zCell for m in ms])
np.savez(out, **res)
print("ok", {k: v.shape for k, v in res.items()})
