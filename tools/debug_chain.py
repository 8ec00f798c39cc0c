"""Step the device and host engines one iteration at a time; print the first divergence."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
ncells, max_cells, seed = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (200, 300, 1)))
prm = tt.define_TDstructrure().replace(max_cells=max_cells)
model = tt.random_model(ncells, seed)
mk = lambda e: tt.Chain(ctx, tt.chain_params(prm, None, seed=seed, chain=1, temperature=1.0, engine=e), model)  # noqa
dev, host = mk(tt.TD_ENGINE_DEVICE), mk(tt.TD_ENGINE_HOST)
prev = None
for it in range(400):
    dev.run(1)
    host.run(1)
    sd, sh = dev.stats(), host.stats()
    if sd["phi"] != sh["phi"] or sd["accepted"] != sh["accepted"] or sd["proposed"] != sh["proposed"]:
        print("diverged at iteration", it)
        print("prev", prev)
        print("dev ", sd)
        print("host", sh)
        break
    prev = sd
else:
    print("no divergence in 400 iterations")
