"""Wave-skew probe (run with TD_LIB_PATH=<a skew build>): the device chain against the host engine on the
test_gpu_chain shapes, printing per launch whether the states agree and the skew build's spin-guard slot
prof[79] (nonzero: a spin wait gave up -- 1 per b_done wait, 1000 per e_done wait, 1e6 per shift_done wait)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tonga  # noqa: E402

tt = tonga.load()
ds = tt.load_data_Tonga()
ctx = tt.TdContext.from_datastruct(ds)
L = tt.lib()
cases = [(8, 12, 600, 4), (200, 300, 400, 1), (1000, 1100, 250, 2), (5000, 5100, 120, 3)]
for ncells, max_cells, iters, seed in cases[:int(os.environ.get("NCASES", "4"))]:
    prm = tt.define_TDstructrure().replace(max_cells=max_cells)
    model = tt.random_model(ncells, seed)
    dev = tt.Chain(ctx, tt.chain_params(prm, None, seed=seed, chain=1, engine=tt.TD_ENGINE_DEVICE), model)
    host = tt.Chain(ctx, tt.chain_params(prm, None, seed=seed, chain=1, engine=tt.TD_ENGINE_HOST), model)
    prof = (ctypes.c_int64 * 80)()
    L.tdt_chain_profile(dev.h, 0, prof)
    for k in range(4):
        t0 = time.time()
        dev.run(iters // 4)
        el = time.time() - t0
        host.run(iters // 4)
        L.tdt_chain_profile(dev.h, 0, prof)
        sd, sh = dev.stats(), host.stats()
        print("cells %d launch %d: %.3f s, same=%s, spin guard %d, phi %r vs %r" % (
            ncells, k, el, sd["phi"] == sh["phi"] and sd["accepted"] == sh["accepted"], prof[79], sd["phi"],
            sh["phi"]), flush=True)
        if prof[79]:  # a wait gave up: the waves' last skew sites (iteration, site), then stop (the state is broken)
            print("  gave up at iteration %d (wave %d); last sites: %s" % (prof[64] >> 8, prof[64] & 255, [
                (prof[56 + w] >> 8, prof[56 + w] & 255) for w in range(8)]), flush=True)
            sys.exit(1)
    dev.close()
    host.close()
