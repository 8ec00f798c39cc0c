import sys, time, json
sys.path.insert(0, '.')
import tonga
tt = tonga.load()
out = {}
for name, nr, nc in (("config3", None, 5000), ("stress", 10000, 20000)):
    ds = tt.load_data_Tonga() if nr is None else tt.synthetic_rays(nr, seed=5)
    ctx = tt.TdContext.from_datastruct(ds)
    ctx.set_nn_method(ctx.NN_BRUTE)
    cells = tt.random_model(nc, 5).cells()
    for _ in range(2): ctx.evaluate(cells)
    ctx.timing(enable=True, reset=True)
    for _ in range(5): ctx.evaluate(cells)
    n, ms = ctx.timing(kernel="nn_partial")
    out[name] = ms / n
    ctx.close()
print(json.dumps(out))
