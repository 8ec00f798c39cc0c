"""td_evaluate's full path as one resident launch (csrc/eval_server.h,
k_eval_server in nn_grid.hip) against the C oracle and the three launches it
replaces (fill, grid search, ray sums): ptS and phi bit for bit
(MCsub.jl:123-185), over cell sets whose size, box and bucket grid change
from call to call, across the launch's idle exit and relaunch, around other
work that stops it, and when its grid barrier fails (the launches answer)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def stats(tt, ctx):
    out = np.zeros(20, dtype=np.int64)
    assert tt.lib().tdt_eval_server_stats(ctx.h, out.ctypes.data) == 0
    return dict(zip(("served", "launches", "failures", "busy_ns", "running", "disabled", "nwg", "lds_pts"),
                    (int(v) for v in out[:8])))


def full_ctx(tt, ds, mode=1, idle_us=0, guard_us=0):
    ctx = tt.TdContext.from_datastruct(ds)
    assert tt.lib().tdt_set_incremental(ctx.h, 0) == 0  # every td_evaluate a full one
    assert tt.lib().tdt_eval_server_config(ctx.h, mode, idle_us, guard_us) == 0
    return ctx


def oracle(orc, ds, cells):
    ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, cells, 0)
    assert ref["rc"] == 0
    return ref


def model_sequence(tt, ds):
    """Cell sets of changing size and extent: the grid's shape, the staged stride and the bucket
    sets' zeroing all change between consecutive calls."""
    seq = []
    for n, seed in ((256, 1), (5000, 2), (300, 3), (8000, 4), (1000, 5), (5000, 6), (2500, 7)):
        seq.append(tt.random_model(n, seed).cells())
    # duplicates later in the list with other values (ties: the first index wins)
    x, y, z, ze = (np.asarray(a, dtype=np.float64) for a in tt.random_model(600, 8).cells())
    x, y, z = (np.concatenate([a, a[::2]]) for a in (x, y, z))
    ze = np.concatenate([ze, ze[::2] + 1.0])
    seq.append((x, y, z, ze))
    # cells on the ray points and a few far outside everything (a sealed box far larger than the rays)
    px, py, pz = (a[~np.isnan(a)] for a in (ds.rayX, ds.rayY, ds.rayZ))
    sel = np.arange(0, len(px), 41)
    x = np.concatenate([px[sel], [1e4, -1e4]])
    y = np.concatenate([py[sel], [0.0, 5e3]])
    z = np.concatenate([pz[sel], [3e3, -2e3]])
    seq.append((x, y, z, np.arange(len(x), dtype=np.float64) % 17))
    return seq


def test_server_equals_oracle_and_launches(tt, orc, ds):
    seq = model_sequence(tt, ds)
    srv = full_ctx(tt, ds)
    got = [srv.evaluate(c)[:2] for c in seq]
    st = stats(tt, srv)
    # one launch, plus one per growth of the cell buffers (the resident launch is stopped before they move)
    assert st["served"] == len(seq) and st["launches"] <= 3 and st["failures"] == 0, st
    assert st["running"] == 1 and st["nwg"] >= 1
    srv.close()
    lau = full_ctx(tt, ds, mode=0)
    for c, (ptS, phi) in zip(seq, got):
        ptS_l, phi_l, _, _ = lau.evaluate(c)
        assert np.array_equal(ptS, ptS_l) and phi == phi_l
    assert stats(tt, lau)["served"] == 0
    lau.close()
    for c, (ptS, phi) in zip(seq, got):
        ref = oracle(orc, ds, c)
        assert np.array_equal(ptS, ref["ptS"]), np.max(np.abs(ptS - ref["ptS"]))
        assert phi == ref["phi"]


def test_server_repeats_and_alternating_models(tt, orc, ds):
    """The same two models alternately, many times: each answer is the first one's (the bucket
    counts of one evaluate are zeroed by the next: a stale count would change an answer)."""
    a, b = tt.random_model(5000, 21).cells(), tt.random_model(3000, 22).cells()
    ra, rb = oracle(orc, ds, a), oracle(orc, ds, b)
    srv = full_ctx(tt, ds)
    for k in range(40):
        c, r = (a, ra) if k % 2 == 0 else (b, rb)
        ptS, phi, _, _ = srv.evaluate(c)
        assert np.array_equal(ptS, r["ptS"]) and phi == r["phi"], k
    st = stats(tt, srv)
    assert st["served"] == 40 and st["launches"] == 1, st
    srv.close()


def test_server_idle_exit_and_relaunch(tt, orc, ds):
    srv = full_ctx(tt, ds, idle_us=2000)  # a 2 ms watchdog
    c1, c2 = tt.random_model(4000, 31).cells(), tt.random_model(4500, 32).cells()
    ptS1, phi1, _, _ = srv.evaluate(c1)
    time.sleep(0.05)  # the launch quits on its own meanwhile
    ptS2, phi2, _, _ = srv.evaluate(c2)  # posted to the quit launch: relaunched, then taken
    st = stats(tt, srv)
    assert st["served"] == 2 and st["launches"] == 2 and st["failures"] == 0, st
    srv.close()
    for c, ptS, phi in ((c1, ptS1, phi1), (c2, ptS2, phi2)):
        ref = oracle(orc, ds, c)
        assert np.array_equal(ptS, ref["ptS"]) and phi == ref["phi"]


def test_server_stopped_by_other_work(tt, orc, ds):
    """An Interpolation (its own launches) and a nearest-index evaluate stop the resident launch
    first; the next full evaluate relaunches it."""
    srv = full_ctx(tt, ds)
    c1, c2 = tt.random_model(2000, 41).cells(), tt.random_model(2200, 42).cells()
    ptS1, phi1, _, _ = srv.evaluate(c1)
    assert stats(tt, srv)["running"] == 1
    vals, _ = srv.interpolate(c1, ds.rayX[:3, 0], ds.rayY[:3, 0], ds.rayZ[:3, 0])
    assert stats(tt, srv)["running"] == 0
    ptS_n, phi_n, _, near = srv.evaluate(c2, want_nearest=True)  # the launches (nearest indices)
    ptS2, phi2, _, _ = srv.evaluate(c2)
    st = stats(tt, srv)
    assert st["served"] == 2 and st["launches"] == 2, st
    srv.close()
    r1, r2 = oracle(orc, ds, c1), oracle(orc, ds, c2)
    assert np.array_equal(ptS1, r1["ptS"]) and phi1 == r1["phi"]
    assert np.array_equal(ptS2, r2["ptS"]) and phi2 == r2["phi"]
    assert np.array_equal(ptS_n, r2["ptS"]) and phi_n == r2["phi"] and np.array_equal(near, r2["nearest"])
    zr, _ = orc.interpolation(c1, ds.rayX[:3, 0], ds.rayY[:3, 0], ds.rayZ[:3, 0])
    assert np.array_equal(vals, zr)


def test_server_small_models_take_the_brute_force(tt, orc, ds):
    srv = full_ctx(tt, ds)
    c = tt.random_model(100, 51).cells()  # below the grid's 256 cells
    ptS, phi, _, _ = srv.evaluate(c)
    assert stats(tt, srv)["served"] == 0
    srv.close()
    ref = oracle(orc, ds, c)
    assert np.array_equal(ptS, ref["ptS"]) and phi == ref["phi"]


def test_server_failed_barrier_falls_back(tt, orc, ds):
    """A 1 us grid-barrier guard: some workgroup gives up waiting (done = -seq), the context turns the
    server off and the launches answer -- the same bits either way."""
    srv = full_ctx(tt, ds, idle_us=2000, guard_us=1)
    cs = [tt.random_model(5000, 61).cells(), tt.random_model(5000, 62).cells()]
    got = [srv.evaluate(c)[:2] for c in cs]
    st = stats(tt, srv)
    assert st["failures"] + st["served"] >= 1, st
    assert st["failures"] == 0 or (st["disabled"] == 1 and st["running"] == 0), st
    srv.close()
    for c, (ptS, phi) in zip(cs, got):
        ref = oracle(orc, ds, c)
        assert np.array_equal(ptS, ref["ptS"]) and phi == ref["phi"]
