"""td_evaluate's incremental path (csrc/incremental.cpp): an unchanged host
that calls evaluate on modeln = model + one edit (TD_inversion_function.jl:
85-88 birth, 132-135 death, 189 change, 234-236 move) gets results bit for
bit equal to the full evaluate, while the context follows the chain on the
device.

* the DROPIN engine (the host loop calling the public td_evaluate /
  td_interpolate, as Julia would) makes exactly the HOST engine's moves (which
  evaluates every proposal in full) and the DEVICE engine's;
* scripted sequences of edits on the last model or the one before it, repeats,
  unrelated models, ties and far-away cells, each checked against a context
  with the incremental path off.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(tt, ds):
    c = tt.TdContext.from_datastruct(ds)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ref_ctx(tt, ds):
    c = tt.TdContext.from_datastruct(ds)
    assert tt.lib().tdt_set_incremental(c.h, 0) == 0
    yield c
    c.close()


def same_models(a, b):
    return (len(a.xCell) == len(b.xCell) and np.array_equal(a.xCell, b.xCell) and np.array_equal(a.yCell, b.yCell)
            and np.array_equal(a.zCell, b.zCell) and np.array_equal(a.zeta, b.zeta))


@pytest.mark.parametrize("ncells,iters,seed,prior", [(200, 400, 1, 1), (1000, 300, 2, 1), (5000, 200, 3, 1),
                                                     (300, 300, 4, 2), (12, 400, 5, 1)])
def test_dropin_engine_follows_host_and_device(tt, ds, ncells, iters, seed, prior):
    ctxs = [tt.TdContext.from_datastruct(ds) for _ in range(3)]
    prm = tt.define_TDstructrure().replace(max_cells=ncells + 300, prior=prior)
    model = tt.random_model(ncells, seed)
    engines = (tt.TD_ENGINE_DROPIN, tt.TD_ENGINE_HOST, tt.TD_ENGINE_DEVICE)
    chains = [tt.Chain(c, tt.chain_params(prm, None, seed=seed, chain=1, engine=e), model)
              for c, e in zip(ctxs, engines)]
    for _ in range(4):
        for ch in chains:
            ch.run(iters // 4)
        st = [ch.stats() for ch in chains]
        assert st[0]["phi"] == st[1]["phi"] == st[2]["phi"], st
        assert st[0]["accepted"] == st[1]["accepted"] == st[2]["accepted"]
    ms = [ch.model() for ch in chains]
    assert same_models(ms[0], ms[1]) and same_models(ms[0], ms[2])
    assert np.array_equal(ms[0].ptS, ms[1].ptS)
    assert sum(st[0]["accepted"]) > 0
    for ch in chains:
        ch.close()
    for c in ctxs:
        c.close()


def edit(rng, cells, box):
    x, y, z, ze = (a.copy() for a in cells)
    n = len(x)
    a = int(rng.integers(1, 5)) if n > 2 else 1
    if a == 1:
        p = [rng.uniform(box[0], box[1]), rng.uniform(box[2], box[3]), rng.uniform(box[4], box[5])]
        return (np.append(x, p[0]), np.append(y, p[1]), np.append(z, p[2]), np.append(ze, rng.uniform(0, 50)))
    k = int(rng.integers(n))
    if a == 2:
        return tuple(np.delete(v, k) for v in (x, y, z, ze))
    if a == 3:
        ze[k] = rng.uniform(0, 50)
    else:
        x[k] += rng.normal(0, 100)
        y[k] += rng.normal(0, 60)
        z[k] += rng.normal(0, 60)
    return x, y, z, ze


def check(ctx, ref_ctx, cells):
    a = ctx.evaluate(cells)
    b = ref_ctx.evaluate(cells)
    assert a[1] == b[1] and np.array_equal(a[0], b[0]) and a[2] == b[2]
    return a


@pytest.mark.parametrize("mode", [2, 1])
def test_edit_sequences_equal_full_evaluate(tt, ds, ref_ctx, mode):
    """A random walk of edits where the 'host' goes on from the proposal (accept)
    or from the previous model (reject) at random, plus repeats of the same
    model (prior-2 deaths call evaluate twice, :141,159), unrelated models,
    a nearest-index request and pauses past the resident server's idle limit
    in between.  mode 2: the resident server (default); 1: a launch per call."""
    import time

    ctx = tt.TdContext.from_datastruct(ds)
    assert tt.lib().tdt_set_incremental(ctx.h, mode) == 0
    rng = np.random.default_rng(11 + mode)
    box = tt.box()
    cur = tt.random_model(400, 11).cells()
    check(ctx, ref_ctx, cur)
    for step in range(600):
        prop = edit(rng, cur, box)
        check(ctx, ref_ctx, prop)
        r = rng.random()
        if r < 0.05:
            check(ctx, ref_ctx, prop)  # the same model again
        if r > 0.97:  # an unrelated model, then back to the walk
            check(ctx, ref_ctx, tt.random_model(int(rng.integers(5, 300)), step).cells())
        if 0.5 < r < 0.52:  # nearest indices requested: always the full path
            _, phi, _, near = ctx.evaluate(prop, want_nearest=True)
            assert near is not None and phi == ref_ctx.evaluate(prop)[1]
        for cells in (prop, cur):  # 1-point Interpolation on the proposal / the model (:81, :146)
            q = [rng.uniform(box[0], box[1]), rng.uniform(box[2], box[3]), rng.uniform(box[4], box[5])]
            if rng.random() < 0.3 and len(cells[0]) > 0:  # exactly on a cell: a tie with its duplicate site
                k = int(rng.integers(len(cells[0])))
                q = [cells[0][k], cells[1][k], cells[2][k]]
            a, _ = ctx.interpolate(cells, [q[0]], [q[1]], [q[2]])
            b, _ = ref_ctx.interpolate(cells, [q[0]], [q[1]], [q[2]])
            assert np.array_equal(a, b), (step, q)
        if rng.random() < 0.55:
            cur = prop
        if step % 150 == 149:
            time.sleep(0.25)  # the server is stopped (host side) / returns by itself; state stays exact
    ctx.close()


def test_adversarial_edits(tt, ctx, ref_ctx):
    """Ties (duplicate cells, a cell moved onto another), cells far outside the
    rays' box, zeta = -0.0, deaths of the first and last cells, a birth exactly
    on an existing cell, several edits at once (full path)."""
    x, y, z, ze = (np.array(a) for a in tt.random_model(60, 21).cells())
    seq = []
    c = (x, y, z, ze)
    seq.append(c)
    c = (np.append(c[0], c[0][5]), np.append(c[1], c[1][5]), np.append(c[2], c[2][5]), np.append(c[3], 7.0))
    seq.append(c)  # birth on top of cell 5: every tie goes to cell 5 (lower position)
    x2 = c[0].copy(); y2 = c[1].copy(); z2 = c[2].copy()
    x2[10], y2[10], z2[10] = x2[3], y2[3], z2[3]
    c = (x2, y2, z2, c[3])
    seq.append(c)  # move onto cell 3
    c = tuple(np.delete(v, 0) for v in c)
    seq.append(c)  # death of the first
    c = tuple(np.delete(v, len(v) - 1) for v in c)
    seq.append(c)  # death of the last
    ze3 = c[3].copy(); ze3[4] = -0.0
    c = (c[0], c[1], c[2], ze3)
    seq.append(c)  # change to -0.0
    c = (np.append(c[0], 5e5), np.append(c[1], -4e5), np.append(c[2], 3e5), np.append(c[3], 20.0))
    seq.append(c)  # a birth far outside (clamped buckets)
    x4 = c[0].copy(); x4[7] = -2e5
    c = (x4, c[1], c[2], c[3])
    seq.append(c)  # a move far outside
    z5 = c[3].copy(); z5[1] = 33.0; z5[2] = 34.0
    c = (c[0], c[1], c[2], z5)
    seq.append(c)  # two changes at once: not one edit (full path)
    c = (np.append(c[0], 400.0), np.append(c[1], 100.0), np.append(c[2], 300.0), np.append(c[3], 1.0))
    seq.append(c)
    for cells in seq:
        check(ctx, ref_ctx, cells)


def test_growth_past_the_shadow_capacity(tt, ctx, ref_ctx):
    """Births beyond twice the starting size: the context rebuilds its shadow
    chain and stays exact."""
    rng = np.random.default_rng(5)
    box = tt.box()
    cur = tt.random_model(20, 5).cells()
    check(ctx, ref_ctx, cur)
    for _ in range(300):
        p = [rng.uniform(box[0], box[1]), rng.uniform(box[2], box[3]), rng.uniform(box[4], box[5])]
        cur = (np.append(cur[0], p[0]), np.append(cur[1], p[1]), np.append(cur[2], p[2]),
               np.append(cur[3], rng.uniform(0, 50)))
        check(ctx, ref_ctx, cur)


def test_incremental_on_many_rays(tt):
    """3000 synthetic rays (the shadow chain's HBM layout)."""
    ds = tt.synthetic_rays(3000, seed=8)
    a = tt.TdContext.from_datastruct(ds)
    b = tt.TdContext.from_datastruct(ds)
    assert tt.lib().tdt_set_incremental(b.h, 0) == 0
    rng = np.random.default_rng(3)
    cur = tt.random_model(700, 3).cells()
    check(a, b, cur)
    for _ in range(80):
        prop = edit(rng, cur, tt.box())
        check(a, b, prop)
        if rng.random() < 0.5:
            cur = prop
    a.close()
    b.close()


def test_sigma_change_drops_the_shadow(tt, ds):
    a = tt.TdContext.from_datastruct(ds)
    b = tt.TdContext.from_datastruct(ds)
    assert tt.lib().tdt_set_incremental(b.h, 0) == 0
    rng = np.random.default_rng(9)
    cur = tt.random_model(300, 9).cells()
    for k in range(40):
        prop = edit(rng, cur, tt.box())
        check(a, b, prop)
        cur = prop
        if k == 20:
            sig = np.asarray(ds.allSig) * 1.5
            a.set_sigma(sig)
            b.set_sigma(sig)
    a.close()
    b.close()


def test_server_reissues_a_command_after_its_watchdog(tt, ds):
    """The host is descheduled between its alive check and the post of a
    command (tdt_set_server_post_delay > the kernel's 200 ms watchdog): the
    kernel has returned, its pending proposal undone; the command is re-issued
    to a new launch (with that proposal as a committed step when the host
    accepted it) and the DROPIN chain still makes the HOST engine's moves."""
    prm = tt.define_TDstructrure().replace(max_cells=500)
    model = tt.random_model(300, 31)
    ctxs = [tt.TdContext.from_datastruct(ds) for _ in range(2)]
    chains = [tt.Chain(c, tt.chain_params(prm, None, seed=31, chain=1, engine=e), model)
              for c, e in zip(ctxs, (tt.TD_ENGINE_DROPIN, tt.TD_ENGINE_HOST))]
    chains[0].run(20)  # the server is up
    assert tt.lib().tdt_set_server_post_delay(260) == 0
    try:
        chains[0].run(8)  # every command (evaluate and one-point query) meets an exited kernel
    finally:
        tt.lib().tdt_set_server_post_delay(0)
    chains[0].run(40)
    chains[1].run(68)
    a, b = chains[0].stats(), chains[1].stats()
    assert a["phi"] == b["phi"] and a["accepted"] == b["accepted"] and a["proposed"] == b["proposed"]
    assert same_models(chains[0].model(), chains[1].model())
    for ch in chains:
        ch.close()
    for c in ctxs:
        c.close()


def test_two_contexts_interleaved_keep_their_pace(tt, ds, ref_ctx):
    """Two contexts of one process, each followed by its resident server,
    called alternately (one Julia worker driving two chains): starting one
    context's work stops the other's resident kernel first (servers_quiesce),
    so no call waits behind a kernel on a shared hardware queue; every result
    equals the full evaluate."""
    import time

    ctxs = [tt.TdContext.from_datastruct(ds) for _ in range(2)]
    rng = np.random.default_rng(17)
    box = tt.box()
    cur = [tt.random_model(500, 17 + k).cells() for k in range(2)]
    times = []
    for step in range(150):
        for k in range(2):
            prop = edit(rng, cur[k], box)
            t0 = time.perf_counter()
            a = ctxs[k].evaluate(prop)
            times.append(time.perf_counter() - t0)
            b = ref_ctx.evaluate(prop)
            assert a[1] == b[1] and np.array_equal(a[0], b[0])
            if rng.random() < 0.5:
                cur[k] = prop
    times = np.array(times[10:])
    assert np.median(times) < 5e-3 and np.mean(times) < 20e-3, (np.median(times), np.mean(times), times.max())
    for c in ctxs:
        c.close()


@pytest.mark.timeout(300)
def test_collective_between_evaluates(tt, tmp_path):
    """An RCCL all_gather between td_evaluate calls (a ray-sharded run's
    pattern), in a fresh child process (world 1 on device 0): same phi in
    modes 1 and 2; mode 1 (what RayShardedContext selects) keeps every call
    short.  Mode 2's per-call times are printed: a resident kernel sharing the
    collective's hardware queue would show as ~200 ms stalls."""
    import json
    import os
    import socket
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    res = {}
    for mode in (1, 2):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        out = tmp_path / ("m%d.json" % mode)
        p = subprocess.run([sys.executable, "-u", os.path.join(here, "collective_worker.py"), str(port), str(out),
                            str(mode)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=240)
        assert p.returncode == 0, p.stdout.decode(errors="replace")[-3000:]
        res[mode] = json.load(open(out))
    assert res[1]["phis"] == res[2]["phis"]
    t1, t2 = np.array(res[1]["times"][5:]), np.array(res[2]["times"][5:])
    print("per call (evaluate + all_gather): mode 1 median %.3f ms max %.3f ms; mode 2 median %.3f ms max %.3f ms"
          % (1e3 * np.median(t1), 1e3 * t1.max(), 1e3 * np.median(t2), 1e3 * t2.max()))
    assert np.median(t1) < 5e-3 and t1.max() < 0.1
