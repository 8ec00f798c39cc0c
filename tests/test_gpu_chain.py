"""GPU parity of the rj-MCMC chain (TD_inversion_function.jl:70-274).

The DEVICE engine (one persistent workgroup, incremental forward model) must
follow the HOST engine -- which evaluates every proposal with a full
td_evaluate exactly as the reference does -- bit for bit: same accepted
proposals, same phi after every run, same final model.  And the cached chain
state must equal a from-scratch evaluate of its model at any time."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(tt, ds):
    return tt.TdContext.from_datastruct(ds)


def make(tt, ctx, prm, model, seed, engine, T=1.0, chain=1):
    p = tt.chain_params(prm, None, seed=seed, chain=chain, temperature=T, engine=engine)
    return tt.Chain(ctx, p, model)


def same_models(a, b):
    return (len(a.xCell) == len(b.xCell) and np.array_equal(a.xCell, b.xCell) and np.array_equal(a.yCell, b.yCell)
            and np.array_equal(a.zCell, b.zCell) and np.array_equal(a.zeta, b.zeta))


@pytest.mark.parametrize("ncells,max_cells,iters,seed", [(200, 300, 400, 1), (1000, 1100, 250, 2),
                                                         (5000, 5100, 120, 3), (8, 12, 600, 4)])
def test_device_engine_follows_host_engine(tt, ds, ctx, ncells, max_cells, iters, seed):
    prm = tt.define_TDstructrure().replace(max_cells=max_cells)
    model = tt.random_model(ncells, seed)
    dev = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_DEVICE)
    host = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_HOST)
    for _ in range(4):
        dev.run(iters // 4)
        host.run(iters // 4)
        sd, sh = dev.stats(), host.stats()
        assert sd["phi"] == sh["phi"], (sd, sh)
        assert sd["accepted"] == sh["accepted"] and sd["proposed"] == sh["proposed"]
        assert sd["ncells"] == sh["ncells"]
    assert same_models(dev.model(), host.model())
    assert sum(sd["accepted"]) > 0


def test_chain_state_equals_full_evaluate(tt, ds, ctx):
    prm = tt.define_TDstructrure().replace(max_cells=2200)
    dev = make(tt, ctx, prm, tt.random_model(2000, 100), 100, tt.TD_ENGINE_DEVICE)
    for _ in range(5):
        dev.run(300)
        m = dev.model()
        ptS, phi, _, _ = ctx.evaluate(m.cells())
        assert phi == m.phi == dev.stats()["phi"]
        assert np.array_equal(ptS, m.ptS)


def test_tempered_chain_matches_host(tt, ds, ctx):
    prm = tt.define_TDstructrure().replace(max_cells=400)
    model = tt.random_model(300, 9)
    dev = make(tt, ctx, prm, model, 9, tt.TD_ENGINE_DEVICE, T=4.0, chain=3)
    host = make(tt, ctx, prm, model, 9, tt.TD_ENGINE_HOST, T=4.0, chain=3)
    dev.run(300)
    host.run(300)
    assert dev.stats()["phi"] == host.stats()["phi"]
    dev.set_temperature(1.5)
    host.set_temperature(1.5)
    dev.run(200)
    host.run(200)
    assert dev.stats()["phi"] == host.stats()["phi"]
    assert same_models(dev.model(), host.model())


def test_debug_prior_samples_prior(tt, ds, ctx):
    prm = tt.define_TDstructrure().replace(debug_prior=1)
    dev = make(tt, ctx, prm, None, 21, tt.TD_ENGINE_DEVICE)
    host = make(tt, ctx, prm, None, 21, tt.TD_ENGINE_HOST)
    counts = []
    for _ in range(20):
        dev.run(500)
        host.run(500)
        m = dev.model()
        counts.append(len(m.xCell))
        assert same_models(m, host.model())
        assert 5 <= len(m.xCell) <= 100
        assert np.all((m.zeta > 0) & (m.zeta < 50))
        assert dev.stats()["phi"] == 1.0
    assert len(set(counts)) > 3  # the dimension actually moves


def test_reference_driver_thinning(tt, ds):
    prm = tt.define_TDstructrure().replace(n_iter=300.0, burn_in=100.0, keep_each=20.0, print_each=100.0,
                                           max_cells=200)
    hist = tt.TD_inversion_function(prm, ds, 1, seed=5)
    assert len(hist) == 10  # (n_iter - burn_in) / keep_each
    for m in hist[::3]:
        m2 = m.copy()
        tt.evaluate(m2, ds, prm)
        assert m2.phi == m.phi


def test_clustered_and_boundary_cells(tt, ds, ctx):
    """Cells packed into one spot (bucket overflow -> full scans) and cells on
    the box faces (clamped buckets): the device engine must still follow the
    host engine bit for bit."""
    xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
    rng = np.random.default_rng(3)
    k = 120
    x = np.concatenate([rng.uniform(400, 401, k), rng.choice([xmin, xmax], 40)])
    y = np.concatenate([rng.uniform(100, 101, k), rng.uniform(ymin, ymax, 40)])
    z = np.concatenate([rng.uniform(300, 301, k), rng.choice([zmin, zmax], 40)])
    zeta = rng.uniform(1, 49, len(x))
    x[5], y[5], z[5] = x[4], y[4], z[4]  # an exact duplicate
    model = tt.Model(float(len(x)), x, y, z, zeta)
    prm = tt.define_TDstructrure().replace(max_cells=400)
    dev = make(tt, ctx, prm, model, 17, tt.TD_ENGINE_DEVICE)
    host = make(tt, ctx, prm, model, 17, tt.TD_ENGINE_HOST)
    for _ in range(3):
        dev.run(200)
        host.run(200)
        assert dev.stats()["phi"] == host.stats()["phi"]
    assert same_models(dev.model(), host.model())


def test_tempering_ladder_device_matches_host(tt, ds, ctx):
    """Three tempered replicas on one GPU exchanging temperatures every 50
    proposals: the device chains make exactly the host chains' moves and swaps."""
    prm = tt.define_TDstructrure().replace(max_cells=300)
    runs = {}
    for eng in (tt.TD_ENGINE_DEVICE, tt.TD_ENGINE_HOST):
        chains = [make(tt, ctx, prm, tt.random_model(150 + 20 * j, 30 + j), 30 + j, eng, chain=1 + j)
                  for j in range(3)]
        lad = tt.TemperingLadder(chains, tmax=8.0, seed=77)
        trace = [list(lad.step(50)) + list(lad.levels) for _ in range(8)]
        runs[eng] = (trace, [c.model() for c in chains], lad.swap_rates())
    assert runs[tt.TD_ENGINE_DEVICE][0] == runs[tt.TD_ENGINE_HOST][0]
    for a, b in zip(runs[tt.TD_ENGINE_DEVICE][1], runs[tt.TD_ENGINE_HOST][1]):
        assert same_models(a, b)


def test_batched_chains_equal_single_launches(tt, ds, ctx):
    """td_chain_run_batch (one workgroup per chain, one launch) gives every
    chain exactly what td_chain_run gives it alone."""
    prm = tt.define_TDstructrure().replace(max_cells=700)
    specs = [(60, 41), (300, 42), (600, 43), (150, 44), (8, 45)]
    solo = []
    for ncell, seed in specs:
        c = make(tt, ctx, prm, tt.random_model(ncell, seed), seed, tt.TD_ENGINE_DEVICE, chain=seed)
        c.run(400)
        solo.append((c.stats(), c.model()))
    batch = [make(tt, ctx, prm, tt.random_model(n, s), s, tt.TD_ENGINE_DEVICE, chain=s) for n, s in specs]
    tt.run_batch(batch, 150)
    tt.run_batch(batch, 250)
    for c, (st, m) in zip(batch, solo):
        assert c.stats()["phi"] == st["phi"] and c.stats()["accepted"] == st["accepted"]
        assert same_models(c.model(), m)


@pytest.mark.parametrize("ncells,iters,seed", [(300, 300, 61), (2000, 200, 62)])
def test_hbm_layout_follows_host_engine(tt, ds, ctx, ncells, iters, seed):
    """The layout larger geometries take (tiles, rays and order in HBM instead
    of LDS: k_chain_run<false>) against the host engine, bit for bit."""
    prm = tt.define_TDstructrure().replace(max_cells=ncells + 200)
    model = tt.random_model(ncells, seed)
    dev = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_DEVICE)
    assert tt.lib().tdt_chain_set_lds_mode(dev.h, 1) == 0
    host = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_HOST)
    for _ in range(3):
        dev.run(iters // 3)
        host.run(iters // 3)
        assert dev.stats()["phi"] == host.stats()["phi"]
        assert dev.stats()["accepted"] == host.stats()["accepted"]
    assert same_models(dev.model(), host.model())
    m = dev.model()
    ptS, phi, _, _ = ctx.evaluate(m.cells())
    assert phi == m.phi and np.array_equal(ptS, m.ptS)


def test_many_rays_chain_follows_host_engine(tt):
    """3000 synthetic rays: tiles, rays and order live in HBM and the chi^2
    tails run through the block-wide exact scan; still bit for bit the host
    engine (one full evaluate per proposal)."""
    ds = tt.synthetic_rays(3000, seed=8)
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=900)
    model = tt.random_model(700, 21)
    dev = make(tt, ctx, prm, model, 21, tt.TD_ENGINE_DEVICE)
    host = make(tt, ctx, prm, model, 21, tt.TD_ENGINE_HOST)
    for _ in range(3):
        dev.run(40)
        host.run(40)
        assert dev.stats()["phi"] == host.stats()["phi"]
        assert dev.stats()["accepted"] == host.stats()["accepted"]
    assert same_models(dev.model(), host.model())
    dev.close()
    host.close()
    ctx.close()


def lds_plan(tt, ch):
    out = (ctypes.c_int64 * 4)()
    assert tt.lib().tdt_chain_lds(ch.h, out) == 0
    return list(out)


def test_bench_config_takes_lds_layout(tt, ds, ctx):
    """bench.py's config 3 (381 rays, 5000 cells, max 10000) fits the LDS layout."""
    prm = tt.define_TDstructrure().replace(max_cells=10000)
    ch = make(tt, ctx, prm, tt.random_model(5000, 3), 3, tt.TD_ENGINE_DEVICE)
    small, big, sup, layout = lds_plan(tt, ch)
    assert small <= 160 * 1024 and layout == 1, (small, big)
    ch.close()


@pytest.mark.parametrize("ncells,rounds,seed", [(2000, 4, 51), (20000, 2, 5)])
def test_stress_geometry_chain_follows_host_engine(tt, ncells, rounds, seed):
    """10k synthetic rays (the stress geometry): the HBM layout with super-tiles
    in LDS and the chi^2 event walk, bit for bit the host engine over a few
    hundred proposals (accepted ones commit the walk's segments and re-mark);
    at 2000 cells and at config 5's full 20k cells (seed 5)."""
    ds = tt.synthetic_rays(10000, seed=5)
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=int(ncells * 1.5))
    model = tt.random_model(ncells, seed)
    dev = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_DEVICE)
    small, big, sup, layout = lds_plan(tt, dev)
    assert layout == 0 and sup == 1, (small, big, sup)
    host = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_HOST)
    for _ in range(rounds):
        dev.run(75)
        host.run(75)
        assert dev.stats()["phi"] == host.stats()["phi"]
        assert dev.stats()["accepted"] == host.stats()["accepted"]
    assert same_models(dev.model(), host.model())
    m = dev.model()
    ptS, phi, _, _ = ctx.evaluate(m.cells())
    assert phi == m.phi and np.array_equal(ptS, m.ptS)
    dev.close()
    host.close()
    ctx.close()


@pytest.mark.parametrize("prior,ncells,iters,seed", [(2, 300, 400, 71), (3, 300, 400, 72), (2, 2000, 200, 73),
                                                     (3, 1000, 200, 74), (2, 0, 400, 75), (3, 0, 400, 76)])
def test_priors_device_follows_host(tt, ds, ctx, prior, ncells, iters, seed):
    """Normal (2) and exponential (3) priors (TD_inversion_function.jl:105-119,
    157-172, 201-212; start MCsub.jl:102-107 when ncells = 0): the device
    engine makes the host engine's decisions bit for bit."""
    prm = tt.define_TDstructrure().replace(prior=prior, max_cells=max(ncells, 100) + 200)
    model = tt.random_model(ncells, seed) if ncells else None
    if model is not None and prior == 2:
        model.zeta[:] = np.random.default_rng(seed).normal(0.0, 50.0, ncells)  # the normal prior's start
    dev = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_DEVICE)
    host = make(tt, ctx, prm, model, seed, tt.TD_ENGINE_HOST)
    m0 = dev.model()
    if ncells == 0:  # build_starting drew the same model in both engines
        assert same_models(m0, host.model())
        if prior == 3:
            assert np.all(m0.zeta > 0)
    for _ in range(4):
        dev.run(iters // 4)
        host.run(iters // 4)
        sd, sh = dev.stats(), host.stats()
        assert sd["phi"] == sh["phi"], (sd, sh)
        assert sd["accepted"] == sh["accepted"] and sd["proposed"] == sh["proposed"]
    assert same_models(dev.model(), host.model())
    assert sum(sd["accepted"]) > 0
    m = dev.model()
    ptS, phi, _, _ = ctx.evaluate(m.cells())
    assert phi == m.phi and np.array_equal(ptS, m.ptS)


def test_resident_rounds_equal_launch_per_round(tt, ds, ctx):
    """td_rounds (one launch resident across the swap rounds, temperatures
    posted through pinned memory) gives exactly the ladder of one
    td_chain_run_batch launch per round -- also when the host pauses past the
    launch's 200 ms idle watchdog between rounds (it returns and is started
    again) and when a round size changes."""
    import time

    prm = tt.define_TDstructrure().replace(max_cells=600)
    runs = []
    for resident in (True, False):
        chains = [make(tt, ctx, prm, tt.random_model(200 + 30 * j, 60 + j), 60 + j, tt.TD_ENGINE_DEVICE,
                       chain=1 + j) for j in range(4)]
        lad = tt.TemperingLadder(chains, tmax=8.0, seed=99, resident=resident)
        assert lad.resident == resident
        trace = []
        for r in range(30):
            k = 10 if r < 20 else 7
            trace.append([list(lad.step(k)), list(lad.levels)])
            if r in (5, 6, 17):
                time.sleep(0.3)
        lad.close()
        runs.append((trace, [c.model() for c in chains], [c.stats() for c in chains], lad.trace_digest()))
        for c in chains:
            c.close()
    (ta, ma, sa, da), (tb, mb, sb, db) = runs
    assert ta == tb and da == db
    for a, b, x, y in zip(ma, mb, sa, sb):
        assert same_models(a, b)
        assert x["phi"] == y["phi"] and x["accepted"] == y["accepted"] and x["proposed"] == y["proposed"]
        assert x["iterations"] == y["iterations"] == 20 * 10 + 10 * 7


def test_resident_rounds_partial_exit(tt, ds, ctx):
    """The watchdog race: some workgroups of the resident launch
    return at a round boundary just as the host posts the next round, while
    the others run it (tdt_rounds_force_exit makes that happen on purpose).
    td_rounds_run must post the round again so that every chain runs it once:
    the ladder equals one launch per round, iteration counts included.  After
    close() every chain sits at its ladder level's temperature: more
    proposals on the chains alone still agree."""
    prm = tt.define_TDstructrure().replace(max_cells=600)
    runs = []
    for resident in (True, False):
        chains = [make(tt, ctx, prm, tt.random_model(200 + 30 * j, 160 + j), 160 + j, tt.TD_ENGINE_DEVICE,
                       chain=1 + j) for j in range(5)]
        lad = tt.TemperingLadder(chains, tmax=8.0, seed=5, resident=resident)
        trace = []
        for r in range(24):
            if resident and r in (1, 7, 8, 15):
                forced = {1: [0], 7: [1, 3], 8: [4], 15: [0, 2, 3]}[r]
                arr = (ctypes.c_int32 * len(forced))(*forced)
                assert tt.lib().tdt_rounds_force_exit(lad.rounds.h, arr, len(forced)) == 0
            trace.append([list(lad.step(10)), list(lad.levels)])
        lad.close()
        for c in chains:  # alone, after the ladder: each at the temperature of its final level
            c.run(60)
        runs.append((trace, [c.model() for c in chains], [c.stats() for c in chains], lad.trace_digest()))
        for c in chains:
            c.close()
    (ta, ma, sa, da), (tb, mb, sb, db) = runs
    assert ta == tb and da == db
    for a, b, x, y in zip(ma, mb, sa, sb):
        assert same_models(a, b)
        assert x["phi"] == y["phi"] and x["accepted"] == y["accepted"] and x["proposed"] == y["proposed"]
        assert x["iterations"] == y["iterations"] == 24 * 10 + 60


def test_resident_rounds_do_not_hold_back_other_streams(tt, ds, ctx):
    """The resident rounds launch spins between rounds on a hardware queue of
    its own (a CU-masked stream): work on other streams -- what an RCCL
    collective's kernel is -- completes at once instead of waiting behind it
    for the 200 ms idle watchdog, and the launch is still there for the next
    round.  Eight ordinary HIP streams (dealt by HIP over its 4 shared
    hardware queues) each run a fill kernel (hipMemsetAsync) while the launch
    waits between rounds.  (Plain HIP through ctypes: the process's HIP
    runtime is the one libtdstar loaded; torch would bring a second one.)"""
    import time

    hip = ctypes.CDLL("libamdhip64.so.7")
    buf = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(1 << 24)) == 0
    streams = []
    for _ in range(8):
        st = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(st)) == 0
        streams.append(st)
    for st in streams:  # warm
        assert hip.hipMemsetAsync(buf, 0, ctypes.c_size_t(1 << 24), st) == 0
        assert hip.hipStreamSynchronize(st) == 0
    prm = tt.define_TDstructrure().replace(max_cells=600)
    chains = [make(tt, ctx, prm, tt.random_model(200 + 30 * j, 260 + j), 260 + j, tt.TD_ENGINE_DEVICE,
                   chain=1 + j) for j in range(4)]
    lad = tt.TemperingLadder(chains, tmax=8.0, seed=3)
    for _ in range(5):
        lad.step(10)
    worst = 0.0
    for r in range(24):
        lad.step(10)  # the launch now waits for the next round
        st = streams[r % len(streams)]
        t0 = time.perf_counter()
        assert hip.hipMemsetAsync(buf, r, ctypes.c_size_t(1 << 24), st) == 0
        assert hip.hipStreamSynchronize(st) == 0
        worst = max(worst, time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(50):
        lad.step(10)
    per_round = (time.perf_counter() - t0) / 50
    lad.close()
    for c in chains:
        c.close()
    for st in streams:
        hip.hipStreamDestroy(st)
    hip.hipFree(buf)
    assert worst < 0.05, worst  # (held back: >= 0.2 s, the watchdog)
    assert per_round < 0.02, per_round


@pytest.mark.parametrize("lds_mode", [0, 1])
def test_exchange_rounds_equal_host_decided(tt, ds, ctx, lds_mode):
    """td_rounds_exchange on one rank (the swaps decided inside the kernel,
    no host in the loop) against the host-decided resident ladder, in both
    layouts (lds_mode 1: the HBM-layout kernel) and two calls of different
    round sizes; then the chains alone, each at its final level's T."""
    prm = tt.define_TDstructrure().replace(max_cells=600)
    runs = []
    for dev_swaps in (True, False):
        chains = [make(tt, ctx, prm, tt.random_model(220 + 25 * j, 300 + j), 300 + j, tt.TD_ENGINE_DEVICE,
                       chain=1 + j) for j in range(5)]
        for c in chains:
            assert tt.lib().tdt_chain_set_lds_mode(c.h, lds_mode) == 0
        lad = tt.TemperingLadder(chains, tmax=6.0, seed=31, device_swaps=dev_swaps)
        assert lad.device_swaps == dev_swaps
        lad.run(30, 10)
        lad.run(13, 3)
        lad.close()
        for c in chains:
            c.run(40)
        runs.append((lad.trace_digest(), list(lad.levels), list(lad.tried), list(lad.accepted), lad.mixing(),
                     [c.model() for c in chains], [c.stats() for c in chains]))
        for c in chains:
            c.close()
    a, b = runs
    assert a[:5] == b[:5]
    assert sum(a[3]) > 0  # swaps happened
    for ma, mb, x, y in zip(a[5], b[5], a[6], b[6]):
        assert same_models(ma, mb)
        assert x["phi"] == y["phi"] and x["accepted"] == y["accepted"] and x["iterations"] == y["iterations"]


def test_library_tempering_loop_equals_round_by_round(tt, ds, ctx):
    """TemperingLadder.run (td_rounds_temper: the resident launch with the swap
    steps decided in the library between rounds, no return to Python per
    round) gives exactly the trace, levels, swap counts, models and stats of
    the same rounds stepped one by one from Python with decide_swaps, in two
    calls of different round sizes."""
    prm = tt.define_TDstructrure().replace(max_cells=600)
    runs = []
    for native in (True, False):
        chains = [make(tt, ctx, prm, tt.random_model(250 + 20 * j, 80 + j), 80 + j, tt.TD_ENGINE_DEVICE,
                       chain=1 + j) for j in range(6)]
        lad = tt.TemperingLadder(chains, tmax=8.0, seed=7, resident=True)
        if native:
            lad.run(25, 10)
            lad.run(11, 4)
        else:
            for r in range(36):
                lad.step(10 if r < 25 else 4)
        lad.close()
        runs.append((lad.trace_digest(), list(lad.levels), list(lad.tried), list(lad.accepted),
                     [c.model() for c in chains], [c.stats() for c in chains], lad.rnd, lad.mixing()))
        for c in chains:
            c.close()
    a, b = runs
    assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2] and a[3] == b[3] and a[6] == b[6] == 36
    assert a[7] == b[7]  # round trips and up-fractions: the library loop observes every round's levels
    for ma, mb, x, y in zip(a[4], b[4], a[5], b[5]):
        assert same_models(ma, mb)
        assert x["phi"] == y["phi"] and x["accepted"] == y["accepted"] and x["proposed"] == y["proposed"]


@pytest.mark.parametrize("lds_mode", [0, 1])
def test_exact_path_of_decisions_on_bounds(tt, ds, ctx, lds_mode):
    """Phase F decides on bounds and leaves an accepted proposal's chi^2 partial
    sums unformed; the exact sums (the committed ones made exact again from
    where accepted proposals left them, with the proposal's own terms in place,
    then the proposal's) run only when a decision falls inside the brackets --
    almost never by itself.  Forced on every k-th decision (k = 1, 2, 3, 7,
    mixing them with bound decisions in every pattern), the chain must be the
    default chain and the HOST engine's, bit for bit, in both layouts, over
    several launches (each ends exact); and the state must equal a from-scratch
    evaluate."""
    prm = tt.define_TDstructrure().replace(max_cells=1200)
    model = tt.random_model(1000, 31)
    L = tt.lib()
    host = make(tt, ctx, prm, model, 31, tt.TD_ENGINE_HOST)
    devs = []
    for k in (0, 1, 2, 3, 7):
        c = make(tt, ctx, prm, model, 31, tt.TD_ENGINE_DEVICE)
        assert L.tdt_chain_set_lds_mode(c.h, lds_mode) == 0
        assert L.tdt_chain_set_exact_every(c.h, k) == 0
        devs.append(c)
    for step in (61, 130, 9):
        host.run(step)
        sh = host.stats()
        for c in devs:
            c.run(step)
            sd = c.stats()
            assert sd["phi"] == sh["phi"], (sd, sh)
            assert sd["accepted"] == sh["accepted"] and sd["proposed"] == sh["proposed"]
    assert sum(sh["accepted"]) > 20
    for c in devs:
        m = c.model()
        assert same_models(m, host.model())
        ptS, phi, _, _ = ctx.evaluate(m.cells())
        assert phi == m.phi and np.array_equal(ptS, m.ptS)
        c.close()
    host.close()


@pytest.mark.parametrize("mode", [2, 3])
def test_two_chains_per_cu_variant_follows_host(tt, ds, ctx, mode):
    """lds_mode 2 / 3: the 256-thread (4-wave) kernel whose <= 80 KB of LDS and
    <= 256 registers let two chains share a CU (td_chain_run_batch packs 2 per
    CU), with the tiles in LDS and the rays and order in HBM (2), or all in
    HBM (3) -- its wave roles differ from the 8-wave kernel's (phase F: the
    tile maxima on one wave, the grid prefetch and the accounting on the
    last).  Alone and batched (more chains than CUs), every chain equals the
    HOST engine and the 8-wave kernel, bit for bit; the state equals a
    from-scratch evaluate."""
    prm = tt.define_TDstructrure().replace(max_cells=1300)
    L = tt.lib()
    specs = [(1000, 71), (400, 72), (1200, 73)]
    host = [make(tt, ctx, prm, tt.random_model(n, s), s, tt.TD_ENGINE_HOST, chain=s) for n, s in specs]
    eight = [make(tt, ctx, prm, tt.random_model(n, s), s, tt.TD_ENGINE_DEVICE, chain=s) for n, s in specs]
    four = [make(tt, ctx, prm, tt.random_model(n, s), s, tt.TD_ENGINE_DEVICE, chain=s) for n, s in specs]
    for c in four:
        assert L.tdt_chain_set_lds_mode(c.h, mode) == 0
    for step in (70, 130):
        for c in host + eight:
            c.run(step)
        tt.run_batch(four, step)
        for h, e, f in zip(host, eight, four):
            sh, se, sf = h.stats(), e.stats(), f.stats()
            assert sf["phi"] == se["phi"] == sh["phi"], (sh, se, sf)
            assert sf["accepted"] == sh["accepted"] and sf["proposed"] == sh["proposed"]
    solo = make(tt, ctx, prm, tt.random_model(1000, 71), 71, tt.TD_ENGINE_DEVICE, chain=71)
    assert L.tdt_chain_set_lds_mode(solo.h, mode) == 0
    solo.run(200)
    assert solo.stats()["phi"] == host[0].stats()["phi"]
    for h, f in zip(host, four):
        m = f.model()
        assert same_models(m, h.model())
        ptS, phi, _, _ = ctx.evaluate(m.cells())
        assert phi == m.phi and np.array_equal(ptS, m.ptS)
    # more chains than CUs in one launch: two resident per CU
    many = [make(tt, ctx, prm, tt.random_model(300, 900 + j), 900 + j, tt.TD_ENGINE_DEVICE, chain=900 + j)
            for j in range(300)]
    for c in many:
        assert L.tdt_chain_set_lds_mode(c.h, mode) == 0
    tt.run_batch(many, 60)
    for j in (0, 137, 299):
        ref = make(tt, ctx, prm, tt.random_model(300, 900 + j), 900 + j, tt.TD_ENGINE_HOST, chain=900 + j)
        ref.run(60)
        assert many[j].stats()["phi"] == ref.stats()["phi"] and same_models(many[j].model(), ref.model())
        ref.close()
    for c in host + eight + four + many + [solo]:
        c.close()


def test_hbm_layout_edge_rays_follow_host_engine(tt):
    """Rays of 1, 2, 3, 16, 17, 18, 34, 35, 140 and 2100 points (every branch of
    the two-rays-per-wave sum, ray_sum.h half_ray_sum, down to Julia's pairwise
    split above 1024 terms), several crossing one region so that proposals
    change many rays at once, in the HBM layout (k_chain_run<false>) against
    the host engine, bit for bit."""
    rng = np.random.default_rng(11)
    lens = [1, 2, 3, 16, 17, 18, 34, 35, 140, 2100, 17, 35, 140, 3, 34, 18, 2]
    m = max(lens)
    rays = []
    for k, n in enumerate(lens):
        a = rng.uniform([-50.0, -50.0, 100.0], [750.0, 350.0, 600.0])
        b = np.array([350.0, 150.0, 300.0]) + rng.normal(0.0, 40.0, 3)  # through one region
        t = np.linspace(0.0, 1.0, n)[:, None]
        rays.append(a + t * (b - a) * (2.0 if k % 2 else 1.0))
    nr = len(rays)
    X, Y, Z = (np.full((m, nr), np.nan) for _ in range(3))
    for i, r in enumerate(rays):
        X[:len(r), i], Y[:len(r), i], Z[:len(r), i] = r[:, 0], r[:, 1], r[:, 2]
    U = np.where(np.isnan(X), np.nan, 0.1 + 0.001 * np.nan_to_num(Z))
    L, Uu = tt.segments(X, Y, Z, U)
    tS = np.linspace(0.1, 0.5, nr)
    sig = np.linspace(0.05, 0.3, nr)
    ds2 = tt.DataStruct(tS, tS, tS, tS, sig, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, tS, X, Y, Z, L, Uu, U)
    c2 = tt.TdContext.from_datastruct(ds2)
    prm = tt.define_TDstructrure().replace(max_cells=400)
    model = tt.random_model(250, 9)
    dev = make(tt, c2, prm, model, 9, tt.TD_ENGINE_DEVICE)
    assert tt.lib().tdt_chain_set_lds_mode(dev.h, 1) == 0
    host = make(tt, c2, prm, model, 9, tt.TD_ENGINE_HOST)
    for _ in range(3):
        dev.run(150)
        host.run(150)
        assert dev.stats()["phi"] == host.stats()["phi"]
        assert dev.stats()["accepted"] == host.stats()["accepted"]
    assert sum(dev.stats()["accepted"]) > 20  # (the models really moved)
    assert same_models(dev.model(), host.model())
    dev.close()
    host.close()
    c2.close()


@pytest.mark.parametrize("clustered", [False, True])
def test_grid_query_forms_agree(tt, ds, ctx, orc, clustered):
    """The chain's grid query reads the grid from its LDS copy and proves its answer first against the
    global bound (h - 2e)^2 (GridGeo); the descriptor-reading form with the query's own face bound
    is kept for comparison (tdt_chain_query_lat modes 0 and 6).  Both must give the same (distance,
    slot, proven) for every query: ray points, points spread over the cells' box and far beyond it,
    the live cells' own sites (distance 0; exact duplicates tie), and (clustered) cells packed into
    one spot plus exact duplicates, where buckets overflow.  And every answer either form calls proven
    must be the exact one: v_nearest's first minimum over the live cells in Julia order
    (MCsub.jl:247-263, the C oracle's interpolation), distance and value bit for bit -- so a bound
    shared by both forms (the sealed box, the global first bound) is checked against a full scan."""
    rng = np.random.default_rng(9 if clustered else 8)
    if clustered:
        xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
        k = 300
        x = np.concatenate([rng.uniform(400, 402, k), rng.uniform(xmin, xmax, 200)])
        y = np.concatenate([rng.uniform(100, 102, k), rng.uniform(ymin, ymax, 200)])
        z = np.concatenate([rng.uniform(300, 302, k), rng.uniform(zmin, zmax, 200)])
        x[7], y[7], z[7] = x[6], y[6], z[6]
        x[k + 5], y[k + 5], z[k + 5] = x[k + 4], y[k + 4], z[k + 4]
        model = tt.Model(float(len(x)), x, y, z, rng.uniform(1, 49, len(x)))
    else:
        model = tt.random_model(5000, 3)
        for a, b in ((10, 11), (200, 4000)):  # exact duplicates: a query at the site ties at distance 0
            model.xCell[b], model.yCell[b], model.zCell[b] = model.xCell[a], model.yCell[a], model.zCell[a]
    prm = tt.define_TDstructrure().replace(max_cells=10000)
    ch = make(tt, ctx, prm, model, 23, tt.TD_ENGINE_DEVICE)
    ch.run(300)
    X, Y, Z = (np.asarray(a, dtype=np.float64).ravel() for a in (ds.rayX, ds.rayY, ds.rayZ))
    ok = ~np.isnan(X)
    X, Y, Z = X[ok], Y[ok], Z[ok]
    sel = rng.integers(0, len(X), 1500)
    lo, hi = np.array([X.min(), Y.min(), Z.min()]), np.array([X.max(), Y.max(), Z.max()])
    box = lo - 50.0 + (hi - lo + 100.0) * rng.random((1500, 3))
    far = lo - 1000.0 + (hi - lo + 2000.0) * rng.random((300, 3))  # well outside the cells' box too
    m = ch.model()
    cells = np.stack([m.xCell, m.yCell, m.zCell], 1)
    sites = cells[rng.integers(0, len(cells), 200)]
    pts = np.ascontiguousarray(np.concatenate([np.stack([X[sel], Y[sel], Z[sel]], 1), box, far, sites]),
                               dtype=np.float64)
    L = tt.lib()
    P = ctypes.POINTER(ctypes.c_double)
    digests = []
    for mode in (0, 6):
        out = (ctypes.c_int64 * 4)()
        assert L.tdt_chain_query_lat(ch.h, pts.ctypes.data_as(P), len(pts), mode, out) == 0
        digests.append(out[3])
    assert digests[0] == digests[1]
    # the proven answers against the exact scan (every live cell, Julia order, first minimum)
    val, ids = orc.interpolation(m.cells(), pts[:, 0], pts[:, 1], pts[:, 2])
    dx, dy, dz = (pts[:, 0] - m.xCell[ids]), (pts[:, 1] - m.yCell[ids]), (pts[:, 2] - m.zCell[ids])
    dref = (dx * dx + dy * dy) + dz * dz
    for mode in (0, 6):
        dist, value = np.zeros(len(pts)), np.zeros(len(pts))
        proven = np.zeros(len(pts), dtype=np.int32)
        assert L.tdt_chain_query_answers(ch.h, pts.ctypes.data_as(P), len(pts), mode, dist.ctypes.data_as(P),
                                         value.ctypes.data_as(P),
                                         proven.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
        pv = proven != 0
        if not clustered:  # (clustered: the packed buckets overflow, and the chain's queries take the full scan)
            assert pv.sum() > len(pts) // 2, (mode, int(pv.sum()))  # (most queries are proven by the grid)
        bad = np.flatnonzero(pv & ((dist != dref) | (value != val)))
        assert bad.size == 0, (mode, bad[:10], dist[bad[:5]], dref[bad[:5]], value[bad[:5]], val[bad[:5]])
    ch.close()
