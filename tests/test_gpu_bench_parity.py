"""The timed path is the tested path: bench.py's exact workloads, at their
full lengths, against the HOST engine (one full td_evaluate of every
proposed model, the reference's structure: TD_inversion_function.jl:70-274,
MCsub.jl:123-185) and against from-scratch evaluates of the chain's model.

* config 3 (the headline): 381 rays x 5000 cells (model seed 3), max_cells
  10000, chain seed 1000, in launches of 5000 proposals -- 125,000
  proposals, the driver's `--steps 20 --warmup 5`; DEVICE == HOST after every
  launch, state == full evaluate every 25,000;
* many_chains: 256 chains (seeds 50000 + j) x 4 launches of 5000 in one
  td_chain_run_batch each; 4 sampled chains == their solo td_chain_run and
  == the HOST engine, final state == full evaluate;
* many_chains_2per_cu: 512 of those chains two per CU (lds_mode 2), 4
  launches of 5000; sampled chains == the same chains alone (8-wave kernel).
* the stress chain (config 5): 10k synthetic rays x 20k cells, 200 + 2000
  proposals, DEVICE == HOST, final state == full evaluate;
* the drop-in leg: the DROPIN engine (public td_evaluate per proposal, its
  resident incremental path) == HOST over bench's 1550 proposals.

The end states are also checked against the C oracle (oracle/tstar_oracle.c,
a scalar restatement of MCsub.jl:123-185), not only against another HIP path:
the 125k-proposal config-3 chain, 4 of the 256 batch chains, the full-size
stress chain (10k rays x 20k cells; oracle.evaluate_threaded splits its rays
over the host cores) and a stress chain on a 1500-ray subset of the config-5
rays at 3000 cells.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BENCH_ITERS = 5000


def same_models(a, b):
    return (len(a.xCell) == len(b.xCell) and np.array_equal(a.xCell, b.xCell) and np.array_equal(a.yCell, b.yCell)
            and np.array_equal(a.zCell, b.zCell) and np.array_equal(a.zeta, b.zeta))


def state_is_full_evaluate(ctx, ch):
    m = ch.model()
    ptS, phi, _, _ = ctx.evaluate(m.cells())
    assert phi == m.phi == ch.stats()["phi"]
    assert np.array_equal(ptS, m.ptS)
    return m


def state_is_oracle(orc, ds, ch):
    """The chain's final (ptS, phi) == the C oracle's evaluate of its model, bit for bit
    (the oracle is the checker here, never the thing measured)."""
    m = ch.model()
    ref = orc.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, m.cells())
    assert ref["rc"] == 0
    assert ref["phi"] == m.phi == ch.stats()["phi"]
    assert np.array_equal(ref["ptS"], m.ptS)
    return m


def agree(a, b):
    sa, sb = a.stats(), b.stats()
    assert sa["phi"] == sb["phi"], (sa, sb)
    assert sa["accepted"] == sb["accepted"] and sa["proposed"] == sb["proposed"]
    assert sa["ncells"] == sb["ncells"]
    return sa


@pytest.fixture(scope="module")
def ctx(tt, ds):
    c = tt.TdContext.from_datastruct(ds)
    c.set_incremental(c.INCR_FULL)  # the checker's evaluates are full ones
    yield c
    c.close()


@pytest.mark.timeout(600)
def test_config3_headline_run_follows_host(tt, ds, ctx, orc):
    prm = tt.define_TDstructrure().replace(max_cells=2 * 5000)
    model = tt.random_model(5000, 3)
    dev = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000, chain=1), model)
    host = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000, chain=1, engine=tt.TD_ENGINE_HOST), model)
    launches = 25  # --warmup 5 + --steps 20
    for k in range(launches):
        dev.run(BENCH_ITERS)
        host.run(BENCH_ITERS)
        st = agree(dev, host)
        if k % 5 == 4:
            m = state_is_full_evaluate(ctx, dev)
            assert same_models(m, host.model())
    assert st["iterations"] == launches * BENCH_ITERS
    assert sum(st["accepted"]) > 10000 and min(st["accepted"]) > 0  # every action was accepted many times
    state_is_oracle(orc, ds, dev)
    dev.close()
    host.close()


@pytest.mark.timeout(600)
def test_many_chains_batch_follows_solo_and_host(tt, ds, ctx, orc):
    prm = tt.define_TDstructrure().replace(max_cells=2 * 5000)
    model = tt.random_model(5000, 3)
    C = 256
    chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model) for j in range(C)]
    launches = 4  # bench: one warm-up launch + 3 timed
    for _ in range(launches):
        tt.run_batch(chains, BENCH_ITERS)
    for j in (0, 85, 170, 255):
        solo = tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model)
        host = tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j, engine=tt.TD_ENGINE_HOST),
                        model)
        for _ in range(launches):
            solo.run(BENCH_ITERS)
            host.run(BENCH_ITERS)
        agree(chains[j], solo)
        agree(chains[j], host)
        m = state_is_full_evaluate(ctx, chains[j])
        assert same_models(m, solo.model()) and same_models(m, host.model())
        state_is_oracle(orc, ds, chains[j])
        solo.close()
        host.close()
    for c in chains:
        c.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("knob", [True, False])
def test_many_chains_two_per_cu_follow_solo(tt, ds, ctx, knob):
    """bench.py's many_chains_2per_cu leg: 512 config-3 chains (seeds 50000 + j)
    in the 4-wave tiles-in-LDS kernel, two per CU (lds_mode 2; or, knob off, the
    launcher's own choice for a batch of more chains than CUs), 4 launches of
    5000; sampled chains equal the same chains run alone in the 8-wave kernel,
    and their state equals a full evaluate."""
    prm = tt.define_TDstructrure().replace(max_cells=2 * 5000)
    model = tt.random_model(5000, 3)
    C = 512
    chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model) for j in range(C)]
    for c in chains:
        if knob:
            assert tt.lib().tdt_chain_set_lds_mode(c.h, 2) == 0
    launches = 4  # bench: one warm-up launch + 3 timed
    for _ in range(launches):
        tt.run_batch(chains, BENCH_ITERS)
    for j in (0, 131, 300, 511):
        solo = tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model)
        for _ in range(launches):
            solo.run(BENCH_ITERS)
        agree(chains[j], solo)
        m = state_is_full_evaluate(ctx, chains[j])
        assert same_models(m, solo.model())
        solo.close()
    for c in chains:
        c.close()


@pytest.mark.timeout(600)
def test_stress_chain_run_follows_host(tt, orc):
    ds = tt.synthetic_rays(10000, seed=5)
    c = tt.TdContext.from_datastruct(ds)
    c.set_incremental(c.INCR_FULL)
    prm = tt.define_TDstructrure().replace(max_cells=40000)
    model = tt.random_model(20000, 5)
    dev = tt.Chain(c, tt.chain_params(prm, ds, seed=77, chain=1), model)
    host = tt.Chain(c, tt.chain_params(prm, ds, seed=77, chain=1, engine=tt.TD_ENGINE_HOST), model)
    for k in (200, 2000):  # bench.stress: ch.run(200) warm, then the timed ch.run(2000)
        dev.run(k)
        host.run(k)
        st = agree(dev, host)
    m = state_is_full_evaluate(c, dev)
    assert same_models(m, host.model())
    assert sum(st["accepted"]) > 500
    # the end state against the C oracle at full size (rays split over the host cores)
    ref = orc.evaluate_threaded(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, m.cells())
    assert ref["rc"] == 0 and ref["phi"] == m.phi == dev.stats()["phi"]
    assert np.array_equal(ref["ptS"], m.ptS)
    dev.close()
    host.close()
    c.close()


@pytest.mark.timeout(600)
def test_dropin_leg_follows_host(tt, ds):
    """bench.dropin: the DROPIN engine's 50 + 1500 proposals, each a public
    td_evaluate (incremental, resident server) and td_interpolate."""
    prm = tt.define_TDstructrure().replace(max_cells=2 * 5000)
    model = tt.random_model(5000, 3)
    ctxs = [tt.TdContext.from_datastruct(ds) for _ in range(2)]
    dropin = tt.Chain(ctxs[0], tt.chain_params(prm, ds, seed=1000, chain=1, engine=tt.TD_ENGINE_DROPIN), model)
    host = tt.Chain(ctxs[1], tt.chain_params(prm, ds, seed=1000, chain=1, engine=tt.TD_ENGINE_HOST), model)
    for k in (50, 1500):
        dropin.run(k)
        host.run(k)
        agree(dropin, host)
    assert same_models(dropin.model(), host.model())
    dropin.close()
    host.close()
    for c in ctxs:
        c.close()


@pytest.mark.timeout(600)
def test_stress_subset_chain_matches_oracle(tt, orc):
    """Config 5's rays, first 1500 (the HBM layout: tiles, rays and order out of
    LDS), 3000 cells, 1500 proposals: DEVICE == HOST, and the final state ==
    the C oracle's evaluate of the final model."""
    full = tt.synthetic_rays(10000, seed=5)
    ds = tt.sub_datastruct(full, 0, 1500)
    c = tt.TdContext.from_datastruct(ds)
    c.set_incremental(c.INCR_FULL)
    prm = tt.define_TDstructrure().replace(max_cells=4500)
    model = tt.random_model(3000, 5)
    dev = tt.Chain(c, tt.chain_params(prm, ds, seed=78, chain=1), model)
    assert tt.lib().tdt_chain_set_lds_mode(dev.h, 1) == 0
    host = tt.Chain(c, tt.chain_params(prm, ds, seed=78, chain=1, engine=tt.TD_ENGINE_HOST), model)
    for k in (300, 1200):
        dev.run(k)
        host.run(k)
        st = agree(dev, host)
    assert sum(st["accepted"]) > 100
    m = state_is_oracle(orc, ds, dev)
    assert same_models(m, host.model())
    dev.close()
    host.close()
    c.close()
