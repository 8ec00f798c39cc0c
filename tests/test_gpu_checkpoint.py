"""Checkpoints and resume (TD_inversion_function.jl:41-67, 275-298).

A chain interrupted after a checkpoint and started again resumes from its
newest JLD checkpoint and returns a model_hist identical, field for field
(cells, phi, ptS, tS, likelihood, action, accept), to the uninterrupted run's:
the counter-based RNG continues exactly.  Both the burn-in checkpoint
(burnin = true: model_hist, saved_#, model_num restored) and the pre-burn-in
one (burnin = false) are exercised.  The JLD files need h5py (the image's
/opt/conda/bin/python3.9); skipped without it."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jld(tt):
    if not tt.jld.available():
        pytest.skip("no interpreter with h5py")
    return tt.jld


def prm(tt, **kw):
    # n_iter / print_each keep 100 * iter / n_iter integral (:291 Int(...) would throw otherwise)
    base = dict(n_iter=500.0, burn_in=200.0, keep_each=20.0, print_each=50.0, max_cells=400)
    base.update(kw)
    return tt.define_TDstructrure().replace(**base)


def same(a, b):
    return (np.array_equal(a.xCell, b.xCell) and np.array_equal(a.yCell, b.yCell) and np.array_equal(a.zCell, b.zCell)
            and np.array_equal(a.zeta, b.zeta) and a.phi == b.phi and np.array_equal(a.ptS, b.ptS)
            and np.array_equal(a.tS, b.tS) and a.likelihood == b.likelihood and a.action == b.action
            and a.accept == b.accept and a.nCells == b.nCells)


@pytest.fixture(scope="module")
def straight(tt, ds, jld, tmp_path_factory):
    d = tmp_path_factory.mktemp("ckA")
    hist = tt.TD_inversion_function(prm(tt), ds, 1, seed=5, model=tt.random_model(250, 5), checkpoint_dir=str(d))
    return hist, d


def test_checkpoint_names_and_contents(tt, ds, jld, straight):
    hist, d = straight
    assert len(hist) == 15  # (n_iter - burn_in) / keep_each
    names = sorted(os.listdir(d), key=lambda f: int(f.split("_iter")[1].split("_")[0]))
    # pre-burn-in every print_each (:291, Int(pct)); after burn-in the 1st saved model and every 10 % (:284)
    assert names[:3] == ["chain1_iter50_10%.jld", "chain1_iter100_20%.jld", "chain1_iter150_30%.jld"]
    assert names[3:] == ["chain1_iter%d_%r%%.jld" % (it, 100 * it / 500.0) for it in (219, 259, 319, 379, 439, 499)]
    c = jld.load_checkpoint(os.path.join(d, "chain1_iter319_63.8%.jld"))
    assert c["burnin"] and c["iter"] == 319.0 and not c["iter_is_int"]
    assert c["saved"] == 6 and c["model_num"] == 120 and len(c["model_hist"]) == 6
    for a, b in zip(c["model_hist"], hist[:6]):
        assert same(a, b)
    assert same(c["model"], hist[5]) and c["model"] is c["model_hist"][-1]  # saved once, referenced twice
    assert np.array_equal(c["ds"]["tS"], ds.tS) and np.array_equal(c["ds"]["rayX"], ds.rayX, equal_nan=True)
    p = jld.load_checkpoint(os.path.join(d, "chain1_iter100_20%.jld"))
    assert not p["burnin"] and p["iter"] == 100 and p["iter_is_int"] and p["model_hist"] == []
    assert {m.action for m in hist} <= {1, 2, 3, 4} and {m.accept for m in hist} <= {0, 1}
    for m in hist[::4]:  # every saved model is what a full evaluate of its cells gives
        m2 = m.copy()
        tt.evaluate(m2, ds, prm(tt))
        assert m2.phi == m.phi and np.array_equal(m2.ptS, m.ptS)


@pytest.mark.parametrize("stop", [350, 170])
def test_kill_and_resume_is_bit_identical(tt, ds, jld, straight, tmp_path, stop):
    hist, _ = straight
    d = str(tmp_path)
    part = tt.TD_inversion_function(prm(tt), ds, 1, seed=5, model=tt.random_model(250, 5), checkpoint_dir=d,
                                    stop_after=stop)  # "crash" after iteration `stop`
    assert len(part) == (7 if stop == 350 else 0)
    resumed = tt.TD_inversion_function(prm(tt), ds, 1, seed=5, model=None, checkpoint_dir=d)
    assert len(resumed) == len(hist)
    for a, b in zip(resumed, hist):
        assert same(a, b)


def test_resume_keeps_newest_two(tt, ds, jld, tmp_path):
    d = str(tmp_path)
    tt.TD_inversion_function(prm(tt), ds, 2, seed=9, model=tt.random_model(100, 9), checkpoint_dir=d, stop_after=330)
    open(os.path.join(d, "chain21_iter10_2%.jld"), "w").close()  # another chain's file: not ours (:41 quirk)
    tt.TD_inversion_function(prm(tt), ds, 2, seed=9, model=None, checkpoint_dir=d, stop_after=331)
    mine = sorted(f for f in os.listdir(d) if f.startswith("chain2_"))
    assert mine == ["chain2_iter259_51.8%.jld", "chain2_iter319_63.8%.jld"]
    assert "chain21_iter10_2%.jld" in os.listdir(d)


def test_burn_in_zero_counts_from_iteration_one(tt, ds):
    """burn_in = 0: model_num = iter, so keep_each = 10 saves iterations 10, 20, ..."""
    p = prm(tt, n_iter=60.0, burn_in=0.0, keep_each=10.0, print_each=10.0)
    m0 = tt.random_model(150, 3)
    hist = tt.TD_inversion_function(p, ds, 1, seed=3, model=m0)
    assert len(hist) == 6
    ctx = tt.context_for(ds)
    ch = tt.Chain(ctx, tt.chain_params(p, ds, seed=3, chain=1), m0)
    for k, m in enumerate(hist):
        ch.run(10)
        m2 = ch.model()
        m2.tS, m2.likelihood = ds.tS, ctx.likelihood_const
        assert same(m2, m), k
    ch.close()
