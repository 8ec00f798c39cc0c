"""GPU: the whole run of main_inversion.jl:11-18 on a small budget -- two
chains on the device engine, the posterior maps, and model.jld written in
JLD and read back to the same saved models (values and aliasing)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_main_inversion_writes_model_jld(tt, ds, tmp_path):
    if not tt.jld.available():
        pytest.skip("no interpreter with h5py")
    prm = tt.define_TDstructrure().replace(n_chains=2, n_iter=3000, burn_in=1000, keep_each=200, print_each=0)
    out = tmp_path / "model.jld"
    models, maps = tt.main_inversion(prm, ds, out=str(out))
    assert [len(c) for c in models] == [10, 10]
    assert maps and all(np.isfinite(v["mean"]).any() for v in maps.values())
    back = tt.jld.load(out)
    for ca, cb in zip(models, back):
        for a, b in zip(ca, cb):
            for k in ("xCell", "yCell", "zCell", "zeta", "ptS", "tS"):
                assert np.array_equal(getattr(a, k), getattr(b, k)), k
            assert a.phi == b.phi and a.nCells == b.nCells and a.likelihood == b.likelihood


def test_chains_run_concurrently_as_pmap(tt, ds):
    """main_inversion's chains (main_inversion.jl:15 pmap) share one
    td_chain_run_batch launch per stretch, and every chain's model_hist is
    the one TD_inversion_function gives it alone."""
    prm = tt.define_TDstructrure().replace(n_chains=3, n_iter=2000, burn_in=500, keep_each=100, print_each=500)
    ctx = tt.context_for(ds)
    ctx.timing(enable=True, reset=True)
    together = tt.run_chains(prm, ds, [1, 2, 3])
    launches3, _ = ctx.timing(kernel="chain_run")
    ctx.timing(enable=True, reset=True)
    alone = [tt.TD_inversion_function(prm, ds, 1)]
    launches1, _ = ctx.timing(kernel="chain_run")
    ctx.timing(enable=False)
    alone += [tt.TD_inversion_function(prm, ds, c) for c in (2, 3)]
    assert [len(h) for h in together] == [len(h) for h in alone] and len(alone[0]) >= 10
    for ha, hb in zip(together, alone):
        for a, b in zip(ha, hb):
            assert a.phi == b.phi and np.array_equal(a.zeta, b.zeta) and np.array_equal(a.xCell, b.xCell)
            assert np.array_equal(a.ptS, b.ptS)
    assert launches3 == launches1  # three chains, one launch per stretch (as many as one chain alone)
