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
