"""The HIP code pinned to the reference's own output file, model.jld.

model.jld holds 100 saved Models of a 487-datum run (2 chains x 50) with
their ptS, tS, phi and likelihood (tests/golden/model_jld_kat.npz).  Its ray
geometry is not shipped, so the nearest search cannot be replayed; but every
device code path that turns a ptS into phi (MCsub.jl:169-172) can be fed the
reference's ptS and must return the reference's phi bit for bit:

  path 0  td_evaluate's chi^2 (the host adds the terms in k order where the
          ray-sum kernel put ptS)
  path 1  td_misfit's block-wide exact scan (k_chi2)
  path 2  the device chain's starting-state prefix sums (k_chi2_prefix)
  path 3  the device chain's proposal-time scan, from k0 = 0 and restarted
          at k0 = n/2 on path 2's prefix

and the likelihood a 487-ray context reports (MCsub.jl:179-182, Julia's
Base.sum association) must be the recorded 163765.04727246414.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIKELIHOOD_KAT = 163765.04727246414


@pytest.fixture(scope="module")
def kat_ctx(tt, kat):
    ds = tt.synthetic_rays(len(kat["tS"]), seed=487)  # any 487-ray geometry: only tS / allSig matter here
    ctx = tt.TdContext(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, kat["tS"], np.full(len(kat["tS"]), 0.2))
    yield ctx
    ctx.close()


def chi2(tt, ctx, ptS, path):
    out = np.zeros(2)
    p = np.ascontiguousarray(ptS, dtype=np.float64)
    tt._lib.check(tt.lib().tdt_chi2(ctx.h, p.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), path,
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), ctx.h)
    return out


@pytest.mark.parametrize("path", [0, 1, 2, 3])
def test_device_chi2_reproduces_model_jld_phi(tt, kat, kat_ctx, path):
    for k in range(len(kat["phi"])):
        out = chi2(tt, kat_ctx, kat["ptS"][k], path)
        assert out[0] == kat["phi"][k], (path, k, out[0], kat["phi"][k])
        if path == 3:
            assert out[1] == kat["phi"][k], (k, out[1], kat["phi"][k])


def test_context_likelihood_is_model_jld_value(tt, kat, kat_ctx):
    assert kat_ctx.likelihood_const == LIKELIHOOD_KAT
    assert np.all(kat["likelihood"] == LIKELIHOOD_KAT)
    # td_evaluate reports the same constant for any model (MCsub.jl:179-182 is model-independent)
    m = tt.random_model(40, 487)
    _, phi, lk, _ = kat_ctx.evaluate(m.cells())
    assert lk == LIKELIHOOD_KAT and np.isfinite(phi)


def test_evaluate_phi_is_chi2_of_its_ptS(tt, kat, kat_ctx, orc):
    """td_evaluate's phi equals the chi^2 code path-0 gives for its own ptS, and
    the oracle's sequential chi^2 of that ptS (pinned to model.jld above)."""
    for seed, ncell in ((1, 5), (2, 27), (3, 300)):
        m = tt.random_model(ncell, seed)
        ptS, phi, _, _ = kat_ctx.evaluate(m.cells())
        assert chi2(tt, kat_ctx, ptS, 0)[0] == phi
        assert orc.chi2(ptS, kat["tS"], np.full(len(ptS), 0.2)) == phi


def test_td_misfit_reproduces_model_jld(tt, kat, kat_ctx):
    """td_misfit (the public chi^2 of a given ptS: the reduction of a ray-sharded
    evaluate) returns the recorded phi and likelihood for all 100 records."""
    sig = np.full(len(kat["tS"]), 0.2)
    for k in range(len(kat["phi"])):
        phi, lk = kat_ctx.misfit(kat["ptS"][k], kat["tS"], sig)
        assert phi == kat["phi"][k] and lk == LIKELIHOOD_KAT, k
