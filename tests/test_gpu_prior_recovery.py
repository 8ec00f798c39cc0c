"""Prior recovery (the reference's own validation mode, debug_prior
= 1, plot_distribution.jl:67-80): the device chain, sampling the prior, must
reach the same distribution of (nCells, zeta, cell sites) as an INDEPENDENT
numpy restatement of the reference loop (oracle/chain_np.py: numpy PCG64
draws, none of the build's code).  The DEVICE and HOST engines share
chain_logic.h (Philox, AS241 quantile, index draw, alpha), so engine-vs-engine
equality cannot catch a bias there; this can.

K independent chains per sampler, each started from build_starting's
distribution (MCsub.jl:86-108) and run `ITERS` iterations; the states at that
iteration are independent across chains, so two-sample tests apply:
chi-square on the nCells histogram, Kolmogorov-Smirnov on the first cell's
zeta and x, the last cell's zeta and one uniformly chosen cell's zeta.  All draws are seeded,
so the outcome is deterministic (no flakes); the threshold p > 1e-4 per
test (15 tests: a family-wise false-alarm rate ~0.1 % for a correct sampler),
while a bias of a few percent in any of these distributions gives p << 1e-4
at K = 8192.
"""
import numpy as np
import pytest
from scipy import stats

from oracle import chain_np

pytestmark = pytest.mark.gpu

K, ITERS = 8192, 400


def nbins(a, b):
    edges = [5, 7, 9, 12, 15, 19, 24, 30, 38, 48, 60, 75, 101]
    ha = np.histogram(a, edges)[0]
    hb = np.histogram(b, edges)[0]
    return np.array([ha, hb])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("prior", [1, 2, 3])
def test_device_chain_recovers_prior_like_numpy_restatement(tt, prior):
    ds = tt.synthetic_rays(4, seed=1)  # geometry is never used in prior sampling (MCsub.jl:134-136)
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(debug_prior=1, prior=prior)
    chains = [tt.Chain(ctx, tt.chain_params(prm, None, seed=7000 + prior, chain=1 + k)) for k in range(K)]
    tt.run_batch(chains, ITERS)
    models = [c.model() for c in chains]
    for c in chains:
        c.close()
    ctx.close()
    n_dev = np.array([len(m.xCell) for m in models])
    z_dev = [m.zeta for m in models]
    x_dev = [m.xCell for m in models]
    n_np, z_np, x_np = chain_np.run(K, ITERS, tt.box(), prior=prior, seed=100 + prior)

    assert n_dev.min() >= 5 and n_dev.max() <= 100
    p_n = stats.chi2_contingency(nbins(n_dev, n_np))[1]
    pick = np.random.default_rng(prior)
    j_dev = [pick.integers(len(z)) for z in z_dev]
    j_np = [pick.integers(len(z)) for z in z_np]
    p_z0 = stats.ks_2samp([z[0] for z in z_dev], [z[0] for z in z_np]).pvalue
    p_zj = stats.ks_2samp([z[j] for z, j in zip(z_dev, j_dev)], [z[j] for z, j in zip(z_np, j_np)]).pvalue
    p_x0 = stats.ks_2samp([x[0] for x in x_dev], [x[0] for x in x_np]).pvalue
    # the last cell: born during the run in most chains (the birth proposal and alpha, :77-124)
    p_zl = stats.ks_2samp([z[-1] for z in z_dev], [z[-1] for z in z_np]).pvalue
    summary = dict(prior=prior, p_n=p_n, p_z0=p_z0, p_zj=p_zj, p_x0=p_x0, p_zl=p_zl, mean_n=(n_dev.mean(), n_np.mean()),
                   mean_z=(np.mean(np.concatenate(z_dev)), np.mean(np.concatenate(z_np))))
    print(summary)
    assert min(p_n, p_z0, p_zj, p_x0, p_zl) > 1e-4, summary
    if prior == 1:  # the uniform prior's support (:92, :195)
        assert all(np.all((z > 0) & (z < 50)) for z in z_dev)
    if prior == 3:
        assert all(np.all(z > 0) for z in z_dev)
    if prior == 2:
        assert any(np.any(z < 0) for z in z_dev)  # the normal prior reaches negative values
