"""Pin the CPU oracle against the reference's own output file (model.jld).

model.jld (2 chains x 50 saved Models, 487 data, written by the reference run)
is the only known-answer data the reference ships.  It pins:
  * the chi^2 reduction MCsub.jl:169-172 (sequential, bit-exact),
  * the likelihood expression MCsub.jl:179 and, through it, the association
    of Julia's Base.sum that the oracle and the GPU kernels use.
"""
import math

import numpy as np
import pytest

from oracle import oracle_np


def test_chi2_bit_exact_all_models(orc, kat):
    sig = np.full(len(kat["tS"]), 0.2)  # the run's allSig (every record reproduces with 0.2)
    for k in range(len(kat["phi"])):
        assert orc.chi2(kat["ptS"][k], kat["tS"], sig) == kat["phi"][k], k
        assert oracle_np.chi2(kat["ptS"][k], kat["tS"], sig) == kat["phi"][k], k


def test_likelihood_bit_exact_all_models(orc, kat):
    sig = np.full(len(kat["tS"]), 0.2)
    lk = orc.likelihood(sig)
    assert np.all(kat["likelihood"] == lk)
    assert oracle_np.likelihood(sig) == lk
    # and it is NOT the strictly sequential sum: the association matters
    c = -math.log(0.2 * math.sqrt(2 * math.pi)) * len(sig)
    seq = 0.0
    for _ in range(len(sig)):
        seq += c
    assert seq != lk


def test_sum_association_is_identified_uniquely(kat):
    """Only 8 lanes x 4 interleaved accumulators reproduces the recorded value."""
    target = kat["likelihood"][0]
    c = -math.log(0.2 * math.sqrt(2 * math.pi)) * 487
    hits = [(vf, ic) for vf in (1, 2, 4, 8) for ic in (1, 2, 4, 8)
            if oracle_np.julia_sum([c] * 487, vf, ic) == target]
    assert hits == [(8, 4)]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 15, 16, 17, 33, 34, 35, 64, 66, 130, 131, 1024, 1025, 1026, 2049, 5000])
def test_julia_sum_c_matches_numpy_restatement(orc, n):
    rng = np.random.default_rng(n)
    a = rng.standard_normal(n) * 10.0 ** rng.integers(-3, 4, n)
    assert orc.julia_sum(a) == oracle_np.julia_sum(a)


def test_kat_cells_are_well_formed(kat):
    off = kat["cell_off"]
    assert len(off) == len(kat["phi"]) + 1
    ncell = np.diff(off)
    assert np.all(ncell == kat["nCells"])
    assert ncell.min() >= 5 and ncell.max() <= 100  # min/max_cells (define_TDstructure.jl:50)
    assert np.all((kat["zeta"] > 0) & (kat["zeta"] < 50))  # uniform prior bounds
