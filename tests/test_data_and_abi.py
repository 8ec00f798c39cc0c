"""Host-side logic that needs no GPU: data loading / slowness / segments vs the
oracle, the C ABI's exported symbols, and the chain's RNG / math / proposal /
acceptance logic (host hooks that run the same source the GPU kernel runs)."""
import ctypes
import math
import os
import re

import numpy as np
import pytest
from scipy import stats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rays381_fixture_shape(ds):
    m, n = ds.rayX.shape
    assert (m, n) == (131, 381)
    npts = (~np.isnan(ds.rayX)).sum(0)
    assert npts.sum() == 16845 and npts.min() == 10 and npts.max() == 131
    assert (npts == m).sum() == 46  # full-length rays


def test_interp1_matches_oracle(tt, orc):
    t = np.load(os.path.join(ROOT, "mcmc-in-tonga_amd", "data", "ak135f.npz"))
    zz = np.concatenate([np.linspace(-5, 700, 3001), t["depth"][:40], [3.0, 3.3, 10.0, 20.0, 35.0]])
    a = tt.interp1(t["depth"], t["vp"], zz)
    b = orc.interp1(t["depth"], t["vp"], zz)
    assert np.array_equal(a, b, equal_nan=True)
    # at a repeated depth the deeper layer's value applies (half-open intervals)
    assert tt.interp1(t["depth"], t["vp"], [3.0])[0] == 1.65


def test_segments_match_oracle(ds, orc):
    L, U = orc.segments(ds.rayX, ds.rayY, ds.rayZ, ds.U)
    assert np.array_equal(L, ds.rayL, equal_nan=True)
    assert np.array_equal(U, ds.rayU, equal_nan=True)


def test_synthetic_stress_rays_layout(tt):
    s = tt.synthetic_rays(50, seed=5)
    npts = (~np.isnan(s.rayX)).sum(0)
    assert np.all(npts >= 2)
    nl = (~np.isnan(s.rayL)).sum(0)
    assert np.array_equal(nl, npts - 1)


def test_reference_parameters_defaults(tt):
    p = tt.define_TDstructrure()
    assert (p.debug_prior, p.add_yVec, p.sig, p.zeta_scale, p.max_cells, p.min_cells) == (0, 1, 10, 50, 100, 5)
    assert (p.interp_style, p.prior, p.n_chains, p.n_iter, p.burn_in, p.keep_each) == (1, 1, 2, 1e3, 5e2, 1e1)


# ----------------------------------------------------------------- ABI ----
def declared_symbols():
    names = []
    for h in ("tdstar.h", "tdstar_testing.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b((?:td|tdt)_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol(tt):
    L = tt.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    from importlib import import_module
    _lib = import_module("mcmc_in_tonga_amd._lib")
    assert sorted(_lib.SIGNATURES) == syms  # the ctypes binding covers exactly the headers


def test_error_message_channel_without_gpu(tt):
    L = tt.lib()
    h = ctypes.c_void_p()
    rc = L.td_create(ctypes.byref(h), 0, None, None, None, None, None, 0, 1, None, None)
    assert rc == 1  # TD_ERR_ARG: m must be >= 1, checked before any HIP call
    assert b"m >= 1" in L.td_last_error(None)


# ------------------------------------------------- chain logic hooks ----
def philox(tt, ctr, key):
    L = tt.lib()
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    L.tdt_philox(c, k, o)
    return list(o)


def test_philox_known_answers(tt):
    # Random123 kat_vectors, philox4x32 10 rounds
    assert philox(tt, [0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert philox(tt, [0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert philox(tt, [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_deterministic_math(tt):
    L = tt.lib()
    rng = np.random.default_rng(0)
    xs = np.concatenate([10.0 ** rng.uniform(-300, 300, 2000), rng.uniform(1e-3, 10, 2000), [1.0, 2.0, 0.5, 1e-310]])
    for x in xs:
        assert abs(L.tdt_det_log(x) - math.log(x)) <= 4e-16 * max(1.0, abs(math.log(x)))
    for x in np.concatenate([rng.uniform(-700, 700, 3000), [0.0, -1e-9, 1e-9]]):
        e = math.exp(x)
        assert abs(L.tdt_det_exp(x) - e) <= 4e-16 * e
    assert L.tdt_det_exp(-800.0) == 0.0 and math.isinf(L.tdt_det_exp(800.0))


def test_normal_quantile(tt):
    L = tt.lib()
    ps = np.concatenate([np.linspace(1e-12, 1 - 1e-12, 4001), [1e-300, 0.5, 0.025, 0.975]])
    for p in ps:
        q = L.tdt_normal_quantile(p)
        r = stats.norm.ppf(p)
        assert abs(q - r) <= 1e-14 * max(1.0, abs(r)), p


def params(tt, **kw):
    prm = tt.define_TDstructrure().replace(**{k: v for k, v in kw.items() if k in ("max_cells", "min_cells", "prior",
                                                                                    "debug_prior")})
    return tt.chain_params(prm, None, seed=kw.get("seed", 3), chain=kw.get("chain", 1),
                           temperature=kw.get("temperature", 1.0))


def test_uniform_draws_and_action_mix(tt):
    L = tt.lib()
    out = (ctypes.c_double * 7)()
    u = np.empty((20000, 7))
    for i in range(20000):
        L.tdt_draws(99, 1, i + 1, out)
        u[i] = list(out)
    assert np.all((u > 0) & (u < 1))
    for j in range(7):  # each stream is U(0,1)
        assert stats.kstest(u[:, j], "uniform").pvalue > 1e-3
    acts = 1 + np.floor(u[:, 0] * 4).astype(int)
    counts = np.bincount(acts, minlength=5)[1:]
    assert stats.chisquare(counts).pvalue > 1e-3  # rand(1:4), TD_inversion_function.jl:72


def propose(tt, prm, it, cells, czeta_birth=0.0):
    L = tt.lib()
    out = (ctypes.c_double * 8)()
    c = [np.ascontiguousarray(a, dtype=np.float64) for a in cells]
    L.tdt_propose(ctypes.byref(prm), it, len(c[0]), *(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) for a in c),
                  czeta_birth, out)
    return list(out)


def test_proposals_follow_reference_branches(tt):
    prm = params(tt, max_cells=100, min_cells=5)
    model = tt.random_model(40, 4)
    xmin, xmax, ymin, ymax, zmin, zmax = tt.box()
    seen = set()
    for it in range(1, 3000):
        a, active, valid, idx, x, y, z, zeta = propose(tt, prm, it, model.cells(), czeta_birth=25.0)
        a = int(a)
        seen.add(a)
        assert active == 1
        if a == 1:  # birth: uniform site in the box, zetanew ~ N(czeta, 5)
            assert xmin <= x <= xmax and ymin <= y <= ymax and zmin <= z <= zmax
            assert valid == (0 < zeta < 50)
        elif a == 3:  # change: N(zeta_k, sig_zeta = 50*10/100)
            assert 0 <= idx < 40 and valid == (0 < zeta < 50)
        elif a == 4:  # move: N(site, 10% of the box), must stay inside
            assert valid == (xmin <= x <= xmax and ymin <= y <= ymax and zmin <= z <= zmax)
    assert seen == {1, 2, 3, 4}
    # at the bounds the birth / death branches are skipped (:77, :127)
    full = tt.random_model(100, 1)
    for it in range(1, 400):
        a, active, *_ = propose(tt, prm, it, full.cells())
        if int(a) == 1:
            assert active == 0
    low = tt.random_model(5, 1)
    for it in range(1, 400):
        a, active, *_ = propose(tt, prm, it, low.cells())
        if int(a) == 2:
            assert active == 0


@pytest.mark.parametrize("prior", [2, 3])
def test_proposal_validity_per_prior(tt, prior):
    """Birth/change zeta validity: normal -- always (:105-109, :201-204);
    exponential -- zeta > 0 (:111, :206)."""
    prm = params(tt, max_cells=100, min_cells=5, prior=prior)
    model = tt.random_model(40, 4)
    model.zeta[:] = 1.0  # near 0: changes often step below it
    n_invalid = 0
    for it in range(1, 3000):
        a, active, valid, idx, x, y, z, zeta = propose(tt, prm, it, model.cells(), czeta_birth=1.0)
        if int(a) in (1, 3):
            assert valid == (1 if prior == 2 else int(zeta > 0))
            n_invalid += valid == 0
    assert (n_invalid == 0) == (prior == 2)


def alpha_reference(action, N, phi, phi_n, czeta=0.0, zetanew=0.0, zeta_killed=0.0, zdn=0.0, T=1.0, prior=1):
    """TD_inversion_function.jl eqs. 14-17, restated in Python for the three
    priors (uniform :96-97,151-152,196; normal :107-108,160-162,202-203;
    exponential :113-114,166-168,207-208); 0 where the reference sets valid = 0
    or alpha = 0.  For change, zetanew is the new value, zeta_killed the old."""
    sig_zeta, zs = 50 * 10 / 100, 50
    d = (phi_n - phi) / (2 * T)
    s2p = math.sqrt(2 * math.pi)
    if action == 1:
        if prior == 1:
            if not (0 < zetanew < zs):
                return 0.0
            a = (N / (N + 1)) * ((sig_zeta * s2p) / zs) * math.exp(((czeta - zetanew) ** 2) / (2 * sig_zeta ** 2) - d)
        elif prior == 2:
            a = (N / (N + 1)) * (sig_zeta / zs) * \
                math.exp(-zetanew ** 2 / zs ** 2 + (czeta - zetanew) ** 2 / (2 * sig_zeta ** 2) - d)
        else:
            if not zetanew > 0:
                return 0.0
            a = (N / (N + 1)) * (s2p * sig_zeta / zs) * \
                math.exp(-zetanew / zs + (czeta - zetanew) ** 2 / (2 * sig_zeta ** 2) - d)
    elif action == 2:
        zk = zeta_killed
        if prior == 1:
            a = (N / (N - 1)) * (zs / (sig_zeta * s2p)) * math.exp(-((zk - zdn) ** 2) / (2 * sig_zeta ** 2) - d)
        elif prior == 2:
            a = (N / (N - 1)) * (zs / sig_zeta) * \
                math.exp(zk ** 2 / (2 * zs ** 2) - (zk - zdn) ** 2 / (2 * sig_zeta ** 2) - d)
        else:
            if not zdn > 0:
                return 0.0
            a = (N / (N - 1)) * (zs / (s2p * sig_zeta)) * \
                math.exp(zk / zs - (zk - zdn) ** 2 / (2 * sig_zeta ** 2) - d)
    elif action == 3:
        zo = zeta_killed
        if prior == 1:
            if not (0 < zetanew < zs):
                return 0.0
            a = math.exp(-d)
        elif prior == 2:
            a = math.exp((zo ** 2 - zetanew ** 2) / (2 * zs ** 2) - d)
        else:
            if not zetanew > 0:
                return 0.0
            a = math.exp((zo - zetanew) / zs - d)
    else:
        a = math.exp(-d)
    return min(1.0, a)


def test_acceptance_matches_reference_formulas(tt):
    L = tt.lib()
    rng = np.random.default_rng(7)
    for prior in (1, 2, 3):
        for T in (1.0, 3.0):
            prm = params(tt, temperature=T, prior=prior)
            for _ in range(3000):
                action = int(rng.integers(1, 5))
                N = int(rng.integers(6, 99))
                phi = rng.uniform(100, 900)
                phi_n = phi + rng.normal(0, 6)
                cz, zn, zk, zd = rng.uniform(-10, 60, 4) if prior != 1 else rng.uniform(0, 50, 4)
                a = alpha_reference(action, N, phi, phi_n, cz, zn, zk, zd, T, prior)
                u = rng.uniform()
                if abs(u - a) < 1e-12:
                    continue
                got = L.tdt_accept(ctypes.byref(prm), action, u, zn, N, phi, phi_n, cz, zk, zd)
                assert got == (1 if u < a else 0), (prior, action, a, u)



def test_decision_prefilter_is_sound(tt):
    """The device decides most proposals from the phi-free part of log alpha and one add (chain_logic.h
    decide_sure) before it evaluates the acceptance rule at the corners of its (phi, phi_n) brackets.  Its
    answer must be the rule's at every point of the bracket: checked on brackets of 1e-16 .. 1e-3
    relative width placed at random and straddling the rule's own threshold (found by bisection)."""
    L = tt.lib()
    rng = np.random.default_rng(11)
    decided = total = 0
    for prior in (1, 2, 3):
        for T in (1.0, 3.0):
            prm = params(tt, temperature=T, prior=prior)
            for _ in range(400):
                action = int(rng.integers(1, 5))
                N = int(rng.integers(6, 99))
                phi = rng.uniform(100, 900)
                cz, zn, zk, zd = rng.uniform(-10, 60, 4) if prior != 1 else rng.uniform(0, 50, 4)
                u = rng.uniform()
                acc = lambda pn, ph=phi: L.tdt_accept(ctypes.byref(prm), action, u, zn, N, ph, pn, cz, zk, zd)
                lo, hi = phi - 200.0, phi + 200.0  # the rule's threshold in phi_n, if inside
                if acc(lo) and not acc(hi):
                    for _ in range(80):
                        mid = 0.5 * (lo + hi)
                        lo, hi = (mid, hi) if acc(mid) else (lo, mid)
                centers = [lo, hi, phi + rng.normal(0, 6)]
                for ci, c in enumerate(centers):
                    for rel in (1e-16, 1e-12, 1e-9, 1e-6, 1e-3):
                        w = abs(c) * rel * rng.uniform(0.5, 2.0)
                        a, b = c - w * rng.uniform(), c + w * rng.uniform()
                        p_lo, p_hi = phi * (1 - rel * rng.uniform()), phi * (1 + rel * rng.uniform())
                        r = L.tdt_decide_sure(ctypes.byref(prm), action, u, zn, N, p_lo, p_hi, a, b, cz, zk, zd)
                        total += ci == 2
                        if r == 1:  # accepted at the bracket's worst corner, hence everywhere
                            decided += ci == 2
                            assert acc(b, p_lo) == 1 and acc(a, p_hi) == 1, (prior, action, c, rel)
                        elif r == -1:
                            decided += ci == 2
                            assert acc(a, p_hi) == 0 and acc(b, p_lo) == 0, (prior, action, c, rel)
    assert decided > 0.9 * total  # (brackets placed at random: nearly all decided without the corners)


def test_td_info_layout_matches_header():
    """td_info (include/tdstar.h) and the ctypes mirror agree: the ABI version and
    the struct's size (num_cus appended in ABI 2)."""
    import ctypes
    import re

    from mcmc_in_tonga_amd import _lib

    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "tdstar.h")).read()
    assert int(re.search(r"#define TDSTAR_ABI_VERSION (\d+)", hdr).group(1)) == 2
    assert [f for f, _ in _lib.TdInfo._fields_][-1] == "num_cus"
    assert ctypes.sizeof(_lib.TdInfo) == 4 + 4 + 8 * 4 + 8 + 32 + 4 + 4  # (tail padding to 8)
