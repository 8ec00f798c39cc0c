"""GPU: the exact sequential sums of exact_sum.h behind chi^2 -- the
block-wide one (long ray lists) and the one-wave one (the chain's tails) --
must equal the strictly left-to-right FP64 loop of MCsub.jl:170-172 bit for
bit whenever they claim success, and claim success on realistic data (the
one-wave sum always does).  Reference: a Python loop of IEEE-754 double adds
(the same operation sequence as the Julia loop)."""
import ctypes
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


WAVE_FALLBACKS = []  # chunks of the one-wave sum that took its slow path, per call


def seq(terms, c0):
    out, c = [], c0
    for t in terms:
        c = c + float(t)
        out.append(c)
    return np.array(out)


def run(tt, terms, c0, wave=False):
    terms = np.ascontiguousarray(terms, dtype=np.float64)
    pre = np.zeros(len(terms))
    ce = ctypes.c_double()
    fast = ctypes.c_int(1)
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    if wave:
        fb = ctypes.c_int()
        assert tt.lib().tdt_wave_seq_sum(0, P(terms), len(terms), float(c0), P(pre), ctypes.byref(ce),
                                         ctypes.byref(fb)) == 0
        WAVE_FALLBACKS.append(fb.value)
    else:
        assert tt.lib().tdt_exact_sum(0, P(terms), len(terms), float(c0), P(pre), ctypes.byref(ce),
                                      ctypes.byref(fast)) == 0
    return bool(fast.value), pre, ce.value


def check(tt, terms, c0):
    """Both sums; returns whether the block-wide one took its fast path."""
    want = seq(terms, c0)
    for wave in (False, True):
        fast, pre, ce = run(tt, terms, c0, wave)
        if fast:
            same = (pre == want) | (np.isnan(pre) & np.isnan(want))
            bad = np.nonzero(~same)[0]
            assert len(bad) == 0, (wave, bad[:5], pre[bad[:5]], want[bad[:5]])
            assert ce == want[-1] or (np.isnan(ce) and np.isnan(want[-1])), wave
        assert fast or not wave
        if not wave:
            block_fast = fast
    return block_fast


def test_chi2_like_terms(tt):
    """(ptS - tS)^2 / sig^2 of a 10k-ray model: the case the kernels meet."""
    rng = np.random.default_rng(0)
    hits = 0
    for trial in range(6):
        n = [2048, 5000, 10000, 10000, 20000, 3000][trial]
        d = rng.normal(0, 0.3, n)
        sig = rng.uniform(0.04, 0.6, n)
        terms = ((d * d) * 1.0) / (sig * sig)
        c0 = 0.0 if trial % 2 == 0 else float(seq(rng.exponential(1.0, 50), 0.0)[-1])
        hits += check(tt, terms, c0)
    assert hits == 6


@pytest.mark.parametrize("cnt", [1, 2, 63, 64, 65, 1023, 1024, 1025, 4097])
def test_sizes(tt, cnt):
    rng = np.random.default_rng(cnt)
    fast = 0
    for trial in range(4):
        terms = rng.exponential(rng.choice([1e-3, 1.0, 40.0]), cnt) * rng.choice([1.0, 1e3], cnt)
        fast += check(tt, terms, 0.0 if trial % 2 == 0 else float(rng.uniform(0, 500)))
    assert fast >= 3


def test_adversarial(tt):
    # exact halfway terms: ties-to-even decided by the running sum's parity
    check(tt, np.full(3000, 2.0 ** -53), 1.0)
    check(tt, np.full(3000, 2.0 ** -53), 1.0 + 2.0 ** -52)
    check(tt, np.full(3000, 3 * 2.0 ** -53), 1.0)
    rng = np.random.default_rng(5)
    half = (rng.integers(1, 9, 4000) * 2 + 1) * 2.0 ** -54  # odd multiples of half an ulp of 1
    assert check(tt, half, 1.0)
    # a binade crossing at every term (more segments than the scan keeps)
    check(tt, 2.0 ** np.arange(300, dtype=np.float64) % 1e300, 1.0)
    # zeros, a zero start, huge and tiny terms mixed
    check(tt, np.zeros(2000), 0.0)
    check(tt, np.concatenate([[0.0, 0.0, 1e-300, 5.0, 0.0, 1e200, 3.0], rng.exponential(1.0, 2000)]), 0.0)
    check(tt, np.concatenate([[1e-310, 2e-310], rng.exponential(1.0, 2000)]), 0.0)
    for _ in range(10):
        check(tt, np.exp(rng.uniform(-40, 40, 3000)), float(rng.uniform(0, 10)))
    # sums landing exactly on powers of two
    check(tt, np.concatenate([[0.5, 0.25, 0.25, 1.0, 2.0, 4.0 - 2.0 ** -50, 2.0 ** -50], np.ones(2000)]), 0.0)


def test_wave_sum_binade_walk(tt):
    """The chain's case: ~381 chi^2-like terms from every starting prefix
    (zero, small, one binade below the top), with NaN/inf/negative terms."""
    rng = np.random.default_rng(11)
    base = rng.exponential(36.0, 381)
    del WAVE_FALLBACKS[:]
    for k0 in (0, 1, 17, 190, 380):
        c0 = float(seq(base[:k0], 0.0)[-1]) if k0 else 0.0
        check(tt, base[k0:], c0)
    assert WAVE_FALLBACKS == [0, 0, 0, 0, 0], WAVE_FALLBACKS
    check(tt, np.concatenate([base[:50], [np.inf], base[50:80]]), 3.0)
    check(tt, np.concatenate([base[:50], [-2.5], base[50:80]]), 3.0)
    check(tt, np.concatenate([base[:70], [np.nan], base[70:90]]), 3.0)
    check(tt, np.full(130, 2.0 ** 60), 2.0 ** 62)            # huge, exact ties
    check(tt, rng.exponential(1e-300, 200), 1e-310)            # subnormal start


def delta_run(tt, terms, old_prefix, changed, c0):
    terms = np.ascontiguousarray(terms, dtype=np.float64)
    old_prefix = np.ascontiguousarray(old_prefix, dtype=np.float64)
    changed = np.ascontiguousarray(changed, dtype=np.int32)
    pre = np.zeros(len(terms))
    ce = ctypes.c_double()
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    assert tt.lib().tdt_wave_delta_sum(0, P(terms), P(old_prefix), changed.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       len(terms), float(c0), P(pre), ctypes.byref(ce)) == 0
    return pre, ce.value


def delta_check(tt, old_terms, new_terms, c0):
    changed = (old_terms != new_terms).astype(np.int32)
    old_prefix = seq(old_terms, c0)
    want = seq(new_terms, c0)
    pre, ce = delta_run(tt, new_terms, old_prefix, changed, c0)
    same = (pre == want) | (np.isnan(pre) & np.isnan(want))
    bad = np.nonzero(~same)[0]
    assert len(bad) == 0, (bad[:5], pre[bad[:5]], want[bad[:5]])
    assert ce == want[-1] or (np.isnan(ce) and np.isnan(want[-1]))


def test_delta_sum_chain_like(tt):
    """The chain's case: a tail of chi^2 terms of which a few changed."""
    rng = np.random.default_rng(21)
    for trial in range(40):
        n = int(rng.choice([1, 5, 63, 64, 65, 381, 1000, 5000]))
        old = rng.exponential(36.0, n)
        new = old.copy()
        idx = rng.choice(n, size=min(n, int(rng.integers(1, 30))), replace=False)
        new[idx] = old[idx] * rng.uniform(0.2, 3.0, len(idx))
        c0 = float(rng.choice([0.0, 1.0, 3000.0, 8191.9, 8192.0, 1e5]))
        delta_check(tt, old, new, c0)


def test_delta_sum_adversarial(tt):
    rng = np.random.default_rng(22)
    base = rng.exponential(36.0, 600)
    # ties everywhere (terms with a set bit just below the unit), offsets odd and even
    ties = (rng.integers(1, 9, 600) * 2 + 1) * 2.0 ** -34
    for d in (2.0 ** -38, 3 * 2.0 ** -38, 1.0, -0.5, 1e-3):
        new = ties.copy()
        new[0] += d
        delta_check(tt, ties, new, 5000.0)
    # the new sum crosses binades the old one does not (and back)
    new = base.copy()
    new[3] += 9000.0
    delta_check(tt, base, new, 100.0)
    new = base.copy()
    new[3] = 0.0
    delta_check(tt, base, new, 8100.0)
    # huge relative changes (inexact offsets), zeros, NaN / inf terms
    new = base.copy()
    new[5] = 1e12
    delta_check(tt, base, new, 0.0)
    new = base.copy()
    new[[7, 300]] = [np.inf, 1.0]
    delta_check(tt, base, new, 10.0)
    new = base.copy()
    new[9] = np.nan
    delta_check(tt, base, new, 10.0)
    z = np.zeros(300)
    new = z.copy()
    new[100] = 5.0
    delta_check(tt, z, new, 0.0)
    # every term changed / none changed
    delta_check(tt, base, base * 1.0000001, 50.0)
    delta_check(tt, base, base.copy(), 50.0)


# ---- the chain's chi^2 walk (exact_sum.h delta_marks / delta_walk / delta_remark / delta_commit) ----
def block_check(tt, old_terms, new_terms, k0=None):
    """old/new terms over the whole ray list (C_{-1} = 0); they may differ only
    from k0 on.  The walk must give the strictly sequential new partial sums."""
    old_terms = np.ascontiguousarray(old_terms, dtype=np.float64)
    new_terms = np.ascontiguousarray(new_terms, dtype=np.float64)
    n = len(old_terms)
    diff = (old_terms != new_terms) & ~(np.isnan(old_terms) & np.isnan(new_terms))
    changed = diff.astype(np.int32)
    if k0 is None:
        k0 = int(np.argmax(diff)) if diff.any() else n
    assert not diff[:k0].any()
    old_prefix = np.array(list(itertools.accumulate(old_terms.tolist())), dtype=np.float64)
    want = np.array(list(itertools.accumulate(new_terms.tolist())), dtype=np.float64)
    pre = np.zeros(n)
    ce = ctypes.c_double()
    ev = ctypes.c_int64()
    ok = ctypes.c_int32()
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    assert tt.lib().tdt_block_delta_sum(0, P(new_terms), P(old_terms), P(old_prefix),
                                        changed.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), k0, n, P(pre),
                                        ctypes.byref(ce), ctypes.byref(ev), ctypes.byref(ok)) == 0
    assert ok.value == 1, "event words kept across the proposal differ from the new state's"
    same = (pre == want) | (np.isnan(pre) & np.isnan(want))
    bad = np.nonzero(~same)[0]
    assert len(bad) == 0, (k0, bad[:5], pre[bad[:5]], want[bad[:5]])
    end = want[-1] if k0 < n else (want[k0 - 1] if k0 > 0 else 0.0)
    assert ce.value == end or (np.isnan(ce.value) and np.isnan(end)), (ce.value, end)
    return ev.value


def test_block_delta_chain_like(tt):
    """The chain's case at the 381-ray and 10k-ray sizes: a few changed rays."""
    rng = np.random.default_rng(31)
    for trial in range(60):
        n = int(rng.choice([1, 2, 63, 64, 65, 381, 1000, 4097, 10000]))
        old = rng.exponential(float(rng.choice([1.0, 36.0, 1e-3])), n)
        new = old.copy()
        idx = rng.choice(n, size=min(n, int(rng.integers(1, 40))), replace=False)
        new[idx] = old[idx] * rng.uniform(0.2, 3.0, len(idx))
        ev = block_check(tt, old, new)
        if n >= 1000:
            assert ev < 200, ev  # O(events): the changed terms and a few binade changes


def test_block_delta_adversarial(tt):
    rng = np.random.default_rng(32)
    base = rng.exponential(36.0, 3000)
    # ties everywhere (odd and even offsets), against a large starting sum
    ties = np.concatenate([[5000.0], (rng.integers(1, 9, 2999) * 2 + 1) * 2.0 ** -34])
    for d in (2.0 ** -38, 3 * 2.0 ** -38, 1.0, -0.5, 1e-3):
        new = ties.copy()
        new[1] += d
        block_check(tt, ties, new)
    # the new sum crosses binades the old one does not (and back), offsets near powers of two
    for k, v in ((3, 9000.0), (3, 0.0), (40, 1e-9), (2000, 7.5e4)):
        new = base.copy()
        new[k] = v
        block_check(tt, base, new)
    near = np.concatenate([[8191.0], np.full(500, 2.0 ** -10)])
    new = near.copy()
    new[0] = 8191.5
    block_check(tt, near, new)
    # huge relative changes, zeros, NaN / inf terms
    for k, v in ((5, 1e12), (7, np.inf), (9, np.nan), (9, -1.0)):
        new = base.copy()
        new[k] = v
        block_check(tt, base, new)
    z = np.zeros(300)
    new = z.copy()
    new[100] = 5.0
    block_check(tt, z, new)
    # every term changed (dense events: the term-by-term path), none changed (empty tail)
    block_check(tt, base, base * 1.0000001)
    block_check(tt, base, base.copy())
    # more events than the segment table holds (materialised into the copy buffer)
    new = base.copy()
    new[::7] *= 1.5
    block_check(tt, base, new)
    # tiny sums: binade changes at nearly every term
    tiny = rng.exponential(1e-300, 2000)
    new = tiny.copy()
    new[10] *= 2
    block_check(tt, tiny, new)
    # a tail start k0 before the first changed term (the chain's k0 is the first changed ray)
    new = base.copy()
    new[1500] += 1.0
    block_check(tt, base, new, k0=1000)
    block_check(tt, base, base.copy(), k0=0)


@pytest.mark.parametrize("n", [20000, 65536])
def test_block_delta_long(tt, n):
    rng = np.random.default_rng(n)
    old = rng.exponential(1.3, n)
    new = old.copy()
    idx = rng.choice(n, size=16, replace=False)
    new[idx] = rng.exponential(1.3, 16)
    assert block_check(tt, old, new) < 200
