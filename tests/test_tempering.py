"""Parallel-tempering exchange: swap decisions, the allgather
over torch.distributed (gloo, world_size 2, CPU), and that a tempered ladder
of toy chains still samples the right cold distribution.  The GPU chains use
the same TemperingLadder (tests/test_gpu_chain.py::test_tempering_ladder_*)."""
import json
import math
import os
import socket

import numpy as np
import pytest

import tonga

tt = tonga.load()
from mcmc_in_tonga_amd import tempering  # noqa: E402


class ToyChain:
    """1-D Metropolis chain with phi(x) = x^2: targets exp(-x^2 / (2T)) = N(0, T)."""

    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)
        self.x = 3.0
        self.T = 1.0
        self.samples = []

    def set_temperature(self, T):
        self.T = T

    def run(self, k):
        for _ in range(k):
            xn = self.x + self.rng.normal() * 1.5
            d = (xn * xn - self.x * self.x) / (2 * self.T)
            if d <= 0 or math.log(self.rng.random()) < -d:
                self.x = xn

    def stats(self):
        return {"phi": self.x * self.x}


def test_ladder_is_geometric():
    t = tempering.geometric_ladder(4, 8.0)
    assert t[0] == 1.0 and abs(t[-1] - 8.0) < 1e-12
    assert np.allclose(t[1:] / t[:-1], 2.0)
    assert list(tempering.geometric_ladder(1)) == [1.0]


def test_swap_rule():
    temps = tempering.geometric_ladder(4, 8.0)
    # a hotter replica with a lower misfit always moves down (log alpha > 0)
    lv, tried, acc = tempering.decide_swaps([100.0, 10.0, 5.0, 1.0], [0, 1, 2, 3], temps, rnd=0, seed=1)
    assert list(lv) == [1, 0, 3, 2] and list(tried) == [1, 0, 1] and list(acc) == [1, 0, 1]
    # odd rounds try the (1,2) pair only
    lv, tried, _ = tempering.decide_swaps([1.0, 5.0, 10.0, 100.0], [0, 1, 2, 3], temps, rnd=1, seed=1)
    assert list(tried) == [0, 1, 0]
    # log alpha = (phi_a - phi_b)(1/2T_a - 1/2T_b)
    assert tempering.swap_log_alpha(3.0, 1.0, 1.0, 2.0) == pytest.approx(2.0 * (0.5 - 0.25))
    # always a permutation, deterministic in (round, seed)
    rng = np.random.default_rng(0)
    lv = np.arange(6)
    for r in range(50):
        phis = rng.uniform(0, 50, 6)
        a, _, _ = tempering.decide_swaps(phis, lv, tempering.geometric_ladder(6), r, 7)
        b, _, _ = tempering.decide_swaps(phis, lv, tempering.geometric_ladder(6), r, 7)
        assert np.array_equal(a, b) and sorted(a) == list(range(6))
        lv = a


def test_swap_acceptance_frequency():
    temps = np.array([1.0, 2.0])
    la = tempering.swap_log_alpha(1.0, 3.0, 1.0, 2.0)  # = -0.5
    hits = sum(tempering.decide_swaps([1.0, 3.0], [0, 1], temps, r, 3)[2][0] for r in range(0, 8000, 2))
    assert abs(hits / 4000 - math.exp(la)) < 0.03


def test_cold_replica_samples_posterior():
    chains = [ToyChain(s) for s in range(4)]
    lad = tempering.TemperingLadder(chains, tmax=16.0, seed=5)
    cold = []
    for r in range(6000):
        lad.step(2)
        j = lad.cold_local()
        cold.append(chains[j].x)
    cold = np.array(cold[500:])
    assert abs(np.mean(cold)) < 0.15
    assert abs(np.var(cold) - 1.0) < 0.15  # N(0, T=1)
    assert all(0.05 < r < 0.95 for r in lad.swap_rates())


def _worker(rank, world, port, outdir, rounds):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    chains = [ToyChain(100 + rank * 2 + j) for j in range(2)]
    lad = tempering.TemperingLadder(chains, tempering.Exchange(dist, "cpu"), tmax=8.0, seed=9)
    trace = []
    for _ in range(rounds):
        phis = lad.step(3)
        trace.append([list(map(float, phis)), list(map(int, lad.levels))])
    with open(os.path.join(outdir, "r%d.json" % rank), "w") as f:
        json.dump({"trace": trace, "temps": [c.T for c in chains]}, f)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_matches_single_process(tmp_path):
    import torch.multiprocessing as mp

    rounds = 40
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), rounds), nprocs=2, join=True)
    r0 = json.load(open(tmp_path / "r0.json"))
    r1 = json.load(open(tmp_path / "r1.json"))
    assert r0["trace"] == r1["trace"]  # every rank saw the same gather and made the same swaps
    # the same 4 replicas in one process (replica g = rank*2 + j, same seeds)
    chains = [ToyChain(100 + g) for g in range(4)]
    lad = tempering.TemperingLadder(chains, tmax=8.0, seed=9)
    for k in range(rounds):
        phis = lad.step(3)
        assert list(map(float, phis)) == r0["trace"][k][0]
        assert list(map(int, lad.levels)) == r0["trace"][k][1]
    assert [c.T for c in chains] == r0["temps"] + r1["temps"]


def test_native_swap_step_is_decide_swaps(tt):
    """td_swap_decide (the library's swap step, which td_rounds_temper runs
    between resident rounds) makes decide_swaps' decisions bit for bit: the
    same SplitMix64 uniforms, the same log alpha, the host libm log -- over
    random ladders, levels and phis, both round parities, and phis that make
    log alpha 0, +-inf or NaN."""
    import ctypes

    from importlib import import_module

    tp = import_module(tt.__name__ + ".tempering")
    L = tt.lib()
    rng = np.random.default_rng(5)
    P64 = ctypes.POINTER(ctypes.c_int64)
    PD = ctypes.POINTER(ctypes.c_double)
    for trial in range(3000):
        R = int(rng.integers(1, 12))
        temps = tp.geometric_ladder(R, float(rng.uniform(1.5, 20.0)))
        levels = rng.permutation(R).astype(np.int64)
        phis = rng.normal(6000.0, float(rng.choice([1.0, 30.0, 3000.0])), R)
        if trial % 7 == 0 and R > 1:
            phis[int(rng.integers(0, R))] = (np.inf, -np.inf, np.nan, phis[0])[trial % 4]
        rnd, seed = int(rng.integers(0, 1 << 40)), int(rng.integers(0, 1 << 62))
        want, wt, wa = tp.decide_swaps(phis, levels, temps, rnd, seed)
        got = np.empty(R, dtype=np.int64)
        t = np.zeros(max(R - 1, 1), dtype=np.int64)
        a = np.zeros(max(R - 1, 1), dtype=np.int64)
        rc = L.td_swap_decide(R, phis.ctypes.data_as(PD), levels.ctypes.data_as(P64), temps.ctypes.data_as(PD), rnd,
                              ctypes.c_uint64(seed), got.ctypes.data_as(P64), t.ctypes.data_as(P64),
                              a.ctypes.data_as(P64))
        assert rc == 0
        assert np.array_equal(got, want), (trial, R, rnd)
        assert np.array_equal(t[:R - 1], wt) and np.array_equal(a[:R - 1], wa)
    bad = np.array([0, 0, 1], dtype=np.int64)  # not a permutation: refused
    out = np.empty(3, dtype=np.int64)
    ph = np.zeros(3)
    tl = tp.geometric_ladder(3)
    assert L.td_swap_decide(3, ph.ctypes.data_as(PD), bad.ctypes.data_as(P64), tl.ctypes.data_as(PD), 0,
                            ctypes.c_uint64(1), out.ctypes.data_as(P64), None, None) != 0


def test_resident_rounds_under_a_gpu_collective():
    """Resident rounds (one spinning launch) also when the gather is an RCCL
    collective: the launch has a hardware queue of its own (a CU-masked
    stream), so the collective's kernels are not held back behind it
    (tests/test_gpu_chain.py::test_resident_rounds_do_not_hold_back_other_streams).
    Device swaps need one rank or the library's communicator."""

    class DeviceStandIn(ToyChain):
        h, ctx = 1, "ctx"

        class params:
            engine = 0

    class FakeDist:
        def __init__(self, world):
            self.w = world

        def get_world_size(self):
            return self.w

        def get_rank(self):
            return 0

    chains = [DeviceStandIn(1), DeviceStandIn(2)]
    assert tempering.TemperingLadder(chains).resident
    assert tempering.TemperingLadder(chains, exchange=tempering.Exchange(FakeDist(2), "cpu")).resident
    assert tempering.TemperingLadder(chains, exchange=tempering.Exchange(FakeDist(2), "cuda:0")).resident
    assert not tempering.TemperingLadder(chains, resident=False).resident
    assert tempering.TemperingLadder(chains, device_swaps=True).device_swaps
    assert not tempering.TemperingLadder(chains, exchange=tempering.Exchange(FakeDist(2), "cuda:0"),
                                         device_swaps=True).device_swaps  # (no communicator)
    assert not tempering.TemperingLadder(chains, resident=False, device_swaps=True).device_swaps


def test_round_trip_counting():
    """mixing(): a replica's 0 -> top -> 0 journey is one round trip; the
    up-fraction histogram labels a visit by the last extreme the replica saw."""
    chains = [ToyChain(s) for s in range(3)]
    lad = tempering.TemperingLadder(chains, tmax=4.0, seed=1)
    # replica 0 climbs to the top and back, replica 2 goes down to 0 and back up (no trip yet)
    seq = [[1, 0, 2], [2, 0, 1], [2, 1, 0], [1, 2, 0], [0, 2, 1]]
    for lv in seq:
        lad._observe(np.array(lv))
        lad.rnd += 1
    m = lad.mixing()
    assert list(lad.trips) == [1, 0, 0] and m["round_trips"] == 1 and m["rounds_per_round_trip"] == 5.0
    assert m["up_fraction"][0] == 1.0 and m["up_fraction"][2] == 0.0


def test_cold_replica_ladder_makes_round_trips():
    chains = [ToyChain(s) for s in range(4)]
    lad = tempering.TemperingLadder(chains, tmax=16.0, seed=5)
    for _ in range(3000):
        lad.step(2)
    m = lad.mixing()
    assert m["round_trips"] > 10
    f = [x for x in m["up_fraction"]]
    assert f[0] == 1.0 and f[-1] == 0.0 and all(a >= b - 0.1 for a, b in zip(f, f[1:]))
