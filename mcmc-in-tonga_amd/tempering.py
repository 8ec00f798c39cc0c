"""Parallel tempering across chains -- the one exchange step of
the multi-GPU path.

The reference runs independent chains (``pmap`` over ``1:n_chains``,
main_inversion.jl:15); each targets exp(-phi/2) times the prior
(TD_inversion_function.jl:95-268).  A tempered replica at temperature T
targets exp(-phi/(2T)) (``td_chain_params.temperature``).  Every ``K``
proposals the replicas exchange temperatures -- never models:

  1. every rank contributes (phi, level) of each local replica;
     ``allgather`` over torch.distributed (RCCL over xGMI on the GPU box,
     gloo in the CPU tests) -- 16 B per replica, latency-bound;
  2. every rank decides the SAME swaps from the gathered vector: in round r
     the adjacent level pairs (l, l+1) with l = r mod 2 are tried with
     u ~ U(0,1), a SplitMix64 hash of (seed, r, l), and accepted when
     log u < (phi_a - phi_b) * (1/(2 T_a) - 1/(2 T_b)) (a at level l, b at
     level l+1: detailed balance for pi_T(m) ~ exp(-phi(m) / (2T))), log =
     chain_logic.h's det_log everywhere (chain_logic.h swap_accept);
  3. each rank sets the new temperature of its replicas
     (``td_chain_set_temperature``) and continues.

Replicas = ranks x chains per rank, so one GPU may hold several (global
replica id g = rank * local + j).  The decision is a pure function of the
gathered vector, the round and the seed (``decide_swaps``), so it is tested
without any GPU (tests/test_tempering.py)."""
import hashlib
import time

import numpy as np


def geometric_ladder(nrep, tmax=8.0):
    """T_l = tmax ** (l / (nrep - 1)), l = 0..nrep-1 (T_0 = 1: the posterior)."""
    if nrep <= 1:
        return np.ones(max(nrep, 1))
    return np.array([float(tmax) ** (l / (nrep - 1)) for l in range(nrep)])


_M64 = 0xFFFFFFFFFFFFFFFF


def _mix64(x):
    """SplitMix64's finaliser (a bijection of 64-bit words with full avalanche)."""
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _uniform(seed, rnd, level):
    """u in (0, 1), a pure function of (seed, round, level): two SplitMix64
    rounds over the key, then (k + 1/2) / 2^52 of the top 52 bits (53 bits
    could round (2^53 - 1) + 1/2 up to exactly 1).  A few
    integer operations (a numpy Philox Generator per draw cost ~25 us, a third
    of a tempering round at 8 replicas x 10 proposals)."""
    x = _mix64((int(seed) * 0x9E3779B97F4A7C15 + int(rnd)) & _M64)
    x = _mix64((x + int(level) * 0xD1B54A32D192ED03 + 1) & _M64)
    return ((x >> 12) + 0.5) / 4503599627370496.0


def _det_log(u):
    """The deterministic log of chain_logic.h (tdt_det_log): the function the
    library's td_swap_decide and the exchange kernel decide with, so every
    side makes the same swap bit for bit (a libm log may differ by an ulp)."""
    from ._lib import lib

    return lib().tdt_det_log(float(u))


def swap_log_alpha(phi_a, phi_b, t_a, t_b):
    return (phi_a - phi_b) * (1.0 / (2.0 * t_a) - 1.0 / (2.0 * t_b))


def decide_swaps(phis, levels, temps, rnd, seed):
    """New level of every replica after round ``rnd``.

    phis[g], levels[g]: gathered over all replicas; temps[l]: the ladder.
    Returns (new_levels, tried, accepted) -- tried/accepted per level pair l
    (index l = pair (l, l+1))."""
    lv = [int(v) for v in levels]  # plain Python on a handful of replicas: ~5x faster than numpy here
    R = len(lv)
    owner = [0] * R
    for g, l in enumerate(lv):
        owner[l] = g  # replica currently at each level
    tried = [0] * max(R - 1, 0)
    acc = [0] * max(R - 1, 0)
    for l in range(int(rnd) % 2, R - 1, 2):
        a, b = owner[l], owner[l + 1]
        tried[l] += 1
        la = swap_log_alpha(float(phis[a]), float(phis[b]), float(temps[l]), float(temps[l + 1]))
        u = _uniform(seed, rnd, l)
        if la >= 0.0 or _det_log(u) < la:
            lv[a], lv[b] = l + 1, l
            owner[l], owner[l + 1] = b, a
            acc[l] += 1
    levels, tried, acc = (np.array(x, dtype=np.int64) for x in (lv, tried, acc))
    return levels, tried, acc


class NativeComm:
    """An RCCL communicator of the job's ranks in libtdstar (td_comm_*,
    include/tdstar.h): what ``TemperingLadder.run`` hands to the exchange
    rounds (td_rounds_exchange), whose allgathers the library issues itself,
    each waiting on a flag the resident kernel raises -- no host in the loop.
    ``from_dist`` ships rank 0's id through torch.distributed; a lone rank
    makes its own."""

    def __init__(self, device=0, nranks=1, rank=0, uid=None):
        import ctypes

        from ._lib import check, lib

        if uid is None:
            if nranks != 1:
                raise ValueError("NativeComm: several ranks need rank 0's id (from_dist)")
            uid = NativeComm.unique_id()
        h = ctypes.c_void_p()
        check(lib().td_comm_create(ctypes.byref(h), int(device), int(nranks), int(rank), bytes(uid)))
        self.h, self.device, self.nranks, self.rank = h, int(device), int(nranks), int(rank)

    @staticmethod
    def unique_id():
        import ctypes

        from ._lib import check, lib

        buf = ctypes.create_string_buffer(128)
        check(lib().td_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def from_dist(cls, dist, device):
        rank, world = dist.get_rank(), dist.get_world_size()
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(device, world, rank, obj[0])

    def allgather(self, vec):
        from ._lib import check, lib, ptr

        vec = np.ascontiguousarray(vec, dtype=np.float64)
        out = np.empty(self.nranks * len(vec), dtype=np.float64)
        check(lib().td_comm_allgather(self.h, ptr(vec), len(vec), ptr(out)))
        return out

    def close(self):
        if getattr(self, "h", None):
            from ._lib import lib

            lib().td_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Exchange:
    """allgather of a small float64 vector per rank (torch.distributed).
    ``device`` = the torch device tensors live on for the backend (cuda for
    nccl/RCCL, cpu for gloo).  Single process: identity -- unless ``force``
    (the collective itself even at world 1: the RCCL path on one GPU).
    ``native``: also make an RCCL communicator in libtdstar (NativeComm) on
    torch device index ``native``, for the device-decided exchange rounds."""

    def __init__(self, dist=None, device="cpu", force=False, native=None):
        self.dist = dist
        self.device = device
        self.force = bool(force)
        self.world = dist.get_world_size() if dist is not None else 1
        self.rank = dist.get_rank() if dist is not None else 0
        self.comm = None
        if native is not None:
            self.comm = NativeComm.from_dist(dist, native) if dist is not None else NativeComm(native)

    def allgather(self, vec):
        vec = np.ascontiguousarray(vec, dtype=np.float64)
        if self.dist is None or (self.world == 1 and not self.force):
            return vec.copy()
        import torch

        t = torch.from_numpy(vec).to(self.device)
        out = torch.empty(self.world * t.numel(), dtype=torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t)
        return out.cpu().numpy()


class TemperingLadder:
    """Parallel tempering over ``chains`` (this rank's replicas) and the
    other ranks' replicas.  Chains need ``run(k)``, ``stats()['phi']`` and
    ``set_temperature(T)`` (``chain.Chain`` or any stand-in)."""

    def __init__(self, chains, exchange=None, tmax=8.0, seed=12345, resident=True, device_swaps=False):
        self.chains = list(chains)
        self.ex = exchange or Exchange()
        self.local = len(self.chains)
        self.R = self.ex.world * self.local
        self.temps = geometric_ladder(self.R, tmax)
        self.seed = seed
        self.rnd = 0
        # replica g starts at level g
        self.levels = np.arange(self.R, dtype=np.int64)
        self.tried = np.zeros(max(self.R - 1, 0), dtype=np.int64)
        self.accepted = np.zeros(max(self.R - 1, 0), dtype=np.int64)
        for j, ch in enumerate(self.chains):
            ch.set_temperature(float(self.temps[self.gid(j)]))
        # the swap trace (gathered phis, new levels) of every round, hashed: equal ladders, equal digests
        self._trace = hashlib.sha256()
        self.gather_s = 0.0  # wall time spent in the allgather (the collective), all rounds
        self.compute_s = 0.0  # step(): wall time of the replicas' proposals (launch or resident round)
        self.decide_s = 0.0  # step(): wall time of the swap decision and bookkeeping
        self.timing = None  # run() with device swaps: the last call's split (td_rounds_exchange timing_out)
        # td_chain replicas of one context run in one launch, one workgroup each
        self.batch = self.local > 1 and all(hasattr(c, "h") and getattr(c, "ctx", None) is self.chains[0].ctx
                                            for c in self.chains)
        # DEVICE td_chain replicas of one context: one launch resident across the rounds (td_rounds),
        # the temperatures posted to it every round instead of a launch per round.  The launch spins
        # between rounds on a high-priority non-blocking stream (comm.cpp dedicated_stream), whose
        # hardware queue nothing else of ours uses, so a GPU collective's kernels (RCCL) are not held
        # back behind it.  The td_comm exchange stream shares that priority pool (GPU_MAX_HW_QUEUES = 4
        # queues per process), so a process holds only a few such streams.
        self.resident = bool(resident) and self.local >= 1 and all(
            hasattr(c, "h") and getattr(c, "ctx", None) is self.chains[0].ctx and
            getattr(getattr(c, "params", None), "engine", None) == 0 for c in self.chains)
        # run(): the swap decisions made inside the resident kernel (td_rounds_exchange): on one rank,
        # or across ranks through the library's RCCL communicator (Exchange(native=...))
        self.device_swaps = bool(device_swaps) and self.resident and (self.ex.world == 1 or
                                                                      self.ex.comm is not None)
        self.rounds = None
        # mixing statistics (_observe): a replica is labelled "up" after it visits level 0 and "down"
        # after it visits the top level; a round trip is a 0 -> top -> 0 journey of one replica
        self.label = np.zeros(self.R, dtype=np.int8)  # 0 none yet, 1 up, -1 down
        self.label[0] = 1
        if self.R > 1:
            self.label[self.R - 1] = -1
        self._went_up = self.label == 1  # visited level 0 before its current "down" label
        self.trips = np.zeros(self.R, dtype=np.int64)  # completed round trips per replica
        self.up_visits = np.zeros(self.R, dtype=np.int64)  # per level: rounds its replica was labelled up
        self.lab_visits = np.zeros(self.R, dtype=np.int64)  # per level: rounds its replica had a label

    def _observe(self, levels):
        """Update the round-trip counts and the up-fraction histogram after a swap round
        (levels[g] = the level of replica g)."""
        if self.R < 2:
            return
        top = self.R - 1
        for g in range(self.R):
            lv = int(levels[g])
            if lv == 0:
                if self.label[g] == -1 and self._went_up[g]:
                    self.trips[g] += 1
                self.label[g] = 1
                self._went_up[g] = True
            elif lv == top:
                self.label[g] = -1
            if self.label[g] != 0:
                self.lab_visits[lv] += 1
                self.up_visits[lv] += self.label[g] == 1

    def mixing(self):
        """Round trips (0 -> top -> 0, all replicas), rounds per round trip, and per level
        the fraction of labelled visits by replicas heading up (1 at T = 1 falling to 0 at
        the top for a ladder whose replicas diffuse over all of it)."""
        n = int(self.trips.sum())
        return {"round_trips": n, "rounds_per_round_trip": round(self.rnd / n, 1) if n else None,
                "up_fraction": [round(float(u) / v, 3) if v else None
                                for u, v in zip(self.up_visits, self.lab_visits)]}

    def gid(self, j):
        return self.ex.rank * self.local + j

    def step(self, k):
        """k proposals on every local replica, then one swap round."""
        tc = time.perf_counter()
        if self.resident:
            if self.rounds is None:
                from .chain import Rounds

                self.rounds = Rounds(self.chains)
            mine = self.rounds.run(k, [self.temps[self.levels[self.gid(j)]] for j in range(self.local)])
        else:
            if self.batch:
                from .chain import run_batch

                run_batch(self.chains, k)  # all local replicas in one launch
            else:
                for ch in self.chains:
                    ch.run(k)
            mine = np.array([ch.stats()["phi"] for ch in self.chains], dtype=np.float64)
        t0 = time.perf_counter()
        self.compute_s += t0 - tc
        allphi = self.ex.allgather(mine)
        t1 = time.perf_counter()
        self.gather_s += t1 - t0
        new, tried, acc = decide_swaps(allphi, self.levels, self.temps, self.rnd, self.seed)
        self._trace.update(np.ascontiguousarray(allphi, dtype=np.float64).tobytes())
        self._trace.update(np.ascontiguousarray(new, dtype=np.int64).tobytes())
        self.tried += tried
        self.accepted += acc
        for j, ch in enumerate(self.chains):
            g = self.gid(j)
            if new[g] != self.levels[g] and not self.resident:  # (resident: posted with the next round)
                ch.set_temperature(float(self.temps[new[g]]))
        self.levels = new
        self._observe(new)
        self.rnd += 1
        self.decide_s += time.perf_counter() - t1
        return allphi

    def run(self, rounds, k):
        """``rounds`` x ``step(k)``.  One process holding every replica in a
        resident launch (BASELINE config 4 on one GPU): the rounds and their
        swap steps run in the library (td_rounds_temper, td_swap_decide: the
        same decisions as decide_swaps, bit for bit) without a return to
        Python per round; the trace is the same.  With ``device_swaps`` the
        kernel itself decides the swaps (td_rounds_exchange): no host in the
        loop at all, across ranks through the library's RCCL allgathers; the
        trace is again the same.  Returns the last gathered phis."""
        rounds = int(rounds)
        if self.device_swaps and rounds > 0:
            return self._run_exchange(rounds, k)
        if not (self.resident and self.ex.world == 1 and rounds > 0):
            out = None
            for _ in range(rounds):
                out = self.step(k)
            return out
        import ctypes

        from ._lib import _pi64, check, lib, ptr

        if self.rounds is None:
            from .chain import Rounds

            self.rounds = Rounds(self.chains)
        R = self.R
        phis = np.empty((rounds, R), dtype=np.float64)
        lv_out = np.empty((rounds, R), dtype=np.int64)
        levels = np.ascontiguousarray(self.levels, dtype=np.int64).copy()
        tried = np.zeros(max(R - 1, 1), dtype=np.int64)
        acc = np.zeros(max(R - 1, 1), dtype=np.int64)
        temps = np.ascontiguousarray(self.temps, dtype=np.float64)
        check(lib().td_rounds_temper(self.rounds.h, rounds, int(k), ptr(temps), ptr(levels, _pi64), int(self.rnd),
                                     ctypes.c_uint64(int(self.seed) & _M64), ptr(phis), ptr(lv_out, _pi64),
                                     ptr(tried, _pi64), ptr(acc, _pi64)), self.chains[0].ctx.h)
        for j in range(rounds):
            self._trace.update(phis[j].tobytes())
            self._trace.update(lv_out[j].tobytes())
            self._observe(lv_out[j])
        self.tried += tried[:R - 1]
        self.accepted += acc[:R - 1]
        self.levels = levels
        self.rnd += rounds
        return phis[-1].copy()

    def _run_exchange(self, rounds, k):
        import ctypes

        from ._lib import _pi64, check, lib, ptr

        if self.rounds is None:
            from .chain import Rounds

            self.rounds = Rounds(self.chains)
        R = self.R
        phis = np.empty((rounds, R), dtype=np.float64)
        lv_out = np.empty((rounds, R), dtype=np.int64)
        levels = np.ascontiguousarray(self.levels, dtype=np.int64).copy()
        tried = np.zeros(max(R - 1, 1), dtype=np.int64)
        acc = np.zeros(max(R - 1, 1), dtype=np.int64)
        temps = np.ascontiguousarray(self.temps, dtype=np.float64)
        tm = np.zeros(7, dtype=np.float64)
        comm = self.ex.comm.h if self.ex.comm is not None else None
        check(lib().td_rounds_exchange(self.rounds.h, comm, rounds, int(k), ptr(temps), ptr(levels, _pi64),
                                       int(self.rnd), ctypes.c_uint64(int(self.seed) & _M64), ptr(phis),
                                       ptr(lv_out, _pi64), ptr(tried, _pi64), ptr(acc, _pi64), ptr(tm)),
              self.chains[0].ctx.h)
        for j in range(rounds):
            self._trace.update(phis[j].tobytes())
            self._trace.update(lv_out[j].tobytes())
            self._observe(lv_out[j])
        self.tried += tried[:R - 1]
        self.accepted += acc[:R - 1]
        self.levels = levels
        self.rnd += rounds
        self.timing = {"call_s": float(tm[0]), "launch_issued_s": float(tm[1]), "exchanges_enqueued_s": float(tm[2]),
                       "exchange_us_per_round": round(float(tm[3]) * 1e6, 3),
                       "proposals_us_per_round": round(float(tm[4]) * 1e6, 3),
                       "slowest_replica_wait_us_per_round": round(float(tm[5]) * 1e6, 3),
                       "kernel_span_s": float(tm[6]), "rounds": rounds}
        return phis[-1].copy()

    def close(self):
        """End the resident launch (the chains' counts and models are current after it).
        A resident round runs at the temperatures posted with it, so the last swap's
        levels reach the chains only here: each chain leaves at its ladder level's T."""
        if self.rounds is not None:
            self.rounds.close()
            self.rounds = None
            for j, ch in enumerate(self.chains):
                ch.set_temperature(float(self.temps[self.levels[self.gid(j)]]))

    def trace_digest(self):
        """sha256 of every round's gathered phis and new levels so far."""
        return self._trace.hexdigest()

    def cold_local(self):
        """Index of the local chain at T = 1, or None (another rank holds it)."""
        for j in range(self.local):
            if self.levels[self.gid(j)] == 0:
                return j
        return None

    def swap_rates(self):
        return [float(a) / t if t else 0.0 for a, t in zip(self.accepted, self.tried)]
