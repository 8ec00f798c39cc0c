"""Ray-sharded evaluate across GPUs (the optional intra-chain
split for the stress configuration).

One proposal's forward model (MCsub.jl:123-185) is independent per ray up to
the chi^2 sum: a point's nearest cell and a ray's t* (MCsub.jl:142-163) need
only that ray and the cells.  So every rank owns a contiguous range of rays
(balanced by ray points, the work of the nearest search) in a context of its
own, and one evaluate is

  1. td_evaluate of the model on the rank's rays (its incremental path
     included: a chain's one-edit-per-call models stay incremental per shard);
  2. one allgather of the shards' ptS (torch.distributed: RCCL over xGMI on
     the GPU box, gloo in the tests), padded to the longest shard;
  3. td_misfit of the gathered ptS, in ray order, against the full tS / allSig
     on every rank: phi is the SEQUENTIAL sum of MCsub.jl:170-172 over all rays,
     bit for bit the one-GPU evaluate (the chi^2 is not split: its order is
     the reference's, and n FP64 terms cost ~20-40 us on one device).

Every rank ends with the same (ptS, phi, likelihood), so a chain can be driven
by every rank in lockstep (same seed) with no further exchange.  Worth it when
one evaluate is much longer than an allgather: the 10k-ray stress geometry,
not the 381-ray configs.  ``shard_rays`` is pure host logic (tested on CPU);
the evaluate path is tests/test_gpu_sharded.py (two processes on one GPU)."""
import numpy as np

from .defstruct import DataStruct
from .forward import TdContext


def ray_points(ds):
    """Valid points per ray (the NaN-terminated columns of rayX, MCsub.jl:312-316)."""
    X = np.asarray(ds.rayX)
    nan = np.isnan(X)
    first = np.where(nan.any(axis=0), nan.argmax(axis=0), X.shape[0])
    return first.astype(np.int64)


def shard_rays(points, world):
    """Contiguous ray ranges [(r0, r1)] of about equal point counts, one per
    rank (ranks may get no rays when there are fewer rays than ranks)."""
    points = np.asarray(points, dtype=np.int64)
    n = len(points)
    if world < 1:
        raise ValueError("world must be >= 1")
    cum = np.concatenate([[0], np.cumsum(points)])
    total = cum[-1]
    bounds = [0]
    for k in range(1, world):
        target = total * k / world
        r = int(np.searchsorted(cum, target, side="left"))
        # the cut nearer to the target; ranges stay non-decreasing
        if r > 0 and abs(cum[r - 1] - target) <= abs(cum[min(r, n)] - target):
            r -= 1
        bounds.append(min(max(r, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[k], bounds[k + 1]) for k in range(world)]


def sub_datastruct(ds, r0, r1):
    """The DataStruct restricted to rays [r0, r1): ray columns and per-ray data
    sliced, everything else shared."""
    def cols(a):
        return np.ascontiguousarray(np.asarray(a)[:, r0:r1])

    def rows(a):
        a = np.asarray(a)
        return a[r0:r1].copy() if a.ndim == 1 and len(a) == ds.rayX.shape[1] else a

    return DataStruct(rows(ds.tS), rows(ds.allaveatten), rows(ds.allLats), rows(ds.allLons), rows(ds.allSig),
                      rows(ds.dataX), rows(ds.dataY), ds.xVec, ds.yVec, ds.zVec, ds.elonsX, ds.elatsY, ds.elons,
                      ds.elats, ds.edep, ds.coastX, ds.coastY, cols(ds.rayX), cols(ds.rayY), cols(ds.rayZ),
                      cols(ds.rayL), cols(ds.rayU), cols(ds.U))


class RayShardedContext:
    """evaluate() over ``exchange.world`` ranks, each owning a ray range
    (``exchange``: tempering.Exchange over torch.distributed; single process =
    the whole geometry on one device)."""

    def __init__(self, ds, exchange, device=-1, make_context=None):
        self.ex = exchange
        self.n = int(np.asarray(ds.rayX).shape[1])
        self.tS = np.ascontiguousarray(ds.tS, dtype=np.float64)
        self.allSig = np.ascontiguousarray(ds.allSig, dtype=np.float64)
        self.bounds = shard_rays(ray_points(ds), self.ex.world)
        r0, r1 = self.bounds[self.ex.rank]
        self.r0, self.r1 = r0, r1
        self.width = max(b - a for a, b in self.bounds)
        # a rank with no rays keeps a one-ray context for td_misfit only
        make = make_context or TdContext.from_datastruct  # (tests inject a host stand-in for the CPU suite)
        self.local = make(sub_datastruct(ds, r0, r1) if r1 > r0 else sub_datastruct(ds, 0, 1), device)
        # an allgather runs between this context's evaluates: no resident kernel may hold
        # the collective's hardware queue (td_set_incremental), one launch per call instead
        if hasattr(self.local, "set_incremental"):
            self.local.set_incremental(TdContext.INCR_LAUNCH)
        self.P_local = self.local.P if r1 > r0 else 0

    def evaluate(self, cells):
        """(ptS[n], phi, likelihood) of the model on all rays: bit-identical to
        one context's td_evaluate."""
        buf = np.full(self.width, np.nan)
        if self.r1 > self.r0:
            ptS_loc, _, _, _ = self.local.evaluate(cells)
            buf[:self.r1 - self.r0] = ptS_loc
        allp = self.ex.allgather(buf).reshape(self.ex.world, self.width)
        ptS = np.concatenate([allp[k, :b - a] for k, (a, b) in enumerate(self.bounds)])
        phi, lk = self.local.misfit(ptS, self.tS, self.allSig)
        return ptS, phi, lk

    def close(self):
        self.local.close()
