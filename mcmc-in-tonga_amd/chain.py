"""rj-MCMC chain -- mirror of TD_inversion_function.jl over the td_chain ABI.

``Chain`` wraps one ``td_chain`` (device-resident loop by default, or the
HOST engine that calls the full ``td_evaluate`` for every proposal exactly as
the reference does).  ``TD_inversion_function(TD_parameters, dataStruct,
chain)`` keeps the reference's signature and bookkeeping: burn-in, thinning
into ``model_hist`` (copies, not the aliased references the reference
pushes, TD_inversion_function.jl:280), progress lines every ``print_each``,
and optional JLD checkpoint/resume (TD_inversion_function.jl:41-67,282-294).
"""
import ctypes
import glob
import os

import numpy as np

from . import _lib
from ._lib import TdChainParams, TdChainStats, check, f64, lib, ptr
from .data import box
from .defstruct import Model
from .forward import context_for

ACTIONS = {1: "birth", 2: "death", 3: "change", 4: "move"}


def chain_params(TD_parameters, dataStruct=None, seed=1, chain=1, temperature=1.0, engine=_lib.TD_ENGINE_DEVICE,
                 extent=None):
    p = TdChainParams()
    p.debug_prior = int(TD_parameters.debug_prior)
    p.sig = int(TD_parameters.sig)
    p.zeta_scale = int(TD_parameters.zeta_scale)
    p.max_cells = int(TD_parameters.max_cells)
    p.min_cells = int(TD_parameters.min_cells)
    p.prior = int(TD_parameters.prior)
    p.n_iter, p.burn_in, p.keep_each = float(TD_parameters.n_iter), float(TD_parameters.burn_in), \
        float(TD_parameters.keep_each)
    if extent is None:
        if dataStruct is not None:  # min(xVec...), max(xVec...) (TD_inversion_function.jl:30-32)
            extent = (float(np.min(dataStruct.xVec)), float(np.max(dataStruct.xVec)),
                      float(np.min(dataStruct.yVec)), float(np.max(dataStruct.yVec)),
                      float(np.min(dataStruct.zVec)), float(np.max(dataStruct.zVec)))
        else:
            extent = box()
    p.xmin, p.xmax, p.ymin, p.ymax, p.zmin, p.zmax = extent
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.chain = int(chain)
    p.temperature = float(temperature)
    p.engine = int(engine)
    return p


class Chain:
    def __init__(self, ctx, params, model=None):
        self.ctx = ctx
        self.params = params
        h = ctypes.c_void_p()
        if model is not None:
            cells = [f64(c) for c in model.cells()]
            check(lib().td_chain_create(ctypes.byref(h), ctx.h, ctypes.byref(params), *(ptr(c) for c in cells),
                                        len(cells[0])), ctx.h)
        else:
            check(lib().td_chain_create(ctypes.byref(h), ctx.h, ctypes.byref(params), None, None, None, None, 0),
                  ctx.h)
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().td_chain_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, iterations):
        check(lib().td_chain_run(self.h, int(iterations)), self.ctx.h)

    def stats(self):
        s = TdChainStats()
        check(lib().td_chain_stats_get(self.h, ctypes.byref(s)), self.ctx.h)
        return dict(iterations=s.iterations, evaluations=s.evaluations, accepted=list(s.accepted)[1:],
                    proposed=list(s.proposed)[1:], phi=s.phi, ncells=s.ncells, bytes=s.bytes,
                    last_action=s.last_action, last_accept=s.last_accept)

    def model(self):
        cap = max(int(self.params.max_cells), self.stats()["ncells"]) + 1
        arrs = [np.zeros(cap) for _ in range(4)]
        n = ctypes.c_int64()
        phi = ctypes.c_double()
        ptS = np.zeros(max(self.ctx.n, 1))
        check(lib().td_chain_get_model(self.h, *(ptr(a) for a in arrs), cap, ctypes.byref(n), ctypes.byref(phi),
                                       ptr(ptS)), self.ctx.h)
        k = n.value
        m = Model(float(k), arrs[0][:k].copy(), arrs[1][:k].copy(), arrs[2][:k].copy(), arrs[3][:k].copy())
        m.phi = phi.value
        m.ptS = ptS[:self.ctx.n].copy()
        st = self.stats()
        if st["last_action"] > 0:  # model.action / model.accept of the last iteration (:73-74)
            m.action, m.accept = st["last_action"], st["last_accept"]
        return m

    def set_temperature(self, T):
        check(lib().td_chain_set_temperature(self.h, float(T)), self.ctx.h)


def run_batch(chains, iterations):
    """``iterations`` proposals on every chain of one context in ONE launch
    (one workgroup per chain, td_chain_run_batch) -- several independent
    chains or tempering replicas per GPU."""
    chains = list(chains)
    if not chains:
        return
    arr = (ctypes.c_void_p * len(chains))(*[c.h for c in chains])
    check(lib().td_chain_run_batch(arr, len(chains), int(iterations)), chains[0].ctx.h)


class Rounds:
    """A resident tempering launch over DEVICE chains of one context
    (td_rounds_*): ``run(K, temps)`` -> every chain's phi after K more
    proposals at those temperatures; no launch per round."""

    def __init__(self, chains):
        self.chains = list(chains)
        arr = (ctypes.c_void_p * len(self.chains))(*[c.h for c in self.chains])
        h = ctypes.c_void_p()
        check(lib().td_rounds_create(ctypes.byref(h), arr, len(self.chains)), self.chains[0].ctx.h)
        self.h = h
        self._phi = np.zeros(len(self.chains))

    def run(self, K, temps):
        t = f64(temps)
        check(lib().td_rounds_run(self.h, int(K), ptr(t), ptr(self._phi)), self.chains[0].ctx.h)
        return self._phi.copy()

    def close(self):
        if getattr(self, "h", None):
            lib().td_rounds_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def build_starting(TD_parameters, dataStruct, seed=1, chain=1):
    """MCsub.jl:76-121 (log-uniform nCells, uniform cells, zeta ~ U(0, zeta_scale)),
    drawn by the chain's RNG; returns (model, dataStruct, valid)."""
    ctx = context_for(dataStruct)
    ch = Chain(ctx, chain_params(TD_parameters, dataStruct, seed=seed, chain=chain))
    m = ch.model()
    ch.close()
    m.tS = dataStruct.tS
    m.likelihood = ctx.likelihood_const if TD_parameters.debug_prior != 1 else 1.0
    return m, dataStruct, 1


def TD_inversion_function(TD_parameters, dataStruct, chain, seed=None, model=None, engine=_lib.TD_ENGINE_DEVICE,  # noqa: N802
                          checkpoint_dir=None, verbose=False, temperature=1.0, stop_after=None):
    """TD_inversion_function.jl:7-305: one chain; returns model_hist (list of Model copies).

    Bookkeeping as the reference's loop (:275-298): from iteration burn_in on,
    model_num counts iterations and every keep_each-th model is saved into
    model_hist; with ``checkpoint_dir`` a JLD checkpoint
    ``chain<c>_iter<it>_<pct>%.jld`` is written at the 1st saved model and at
    every 10 % of them (:282-287: model, dataStruct, iter, saved_#,
    model_num, model_hist, burnin = true), and before burn-in every
    print_each iterations (:289-294: model, dataStruct, iter, burnin =
    false).  At the start the newest checkpoint of this chain is resumed
    (:41-67); all but the newest two are deleted (:53-55).

    Deliberate differences: the resumed loop starts at iter + 1 (the
    reference re-runs the saved iteration, :59,70; with the counter-based RNG
    starting after it continues the interrupted chain exactly); "newest" is the
    highest iteration number, not the last name in lexicographic order (:51,
    which ranks iter1000 before iter900), and only this chain's files match
    (glob("chain1*") also matches chain10..., :41).  The geometry of the
    checkpoint's dataStruct is the caller's (it never changes: action 5 is
    unreachable, :72).  ``stop_after``: return after that iteration (testing a
    crash and resume)."""
    drv = _ChainDriver(TD_parameters, dataStruct, chain, seed, model, engine, checkpoint_dir, verbose, temperature,
                       stop_after)
    while True:
        k = drv.next_stretch()
        if k is None:
            return drv.finish()
        drv.ch.run(k)
        drv.after_stretch()


class _ChainDriver:
    """One chain of TD_inversion_function as a sequence of stretches: the
    iterations between two bookkeeping points run in ONE device launch;
    ``next_stretch`` says how many, ``after_stretch`` does the bookkeeping.
    Several drivers can share launches (main_inversion: td_chain_run_batch)."""

    def __init__(self, TD_parameters, dataStruct, chain, seed, model, engine, checkpoint_dir, verbose, temperature,
                 stop_after):
        from . import jld

        self.jld = jld
        self.prm_ref = TD_parameters
        self.ds = dataStruct
        self.chain = chain
        self.ctx = ctx = context_for(dataStruct)
        seed = chain * 7919 + 1 if seed is None else seed
        prm = chain_params(TD_parameters, dataStruct, seed=seed, chain=chain, temperature=temperature, engine=engine)
        self.n_iter, self.keep = int(TD_parameters.n_iter), int(TD_parameters.keep_each)
        self.B = float(TD_parameters.burn_in)
        self.print_each = int(TD_parameters.print_each)
        self.num_models = int((TD_parameters.n_iter - TD_parameters.burn_in) / TD_parameters.keep_each)  # :25
        self.model_hist, it0, self.model_num, self.used_num = [], 1, 0, 0
        self.ckdir = checkpoint_dir
        self.verbose = verbose
        ckpt = _latest_checkpoint(checkpoint_dir, chain) if checkpoint_dir else None
        if ckpt is not None:  # :41-67 resume
            c = jld.load_checkpoint(ckpt)
            model = c["model"]
            it0 = int(c["iter"]) + 1
            if c["burnin"]:
                self.model_hist, self.used_num, self.model_num = list(c["model_hist"]), c["saved"], c["model_num"]
        prm.start_iter = it0  # the counter-based RNG continues exactly where the checkpoint stopped
        self.ch = Chain(ctx, prm, model)
        self.last = self.n_iter if stop_after is None else min(self.n_iter, int(stop_after))
        self.it = it0
        self.nxt = None

    def current(self):
        m = self.ch.model()
        m.tS = self.ds.tS
        m.likelihood = self.ctx.likelihood_const if self.prm_ref.debug_prior != 1 else 1.0
        return m

    def next_stretch(self):
        """Iterations to run up to the next one with bookkeeping (None: done)."""
        it = self.it
        if it > self.last:
            return None
        nxt = self.last
        if it < self.B:  # pre-burn-in: checkpoints every print_each (:289)
            nxt = min(nxt, int(np.ceil(self.B)) - 1)
        elif self.keep > 0:  # the next saved model: model_num + (nxt - it + 1) = 0 mod keep
            nxt = min(nxt, it + (self.keep - self.model_num % self.keep) - 1)
        if self.print_each > 0:
            nxt = min(nxt, ((it + self.print_each - 1) // self.print_each) * self.print_each)
        self.nxt = max(nxt, it)
        return self.nxt - it + 1

    def after_stretch(self):
        it, nxt, jld = self.it, self.nxt, self.jld
        TD = self.prm_ref
        if nxt >= self.B:  # :276-288
            self.model_num += nxt - it + 1
            if self.keep > 0 and self.model_num % self.keep == 0:
                self.used_num += 1
                m = self.current()
                self.model_hist.append(m)
                # used_num == 1 first: with n_iter == burn_in num_models is 0 (Julia gives Inf, no error)
                if self.ckdir and (self.used_num == 1 or
                                   (self.num_models > 0 and (100 * self.used_num / self.num_models) % 10 < 1e-9)):
                    os.makedirs(self.ckdir, exist_ok=True)
                    name = "chain%d_iter%d_%r%%.jld" % (self.chain, nxt, 100 * float(nxt) / float(TD.n_iter))
                    jld.save_checkpoint(os.path.join(self.ckdir, name), m, self.ds, float(nxt), True,
                                        self.model_hist, self.used_num, self.model_num)
        elif self.ckdir and self.print_each > 0 and nxt % self.print_each == 0:  # :289-294
            os.makedirs(self.ckdir, exist_ok=True)
            name = "chain%d_iter%d_%d%%.jld" % (self.chain, nxt, int(100 * nxt / TD.n_iter))
            jld.save_checkpoint(os.path.join(self.ckdir, name), self.current(), self.ds, nxt, False)
        if self.verbose and self.print_each > 0 and nxt % self.print_each == 0:  # :296-298
            print("Chain #%d at %r%% with a phi of %r" % (self.chain, 100 * nxt / TD.n_iter, self.ch.stats()["phi"]))
        self.it = nxt + 1

    def finish(self):
        self.ch.close()
        return self.model_hist


def _ckpt_iter(f):
    return int(os.path.basename(f).split("_iter")[1].split("_")[0])


def _latest_checkpoint(d, chain):
    """The newest checkpoint of this chain (highest iteration); all but the
    newest two are removed, as TD_inversion_function.jl:53-55 does."""
    files = [f for f in glob.glob(os.path.join(d, "chain%d_iter*.jld" % chain))
             if os.path.basename(f).startswith("chain%d_iter" % chain)]
    files.sort(key=_ckpt_iter)
    for f in files[:-2]:
        os.remove(f)
    return files[-1] if files else None


def delete_checkpoints(d):
    """main_inversion.jl:21-22: remove every chain*jld checkpoint after the run."""
    for f in glob.glob(os.path.join(d, "chain*.jld")):
        os.remove(f)


def run_chains(TD_parameters, dataStruct, chains, engine=_lib.TD_ENGINE_DEVICE, checkpoint_dir=None,
               verbose=False, seeds=None):
    """``pmap(x -> TD_inversion_function(TD_parameters, dataStruct, x), chains)``
    (main_inversion.jl:15) on this GPU: every chain's stretch between two
    bookkeeping points runs in ONE td_chain_run_batch launch with the others
    (one workgroup per chain, concurrently, as the reference's workers run);
    chains whose stretches differ (resumed from different checkpoints) run in
    separate launches.  Each chain's model_hist is the one TD_inversion_function
    returns for it alone.

    HOST and DROPIN chains call the context's td_evaluate per proposal: they
    share its incremental shadow (one model at a time), so they run one chain
    after another, as separate workers would, instead of interleaved stretches
    that would rebuild the shadow at every switch."""
    chains = list(chains)
    seeds = seeds or [None] * len(chains)
    if engine != _lib.TD_ENGINE_DEVICE:
        out = []
        for c, s in zip(chains, seeds):
            d = _ChainDriver(TD_parameters, dataStruct, c, s, None, engine, checkpoint_dir, verbose, 1.0, None)
            while True:
                k = d.next_stretch()
                if k is None:
                    break
                d.ch.run(k)
                d.after_stretch()
            out.append(d.finish())
        return out
    drv = [_ChainDriver(TD_parameters, dataStruct, c, s, None, engine, checkpoint_dir, verbose, 1.0, None)
           for c, s in zip(chains, seeds)]
    live = list(drv)
    while live:
        want = {}
        for d in live:
            k = d.next_stretch()
            if k is not None:
                want.setdefault(k, []).append(d)
        live = [d for ds_ in want.values() for d in ds_]
        for k, group in want.items():
            run_batch([d.ch for d in group], k)
            for d in group:
                d.after_stretch()
    return [d.finish() for d in drv]


def main_inversion(TD_parameters=None, dataStruct=None, out="model.jld", checkpoint_dir=None,  # noqa: N803
                   engine=_lib.TD_ENGINE_DEVICE):
    """main_inversion.jl:11-18: the chains (concurrently on this GPU, one
    td_chain_run_batch launch per stretch: run_chains; one rank per GPU for
    more, see tempering/bench), the posterior maps of plot_model_hist (numbers
    only) and ``save(out, "model", models)`` in JLD.  Returns (models, maps)."""
    from . import jld
    from .config import define_TDstructrure
    from .data import load_data_Tonga
    from .posterior import plot_model_hist
    TD_parameters = TD_parameters or define_TDstructrure()
    dataStruct = dataStruct or load_data_Tonga(TD_parameters)
    models = run_chains(TD_parameters, dataStruct, range(1, int(TD_parameters.n_chains) + 1), engine=engine,
                        checkpoint_dir=checkpoint_dir)
    maps = plot_model_hist(models, dataStruct, TD_parameters, 20.0)
    if out:
        jld.save(out, models)
    if checkpoint_dir:
        delete_checkpoints(checkpoint_dir)
    return models, maps
