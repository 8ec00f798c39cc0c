#!/usr/bin/env python3
"""bench.py -- MCMC proposals/s of the rj-MCMC t* chain on MI355X.

Metric (BASELINE.json): MCMC proposals/sec (likelihood evaluations/sec) at 381
rays x N cells.  Workload (BASELINE configs[2], the north-star target): the
381 shipped rays, a 5000-cell starting model (seed 3), one chain per GPU
running the reference's birth/death/change/move mix
(TD_inversion_function.jl:72) with the DEVICE engine.  max_cells is raised to
2N so births stay active (the reference default of 100 would freeze N).

A "step" = --iters-per-step chain iterations (proposals), each one a complete
forward-model evaluation of the proposed model -- bit-identical to a full
evaluate (tests/test_gpu_chain.py) -- plus the Metropolis-Hastings decision.
Inputs are resident in HBM before the timed region.  value = proposals of
all ranks / max-over-ranks wall time (weak scaling: one chain per GPU,
independent chains, no data-path collective).

Also reported:
  roofline      -- k_chain_run (the only kernel in the timed region).  Its
                   bound is LATENCY (one persistent workgroup per chain: a
                   chain of dependent barriers and LDS/L2 round trips per
                   proposal); `latency` gives the measured phase cycles.  The
                   headline's HBM line prices SURVEY 8(d)'s algorithmic bytes
                   of one evaluate per proposal against HBM peak;
                   `incremental_*` beside it is what the incremental proposals
                   actually read (counted in-kernel: tile boxes, candidate
                   points, grid queries, re-summed ray points, chi^2 terms),
                   and every other chain block's `frac` is that counted figure
                   (chain_roofline: no `frac` above 1).
  full_evaluate -- the drop-in td_evaluate path (brute-force P x N nearest
                   search, MCsub.jl:123-185) on the same model: latency and
                   the FP64-VALU roofline of its dominant kernel.
  cpu_baseline  -- the CPU oracle (scalar C restatement of evaluate), one
                   chain per host core of the job's share (and on 1 core),
                   ~--cpu-seconds in all: the reference's structure does one
                   full evaluate per proposal.
At N > 1 ranks every rank also runs BASELINE config 4 (`config4_ranks`: one
tempered replica per rank, a swap round every 10 proposals through the
allgather -- RCCL over xGMI) and config 5 (`stress_chains`: one 10k x 20k
stress chain per rank).  Each multi-rank leg runs under a deadline the ranks
agree on (run_leg): a stalled collective makes rank 0 print the line it has,
with that leg as an error, and every rank exit non-zero, instead of hanging.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md (spec; 6.3 TB/s measured copy)
FP64_VALU_PEAK_TFLOPS = 78.6   # FP64 vector, FMA counted as 2 (spec)
# the distance kernel may not use FMA (bit-exactness), so its roof is half that
FP64_NOFMA_PEAK_TFLOPS = FP64_VALU_PEAK_TFLOPS / 2


def measured_traffic(key):
    """HBM bytes per launch from the committed rocprofv3 PMC passes
    (profiles/traffic.json, written by profiles/make_traffic.py from
    tools/profile.sh output: FETCH_SIZE x2 + WRITE_SIZE per
    MI355X_MICROARCH.md) and that profile's kernel-trace average launch time;
    (None, None, None) when absent.  Not measured in this run."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            t = json.load(f)[key]
        return round(float(t["traffic_bytes_per_launch"]), 1), t["source"], t.get("avg_launch_us")
    except (OSError, KeyError, ValueError):
        return None, None, None


def model_bytes(P, n, N):
    """SURVEY 8(d)'s algorithmic (compulsory) bytes of one full evaluate:
    24 P (points) + 8 S (w = l*u per segment) + 32 N (cells) + 24 n (tS, sigma,
    ptS), S = P - n segments.  The chain's proposals are evaluated
    incrementally, so this is the byte count the reference's structure needs
    per proposal, not what the incremental kernel reads."""
    S = P - n
    return 24 * P + 8 * S + 32 * N + 24 * n


def chain_roofline(kernel, ref_bytes_per_proposal, proposals_per_launch, avg_launch_s, counted_bytes_per_launch,
                   traffic_key, match, headline=False):
    """roofline block of a chain kernel.  bound = latency.
    Two byte counts per launch, both over the launch's HIP-event time:
    SURVEY 8(d)'s algorithmic bytes of one evaluate (24 P + 8 S + 32 N + 24 n,
    model_bytes) x the proposals of one launch -- what the reference's
    structure must move per proposal (`equiv_full_evaluate_*`) -- and the bytes
    the incremental proposals actually read, counted in-kernel (tile boxes 32 B
    per tested tile, 36 B per candidate point, 27 x 8 x 32 B per grid query,
    17 B per re-summed ray point, 28 B per chi^2 term; `incremental_*`).
    `achieved` / `frac` is the headline's 8(d) figure (headline=True: one chain,
    the bench's own workload) and the counted bytes for every other block: a
    many-chain launch does 8(d)'s work per proposal at a rate whose bytes would
    exceed the HBM peak (it does not move them), so pricing those bytes against
    the peak is no roofline fraction.  No `frac` exceeds 1 (if the 8(d) figure
    ever did, the counted bytes are used and `frac_basis` says so).
    `traffic` = the PMC-measured HBM bytes per launch from the committed
    rocprofv3 profile of the same command (`traffic_source`)."""
    alg = float(ref_bytes_per_proposal) * proposals_per_launch
    equiv = alg / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    inc = counted_bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    use_8d = headline and equiv <= HBM_PEAK_GBS
    achieved = equiv if use_8d else inc
    out = {"kernel": kernel, "bound": "latency",
           "limiter": "one persistent workgroup per chain: dependent barriers and LDS/L2 round trips "
                      "(DESIGN.md 4.2); HBM line below",
           "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None, "traffic_source": None,
           "frac_basis": ("SURVEY 8(d) bytes of one full evaluate per proposal" if use_8d else
                          "bytes the incremental proposals read, counted in-kernel"),
           "bytes_model": "SURVEY 8(d): 24 P + 8 S + 32 N + 24 n bytes per proposal (one evaluate)",
           "algorithmic_bytes_per_proposal": ref_bytes_per_proposal,
           "algorithmic_bytes_per_launch": round(alg, 1),
           "equiv_full_evaluate_achieved": round(equiv, 3),
           "equiv_full_evaluate_frac": round(equiv / HBM_PEAK_GBS, 6),
           "incremental_bytes_per_launch": round(counted_bytes_per_launch, 1),
           "incremental_achieved": round(inc, 3), "incremental_frac": round(inc / HBM_PEAK_GBS, 6),
           "proposals_per_launch": proposals_per_launch, "avg_launch_ms": round(avg_launch_s * 1e3, 4),
           "us_per_proposal": round(avg_launch_s / max(proposals_per_launch, 1) * 1e6, 4)}
    if equiv > HBM_PEAK_GBS:  # (many chains: one evaluate per proposal could not run at this rate)
        out["note"] = ("equiv_full_evaluate_frac > 1: the reference's one-evaluate-per-proposal bytes at this "
                       "proposal rate exceed the HBM peak -- a rate comparison, not a roofline fraction; frac is "
                       "the counted incremental bytes, traffic the PMC-measured HBM bytes")
    if match:
        tr, src, prof_us = measured_traffic(traffic_key)
        if tr is not None:
            out["traffic"], out["traffic_source"] = tr, src
            out["traffic_frac_of_peak"] = round(tr / avg_launch_s / 1e9 / HBM_PEAK_GBS, 6)
            if prof_us:
                out["profile_avg_launch_ms"] = round(prof_us / 1e3, 4)
    return out


PHASES = ["loop top", "B tiles + query", "C points", "D orphans", "E ray sums", "F chi2 + decision", "G commit + next"]


def phase_cycles(tt, ch, iters):
    """The chain's s_memtime phase stamps (a diagnostic mode of k_chain_run,
    DESIGN.md 4.2) over `iters` more proposals, after the timed region:
    cycles per proposal of each phase and the stamp clock (cycles / wall s)."""
    import ctypes

    L = tt.lib()
    a, b = (ctypes.c_int64 * 80)(), (ctypes.c_int64 * 80)()
    L.tdt_chain_profile(ch.h, 1, a)
    t0 = time.perf_counter()
    ch.run(iters)
    el = time.perf_counter() - t0
    L.tdt_chain_profile(ch.h, 0, b)
    cyc = [float(b[k] - a[k]) for k in range(7)]
    cyc[6] += float((b[12] - a[12]) + (b[13] - a[13]))
    tot = sum(cyc)
    return {"proposals": iters, "cycles_per_proposal": round(tot / iters, 1),
            "phases": {p: round(c / iters, 1) for p, c in zip(PHASES, cyc)},
            "stamp_clock_ghz": round(tot / el / 1e9, 3), "us_per_proposal_stamped": round(el / iters * 1e6, 3),
            "note": "stamped run (+~5 %), after the timed region; per-phase cycles are the latency yardstick"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cells", type=int, default=5000)
    ap.add_argument("--iters-per-step", type=int, default=5000)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-evaluate", action="store_true")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in leg (td_evaluate called per proposal by a host loop)")
    ap.add_argument("--chains-per-gpu", type=int, default=1,
                    help="independent chains per rank, one workgroup each, one launch (td_chain_run_batch)")
    ap.add_argument("--swap-every", type=int, default=0,
                    help="parallel tempering: exchange temperatures every K proposals (RCCL allgather); 0 = "
                         "independent chains as the reference's pmap")
    ap.add_argument("--tmax", type=float, default=8.0)
    ap.add_argument("--batch-chains", type=int, default=256,
                    help="size of the extra many-chains-per-GPU measurement on rank 0 (0 = skip)")
    ap.add_argument("--batch-iters", type=int, default=5000)
    ap.add_argument("--no-config4", dest="config4", action="store_false",
                    help="skip the config-4 block (8 tempered replicas x 2000 cells, swap every 10, one GPU)")
    ap.add_argument("--no-stress", action="store_true",
                    help="skip the config-5 stress block (10k synthetic rays x 20k cells)")
    ap.add_argument("--config4-rounds", type=int, default=300, help="timed swap rounds of the config-4 blocks")
    ap.add_argument("--stress-iters", type=int, default=2000, help="timed proposals of the stress chain(s)")
    ap.add_argument("--no-phases", action="store_true", help="skip the stamped phase-cycle run")
    ap.add_argument("--leg-deadline", type=float, default=100.0,
                    help="seconds each multi-rank leg (config4_ranks, stress_chains, stress_sharded) may take at N > 1 "
                         "before rank 0 prints the line with that leg as an error and every rank exits non-zero")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher self-test: the ranks meet over gloo and rank 0 prints the world it saw "
                         "(no GPU call; tests/test_bench_launch.py)")
    return ap.parse_args()


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) started without a launcher: start N fresh
    rank processes through torch.distributed.run (one per GPU, rendezvous on
    127.0.0.1) and wait for them.  Called before anything touches the GPU
    (this process imports neither torch nor the library), so every rank
    initialises its own device.  Rank 0's stdout -- the JSON line -- passes
    straight through; the exit code is torch.distributed.run's, which is
    non-zero when any rank failed (the reference's chains are one `pmap`
    worker each, main_inversion.jl:15)."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + argv
    return subprocess.run(cmd, env=env).returncode


PG_TIMEOUT_S = 120  # every collective of the process group (a stalled one raises instead of waiting 10 min)


def launch_check(world, rank, deadline_s):
    """The launcher self-test: no GPU, gloo only.  Every rank contributes one;
    rank 0 prints the world size and the sum.  Then one multi-rank leg under
    run_leg's deadline (an all-reduce; TD_BENCH_STALL_LEG can stall a rank in
    it: tests/test_bench_launch.py)."""
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", timeout=timedelta(seconds=PG_TIMEOUT_S))
    t = torch.ones(1, dtype=torch.int64)
    dist.all_reduce(t)
    out = {"launch_check": True, "n_gpus": world, "ranks_seen": int(t.item()), "pid_parent": os.getppid()}

    def leg():
        u = torch.ones(1, dtype=torch.int64)
        dist.all_reduce(u)
        return {"ranks": int(u.item())}

    res = run_leg("leg_check", leg, dist, "cpu", rank, out, deadline_s, [])
    if rank == 0:
        out["leg_check"] = res
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def run_leg(name, fn, dist, coll_dev, rank, out, deadline_s, later):
    """One multi-rank leg of an N > 1 run under a deadline the ranks agree on:
    rank 0's wall clock + deadline_s, taken as the MAX over the ranks (one host,
    one clock; until they have agreed, each rank's own clock + deadline_s).  A
    leg that stalls -- a collective some rank never joins (the first
    multi-rank RCCL traffic over xGMI happens here) -- cannot be left inside
    its process: a watchdog thread then has rank 0 print the JSON line with
    everything measured so far (the headline first), this leg as
    {"error": "deadline"} and the `later` legs as skipped, and every rank exit
    with status 3.  A leg that raises is reported as {"error": ...} and the
    run goes on.  Testing: TD_BENCH_STALL_LEG="name:rank" stalls that rank in
    that leg before its first collective."""
    import threading

    import torch

    state = {"until": time.time() + deadline_s}
    done = threading.Event()

    def expire():
        while not done.wait(0.25):
            if time.time() < state["until"]:
                continue
            if rank == 0:
                o = dict(out)
                o[name] = {"error": "deadline", "deadline_s": deadline_s,
                           "note": "a rank did not finish this leg in time (stalled collective?); the process exits"}
                for k in later:
                    o[k] = {"error": "skipped: an earlier multi-rank leg passed its deadline"}
                sys.stdout.write(json.dumps(o) + "\n")
                sys.stdout.flush()
            sys.stderr.write("bench.py rank %d: leg %s passed its deadline (%.0f s); exiting\n" % (rank, name, deadline_s))
            sys.stderr.flush()
            os._exit(3)

    threading.Thread(target=expire, name="leg-deadline-" + name, daemon=True).start()
    try:
        t = torch.tensor([state["until"]], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        state["until"] = float(t.item())
        if os.environ.get("TD_BENCH_STALL_LEG") == "%s:%d" % (name, rank):
            while True:
                time.sleep(1.0)
        return fn()
    except Exception as e:  # (a leg that fails on this rank; a rank left waiting for it hits the deadline)
        return {"error": repr(e)[:300]}
    finally:
        done.set()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != a.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks" % (a.gpus, world))
    if a.launch_check:
        launch_check(world, rank, a.leg_deadline)
        return
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        # rehearsal knobs (one GPU box): TD_BENCH_BACKEND=gloo TD_BENCH_DEVICE=0 runs every rank on
        # device 0 with CPU collectives; the driver's runs use RCCL, one rank per GPU
        backend = os.environ.get("TD_BENCH_BACKEND", "nccl")
        local = int(os.environ.get("TD_BENCH_DEVICE", local))
        from datetime import timedelta

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=timedelta(seconds=PG_TIMEOUT_S))
        else:
            dist.init_process_group(backend, timeout=timedelta(seconds=PG_TIMEOUT_S))
    coll_dev = "cuda" if os.environ.get("TD_BENCH_BACKEND", "nccl") == "nccl" else "cpu"

    import tonga

    tt = tonga.load()
    ds = tt.load_data_Tonga()
    N = a.cells
    model = tt.random_model(N, 3)  # config 3: seed 3
    ctx = tt.TdContext.from_datastruct(ds, device=local)
    prm = tt.define_TDstructrure().replace(max_cells=2 * N)
    C = max(1, a.chains_per_gpu)
    chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000 + rank * C + j, chain=1 + rank * C + j), model)
              for j in range(C)]
    ladder = None
    if a.swap_every > 0:
        ex = tt.Exchange(dist, coll_dev) if dist is not None else tt.Exchange()
        ladder = tt.TemperingLadder(chains, ex, tmax=a.tmax, seed=4242)

    def run_step(k):
        if ladder is not None:
            done = 0
            while done < k:
                kk = min(a.swap_every, k - done)
                ladder.step(kk)
                done += kk
        elif C > 1:
            tt.run_batch(chains, k)
        else:
            chains[0].run(k)  # synchronous: returns after the kernel finished

    def agg(key):
        st = [c.stats() for c in chains]
        if key in ("accepted", "proposed"):
            return [sum(x[key][i] for x in st) for i in range(4)]
        return sum(x[key] for x in st)

    def barrier_sync():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(a.warmup):
        run_step(a.iters_per_step)
    s0 = {k: agg(k) for k in ("accepted", "proposed", "bytes")}
    ctx.timing(enable=True, reset=True)
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run_step(a.iters_per_step)
    barrier_sync()
    el = time.perf_counter() - t0
    s1 = {k: agg(k) for k in ("accepted", "proposed", "bytes")}
    s1["ncells"] = chains[0].stats()["ncells"]
    launches, kms = ctx.timing(kernel="chain_run")
    ctx.timing(enable=False)
    if dist is not None:
        import torch

        t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    iters = a.steps * a.iters_per_step
    total = iters * world * C
    value = total / el
    P = ctx.P
    acc = [x - y for x, y in zip(s1["accepted"], s0["accepted"])]
    prop = [x - y for x, y in zip(s1["proposed"], s0["proposed"])]
    nbytes = s1["bytes"] - s0["bytes"]
    if ladder is not None:
        launches = max(launches, 1)
    bytes_per_launch = nbytes / max(launches, 1)
    avg_s = kms / 1e3 / max(launches, 1)
    out = {
        "metric": "MCMC proposals/sec (likelihood evals/sec) at 381 rays x N cells",
        "value": round(value, 1),
        "unit": "proposals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "381 shipped rays (Data/381raypaths.jld), ak135 slowness substitute, synthetic seeded cells",
        "config": {"workload": "config3: 381 rays x %d cells, %d chain/GPU, birth/death/change/move%s"
                               % (N, C, ", tempering swap every %d (RCCL allgather)" % a.swap_every
                                  if ladder is not None else ""),
                   "rays": int(ctx.n), "points": P, "cells_start": N, "cells_end": int(s1["ncells"]),
                   "iters_per_step": a.iters_per_step, "engine": "device",
                   "parallelism": "chains%d" % (world * C)},
        # point x cell distance pairs a brute-force evaluate per proposal would need
        "nn_pair_evals_per_s_equiv": round(value * P * N, 1),
        "acceptance": {"birth/death/change/move accepted": acc, "proposed": prop,
                       "rate": round(sum(acc) / max(sum(prop), 1), 4)},
        "roofline": chain_roofline("k_chain_run", model_bytes(P, int(ctx.n), N), a.iters_per_step * C, avg_s,
                                   bytes_per_launch, "k_chain_run/single",
                                   C == 1 and ladder is None and N == 5000 and a.iters_per_step == 5000,
                                   headline=True),
    }
    if C == 1 and ladder is None and not a.no_phases:  # the latency yardstick, measured after the timed region
        out["roofline"]["latency"] = phase_cycles(tt, chains[0], min(a.iters_per_step, 5000))
    if ladder is not None:
        out["tempering"] = {"replicas": ladder.R, "temps": [round(t, 4) for t in ladder.temps],
                            "swap_rates": [round(r, 3) for r in ladder.swap_rates()]}
    legs = []  # the multi-rank legs, each under a deadline (run_leg): the headline above is already measured
    if dist is not None and a.config4:  # every rank: config 4, one tempered replica per rank, RCCL allgather
        legs.append(("config4_ranks", lambda: config4_ranks(tt, ds, dist, coll_dev, rank, world, local,
                                                            rounds=a.config4_rounds)))
    if dist is not None and not a.no_stress:  # every rank: config 5, one stress chain per rank
        legs.append(("stress_chains", lambda: stress_chains(tt, dist, coll_dev, rank, world, local, a.stress_iters)))
        # every rank: the stress evaluate split over the ranks' rays
        legs.append(("stress_sharded", lambda: stress_sharded(tt, tt.Exchange(dist, coll_dev), dist, coll_dev, local)))
    for k, (name, fn) in enumerate(legs):
        res = run_leg(name, fn, dist, coll_dev, rank, out, a.leg_deadline, [n for n, _ in legs[k + 1:]])
        if rank == 0:
            out[name] = res
    if rank == 0 and not a.no_full_evaluate:
        out["full_evaluate"] = full_evaluate(tt, ctx, model, N)
    if rank == 0 and not a.no_dropin:
        out["dropin"] = dropin(tt, ds, model)
    if rank == 0 and not a.no_stress:
        out["stress"] = stress(tt, a.stress_iters)
    if rank == 0 and a.config4:
        out["config4_tempering"] = tempering_config4(tt, ctx, ds, rounds=a.config4_rounds)
        out["exchange_cost"] = exchange_cost(tt, ctx, ds, rounds=a.config4_rounds)
    if rank == 0 and not a.no_full_evaluate:  # SURVEY 8f rows 2 and 4, measured beside their CPU restatements
        out["posterior_maps"] = posterior_maps(tt, ctx, ds)
        out["ingest_trilinear"] = ingest_trilinear(tt)
    if rank == 0 and a.batch_chains > 0:
        out["many_chains"] = many_chains(tt, ctx, ds, prm, model, a.batch_chains, a.batch_iters)
        # more chains than CUs: td_chain_run_batch packs two per CU by itself
        out["many_chains_2per_cu"] = many_chains(tt, ctx, ds, prm, model, 2 * a.batch_chains, a.batch_iters)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:  # the host-core baseline: N = 1 only
        out["cpu_baseline"] = cpu_baseline(ds, model, a.cpu_seconds, tt if not a.no_full_evaluate else None)
        if out["cpu_baseline"]["value"] > 0:
            out["speedup_vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
        aux = out["cpu_baseline"].get("aux", {})
        for key, unit in (("posterior_maps", "ms_per_section"), ("ingest_trilinear", "ms")):
            if key in aux and key in out and out[key][unit] > 0:
                out[key]["cpu_baseline"] = aux[key]
                out[key]["speedup_vs_cpu_baseline"] = round(aux[key][unit] / out[key][unit], 1)
    for c in chains:
        c.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def ladder_modes(tt, device):
    """The three ways one process runs a resident ladder: the swaps decided by
    the host between posted rounds (td_rounds_temper), decided inside the
    kernel with the phis meeting in device memory (td_rounds_exchange, no
    collective), and decided inside the kernel after an RCCL allgather of the
    library's own one-rank communicator (the exchange stream waiting on the
    kernel's flag: the mechanism a rank uses at N GPUs)."""
    return [("host_decided", False, None), ("device_swaps", True, None),
            ("device_swaps_rccl", True, tt.NativeComm(device))]


def run_ladder(tt, chains, device_swaps, comm, swap_every, rounds, warm=20):
    ex = tt.Exchange()
    ex.comm = comm
    lad = tt.TemperingLadder(chains, ex, tmax=8.0, seed=4242, device_swaps=device_swaps)
    lad.run(warm, swap_every)
    t0 = time.perf_counter()
    lad.run(rounds, swap_every)  # one resident launch: the swap steps in the library or in the kernel
    el = time.perf_counter() - t0
    lad.close()
    out = {"ms_per_round": round(el / rounds * 1e3, 4),
           "proposals_per_s": round(len(chains) * swap_every * rounds / el, 1),
           "trace_sha256": lad.trace_digest()}
    if lad.timing:
        out["split_us_per_round"] = {k: lad.timing[k] for k in ("exchange_us_per_round", "proposals_us_per_round",
                                                                 "slowest_replica_wait_us_per_round")}
    return out, lad


def tempering_config4(tt, ctx, ds, nrep=8, ncells=2000, swap_every=10, rounds=300):
    """BASELINE config 4's ladder on ONE GPU: 8 tempered replicas x 2000 cells
    (seeds 100 + replica), geometric T in [1, 8], a swap round every 10
    proposals, one resident launch -- in each of ladder_modes' three ways,
    which must leave the same trace (the top-level numbers: host_decided).
    The N-GPU runs put one rank per GPU (config4_ranks)."""
    res = {"replicas": nrep, "cells": ncells, "swap_every": swap_every, "rounds": rounds, "modes": {}}
    digests = set()
    for name, dev_swaps, comm in ladder_modes(tt, ctx.device):
        chains = config4_replicas(tt, ctx, ds, 0, nrep, ncells)
        out, lad = run_ladder(tt, chains, dev_swaps, comm, swap_every, rounds)
        digests.add(out["trace_sha256"])
        res["modes"][name] = out
        if name == "host_decided":
            res.update({"proposals_per_s": out["proposals_per_s"], "ms_per_round": out["ms_per_round"],
                        "rounds_by": "one resident k_chain_run launch; swap steps in the library between rounds "
                                     "(td_rounds_temper, no return to Python per round)",
                        "temps": [round(t, 4) for t in lad.temps],
                        "swap_rates": [round(r, 3) for r in lad.swap_rates()],
                        "mixing": lad.mixing(), "cold_phi": chains[lad.cold_local()].stats()["phi"]})
        for c in chains:
            c.close()
        if comm is not None:
            comm.close()
    res["modes_same_trace"] = len(digests) == 1
    res["calibrated"] = calibrated_ladder(tt, ctx, ds, nrep, ncells, swap_every)
    return res


def calibrated_ladder(tt, ctx, ds, nrep=8, ncells=2000, swap_every=10, tmax=1.1, burn=200, rounds=2000):
    """Beside BASELINE's ladder (T in [1, 8]: its replicas' misfits differ by
    thousands, so neighbours almost never swap), the same 8 replicas on a
    ladder that mixes at this model size: T_max = 1.1, chosen from the sweep in
    profiles/r04/ladder_calibration.json (tools/calibrate_ladder.py) as the
    widest ladder with every adjacent swap rate well above 20 % and replicas
    completing round trips.  Device-decided rounds; a burn-in, then the
    measured rounds."""
    chains = config4_replicas(tt, ctx, ds, 0, nrep, ncells)
    lad = tt.TemperingLadder(chains, tmax=tmax, seed=4242, device_swaps=True)
    lad.run(burn, swap_every)
    tried0, acc0, trips0 = lad.tried.copy(), lad.accepted.copy(), int(lad.trips.sum())
    t0 = time.perf_counter()
    lad.run(rounds, swap_every)
    el = time.perf_counter() - t0
    lad.close()
    rates = [float(a) / t if t else 0.0 for a, t in zip(lad.accepted - acc0, lad.tried - tried0)]
    for c in chains:
        c.close()
    return {"tmax": tmax, "temps": [round(t, 4) for t in lad.temps], "burn_rounds": burn, "rounds": rounds,
            "ms_per_round": round(el / rounds * 1e3, 4), "swap_rates": [round(r, 3) for r in rates],
            "round_trips": int(lad.trips.sum()) - trips0, "mixing": lad.mixing()}


def exchange_cost(tt, ctx, ds, swap_every=10, rounds=300, ncells=2000):
    """What the exchange step costs a rank of config 4 at N GPUs, measured on
    one: ONE replica (replica 0), a round of 10 proposals, in ladder_modes'
    three ways.  host_decided is the resident round with a host handshake;
    device_swaps_rccl adds the real collective machinery (flag -> stream wait
    -> ncclAllGather -> stream write -> kernel) that every round of a rank
    pays, minus only the xGMI hop of a multi-GPU allgather."""
    res = {"replicas": 1, "cells": ncells, "swap_every": swap_every, "rounds": rounds}
    for name, dev_swaps, comm in ladder_modes(tt, ctx.device):
        chains = config4_replicas(tt, ctx, ds, 0, 1, ncells)
        out, _ = run_ladder(tt, chains, dev_swaps, comm, swap_every, rounds)
        out.pop("trace_sha256")
        res[name] = out
        for c in chains:
            c.close()
        if comm is not None:
            comm.close()
    base = res["host_decided"]["ms_per_round"]
    res["rccl_round_over_resident_round"] = round(res["device_swaps_rccl"]["ms_per_round"] / base, 4)
    return res


def config4_replicas(tt, ctx, ds, first, count, ncells=2000):
    """BASELINE config 4's replicas g = first .. first + count - 1: seed
    100 + g, chain id 1 + g, model random_model(ncells, 100 + g), max_cells
    2 ncells (tests/tempering_worker.py builds the same)."""
    prm = tt.define_TDstructrure().replace(max_cells=2 * ncells)
    return [tt.Chain(ctx, tt.chain_params(prm, ds, seed=100 + g, chain=1 + g), tt.random_model(ncells, 100 + g))
            for g in range(first, first + count)]


def config4_ranks(tt, ds, dist, coll_dev, rank, world, device, swap_every=10, rounds=300, warm=20):
    """BASELINE config 4 across the ranks: one tempered replica per rank
    (replica g = rank), geometric T in [1, 8] over the world, a swap round
    every 10 proposals.  Two ways, each timed over the same rounds, value =
    all ranks' proposals / the max-over-ranks time:

    * device_swaps (RCCL only): ONE resident launch per rank for all rounds;
      each round the kernel raises a flag, the library's exchange stream
      (waiting on it) runs ncclAllGather of every rank's phi over xGMI and
      writes the round's done word, and the kernel decides the swaps itself
      (td_rounds_exchange) -- no host in the loop;
    * host_loop: TemperingLadder.step -- the resident round posted by the host,
      Exchange.allgather through torch.distributed (RCCL, or gloo in the
      one-GPU rehearsal), the decision in Python.

    Rank 0 then replays the same ladder in ONE process (all `world` replicas
    on its GPU): the swap traces' digests must be equal.  Each mode carries a
    roofline block for the replica's kernel (latency-bound; the in-kernel byte
    count over the timed region against HBM) and its per-round split."""
    import torch

    ctx = tt.TdContext.from_datastruct(ds, device=device)
    res = {"replicas": world, "ranks": world, "cells": 2000, "swap_every": swap_every, "rounds": rounds,
           "collective": "allgather of 8 B per rank (%s)" % ("RCCL" if coll_dev == "cuda" else "gloo"), "modes": {}}
    modes = (["device_swaps"] if coll_dev == "cuda" else []) + ["host_loop"]
    digest = None
    for mode in modes:
        chains, ex, lad, err = [], None, None, None
        try:
            chains = config4_replicas(tt, ctx, ds, rank, 1)
            if mode == "device_swaps":
                ex = tt.Exchange(dist, coll_dev, native=device)
                lad = tt.TemperingLadder(chains, ex, tmax=8.0, seed=4242, device_swaps=True)
                lad.run(warm, swap_every)
            else:
                ex = tt.Exchange(dist, coll_dev)
                lad = tt.TemperingLadder(chains, ex, tmax=8.0, seed=4242)
                for _ in range(warm):
                    lad.step(swap_every)
            b0 = chains[0].stats()["bytes"]
            c0, g0, d0 = lad.compute_s, lad.gather_s, lad.decide_s
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            if mode == "device_swaps":
                lad.run(rounds, swap_every)
            else:
                for _ in range(rounds):
                    lad.step(swap_every)
            el = time.perf_counter() - t0
            lad.close()
            nbytes = chains[0].stats()["bytes"] - b0
            t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_max = float(t[0].item())
            out = {"proposals_per_s": round(world * swap_every * rounds / el_max, 1),
                   "ms_per_round": round(el_max / rounds * 1e3, 4), "trace_sha256": lad.trace_digest()}
            if mode == "device_swaps":
                tm = lad.timing
                out["split_us_per_round"] = {"exchange": tm["exchange_us_per_round"],
                                             "proposals": tm["proposals_us_per_round"],
                                             "launch_amortized": round((tm["call_s"] - tm["kernel_span_s"]) / rounds * 1e6,
                                                                       3)}
            else:
                out["split_us_per_round"] = {"compute": round((lad.compute_s - c0) / rounds * 1e6, 3),
                                             "gather": round((lad.gather_s - g0) / rounds * 1e6, 3),
                                             "decide": round((lad.decide_s - d0) / rounds * 1e6, 3)}
            out["roofline"] = chain_roofline("k_chain_run (config-4 replica, resident rounds)",
                                             model_bytes(int(ctx.P), int(ctx.n), 2000), swap_every * rounds, el, nbytes,
                                             None, False)
            out["roofline"]["latency"] = phase_cycles(tt, chains[0], 2000)
            if digest is None:
                digest = out["trace_sha256"]
                res.update({"temps": [round(x, 4) for x in lad.temps], "swap_rates": [round(r, 3) for r in lad.swap_rates()],
                            "mixing": lad.mixing()})
            res["modes"][mode] = out
        except Exception as e:  # (a mode that fails on every rank, e.g. an exchange watchdog, is reported)
            err = repr(e)[:300]
            try:
                if lad is not None:
                    lad.close()
            except Exception:
                pass
        for c in chains:
            c.close()
        if ex is not None and ex.comm is not None:
            ex.comm.close()
        flag = torch.tensor([1.0 if err else 0.0], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if float(flag[0].item()) > 0:
            res["modes"][mode] = {"error": err or "failed on another rank"}
    good = [m for m in res["modes"].values() if "error" not in m]
    if not good:
        ctx.close()
        return res
    best = min(good, key=lambda m: m["ms_per_round"])
    res["proposals_per_s"], res["ms_per_round"] = best["proposals_per_s"], best["ms_per_round"]
    res["roofline"] = best["roofline"]
    if rank == 0:  # the one-process ladder of the same replicas
        ref = config4_replicas(tt, ctx, ds, 0, world)
        lad1 = tt.TemperingLadder(ref, tmax=8.0, seed=4242)
        lad1.run(warm + rounds, swap_every)
        lad1.close()
        res["trace_sha256"] = digest
        res["trace_matches_single_process"] = all(m["trace_sha256"] == lad1.trace_digest() for m in good)
        for c in ref:
            c.close()
    ctx.close()
    return res


def stress_chains(tt, dist, coll_dev, rank, world, device, iters):
    """BASELINE config 5 across the ranks: 10k synthetic rays x 20k cells,
    one chain per rank (seed 77 + rank), `iters` proposals each; value = all
    ranks' proposals / the max-over-ranks time (weak scaling)."""
    import torch

    ds = tt.synthetic_rays(10000, seed=5)
    ctx = tt.TdContext.from_datastruct(ds, device=device)
    prm = tt.define_TDstructrure().replace(max_cells=40000)
    ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=77 + rank, chain=1 + rank), tt.random_model(20000, 5))
    ch.run(200)
    b0 = ch.stats()["bytes"]
    torch.cuda.synchronize()
    dist.barrier()
    ctx.timing(enable=True, reset=True)
    t0 = time.perf_counter()
    ch.run(iters)
    el = time.perf_counter() - t0
    launches, kms = ctx.timing(kernel="chain_run")
    ctx.timing(enable=False)
    nbytes = ch.stats()["bytes"] - b0
    t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    res = {"chains": world, "rays": int(ctx.n), "cells": 20000, "iters_per_chain": iters,
           "proposals_per_s": round(world * iters / el, 1), "per_chain_proposals_per_s": round(iters / el, 1),
           "phi_rank0": ch.stats()["phi"],
           "roofline": chain_roofline("k_chain_run<false, false> (rays in HBM), this rank's chain",
                                      model_bytes(int(ctx.P), int(ctx.n), 20000), iters,
                                      kms / 1e3 / max(launches, 1), nbytes, "k_chain_run/stress", iters == 2000)}
    ch.close()
    ctx.close()
    return res


def many_chains(tt, ctx, ds, prm, model, C, iters, steps=3, lds_mode=0):
    """Occupancy mode (SURVEY 7 / 8d "batched multi-chain streams"): C
    independent config-3 chains on this GPU, one workgroup each, one launch
    per step.  More chains than CUs: two per CU (the 4-wave tiles-in-LDS
    kernel, the launcher's own choice; lds_mode 2 forces it).
    Reported beside the headline, never as `value`."""
    chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model) for j in range(C)]
    for c in chains:
        if lds_mode:
            tt.lib().tdt_chain_set_lds_mode(c.h, lds_mode)
    # two chains per CU: forced (lds_mode 2), or the launcher's own choice for more chains than CUs
    packed = lds_mode == 2 or (lds_mode == 0 and C > ctx.num_cus)
    tt.run_batch(chains, iters)  # warmup
    b0 = sum(c.stats()["bytes"] for c in chains)
    ctx.timing(enable=True, reset=True)
    t0 = time.perf_counter()
    for _ in range(steps):
        tt.run_batch(chains, iters)
    el = time.perf_counter() - t0
    launches, kms = ctx.timing(kernel="chain_run")
    ctx.timing(enable=False)
    nbytes = sum(c.stats()["bytes"] for c in chains) - b0
    for c in chains:
        c.close()
    value = C * iters * steps / el
    avg_s = kms / 1e3 / max(launches, 1)
    roof = chain_roofline("k_chain_run (grid = %d chains)" % C, model_bytes(int(ctx.P), int(ctx.n), len(model.xCell)),
                          C * iters, avg_s, nbytes / max(launches, 1),
                          "k_chain_run/many%d%s" % (C, "x2" if packed else ""), iters == 5000)
    return {"chains": C, "chains_per_cu": 2 if packed else 1, "proposals_per_s": round(value, 1), "per_chain_proposals_per_s": round(value / C, 1),
            "ms_per_launch": round(kms / max(launches, 1), 4), "iters_per_launch": iters, "roofline": roof}


def dropin(tt, ds, model, iters=1500, host_iters=300):
    """The drop-in boundary as an unchanged Julia host drives it: the
    reference's loop on the host (TD_inversion_function.jl:70-274), one
    td_evaluate of the proposed model per proposal and a td_interpolate per
    birth/death query (:81, :146) -- TD_ENGINE_DROPIN, whose td_evaluate calls
    take the incremental path -- beside the same loop with every evaluate in
    full (TD_ENGINE_HOST, what td_evaluate cost before the incremental path)."""
    prm = tt.define_TDstructrure().replace(max_cells=2 * len(model.xCell))
    out = {}
    for name, engine, k in (("incremental", tt.TD_ENGINE_DROPIN, iters), ("full_evaluate", tt.TD_ENGINE_HOST,
                                                                          host_iters)):
        ctx = tt.TdContext.from_datastruct(ds)
        ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000, chain=1, engine=engine), model)
        ch.run(50)
        e0 = ch.stats()["evaluations"]
        ctx.timing(enable=True, reset=True)
        dt = np.zeros(18, dtype=np.int64)
        tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data_as(tt._lib._pi64))
        t0 = time.perf_counter()
        ch.run(k)
        el = time.perf_counter() - t0
        tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data_as(tt._lib._pi64))
        ne = ch.stats()["evaluations"] - e0
        res = {"proposals_per_s": round(k / el, 1), "us_per_proposal": round(el / k * 1e6, 2), "evaluates": ne,
               "proposals": k}
        if engine == tt.TD_ENGINE_DROPIN:
            res["served_by"] = ("one resident k_chain_run per shadow chain, fed each td_evaluate / td_interpolate "
                                "through a pinned mailbox (no launch per call)")
            us = lambda v: round(float(v) / 1e3 / k, 3)  # noqa: E731  (ns summed -> us per proposal)
            ev, ip = dt[0], dt[3]
            res["breakdown_us_per_proposal"] = {
                "td_evaluate": us(ev), "evaluate_classify": us(dt[1]), "evaluate_server_round_trip": us(dt[2]),
                "evaluate_rest": us(ev - dt[1] - dt[2]),
                "td_interpolate_1pt": us(ip), "interpolate_classify": us(dt[4]),
                "interpolate_server_round_trip": us(dt[5]), "interpolate_rest": us(ip - dt[4] - dt[5]),
                "host_loop_modeln_copy": us(dt[9]), "host_loop_rest": us(dt[10] - ev - ip - dt[9]),
                "server_busy_evaluate": us(dt[16]), "server_busy_interpolate": us(dt[17]),
                "calls_per_proposal": {"td_evaluate": round(float(dt[6]) / k, 3),
                                       "td_interpolate": round(float(dt[7]) / k, 3),
                                       "full_evaluates": int(dt[8])}}
        ctx.timing(enable=False)
        out[name] = res
        ch.close()
        ctx.close()
    out["speedup"] = round(out["incremental"]["proposals_per_s"] / out["full_evaluate"]["proposals_per_s"], 2)
    return out


def full_evaluate(tt, ctx, model, N, reps=50):
    """The drop-in td_evaluate (MCsub.jl:123-185) on the same model, both
    nearest-cell methods: the bucket grid (default from 256 cells) and the
    reference-shaped brute force (every point x every cell), whose dominant
    kernel nn_tile is FP64-VALU bound (no FMA: 39.3 TFLOP/s roof)."""
    cells = model.cells()
    E = ctx.P * N
    out = {}
    kernels = {"grid": ["nn_grid_build", "nn_grid", "ray_sums"],
               "brute_force": ["nn_tile", "nn_partial", "nn_merge", "ray_sums"]}
    tt.lib().tdt_set_incremental(ctx.h, 0)  # every call a full evaluate (repeats would hit the shadow's cache)
    for name, method in (("grid", ctx.NN_GRID), ("brute_force", ctx.NN_BRUTE)):
        ctx.set_nn_method(method)
        for _ in range(3):
            ctx.evaluate(cells)
        t0 = time.perf_counter()  # wall time per call, no event timing
        for _ in range(reps):
            ctx.evaluate(cells)
        el = (time.perf_counter() - t0) / reps
        dt = np.zeros(18, dtype=np.int64)
        tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data_as(tt._lib._pi64))
        for _ in range(reps):
            ctx.evaluate(cells)
        tt.lib().tdt_dropin_timing(ctx.h, 1, dt.ctypes.data_as(tt._lib._pi64))
        host = {k: round(float(dt[i]) / 1e3 / reps, 3) for k, i in (("pack_cells", 12), ("issue_kernels", 13),
                                                                    ("wait_kernels", 14), ("chi2_copy_out", 15))}
        ctx.timing(enable=True, reset=True)  # then the kernels, timed with HIP events
        for _ in range(reps):
            ctx.evaluate(cells)
        km = {}
        for k in kernels[name]:
            nl, ms = ctx.timing(kernel=k)
            if nl:
                km[k] = round(ms / nl, 4)
        ctx.timing(enable=False)
        out[name] = {"evaluate_ms": round(el * 1e3, 4), "evaluates_per_s": round(1.0 / el, 1),
                     "nn_pair_evals_per_s_equiv": round(E / el, 1), "kernel_ms": km, "host_us": host}
    ctx.set_nn_method(ctx.NN_AUTO)
    tt.lib().tdt_set_incremental(ctx.h, 1)
    # the dominant kernel: the one-launch tile search (the split search only when forced)
    km = out["brute_force"]["kernel_ms"]
    kname = "nn_tile" if "nn_tile" in km else "nn_partial"
    t_nn = km.get(kname, 0.0) / 1e3
    flops = 8.0 * E  # 3 sub + 3 mul + 2 add per distance, no FMA allowed
    tf = flops / t_nn / 1e12 if t_nn > 0 else 0.0
    out["brute_force"]["roofline"] = {"kernel": kname, "bound": "valu-fp64", "achieved": round(tf, 3),
                                      "peak": FP64_NOFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                      "frac": round(tf / FP64_NOFMA_PEAK_TFLOPS, 4), "flops_per_launch": flops}
    tr, src, _ = measured_traffic("k_%s/%s" % (kname, "config3" if ctx.P < 100000 else "stress"))
    if tr is not None:
        out["brute_force"]["roofline"]["traffic"] = tr
        out["brute_force"]["roofline"]["traffic_source"] = src
        out["brute_force"]["roofline"]["compulsory_bytes"] = 24 * ctx.P + 32 * N + 20 * ctx.P
    return out


def stress(tt, chain_iters=2000):
    """BASELINE config 5 on one GPU: 10k synthetic rays (seed 5) x 20k cells.
    The drop-in evaluate with both nearest-cell methods, and the device chain
    (its tiles / rays / order no longer fit in LDS: the HBM layout)."""
    ds = tt.synthetic_rays(10000, seed=5)
    ctx = tt.TdContext.from_datastruct(ds)
    model = tt.random_model(20000, 5)
    res = {"rays": int(ctx.n), "points": int(ctx.P), "cells": 20000}
    res["evaluate"] = full_evaluate(tt, ctx, model, 20000, reps=5)
    prm = tt.define_TDstructrure().replace(max_cells=40000)
    ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=77, chain=1), model)
    ch.run(200)
    b0 = ch.stats()["bytes"]
    ctx.timing(enable=True, reset=True)
    t0 = time.perf_counter()
    ch.run(chain_iters)
    el = time.perf_counter() - t0
    launches, kms = ctx.timing(kernel="chain_run")
    ctx.timing(enable=False)
    res["chain"] = {"proposals_per_s": round(chain_iters / el, 1), "iters": chain_iters,
                    "layout": "hbm (tiles, rays, order do not fit in LDS)",
                    "roofline": chain_roofline("k_chain_run<false, false> (rays in HBM)", model_bytes(int(ctx.P), int(ctx.n), 20000),
                                               chain_iters, kms / 1e3 / max(launches, 1), ch.stats()["bytes"] - b0,
                                               "k_chain_run/stress", chain_iters == 2000)}
    ch.close()
    ctx.close()
    return res


def stress_sharded(tt, ex, dist, coll_dev, device, reps=10):
    """SURVEY 8e's optional intra-chain split, on config 5's evaluate: every
    rank owns a ray range of the 10k synthetic rays (sharded.py), one evaluate
    = td_evaluate of its shard + an allgather of ptS + td_misfit of all rays
    (bit-identical to one GPU's evaluate: tests/test_gpu_sharded.py).  Full
    evaluates (no incremental path), time = max over ranks."""
    import torch

    ds = tt.synthetic_rays(10000, seed=5)
    sc = tt.RayShardedContext(ds, ex, device=device)
    tt.lib().tdt_set_incremental(sc.local.h, 0)
    cells = tt.random_model(20000, 5).cells()
    for _ in range(2):
        sc.evaluate(cells)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        _, phi, _ = sc.evaluate(cells)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    res = {"ranks": ex.world, "rays": int(sc.n), "cells": 20000, "evaluate_ms": round(el / reps * 1e3, 4),
           "evaluates_per_s": round(reps / el, 1), "rays_per_rank": [b - a for a, b in sc.bounds], "phi": phi,
           "note": "td_evaluate of each rank's rays + allgather of ptS + td_misfit (sequential chi^2 of all rays); "
                   "compare stress.evaluate.grid.evaluate_ms (one GPU, all rays)"}
    sc.close()
    return res


def posterior_inputs(tt, ds, nmodels=100, ncells=5000):
    """plot_model_hist's workload (MCsub.jl:753-781): one xz section at the
    reference's node grid (xVec x zVec, y = 100 km) over `nmodels` saved models
    of `ncells` cells (synthetic, seeded)."""
    models = [tt.random_model(ncells, 700 + k).cells() for k in range(nmodels)]
    xv, zv = np.asarray(ds.xVec, dtype=np.float64), np.asarray(ds.zVec, dtype=np.float64)
    qx, qz = np.tile(xv, len(zv)), np.repeat(zv, len(xv))
    return models, qx, np.full(qx.shape, 100.0), qz


def posterior_maps(tt, ctx, ds):
    """SURVEY 8f row 2, plot_model_hist (MCsub.jl:753-781): every node's
    v_nearest value in every saved model, then mean and std over the models
    (td_rasterize, posterior_inputs).  Its CPU leg is timed in cpu_baseline."""
    models, qx, qy, qz = posterior_inputs(tt, ds)
    ncells = len(models[0][0])
    ctx.rasterize(models[:2], qx, qy, qz)  # warm
    reps = 3
    ctx.timing(enable=True, reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.rasterize(models, qx, qy, qz)
    el = (time.perf_counter() - t0) / reps
    nl, kms = ctx.timing(kernel="raster_brute")
    ctx.timing(enable=False)
    flops = 8.0 * len(qx) * ncells * len(models)  # 3 sub + 3 mul + 2 add per distance, no FMA
    k_s = kms / 1e3 / max(nl, 1) if nl else 0.0
    tf = flops / k_s / 1e12 if k_s > 0 else 0.0
    roof = {"kernel": "k_raster_brute", "bound": "valu-fp64", "achieved": round(tf, 3),
            "peak": FP64_NOFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / FP64_NOFMA_PEAK_TFLOPS, 4),
            "flops_per_launch": flops,
            # every model's cells x, y, z once, its zeta per node, the nodes, the values written
            "compulsory_bytes": 24 * ncells * len(models) + 8 * len(qx) * len(models) + 24 * len(qx) +
                                8 * len(qx) * len(models)}
    tr, src, _ = measured_traffic("k_raster_brute/section")
    if tr is not None and len(models) == 100 and ncells == 5000:
        roof["traffic"], roof["traffic_source"] = tr, src
    return {"nodes": int(len(qx)), "models": len(models), "cells": ncells, "ms_per_section": round(el * 1e3, 3),
            "kernel_ms_per_section": round(kms / max(nl, 1), 4) if nl else None, "roofline": roof,
            "note": "ms_per_section: the whole call from host arrays (cells packed into pinned memory, one copy); "
                    "kernel: every model at every node in one launch (k_raster_brute)",
            "node_model_pairs_per_s": round(len(qx) * len(models) / el, 1),
            "nn_pair_evals_per_s_equiv": round(float(len(qx)) * ncells * len(models) / el, 1)}


def trilinear_inputs(tt, grid=(120, 70, 40), seed=3):
    """The ray points of the 10k synthetic stress rays and a seeded slowness
    grid of `grid` knots covering them (pre_process_data.jl:34's workload)."""
    s = tt.synthetic_rays(10000, seed=5)
    px, py, pz = (a.T[~np.isnan(s.rayX.T)] for a in (s.rayX, s.rayY, s.rayZ))
    rng = np.random.default_rng(seed)
    lo = [min(a.min(), 0.0) - 1.0 for a in (px, py, pz)]
    hi = [a.max() + 1.0 for a in (px, py, pz)]
    xs, ys, zs = (np.sort(np.concatenate([[l, h], rng.uniform(l, h, n - 2)])) for l, h, n in zip(lo, hi, grid))
    return xs, ys, zs, 1.0 / rng.uniform(5.0, 9.0, grid), px, py, pz


def ingest_trilinear(tt):
    """SURVEY 8f row 4, the ray points' slowness (Gridded(Linear()) of
    load_3Dvel.jl:32): td_trilinear over every stress ray point; host buffers
    in and out (PCIe included).  Its CPU leg is timed in cpu_baseline."""
    from importlib import import_module
    xs, ys, zs, vals, px, py, pz = trilinear_inputs(tt)
    itp = import_module(tt.__name__ + ".ingest").Gridded(xs, ys, zs, vals, device=0)
    itp(px[:1000], py[:1000], pz[:1000])  # warm
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        itp(px, py, pz)
    el = (time.perf_counter() - t0) / reps
    return {"points": int(len(px)), "grid": [len(xs), len(ys), len(zs)], "ms": round(el * 1e3, 3),
            "points_per_s": round(len(px) / el, 1), "note": "host arrays in and out: PCIe-inclusive"}


def host_cores():
    """The host cores this job may use, read from the OS: the CPUs in this
    process's affinity mask (os.sched_getaffinity), capped by the CPU share
    the box exports in OMP_NUM_THREADS when that is smaller (the GPU box's
    mask and os.cpu_count() show the whole machine, its share is 16).
    Returns (cores used, the facts they were chosen from)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    used = min(aff, omp) if omp > 0 else aff
    src = "OMP_NUM_THREADS (the job's CPU share)" if 0 < omp < aff else "os.sched_getaffinity(0)"
    return max(1, used), {"sched_getaffinity": aff, "os_cpu_count": os.cpu_count(),
                          "OMP_NUM_THREADS": omp if omp > 0 else None, "cores_from": src}


def cpu_baseline(ds, model, seconds, tt=None):
    """The reference's structure on the host: one full evaluate per proposal
    (oracle/tstar_oracle.c, the scalar restatement of MCsub.jl:123-185), one
    chain per core as main_inversion.jl:15's pmap runs them.  Threads call the
    C oracle through ctypes, which releases the GIL, so they run in parallel.
    Timed on 1 core, then on every core of the job's share."""
    import threading

    import oracle  # CPU baseline leg only

    oracle.lib()
    cells = model.cells()

    def leg(threads, secs):
        counts = [0] * threads
        t0 = time.perf_counter()

        def work(k):
            while time.perf_counter() - t0 < secs:
                oracle.evaluate(ds.rayX, ds.rayY, ds.rayZ, ds.rayL, ds.rayU, ds.tS, ds.allSig, cells)
                counts[k] += 1

        ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return sum(counts), time.perf_counter() - t0

    n1, el1 = leg(1, seconds * 0.5)
    cores, core_facts = host_cores()
    nc, elc = leg(cores, seconds * 0.5)
    aux = {}
    if tt is not None:  # the CPU legs of SURVEY 8f rows 2 and 4: the checker's numpy restatements, one core
        from oracle import oracle_np

        models, qx, qy, qz = posterior_inputs(tt, ds)
        k = 10
        t0 = time.perf_counter()
        oracle_np.rasterize(models[:k], qx, qy, qz)
        el = (time.perf_counter() - t0) * len(models) / k
        aux["posterior_maps"] = {"ms_per_section": round(el * 1e3, 1), "cores": 1, "kind": "port (numpy)",
                                 "sample": "%d of the %d models, scaled" % (k, len(models))}
        xs, ys, zs, vals, px, py, pz = trilinear_inputs(tt)
        t0 = time.perf_counter()
        oracle_np.trilinear(xs, ys, zs, vals, px, py, pz)
        aux["ingest_trilinear"] = {"ms": round((time.perf_counter() - t0) * 1e3, 1), "cores": 1,
                                   "kind": "port (numpy)", "sample": "all %d points" % len(px)}
    return {"value": round(nc / elc, 3), "unit": "proposals/s", "cores": cores, "host": core_facts,
            "kind": "port", "aux": aux,
            "single_core_value": round(n1 / el1, 3),
            "sample": "full evaluates (oracle/tstar_oracle.c, scalar FP64, -O2) of the same 381-ray x %d-cell "
                      "model, one chain per core: %d in %.1f s on %d cores, %d in %.1f s on 1 core; the reference "
                      "evaluates every proposal in full" % (len(cells[0]), nc, elc, cores, n1, el1)}


if __name__ == "__main__":
    main()
