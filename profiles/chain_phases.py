#!/usr/bin/env python3
"""Diagnostic: where one DEVICE-engine chain iteration spends its cycles.

Runs the config-3 chain (381 rays x 5000 cells) with the kernel's s_memtime
phase stamps enabled (a diagnostic mode; never used for bench numbers) and
prints the per-phase share of shader cycles and cycles per iteration."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tonga  # noqa: E402

# k_chain_run phases A..G (chain_kernels.hip, STAMP(0..6))
PHASES = ["(loop top)", "B tiles + birth/death query", "C points", "D orphans", "E ray sums",
          "F chi2 + accept || next proposal, tile maxima", "G commit + grid update + next proposal"]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    nrays = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # > 0: synthetic rays (the stress geometry: 10000)
    tt = tonga.load()
    ds = tt.synthetic_rays(nrays, seed=5) if nrays > 0 else tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=2 * N)
    ch = tt.Chain(ctx, tt.chain_params(prm, ds, seed=1000, chain=1), tt.random_model(N, 3))
    ch.run(2000 if nrays == 0 else 200)
    L = tt.lib()
    out0 = (ctypes.c_int64 * 80)()
    L.tdt_chain_profile(ch.h, 1, out0)
    st0 = ch.stats()
    t0 = time.perf_counter()
    ch.run(iters)
    el = time.perf_counter() - t0
    out = (ctypes.c_int64 * 80)()
    L.tdt_chain_profile(ch.h, 0, out)
    cyc = np.array(out[:7], dtype=np.float64) - np.array(out0[:7], dtype=np.float64)
    cyc[6] += (out[12] - out0[12]) + (out[13] - out0[13])  # G = commit + next proposal + barrier
    fallbacks = int(out[15] - out0[15])
    tot = cyc.sum()
    st1 = ch.stats()
    prop = np.array(st1["proposed"], dtype=np.float64) - np.array(st0["proposed"], dtype=np.float64)
    act = np.array(out[8:12], dtype=np.float64) - np.array(out0[8:12], dtype=np.float64)
    per_action = {a: round(c / max(k, 1), 1) for a, c, k in zip(["birth", "death", "change", "move"], act, prop)}
    res = {"cells": N, "iters": iters, "us_per_iter_wall": el / iters * 1e6,
           "cycles_per_iter": tot / iters, "grid_fallbacks": fallbacks,
           "phases": {p: {"share": round(c / tot, 4), "cycles_per_iter": round(c / iters, 1)}
                      for p, c in zip(PHASES, cyc)},
           "cycles_per_proposal_by_action": per_action,
           "early_rejections": int(out[14] - out0[14]),
           "rejections": int(sum(prop) - (sum(ch.stats()["accepted"]) - sum(st0["accepted"]))),
           "G sub-phases per iter (tid 0)": {
               "commit": round((out[12] - out0[12]) / iters, 1),
               "next proposal": round((out[13] - out0[13]) / iters, 1),
               "final barrier": round((out[6] - out0[6]) / iters, 1)}}
    # the same phases split by action: cycles per proposal of that action
    names = PHASES[:6] + ["G commit", "G next proposal", "final barrier"]
    res["phases_by_action (cycles per proposal)"] = {
        a: {names[j]: round((out[16 + 10 * i + j] - out0[16 + 10 * i + j]) / max(prop[i], 1), 1) for j in range(9)}
        for i, a in enumerate(["birth", "death", "change", "move"])}
    res["F per wave (cycles per iter): chi2 scan, next proposal, tile maxima x4, bound, grid prefetch"] = [
        round((out[56 + w] - out0[56 + w]) / iters, 1) for w in range(8)]
    ev = max(sum(prop), 1)
    res["chi2 tail terms per proposal"] = round((out[64] - out0[64]) / ev, 1)
    res["chi2 scan rounds per proposal"] = round((out[65] - out0[65]) / ev, 2)
    res["per evaluated proposal: tiles hit, points seen, points changed, rays changed"] = [
        round((out[k] - out0[k]) / ev, 1) for k in (68, 69, 70, 71)]
    res["chi2 walk (rays in HBM) per proposal: events, batch-load cycles, walk cycles, terms one by one"] = [
        round((out[k] - out0[k]) / ev, 1) for k in (72, 73, 74, 75)]
    res["F wave 0: cycles to scan end / to decision (per iter)"] = [round((out[k] - out0[k]) / iters, 1)
                                                                     for k in (66, 67)]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
