// chain_dev.h -- device state of one rj-MCMC chain (TD_ENGINE_DEVICE).
//
// Cells live in SLOTS (stable storage); order[pos] = slot and rank[slot] =
// pos keep the Julia order (birth appends, death deleteat!-shifts), which
// decides nearest-cell ties.  Per ray point the chain caches the exact FP64
// (slot, squared distance, zeta) of its nearest cell -- exactly what a full
// v_nearest scan would give -- so a proposal only touches:
//   birth : points the new cell captures (d < cached d)
//   death : points whose cell is the killed one (full re-search of those)
//   change: points whose cell is the changed one (zeta only)
//   move  : points of the moved cell (re-search) + points it captures
// Candidate points are found through 16-point ray tiles whose FP64 bounding
// boxes give an exact lower bound of the distance (computed with the same
// rounded operations as the distance itself, so LB <= d holds bit-wise).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "chain_logic.h"
#include "internal.h"

namespace tdstar {

constexpr int kTilePts = 16;
constexpr int kChainThreads = 1024;

struct ChainScalars {
    int64_t iter;          // next iteration index
    int64_t evaluations;
    int64_t accepted[5];
    int64_t proposed[5];
    double phi;
    int64_t bytes;         // algorithmic global-memory bytes the proposals needed (roofline)
    int ncells;            // cells in the model
    int nslots;            // slot high-water mark
    int nfree;             // free-slot stack depth
    int pad;
};

struct DevChain {
    // geometry (owned by the td_ctx)
    const double *px, *py, *pz, *w, *tS, *sig;
    const int *ray_off, *pt_ray;
    int P, n;
    // tiles of <= kTilePts consecutive points of one ray
    const int *tile_start;  // [ntiles+1]
    const int *tile_of;     // [P]
    const double *tile_lo, *tile_hi;  // [3][ntiles] SoA
    double *tile_maxd;      // [ntiles] max cached distance of the tile's points
    int ntiles;
    // cells by slot
    double *cx, *cy, *cz, *czeta;  // [cap]
    int *order, *rank, *free_slots, *order_tmp;  // [cap]
    int cap;
    // per-point cache (current state) and candidate overlay
    int *best_s;
    double *best_d, *zeta0;
    int *cand_s;
    double *cand_d, *cand_z;
    unsigned char *cand_flag;
    int *changed, *orphans, *tiles_hit;
    // rays
    double *ptS, *cand_ptS, *prefix, *cand_prefix;  // prefix[k] = chi^2 partial sum through ray k
    int *rays_hit;
    int *ray_flag;
    ChainScalars *st;
    tdchain::Params params;
    uint64_t seed;
    uint32_t chain;
};

// Build the cache from scratch for the cells currently in slots 0..ncells-1
// (order = rank = identity): nearest search, ray sums, chi^2 prefix, tile maxima.
hipError_t chain_full_state(DevChain &d, int ncells, NNWork &work, int num_cus, hipStream_t s);
// Run `iters` iterations inside one persistent workgroup.
hipError_t chain_run(const DevChain &d, int64_t iters, hipStream_t s);

}  // namespace tdstar
