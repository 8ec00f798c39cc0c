// chain_kernels.hip -- the device-resident rj-MCMC chain (TD_ENGINE_DEVICE).
//
// One persistent 1024-thread workgroup runs `iters` iterations of
// TD_inversion_function.jl:70-274 without returning to the host: draw the
// proposal (chain_logic.h, shared with the host engine), evaluate it
// incrementally against the cached per-point nearest cells (chain_dev.h),
// recompute t* only for the rays whose points changed (Julia sum order,
// ray_sum.h) and chi^2 only from the first changed ray on (the cached prefix
// sums ARE the reference's sequential partial sums), then accept or reject.
// Every phi it produces is bit-identical to a full evaluate of the proposed
// model (tests/test_gpu_chain.py checks it against the host engine).
//
// Why one workgroup: a proposal touches ~P/N points and a few rays, i.e.
// microseconds of latency-bound work; a grid-wide barrier costs 4-10 us on
// MI355X (MI355X_MICROARCH.md, barrier-xcd) and a kernel boundary ~1.5 us.
// One CU keeps the loop free of both.  What bounds an iteration is then the
// chain of dependent memory round trips and barriers, so:
//   * tile boxes (FP32, outward-rounded), tile maxima, every per-ray array and
//     the position->slot map live in LDS when they fit (SMALL: the 381-ray
//     configs) and are written back to HBM when the launch ends;
//   * the RNG draws of 64 iterations are computed ahead, one lane each;
//   * nearest-cell queries go through the bucket grid, one wave per query,
//     one round of loads, and overlap the tile pass;
//   * candidate flags are cleared, and the bucket grid updated, at the start of
//     the NEXT iteration, off the critical path;
//   * the sequential chi^2 tail runs on one lane from LDS, 8 terms per trip.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstddef>
#include <cstdlib>

#include "chain_dev.h"
#include "exact_sum.h"
#include "internal.h"
#include "ray_sum.h"
#include "wave_ops.h"

namespace tdstar {

namespace {

using tdchain::Proposal;

constexpr int kWaves = kChainThreads / 64;
static_assert(kTilePts == 16, "a tile is one 16-lane DPP row (row_max_u64)");
constexpr int kOrphanLds = 96;  // orphan records kept in LDS (more: read back from HBM)
constexpr int kPre = 64 / kTilePts;  // LDS layout: hit tiles per wave whose points phase B preloads
static_assert(kPre == 4, "the preload slots are four registers");
constexpr int kCtmLds = 256;    // tiles in LDS, rays in HBM: hit tiles' candidate maxima kept in LDS
constexpr int kListLds = 1024;
// LDS layout, phase D: from this many orphans on, one search for all of them (the bucket region
// around them staged once in LDS, a thread per orphan) instead of one wave's grid search each
constexpr int kBatchOrphans = 64;
constexpr int kBatchCand = 192;     // cell entries staged (phase E's idle ray scratch: 28 B each)
constexpr int kBatchBuckets = 512;  // buckets in the region at most  // rays in HBM: hit tiles / changed rays / hit super-tiles kept in LDS
// Phase C leaves lanes idle (16 per hit tile, ~8 tiles): wave 7 lane 0 forms the decision's
// phi_n-free parts; wave 6 lane 0 (LDS layout) begins the next proposal's guess -- its global loads
// fly across the phase barriers until phase F finishes it there
// The LDS layout could sum chi^2 with the event walk too; its tails are ~60 terms and the
// one-wave binade scan with the early-rejection bound is faster there (measured: the walk
// costs ~1.2k more cycles per proposal at 381 rays x 5000 cells)
constexpr bool kSmallWalk = false;

// A changed point's candidate (what mark() stores in the overlay), kept in LDS for the first kChgLds of
// a proposal: phase G commits them from here with stores only -- no dependent round trips to the
// changed list and the overlay in HBM
struct ChgRec {
    int q, s;
    double d, z;
};
constexpr int kChgLds = 64;

// A point whose nearest cell is removed or moved: re-searched in phase D.
struct OrphanRec {
    double x, y, z;
    int q, ray;
};

__device__ __forceinline__ double dist2(double cx, double cy, double cz, double x, double y, double z) {
    // (mx-x)^2 + (my-y)^2 + (mz-z)^2, MCsub.jl:254 -- same ops as k_nn_partial
    const double dx = cx - x, dy = cy - y, dz = cz - z;
    double d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

// (distance, Julia position) lexicographic order; a cell must also beat the
// 1e9 sentinel strictly (MCsub.jl:250,255).
template <class R>
__device__ __forceinline__ bool better(double d, R r, double bd, R br) {
    return d < bd || (d == bd && d < kSentinel && r < br);
}

struct OverlayZeta {
    const unsigned char *flag;
    const double *cand, *cur;
    __device__ __forceinline__ double operator()(int k) const {
        const double a = cand[k], b = cur[k];  // both loads issued at once, then select
        return flag[k] ? a : b;
    }
};

// A proposal with what it needs from the model (tid 0 builds it).
struct PState {
    Proposal p;
    double kx, ky, kz, zeta_killed;  // site and value of the selected cell (not birth)
    int slot_k, new_slot, eval;
};

// TD_inversion_function.jl:72-80,127-128,184-188,221-232: the proposal of one
// iteration from its draws and the model.  slot_at(pos) = slot at Julia
// position pos.
// In two halves: the draws' proposal and the loads of what it needs from the
// model (the selected cell, or the slot a birth takes), then the rest -- so the
// loads of a guessed next proposal can fly while other work runs.
struct ProposalLoads {
    Proposal q;
    int s, new_slot;
    double x, y, z, ze;
};
template <class SlotAt>
__device__ __forceinline__ ProposalLoads proposal_begin(const tdchain::Params &P, const tdchain::Draws &dr,
                                                        int ncells, int nfree, int nslots, const int *free_slots,
                                                        const double *cx, const double *cy, const double *cz,
                                                        const double *czeta, SlotAt slot_at) {
    ProposalLoads l;
    l.q = tdchain::propose(P, dr, ncells);
    l.s = -1;
    l.new_slot = -1;
    l.x = l.y = l.z = l.ze = 0.0;
    if (l.q.active && l.q.action != tdchain::kBirth) {  // (global loads: no LDS wait or barrier waits for them)
        l.s = slot_at((int)l.q.index);
        l.x = gload(cx + l.s);
        l.y = gload(cy + l.s);
        l.z = gload(cz + l.s);
        l.ze = gload(czeta + l.s);
    }
    if (l.q.active && l.q.action == tdchain::kBirth) l.new_slot = nfree > 0 ? gload(free_slots + nfree - 1) : nslots;
    return l;
}
__device__ __forceinline__ void proposal_end(PState &o, const tdchain::Params &P, const tdchain::Draws &dr,
                                             ProposalLoads l) {
    Proposal q = l.q;
    o.slot_k = -1;
    o.new_slot = l.new_slot;
    if (q.active && q.action != tdchain::kBirth) {
        o.slot_k = l.s;
        o.kx = l.x;
        o.ky = l.y;
        o.kz = l.z;
        o.zeta_killed = l.ze;
        tdchain::complete_proposal(P, dr, q, l.x, l.y, l.z, l.ze);
    }
    o.p = q;
    // forward evaluation needed (birth validity is only known after its query)
    o.eval = q.active && (q.valid || q.action == tdchain::kBirth) && P.debug_prior != 1;
}
template <class SlotAt>
__device__ __forceinline__ void make_proposal(PState &o, const tdchain::Params &P, const tdchain::Draws &dr,
                                              int ncells, int nfree, int nslots, const int *free_slots,
                                              const double *cx, const double *cy, const double *cz,
                                              const double *czeta, SlotAt slot_at) {
    proposal_end(o, P, dr, proposal_begin(P, dr, ncells, nfree, nslots, free_slots, cx, cy, cz, czeta, slot_at));
}

// A scripted step (td_evaluate's incremental path) as the proposal: always
// active and valid, no draws; birth's zeta is given (birth_zeta is not called).
template <class SlotAt>
__device__ __forceinline__ void script_proposal(PState &o, const ScriptStep &st, int nfree, int nslots,
                                               const int *free_slots, SlotAt slot_at) {
    Proposal q{};
    q.action = st.action;
    q.active = 1;
    q.valid = 1;
    q.index = st.index;
    q.x = st.x;
    q.y = st.y;
    q.z = st.z;
    q.zeta = st.zeta;
    o.slot_k = -1;
    o.new_slot = -1;
    if (q.action != tdchain::kBirth) {
        const int s = slot_at(st.index);
        o.slot_k = s;
        o.kx = st.old[0];  // the cell's values came with the step (a round trip to the cell arrays saved)
        o.ky = st.old[1];
        o.kz = st.old[2];
        o.zeta_killed = st.old[3];
        if (q.action == tdchain::kChange) {  // the site stays; only zeta is new
            q.x = o.kx;
            q.y = o.ky;
            q.z = o.kz;
        } else if (q.action == tdchain::kMove) {
            q.zeta = o.zeta_killed;
        }
    } else {
        o.new_slot = nfree > 0 ? free_slots[nfree - 1] : nslots;
    }
    o.p = q;
    o.eval = 1;
}

// The bucket grid's geometry and arrays, copied into LDS when a launch starts: a query reads them in
// one round of LDS loads rather than one scalar load (and wait) per descriptor field, and bounds the
// block without branches (wave_grid_search)
struct GridGeo {
    double x0, y0, z0, ix, iy, iz, hx, hy, hz, ex, ey, ez;
    double lo[3], hi[3];
    // a bound every query may use first: each face of a query's 3x3x3 block is at least h - e (the
    // cells' allowance) - e (the query's own bucket rounding, within the same allowance) away on its
    // axis, so every cell outside the block is at least lb0 away (+inf when no axis can have a face)
    double lb0;
    const int *count;
    const CellEntry *buckets;
    const int *bslot;
    int gx, gy, gz, sealed;
};
__device__ __forceinline__ void geo_fill(GridGeo &g, const DevChain &d) {
    const CellGrid &G = d.grid;
    g.x0 = G.x0; g.y0 = G.y0; g.z0 = G.z0;
    g.ix = G.ix; g.iy = G.iy; g.iz = G.iz;
    g.hx = G.hx; g.hy = G.hy; g.hz = G.hz;
    g.ex = G.ex; g.ey = G.ey; g.ez = G.ez;
    for (int a = 0; a < 3; ++a) {
        g.lo[a] = G.lo[a];
        g.hi[a] = G.hi[a];
    }
    g.count = d.bucket_count;
    g.buckets = d.buckets;
    g.bslot = d.bslot;
    g.gx = G.gx; g.gy = G.gy; g.gz = G.gz;
    g.sealed = G.sealed;
    const double h3[3] = {G.hx, G.hy, G.hz}, e3[3] = {G.ex, G.ey, G.ez};
    const int g3[3] = {G.gx, G.gy, G.gz};
    double lb0 = __builtin_huge_val();
    for (int a = 0; a < 3; ++a) {
        if (g3[a] < 3) continue;  // the block spans the axis: no face on it
        const double gap = (h3[a] - 2.0 * e3[a]) * (1.0 - 0x1p-30);
        const double f = gap > 0.0 ? gap * gap : 0.0;
        lb0 = f < lb0 ? f : lb0;
    }
    g.lb0 = grid_lb_close(lb0);
}

struct Shared {
    GridGeo geo;       // the bucket grid (geo_fill at a launch's start)
    PState ps[2];      // this iteration's proposal (ps[cur]) and the next one guessed in phase F
    int cur, spec_ok;
    int defer;  // phase F: accepted on bounds (LDS layout): the new chi^2 partial sums are not formed
    double phi_n;
    // decisions on bounds (phase F; wave 0): prefix[] exact below ex_upto, phi_r an
    // estimate in [phi_lo, phi_hi] (held here, not in registers: the kernel is at its VGPR limit)
    int ex_upto;
    double phi_lo, phi_hi, b_lo, b_hi;
    // The proposal's counters (atomic adds in phases B-E; wave 0 clears them at the iteration's end for the
    // next one).  No wave reads them after phase F's barrier: phase G reads the snapshot gs instead.
    int n_tiles, n_changed, n_orphans, n_rays, k0;
    // What phase G needs of the proposal, taken by tid 0 in phase F before its barrier (the counters are
    // final by then: n_tiles after B, the others after D) and read after it; written again only in the next
    // iteration's phase F, after the iteration-end barrier -- so nothing writes it while a wave may read it,
    // and the counters above can be cleared at the iteration's end whatever the waves' skew.  accept: the
    // decision (phase F), or a server's next command (phase G, wave 0, then a block barrier).
    struct GSnap {
        int nc, nr, nt, k0, accept;
    } gs;
    int ob_lo[3], ob_hi[3], ob_ncand, ob_nfb;  // phase D's orphan-batch search (LDS layout)
    int n_super[2];  // rays in HBM: super-tiles hit, by iteration parity (the next iteration refreshes their maxima)
    int pts_seen, ray_pts;
    int e_done;  // LDS layout: waves done with their phase-E rays (waves 1..; wave 0 waits for them)
    int b_done;  // LDS layout: waves done with their phase-B tile pass (phase B without its barrier)
    // bucket-grid update of an accepted proposal (applied by the last wave in phase G)
    int g_op, g_slot;           // bit 1: remove at old site, bit 2: insert at new site, bit 4: new value in place
    // what the update needs from the grid, read during phase F (G only writes)
    int gp_bo, gp_co, gp_pos, gp_bn, gp_cn;
    CellEntry gp_last;
    int gp_last_slot;
    double g_nzeta;
    double g_ox, g_oy, g_oz, g_nx, g_ny, g_nz;
    // chain scalars, resident for the whole launch
    long long iter, evaluations, bytes;
    long long proposed[5], accepted[5];
    double phi;
    int ncells, nslots, nfree;
    long long next_stamp;  // the next birth's stamp (tid 0)
    double lnN[3];     // logN[ncells - 1 .. ncells + 1]
    double lnN_far[2];  // logN[ncells - 2], logN[ncells + 2]: read during phase F for a birth/death commit
    double q_zeta;         // result of the birth/death Interpolation query
    int grid_fallbacks32;  // grid searches that needed the full scan
    int grid_ovf;          // LDS copy of *d.grid_overflow
    // scripted / server steps: the current step, a server command's steps
    ScriptStep step_cur;
    ScriptStep srv_step[kMaxScript];
    int srv_n, srv_k, srv_quit;
    // resident tempering rounds: the temperature of the current round (for reject_bound) and its last seq
    double rT, rinv2t;
    long long rseq;
    int rK, rskip;
    long long srv_seq, srv_busy_c, srv_busy_w;
    long long mbox[40];  // server mode: the last command read from the mailbox
    OrphanRec orph[kOrphanLds];
    ChgRec chg[kChgLds];
    tdchain::AlphaParts ap;  // the decision's phi-free part (phase C, last wave), for phase F
    DeltaSegs dseg;  // rays in HBM: phase F's new chi^2 partial sums as segments over the old ones
    long long prof[kProfSlots], t_last, t_iter;  // diagnostic phase stamps
    // rays in HBM: the committed terms' sum kept in any order, |tsum - (the exact real sum)| <=
    // terr; a proposal adds dsum = its terms' changes (any order), dabs = their magnitudes (phase E)
    double tsum, terr, dsum, dabs, b_T, b_E;
    double wpart[kChainThreads / 64];  // each wave's part of a block-wide any-order sum of the terms
    // a death, rays in LDS, free-running: phase G's deleteat! shift (shift_range) by waves 1.. -- each
    // wave's last source read in phase F (shift_edge), the waves done counted in shift_done, which wave 0
    // waits for before it reads the order for the next proposal
    int shift_done;
    int shift_edge[kChainThreads / 64];
    int dbg_site[kChainThreads / 64];  // the skew build's trail: each wave's last skew site (SKEW)
};

// deleteat! at Julia position `index` (rays in LDS, free-running): positions index+1 .. ncells-1 move down
// one, wave w (1 .. nw) taking the source positions [a, b).  Each wave reads its sources and writes
// them one lower in passes of 64 (a pass reads before it writes); the one source another wave writes
// over -- position b-1, the next wave's first target -- was read in phase F (Shared::shift_edge).
__device__ __forceinline__ void shift_range(int index, int ncells, int w, int nw, int &a, int &b) {
    const int first = index + 1, C = (ncells - first + nw - 1) / nw;
    a = first + (w - 1) * C;
    b = min(a + C, ncells);
}

// Diagnostic phase stamp (lane 0 of wave 0, right after a barrier): cycles
// since the previous stamp are charged to phase k.  Off unless d.profile.
#define STAMP(k)                                   \
    do {                                           \
        if (prof_on && tid == 0) {                 \
            const long long t_ = clock64();        \
            sh.prof[k] += t_ - sh.t_last;          \
            sh.prof[16 + 10 * (action - 1) +       \
                    ((k) <= 5 ? (k) : (k) == 12 ? 6 : (k) == 13 ? 7 : 8)] += t_ - sh.t_last; \
            sh.t_last = t_;                        \
        }                                          \
    } while (0)

// Wave-skew testing build (-DTD_CHAIN_SKEW, tools/build_skew.sh): after every block barrier and every
// barrier-free phase end of the chain loop, one wave -- rotating with the iteration and the site --
// sleeps 8k-16k cycles (a whole phase or more), so any shared word read without a synchronisation
// that orders it shows up as a wrong answer in the chain parity tests.  Off in the product build.
#ifdef TD_CHAIN_SKEW
#define SKEW(site)                                                                      \
    do {                                                                                \
        if (lane == 0) sh.dbg_site[wv] = (int)((it << 8) | (site));                     \
        if (wv == (int)(((unsigned long long)it * 5ull + (site)) % (unsigned)kWv)) {    \
            __builtin_amdgcn_s_sleep(127);                                              \
            if (((it + (site)) & 1) != 0) __builtin_amdgcn_s_sleep(127);                \
        }                                                                               \
    } while (0)
#else
#define SKEW(site) \
    do {           \
    } while (0)
#endif
// The chain's spin waits (a wave waiting for other waves' counts in LDS).  In the skew build each gives up
// after ~0.5 s, adds `site` to the diagnostic slot prof[79] (tdt_chain_profile) and goes on, so a wait that
// can never end shows up as a wrong answer and a nonzero slot instead of a hung launch.
#ifdef TD_CHAIN_SKEW
// (the first time one gives up, prof[56 + w] holds wave w's last skew site, as it << 8 | site, and
// prof[64] the iteration << 8 | the giving-up wave)
#define SPIN_WAIT(cond, site)                                                                        \
    do {                                                                                             \
        long long n_ = 0;                                                                            \
        while (cond) {                                                                               \
            __builtin_amdgcn_s_sleep(1);                                                             \
            if (++n_ > (1ll << 23)) {                                                                \
                if (lane == 0) {                                                                     \
                    if (atomicAdd((unsigned long long *)&sh.prof[79], (unsigned long long)(site)) == 0ull) { \
                        for (int w_ = 0; w_ < kWv; ++w_) sh.prof[56 + w_] = sh.dbg_site[w_];       \
                        sh.prof[64] = (it << 8) | wv;                                                \
                    }                                                                                \
                }                                                                                    \
                break;                                                                               \
            }                                                                                        \
        }                                                                                            \
    } while (0)
#else
#define SPIN_WAIT(cond, site)                      \
    do {                                           \
        while (cond) __builtin_amdgcn_s_sleep(1);  \
    } while (0)
#endif

// Phase-B probe build (-DTD_B_PROBE, diagnostics only): tid 0's cycles from the phase's start (STAMP(0)) to
// points inside phase B, summed into prof[72 + k] (those slots' preamble use is off in that build).
#ifdef TD_B_PROBE
#define BPROBE(k)                                                       \
    do {                                                                \
        if (prof_on && tid == 0) sh.prof[72 + (k)] += clock64() - sh.t_last; \
    } while (0)
#else
#define BPROBE(k) \
    do {          \
    } while (0)
#endif

// LDS carve-up (host and device agree on it through this function).
struct LdsPlan {
    size_t scratch, draws, smask, cmask, slo, shi, smax, shit, hrec, rhitl, tlo, thi, tmaxd, tstart, thit, ctm, tray, rayoff, ptS, prefix, cptS, cprefix, term, cterm,
        tS, sig, rflag, rhit, ord, total;
    bool super_lds;  // rays in HBM: super-tile boxes, maxima and hit lists in LDS
    bool lists_lds;  // rays in HBM: the first kListLds hit tiles (as records) and changed rays in LDS
};

constexpr size_t kLdsBudget = 160 * 1024;
constexpr size_t kDrawsBudget = (size_t)256 << 20;  // precomputed draws of one launch, at most (chain_run)

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// small: the tiles in LDS (and, rays_lds, the per-ray arrays and the order too -- else those stay in
// HBM, and the first kCtmLds hit tiles' candidate maxima are in LDS: the 4-wave two-chains-per-CU
// kernel's "tiles" layout)
__host__ __device__ inline LdsPlan lds_plan(int ntiles, int n, int cap, bool small, int waves = kWaves,
                                            bool rays_lds = true) {
    LdsPlan L{};
    size_t o = align16(sizeof(Shared));
    L.scratch = o; o += align16(sizeof(double) * waves * (small ? 96 : 192));  // (HBM layout: two rays a wave)
    L.draws = o; o += align16(sizeof(tdchain::Draws) * 64);                     // 64 iterations ahead
    if (!small || kSmallWalk) {  // the chi^2 walk's event words (exact_sum.h): static ones, kept; changed rays
        L.smask = o; o += align16(sizeof(unsigned long long) * delta_words(n));
        L.cmask = o; o += align16(sizeof(unsigned long long) * delta_words(n));
    }
    if (small) {
        L.tlo = o; o += align16(sizeof(float) * 3 * ntiles);
        L.thi = o; o += align16(sizeof(float) * 3 * ntiles);
        L.tmaxd = o; o += align16(sizeof(double) * ntiles);
        L.tstart = o; o += align16(sizeof(int) * (ntiles + 1));
        L.thit = o; o += align16(sizeof(int) * (ntiles + 1));
        L.ctm = o; o += align16(sizeof(double) * (rays_lds ? ntiles + 1 : kCtmLds));
        L.tray = o; o += align16(sizeof(int) * ntiles);
        if (rays_lds) {
            L.rayoff = o; o += align16(sizeof(int) * (n + 1));
            L.ptS = o; o += align16(sizeof(double) * n);
            L.prefix = o; o += align16(sizeof(double) * n);
            L.cptS = o; o += align16(sizeof(double) * n);
            L.cprefix = o; o += align16(sizeof(double) * n);
            L.term = o; o += align16(sizeof(double) * n);
            L.cterm = o; o += align16(sizeof(double) * n);
            L.tS = o; o += align16(sizeof(double) * n);
            L.sig = o; o += align16(sizeof(double) * n);
            L.rflag = o; o += align16(sizeof(int) * n);
            L.rhit = o; o += align16(sizeof(int) * n);
            L.ord = o; o += align16(sizeof(int) * cap);
        }
    } else {
        // the first hit tiles as {tile, start << 5 | count, ray} records, the first changed rays
        size_t q = o;
        L.hrec = q; q += align16(sizeof(int4) * kListLds);
        L.rhitl = q; q += align16(sizeof(int) * kListLds);
        L.lists_lds = q <= kLdsBudget;
        if (L.lists_lds) o = q;
        // super-tiles (16 tiles each): boxes, maxima (FP32, rounded up), two hit lists
        const int ns = (ntiles + kTilePts - 1) / kTilePts;
        q = o;
        L.slo = q; q += align16(sizeof(float) * 3 * ns);
        L.shi = q; q += align16(sizeof(float) * 3 * ns);
        L.smax = q; q += align16(sizeof(float) * ns);
        L.shit = q; q += align16(sizeof(int) * 2 * kListLds);
        L.super_lds = q <= kLdsBudget;
        if (L.super_lds) o = q;
    }
    L.total = o;
    return L;
}

// Views of the arrays a launch works on: LDS copies in SMALL mode, else HBM.
struct Views {
    const float *tlo, *thi;
    double *tmaxd, *ptS, *prefix, *cptS, *cprefix, *term, *cterm;
    const double *tS, *sig;
    const int *tstart, *ray_off, *tray;
    int *thit, *rflag, *rhit, *ord;
    // rays in HBM: the first kListLds changed rays in LDS (rhit), the rest in rhit_g;
    // the first kListLds hit tiles also as LDS records
    int *rhit_g;
    int rhit_cap;
    int4 *hrec;
    int hrec_cap;
    // hit tile i's maximum if the proposal is accepted: the first ctm_cap in LDS (ctm), the rest in ctm_g
    double *ctm, *ctm_g;
    int ctm_cap;
    __device__ __forceinline__ double ctm_at(int i) const { return i < ctm_cap ? ctm[i] : ctm_g[i]; }
    __device__ __forceinline__ void ctm_put(int i, double x) const {
        if (i < ctm_cap) ctm[i] = x;
        else ctm_g[i] = x;
    }
    __device__ __forceinline__ int ray_at(int i) const { return i < rhit_cap ? rhit[i] : rhit_g[i]; }
    __device__ __forceinline__ void ray_put(int i, int r) const {
        if (i < rhit_cap) rhit[i] = r;
        else rhit_g[i] = r;
    }
    // hit tile i: {tile, start << 5 | count, ray}
    __device__ __forceinline__ int4 tile_rec(int i) const {
        if (i < hrec_cap) return hrec[i];
        const int t = thit[i] & 0x7fffffff;  // LDS layout: the high bit marks a tile preloaded in phase B
        return int4{t, tstart[t], tray[t], 0};
    }
};

// Result of one nearest-cell query, the same in every lane of the wave.
struct Nearest {
    double d, z;  // squared distance (1e9 sentinel if none) and the cell's value (0.0 if none)
    int s;        // slot (-1 if none)
    bool proven;
};

// Exact nearest live cell by scanning every slot, ONE wave: lexicographic
// (distance, Julia position), which is what v_nearest's first-index rule
// gives (MCsub.jl:250-258) -- positions compared through the slots' stamps,
// which are in Julia order (chain_dev.h).  Fallback of the grid search (rare:
// out of line).
__device__ __attribute__((noinline)) Nearest wave_full_scan(const long long *__restrict__ stamp,
                                                           const double *__restrict__ cx,
                                                           const double *__restrict__ cy,
                                                           const double *__restrict__ cz,
                                                           const double *__restrict__ czeta, int cap, int nslots,
                                                           int lane, double x, double y, double z, int skip,
                                                           int moved, double mx, double my, double mz) {
    double bd = kSentinel;
    long long br = LLONG_MAX;
    int bs = -1;
    constexpr int kScanUnroll = 8;  // all loads of a round issued before any use
    for (int s0 = lane; s0 < nslots; s0 += kScanUnroll * 64) {
        long long r[kScanUnroll];
        double px[kScanUnroll], py[kScanUnroll], pz[kScanUnroll];
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
            // unconditional loads from a clamped slot, masked afterwards
            const int s = min(s0 + u * 64, cap - 1);
            r[u] = stamp[s];
            px[u] = cx[s];
            py[u] = cy[s];
            pz[u] = cz[s];
        }
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
            const int s = s0 + u * 64;
            if (s >= nslots || r[u] < 0 || s == skip) continue;  // free slot / killed cell
            if (s == moved) {
                px[u] = mx;
                py[u] = my;
                pz[u] = mz;
            }
            const double dd = dist2(px[u], py[u], pz[u], x, y, z);
            if (better(dd, r[u], bd, br)) {
                bd = dd;
                br = r[u];
                bs = s;
            }
        }
    }
    // lexicographic min: the distance first, then the position among equals
    const unsigned long long kd = wave_min_u64((unsigned long long)__double_as_longlong(bd));
    const bool at_min = (unsigned long long)__double_as_longlong(bd) == kd;
    const unsigned long long kr = wave_min_u64(at_min ? (unsigned long long)br : ~0ull);
    Nearest res;
    res.d = __longlong_as_double((long long)kd);
    res.proven = true;
    if (res.d < kSentinel && kr != ~0ull) {  // (stamps are unique: one lane holds the winner)
        const unsigned long long who = __ballot(at_min && (unsigned long long)br == kr);
        res.s = __builtin_amdgcn_readlane(bs, __builtin_ctzll(who));
        res.z = czeta[res.s];
    } else {
        res.s = -1;
        res.z = 0.0;
    }
    return res;
}

// Nearest live cell through the bucket grid, ONE wave, no block barrier.
// Lanes 0..53 cover the 3x3x3 buckets around the query, 8 entries per bucket
// (entries hold the cell coordinates inline: ONE round of loads).  The answer
// is proven when its distance is strictly below the squared distance to the
// outer faces of the block (every cell outside lies beyond a face), no other
// entry ties it and no bucket holds more than 8 entries.  `skip` = the killed
// slot; slot `moved` is taken at (mx,my,mz) instead of its stored site.
__device__ __forceinline__ Nearest wave_grid_search(const DevChain &d, bool ovf, int lane, double x, double y,
                                                    double z, int skip, int moved, double mx, double my, double mz,
                                                    double mzeta) {
    const CellGrid &G = d.grid;
    const int bi = grid_axis(x, G.x0, G.ix, G.gx), bj = grid_axis(y, G.y0, G.iy, G.gy),
              bk = grid_axis(z, G.z0, G.iz, G.gz);
    const int nb = lane % 27, grp = lane / 27;
    const int ii = bi + nb % 3 - 1, jj = bj + (nb / 3) % 3 - 1, kk = bk + nb / 9 - 1;
    const bool inb = lane < 54 && ii >= 0 && ii < G.gx && jj >= 0 && jj < G.gy && kk >= 0 && kk < G.gz;
    const int b = inb ? (kk * G.gy + jj) * G.gx + ii : 0;
    // global_ loads (vmcnt only): the scalar loads of the grid's fields below wait on lgkmcnt, which a
    // flat_ load would hold until these loads are back
    const int cnt = gload(d.bucket_count + b);
    CellEntry e[4];
    int sl[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const CellEntry *ep = d.buckets + b * kBucketCap + grp * 4 + u;
        e[u].x = gload(&ep->x);
        e[u].y = gload(&ep->y);
        e[u].z = gload(&ep->z);
        e[u].zeta = gload(&ep->zeta);
        sl[u] = gload(d.bslot + b * kBucketCap + grp * 4 + u);
    }
    // every cell outside the 3x3x3 block is at least sqrt(lb) away: computed while the loads fly
    const double lb = grid_block_lb(G, x, y, z, 1);
    double bd = kSentinel, bz = 0.0;
    int bs = -1;
    bool tie = false;
    const bool overfull = inb && cnt > 8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const bool ok = inb && grp * 4 + u < cnt && sl[u] != skip && sl[u] != moved;
        const double dd = dist2(e[u].x, e[u].y, e[u].z, x, y, z);
        if (ok) {
            if (dd < bd) {
                bd = dd;
                bs = sl[u];
                bz = e[u].zeta;
                tie = false;
            } else if (dd == bd && dd < kSentinel) {
                tie = true;
            }
        }
    }
    if (lane == 63 && moved >= 0) {  // the moved cell, at its proposed site
        const double dd = dist2(mx, my, mz, x, y, z);
        if (dd < bd) {
            bd = dd;
            bs = moved;
            bz = mzeta;
            tie = false;
        } else if (dd == bd && dd < kSentinel) {
            tie = true;
        }
    }
    const unsigned long long key = (unsigned long long)__double_as_longlong(bd);
    const unsigned long long kmin = wave_min_u64(key);
    const unsigned long long who = __ballot(key == kmin);
    const int win = __builtin_ctzll(who);
    Nearest res;
    res.d = __longlong_as_double((long long)kmin);
    const bool found = res.d < kSentinel;
    // distinct slots at the minimum (a slot sits in one lane only), or a tie inside the winner
    const bool tied = found && (__popcll(who) > 1 || __builtin_amdgcn_readlane((int)tie, win) != 0);
    const bool any_over = __ballot(overfull) != 0ull;
    res.s = found ? __builtin_amdgcn_readlane(bs, win) : -1;
    res.z = found ? readlane_f64(bz, win) : 0.0;
    res.proven = !ovf && !tied && !any_over && res.d < lb;
    return res;
}

// wave_grid_search on the LDS copy of the grid: the same loads, the same answer and the same proof
// (grid_block_lb's bound, R = 1, each face taken by a select instead of a branch)
__device__ __forceinline__ Nearest wave_grid_search(const GridGeo &gl, bool ovf, int lane, double x, double y,
                                                    double z, int skip, int moved, double mx, double my, double mz,
                                                    double mzeta) {
    const GridGeo G = gl;  // (one round of LDS loads, every lane the same words)
    const int bi = grid_axis(x, G.x0, G.ix, G.gx), bj = grid_axis(y, G.y0, G.iy, G.gy),
              bk = grid_axis(z, G.z0, G.iz, G.gz);
    const int nb = lane % 27, grp = lane / 27;
    const int ii = bi + nb % 3 - 1, jj = bj + (nb / 3) % 3 - 1, kk = bk + nb / 9 - 1;
    const bool inb = lane < 54 && ii >= 0 && ii < G.gx && jj >= 0 && jj < G.gy && kk >= 0 && kk < G.gz;
    const int b = inb ? (kk * G.gy + jj) * G.gx + ii : 0;
    const int cnt = gload(G.count + b);
    CellEntry e[4];
    int sl[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const CellEntry *ep = G.buckets + b * kBucketCap + grp * 4 + u;
        e[u].x = gload(&ep->x);
        e[u].y = gload(&ep->y);
        e[u].z = gload(&ep->z);
        e[u].zeta = gload(&ep->zeta);
        sl[u] = gload(G.bslot + b * kBucketCap + grp * 4 + u);
    }
    double bd = kSentinel, bz = 0.0;
    int bs = -1;
    bool tie = false;
    const bool overfull = inb && cnt > 8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const bool ok = inb && grp * 4 + u < cnt && sl[u] != skip && sl[u] != moved;
        const double dd = dist2(e[u].x, e[u].y, e[u].z, x, y, z);
        if (ok) {
            if (dd < bd) {
                bd = dd;
                bs = sl[u];
                bz = e[u].zeta;
                tie = false;
            } else if (dd == bd && dd < kSentinel) {
                tie = true;
            }
        }
    }
    if (lane == 63 && moved >= 0) {  // the moved cell, at its proposed site
        const double dd = dist2(mx, my, mz, x, y, z);
        if (dd < bd) {
            bd = dd;
            bs = moved;
            bz = mzeta;
            tie = false;
        } else if (dd == bd && dd < kSentinel) {
            tie = true;
        }
    }
    const unsigned long long key = (unsigned long long)__double_as_longlong(bd);
    const unsigned long long kmin = wave_min_u64_2p(key);
    const unsigned long long who = __ballot(key == kmin);
    const int win = __builtin_ctzll(who);
    Nearest res;
    res.d = __longlong_as_double((long long)kmin);
    const bool found = res.d < kSentinel;
    const bool tied = found && (__popcll(who) > 1 || __builtin_amdgcn_readlane((int)tie, win) != 0);
    const bool any_over = __ballot(overfull) != 0ull;
    res.s = found ? __builtin_amdgcn_readlane(bs, win) : -1;
    res.z = found ? readlane_f64(bz, win) : 0.0;
    res.proven = !ovf && !tied && !any_over && res.d < G.lb0;
    if (!res.proven && !ovf && !tied && !any_over) {  // (wave-uniform; rare) the query's own block bound
        double lb;
        {
            const double v[3] = {x, y, z}, e3[3] = {G.ex, G.ey, G.ez};
            double o2[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {  // grid_out2
                const double below = G.lo[a] - v[a], above = v[a] - G.hi[a];
                const double o = (below > above ? below : above) - e3[a];
                o2[a] = (G.sealed && o > 0.0) ? o * o : 0.0;
            }
            lb = __builtin_huge_val();
            auto face = [&lb](double w, double w0, double h, double e1, int g, int i, double other) {
                const double gl0 = (w - (w0 + (double)(i - 1) * h)) - e1;
                const double gh0 = ((w0 + (double)(i + 2) * h) - w) - e1;
                const double fl = (gl0 > 0.0 ? gl0 * gl0 : 0.0) + other;
                const double fh = (gh0 > 0.0 ? gh0 * gh0 : 0.0) + other;
                lb = (i - 1 > 0 && fl < lb) ? fl : lb;
                lb = (i + 1 < g - 1 && fh < lb) ? fh : lb;
            };
            face(x, G.x0, G.hx, G.ex, G.gx, bi, o2[1] + o2[2]);
            face(y, G.y0, G.hy, G.ey, G.gy, bj, o2[0] + o2[2]);
            face(z, G.z0, G.hz, G.ez, G.gz, bk, o2[0] + o2[1]);
            lb = grid_lb_close(lb);
        }
        res.proven = res.d < lb;
    }
    return res;
}

// Nearest live cell for one query, one wave: grid first, full scan if unproven.
__device__ __forceinline__ Nearest wave_nearest(const DevChain &d, const Views &v, Shared &sh, int lane, double x,
                                                double y, double z, int skip, int moved, double mx, double my,
                                                double mz, double mzeta) {
    Nearest r = wave_grid_search(sh.geo, sh.grid_ovf != 0, lane, x, y, z, skip, moved, mx, my, mz, mzeta);
    if (!r.proven) {
        if (lane == 0) atomicAdd(&sh.grid_fallbacks32, 1);
        r = wave_full_scan(d.stamp, d.cx, d.cy, d.cz, d.czeta, d.cap, sh.nslots, lane, x, y, z, skip, moved,
                           mx, my, mz);
    }
    return r;
}

// Read what the bucket-grid update of an accepted proposal will need (one
// wave, during phase F, before the decision): the old site's bucket, count,
// the slot's position in it and its last entry; the new site's bucket and count.
__device__ void grid_prefetch(const DevChain &d, Shared &sh, int lane, int action, int slot, double ox, double oy,
                              double oz, double nx, double ny, double nz) {
    const bool rm = action == tdchain::kDeath || action == tdchain::kMove;
    const bool ins = action == tdchain::kBirth || action == tdchain::kMove;
    const bool upd = action == tdchain::kChange;  // the entry's value, in place
    int bo = 0, co = 0, pos = -1, bn = 0, cn = 0;
    if (rm || upd) {
        bo = grid_bucket(d.grid, ox, oy, oz);
        co = d.bucket_count[bo];
        const int s = lane < kBucketCap ? d.bslot[bo * kBucketCap + lane] : -1;
        const unsigned long long m = __ballot(lane < co && s == slot);
        pos = m ? __builtin_ctzll(m) : -1;
        if (rm && lane == 0 && co > 0) {
            sh.gp_last = d.buckets[bo * kBucketCap + co - 1];
            sh.gp_last_slot = d.bslot[bo * kBucketCap + co - 1];
        }
    }
    if (ins) {
        bn = grid_bucket(d.grid, nx, ny, nz);
        cn = d.bucket_count[bn];
    }
    if (lane == 0) {
        sh.gp_bo = bo;
        sh.gp_co = co;
        sh.gp_pos = pos;
        sh.gp_bn = bn;
        sh.gp_cn = cn;
    }
}

// Apply the accepted proposal's bucket-grid update from the prefetched data
// (lane 0 of one wave; stores only).
__device__ void grid_apply(const DevChain &d, Shared &sh) {
    const int op = sh.g_op;
    int co = sh.gp_co;
    if (op & 1) {  // remove g_slot: the bucket's last entry takes its place
        const int b = sh.gp_bo, pos = sh.gp_pos;
        if (pos < 0) {
            *d.grid_overflow = 1;  // bookkeeping lost track: stop trusting the grid
            sh.grid_ovf = 1;
        } else {
            d.buckets[b * kBucketCap + pos] = sh.gp_last;
            d.bslot[b * kBucketCap + pos] = sh.gp_last_slot;
            d.bucket_count[b] = co - 1;
            co -= 1;
        }
    }
    if (op & 4) {  // a change: the entry's value
        const int pos = sh.gp_pos;
        if (pos < 0) {
            *d.grid_overflow = 1;
            sh.grid_ovf = 1;
        } else {
            d.buckets[sh.gp_bo * kBucketCap + pos].zeta = sh.g_nzeta;
        }
    }
    if (op & 2) {  // insert at the new site
        const int b = sh.gp_bn;
        const int cnt = ((op & 1) && b == sh.gp_bo) ? co : sh.gp_cn;  // a move inside one bucket
        if (cnt < kBucketCap) {
            d.buckets[b * kBucketCap + cnt] = CellEntry{sh.g_nx, sh.g_ny, sh.g_nz, sh.g_nzeta};
            d.bslot[b * kBucketCap + cnt] = sh.g_slot;
            d.bucket_count[b] = cnt + 1;
        } else {
            *d.grid_overflow = 1;
            sh.grid_ovf = 1;
        }
    }
}

__device__ __forceinline__ void mark(const DevChain &d, const Views &v, Shared &sh, int p, int r, int s, double dd,
                                     double z) {
    d.cand_s[p] = s;
    d.cand_d[p] = dd;
    d.cand_z[p] = z;
    d.cand_flag[p] = 1;
    const int c = atomicAdd(&sh.n_changed, 1);
    d.changed[c] = p;
    if (c < kChgLds) sh.chg[c] = ChgRec{p, s, dd, z};
    if (atomicExch(&v.rflag[r], 1) == 0) {
        v.ray_put(atomicAdd(&sh.n_rays, 1), r);
        atomicMin(&sh.k0, r);
    }
}

// Tile test in FP32: can some point p of tile t have dist2(q, p) <= thr?
// Every rounding is taken against the answer (the query rounded to FP32 moves
// by <= |q| 2^-24, each FP32 operation errs by <= 2^-24 relative), so the test
// never says "no" for a tile that holds such a point; it may say "yes" for a
// tile that does not (its points are then checked exactly in FP64).
struct TileQuery {
    float x, y, z, ex, ey, ez;  // coordinates and their rounding allowance
};
__device__ __forceinline__ TileQuery tile_query(double x, double y, double z) {
    TileQuery q;
    q.x = (float)x;
    q.y = (float)y;
    q.z = (float)z;
    q.ex = fabsf(q.x) * 0x1p-23f;
    q.ey = fabsf(q.y) * 0x1p-23f;
    q.ez = fabsf(q.z) * 0x1p-23f;
    return q;
}
__device__ __forceinline__ float gap_lb(float q, float e, float l, float h) {
    const float g = fmaxf(fmaxf(l - q, q - h), 0.0f);
    return fmaxf(g * (1.0f - 0x1p-20f) - e, 0.0f);
}
// thr: an FP32 bound >= the FP64 threshold (tile_thr)
__device__ __forceinline__ bool tile_may_hit(const float *lo, const float *hi, int nt, int t, const TileQuery &q,
                                             float thr) {
    const float gx = gap_lb(q.x, q.ex, lo[t], hi[t]);
    const float gy = gap_lb(q.y, q.ey, lo[nt + t], hi[nt + t]);
    const float gz = gap_lb(q.z, q.ez, lo[2 * nt + t], hi[2 * nt + t]);
    float s = gx * gx;
    s = s + gy * gy;
    s = s + gz * gz;
    return s * (1.0f - 0x1p-20f) <= thr;
}
__device__ __forceinline__ float tile_thr(double mx) { return (float)mx * (1.0f + 0x1p-20f); }

// The same filter in about half the VALU operations (phase B's tile pass, LDS layout; TD_TILE2): the
// query's rounding folded into two per-query bounds per axis, one max3 per axis, the squares summed with
// FMAs.  Never says "no" for a tile holding a point p with dist2(q, p) <= mx (FP64), thr = tile_thr(mx):
// with E = max_a |(float)q_a| 2^-23 >= |q_a - (float)q_a| on every axis, up = fl((float)q + 2E) >= q and
// dn = fl((float)q - 2E) <= q (the rounding of the add is at most E/2); for p in the outward-rounded box,
// |p_a - q_a| >= max(lo - up, dn - hi, 0) >= g_a (1 - 2^-24) with g_a the rounded max3; the FMA sum s
// errs by at most 3 ulps, so the real sum of the squared gaps -- a lower bound of the exact squared
// distance, itself within 2^-50 of the FP64 one -- is >= s (1 - 2^-21); and thr >= mx (1 - 2^-24)^2
// (1 + 2^-20), so s > thr implies dist2(q, p) > mx for every point of the tile.
#ifndef TD_TILE2
#define TD_TILE2 1
#endif
struct TileQuery2 {
    float ux, uy, uz, dx, dy, dz;  // the query's upper and lower bounds per axis
};
__device__ __forceinline__ TileQuery2 tile_query2(double x, double y, double z) {
    const float fx = (float)x, fy = (float)y, fz = (float)z;
    const float e2 = fmaxf(fmaxf(fabsf(fx), fabsf(fy)), fabsf(fz)) * 0x1p-22f;  // 2E
    return TileQuery2{fx + e2, fy + e2, fz + e2, fx - e2, fy - e2, fz - e2};
}
struct TileBox {
    float lx, ly, lz, hx, hy, hz, thr;
};
__device__ __forceinline__ TileBox tile_box(const float *lo, const float *hi, const double *maxd, int nt, int t) {
    return TileBox{lo[t], lo[nt + t], lo[2 * nt + t], hi[t], hi[nt + t], hi[2 * nt + t], tile_thr(maxd[t])};
}
__device__ __forceinline__ bool tile_may_hit2(const TileBox &b, const TileQuery2 &q) {
    const float gx = fmaxf(fmaxf(b.lx - q.ux, q.dx - b.hx), 0.0f);
    const float gy = fmaxf(fmaxf(b.ly - q.uy, q.dy - b.hy), 0.0f);
    const float gz = fmaxf(fmaxf(b.lz - q.uz, q.dz - b.hz), 0.0f);
    float s = gx * gx;
    s = __builtin_fmaf(gy, gy, s);
    s = __builtin_fmaf(gz, gz, s);
    return s <= b.thr;
}
// x rounded up to FP32 (x >= 0; the super-tile maxima)
__device__ __forceinline__ float f32_up(double x) {
    const float f = (float)x;
    return (double)f < x ? __int_as_float(__float_as_int(f) + 1) : f;  // f >= 0 finite: the next float up
}

// System-scope access to the mailbox (pinned host memory, the host polls it)
__device__ __forceinline__ long long mb_load(const long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void mb_store(long long *p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Server mode, wave 0: wait for the next EVAL or QUIT command, answering
// QUERY commands (one-point Interpolation on the committed model or the model
// plus one edit -- the state here is the committed one, a pending proposal
// lives only in the candidate overlay) meanwhile.  EVAL: its steps into
// sh.srv_*, the pending proposal's fate into sh.gs.accept; QUIT or silence:
// sh.srv_quit (and undo).
__device__ void server_wait(Mailbox *mb, const DevChain &d, const Views &v, Shared &sh, int lane) {
    constexpr int kWords = (int)(offsetof(Mailbox, done) / sizeof(long long));
    static_assert(kWords <= 64 && kWords <= (int)(sizeof(sh.mbox) / sizeof(long long)), "mailbox payload");
    long long seen = sh.srv_seq;
    long long t0 = (long long)wall_clock64();
    if (lane == 0 && sh.srv_busy_c) {  // diagnostic: the busy interval that ends here (clock rate)
        mb_store(&mb->diag[0], clock64() - sh.srv_busy_c);
        mb_store(&mb->diag[1], t0 - sh.srv_busy_w);
    }
    static_assert(kMailboxCheckWord == kWords - 1, "the check is the command's last word");
    long long polls = 0;
    while (true) {
        // every poll reads the whole command, one word per lane (as cheap as seq alone: one round
        // trip); a new seq is taken only with a matching check -- the poll may have caught the
        // host between its words (then the next poll reads them again)
        // (no system-scope acquire: the command is read through system-scope atomics, and one
        // would invalidate this XCD's L2, the chain's working set, at every call)
        const long long w = lane < kWords ? mb_load(reinterpret_cast<const long long *>(mb) + lane) : 0;
        const long long sq = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(w >> 32), 0) << 32) |
                                         (unsigned)__builtin_amdgcn_readlane((int)w, 0));
        ++polls;
        bool fresh = sq != seen;
        if (fresh) {  // (a torn read: not yet -- the next poll reads the words again)
            const unsigned long long h =
                wave_xor_u64(lane >= 1 && lane < kWords - 1 ? mailbox_word_mix((unsigned long long)w, lane, sq) : 0ull);
            const unsigned long long chk =
                ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(w >> 32), kWords - 1) << 32) |
                (unsigned)__builtin_amdgcn_readlane((int)w, kWords - 1);
            fresh = h == chk;
        }
        if (fresh) {
            seen = sq;
            if (lane == 0) {
                sh.srv_busy_c = clock64();
                sh.srv_busy_w = (long long)wall_clock64();
                mb_store(&mb->diag[2], polls);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (lane < kWords) sh.mbox[lane] = w;
            wave_sync_lds();
            const Mailbox &c = *reinterpret_cast<const Mailbox *>(sh.mbox);
            if (c.type == kCmdQuery) {
                const double x = c.q[0], y = c.q[1], z = c.q[2];
                const bool has_edit = c.has_edit != 0;
                const ScriptStep e = c.qedit;
                int skip = -1, moved = -1, slot_k = -1;
                if (has_edit && e.action != tdchain::kBirth) slot_k = v.ord[e.index];
                if (has_edit && e.action == tdchain::kDeath) skip = slot_k;  // the reduced model (:132-135)
                if (has_edit && e.action == tdchain::kMove) moved = slot_k;  // the cell at its new site
                const Nearest r = wave_nearest(d, v, sh, lane, x, y, z, skip, moved, e.x, e.y, e.z,
                                               moved >= 0 ? d.czeta[moved] : 0.0);
                double val = r.z;
                if (has_edit && e.action == tdchain::kChange && r.s == slot_k) val = e.zeta;
                if (has_edit && e.action == tdchain::kBirth) {  // the appended cell wins only strictly (last position)
                    const double dd = dist2(e.x, e.y, e.z, x, y, z);
                    if (dd < r.d && dd < kSentinel) val = e.zeta;
                }
                if (lane == 0) {
                    mb_store(reinterpret_cast<long long *>(&mb->qval), __double_as_longlong(val));
                    __builtin_amdgcn_s_waitcnt(0);  // the answer acknowledged before done (no L2 write-back)
                    mb_store(&mb->done, sq);
                }
                wave_sync_lds();
                t0 = (long long)wall_clock64();
                continue;
            }
            if (lane == 0) {
                sh.srv_seq = sq;
                if (c.type == kCmdEval) {
                    const int ns = min(max(c.nsteps, 1), kMaxScript);
                    for (int k = 0; k < ns; ++k) sh.srv_step[k] = c.step[k];
                    sh.srv_n = ns;
                    sh.srv_k = 0;
                    sh.gs.accept = c.decision != 0 ? 1 : 0;
                    sh.srv_quit = 0;
                } else {  // quit: the pending proposal (if any) is undone
                    sh.gs.accept = 0;
                    sh.srv_quit = 1;
                }
            }
            wave_sync_lds();
            return;
        }
        if ((long long)wall_clock64() - t0 > kServerIdleTicks) {  // no host: undo and return
            if (lane == 0) {
                sh.gs.accept = 0;
                sh.srv_quit = 1;
            }
            wave_sync_lds();
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Resident tempering rounds, wave 0 at a round boundary: publish the chain's
// phi for the round just finished (done = its seq), then wait for the next
// command: RUN (K proposals at the slot's new temperature) or QUIT; silence
// past the idle watchdog is a QUIT (the state is consistent between rounds).
// Results in sh.rK / sh.rT / sh.rinv2t / sh.srv_quit.
// A RUN posted with the slot's `skip` set (the chain ran that round in a launch
// the host lost, chain.cpp td_rounds_run) is answered with phi at once and
// waited past: the chain runs each round exactly once.  `phi` = the chain's
// exact phi (the launch's first wait: its stored one).
__device__ void round_wait(RoundBox *rb, int b, Shared &sh, int lane, bool publish, double phi) {
    RoundSlot *slot = &rb->slot[b];
    // The mailbox is coherent pinned host memory and every access to it is a system-scope atomic,
    // so no system-scope fence is needed -- one would write back (release) or invalidate (acquire)
    // this XCD's whole L2, the chain's working set, at every round.  phi is acknowledged before
    // done is written (the host reads done, then phi).
    if (publish && lane == 0) {
        mb_store(reinterpret_cast<long long *>(&slot->phi), __double_as_longlong(phi));
        __builtin_amdgcn_s_waitcnt(0);
        mb_store(&slot->done, sh.rseq);
    }
    long long seen = sh.rseq;
    long long idle = kServerIdleTicks;
    if (!publish) {  // a launch's first wait: the testing override of the watchdog
        const long long o = mb_load(&slot->idle);
        if (o > 0) idle = o;
    }
    long long t0 = (long long)wall_clock64();
    while (true) {
        const long long sq = mb_load(&rb->seq);
        if (sq != seen) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (lane == 0) {
                // (the host wrote them before seq: four loads in flight together)
                const long long w = mb_load(reinterpret_cast<const long long *>(rb) + 1);  // cmd | K << 32
                const long long tb = mb_load(reinterpret_cast<const long long *>(&slot->T));
                const long long ib = mb_load(reinterpret_cast<const long long *>(&slot->inv_2t));
                const long long sk = mb_load(&slot->skip);
                const int cmd = (int)(w & 0xffffffffll), K = (int)(w >> 32);
                sh.rseq = sq;
                sh.rskip = 0;
                if (cmd == kRoundRun && K > 0 && sk) {  // ran already: report it again
                    mb_store(reinterpret_cast<long long *>(&slot->phi), __double_as_longlong(phi));
                    __builtin_amdgcn_s_waitcnt(0);
                    mb_store(&slot->done, sq);
                    sh.rskip = 1;
                } else if (cmd == kRoundRun && K > 0) {
                    sh.rK = K;
                    sh.rT = __longlong_as_double(tb);
                    sh.rinv2t = __longlong_as_double(ib);
                    sh.srv_quit = 0;
                } else {
                    sh.srv_quit = 1;
                }
            }
            wave_sync_lds();
            if (sh.rskip) {
                seen = sq;
                t0 = (long long)wall_clock64();
                continue;
            }
            return;
        }
        if ((long long)wall_clock64() - t0 > idle) {
            if (lane == 0) sh.srv_quit = 1;
            wave_sync_lds();
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Exchange rounds (chain_dev.h RoundX), wave 0 at the end of round j with the
// chain's exact phi: publish it, wait for every replica's phi of the round,
// make the round's swap decisions (all of them, the same in every workgroup
// of every rank: chain_logic.h swap_accept on the gathered vector) and take
// this chain's new temperature (sh.rT, sh.rinv2t).  sh.srv_quit = 1 when an
// exchange never came (x.err set).  R <= 64: lane g holds replica g.
__device__ void round_exchange(const RoundX &x, int b, long long j, Shared &sh, int lane, double phi) {
    const int R = x.R;
    const unsigned long long tag = x.ready_base + (unsigned long long)j + 1ull;
    if (b == 0 && lane == 0) x.log_t[3 * j] = (long long)wall_clock64();
    if (lane == 0) {  // phi acknowledged before the flag (the readers load the flag, then phi)
        mb_store(reinterpret_cast<long long *>(&x.xin[(j & 1) * x.local + b]), __double_as_longlong(phi));
        __builtin_amdgcn_s_waitcnt(0);
        mb_store(reinterpret_cast<long long *>(&x.rdy[b]), (long long)tag);
    }
    const bool one = x.gdone == nullptr;  // one rank: xout is xin, every replica's flag is local
    const int nflags = one ? R : x.local;
    bool ok = true;
    if (one || b == 0) {  // wait for the flags (lane g reads flag g)
        const long long t0 = (long long)wall_clock64();
        while (true) {
            const unsigned long long f =
                lane < nflags ? (unsigned long long)mb_load(reinterpret_cast<const long long *>(&x.rdy[lane])) : tag;
            if (__all(f >= tag)) break;
            if ((long long)wall_clock64() - t0 > kExchangeTicks) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (!one && ok && lane == 0)  // this rank's phis are in: the exchange stream may gather
            mb_store(reinterpret_cast<long long *>(x.ready), (long long)tag);
        if (b == 0 && lane == 0) x.log_t[3 * j + 1] = (long long)wall_clock64();
    }
    if (!one && ok) {  // the allgather of round j done (the exchange stream's write)
        const unsigned long long want = x.gdone_base + (unsigned long long)j + 1ull;
        const long long t0 = (long long)wall_clock64();
        while ((unsigned long long)mb_load(reinterpret_cast<const long long *>(x.gdone)) < want) {
            if ((long long)wall_clock64() - t0 > kExchangeTicks) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (!ok) {
        if (lane == 0) {
            mb_store(x.err, 1ll);
            sh.srv_quit = 1;
        }
        wave_sync_lds();
        return;
    }
    if (b == 0 && lane == 0) x.log_t[3 * j + 2] = (long long)wall_clock64();
    // every replica's phi and level (system-scope loads: the gathered vector bypasses the L2s)
    const bool in = lane < R;
    const double ph =
        in ? __longlong_as_double(mb_load(reinterpret_cast<const long long *>(&x.xout[(j & 1) * R + lane]))) : 0.0;
    const int lv = in ? x.lev[b * R + lane] : lane;
    // owner of level l (lane l): the replica at that level -- a forward permute of the levels
    const int owner = __builtin_amdgcn_ds_permute(lv * 4, lane);
    const unsigned long long rnd = (unsigned long long)(x.rnd0 + j);
    const int par = (int)(rnd & 1ull);
    // pair leaders l = par, par + 2, ... < R - 1 decide the disjoint pairs (l, l + 1)
    const bool leader = lane >= par && ((lane - par) & 1) == 0 && lane + 1 < R;
    const int owner_hi = __shfl(owner, (lane + 1) & 63);
    const double pa = __shfl(ph, owner & 63), pb = __shfl(ph, owner_hi & 63);
    bool acc = false;
    if (leader) acc = tdchain::swap_accept(pa, pb, x.temps[lane], x.temps[lane + 1], x.seed, rnd, (uint64_t)lane);
    // every replica: its pair (led by its level, or by the level below) and that pair's fate
    int lead = -1;
    if (in) {
        if (lv >= par && ((lv - par) & 1) == 0 && lv + 1 < R) lead = lv;
        else if (lv - 1 >= par && ((lv - 1 - par) & 1) == 0) lead = lv - 1;
    }
    const int acc_i = __shfl((int)acc, lead < 0 ? 0 : lead);
    const int nl = (lead >= 0 && acc_i) ? (lv == lead ? lead + 1 : lead) : lv;
    if (in) {
        x.lev[b * R + lane] = nl;
        if (b == 0) {
            x.log_phi[j * R + lane] = ph;
            x.log_lev[j * R + lane] = nl;
        }
    }
    const int me = x.rank * x.local + b;
    const int my_level = __shfl(nl, me);
    if (lane == 0) {
        const double T = x.temps[my_level];
        sh.rT = T;
        sh.rinv2t = 1.0 / (2.0 * T);  // = params_derived's inv_2t
    }
    wave_sync_lds();
}

// One array of a fused block copy: U elements per thread per round, loaded
// into registers by load(), written by store().  Several Segs loaded before
// any is stored keep all their loads in flight at once: the launch preamble
// is a handful of memory round trips whatever the number of arrays.  S = the
// block's thread count (the caller's loop steps by U * S).
template <class T, int U, int S = kChainThreads>
struct CopySeg {
    T *dst;
    const T *src;
    int n;
    T v[U];
    __device__ __forceinline__ void load(int b) {
        if (n <= 0) return;
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[min(b + u * S, n - 1)];
    }
    __device__ __forceinline__ void store(int b) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (b + u * S < n) dst[b + u * S] = v[u];
    }
};

// The decisions on bounds (phase F): 2u, u = 2^-53 the unit roundoff -- every rounding bound below is
// taken twice over
constexpr double kSumSlack = 2.3e-16;

// LDS layout, one wave (the rare paths of the decisions on bounds, phase F):
// prefix[ex_upto..n) exact again -- the committed terms added in k order
// (MCsub.jl:170-172, exact_sum.h) -- and the committed phi returned; then, if
// k0 < n, the proposal's partial sums from k0 into cprefix, its phi_n in
// *phi_n.  `overlay`: a proposal's terms are in place (its rays flagged, their
// committed terms in cterm), staged through cprefix.  Out of line: it is
// rare, and the kernel is at its register limit.
// (The arrays by value: a Views passed by reference would be spilled to scratch in the caller; phi_n
// comes back in the result for the same reason -- an out-pointer would keep the caller's phi_n in scratch.)
struct ExactPhis {
    double phi, phi_n;
};
__device__ __attribute__((noinline)) ExactPhis exact_sums(const double *term, double *prefix, double *cprefix,
                                                          const double *cterm, const int *rflag, Shared &sh, int n,
                                                          int lane, bool overlay, int k0, double phi, double phi_n) {
    const int ex_upto = sh.ex_upto;
    if (ex_upto < n) {
        const double C0 = ex_upto > 0 ? prefix[ex_upto - 1] : 0.0;
        const double *t = term + ex_upto;
        if (overlay) {
            for (int k = ex_upto + lane; k < n; k += 64) cprefix[k] = rflag[k] ? cterm[k] : term[k];
            wave_sync_lds();
            t = cprefix + ex_upto;
        }
        bool stopped = false;
        phi = wave_seq_sum(t, n - ex_upto, C0, prefix + ex_upto, lane, nullptr, &stopped);
        wave_sync_lds();
        if (lane == 0) {
            sh.ex_upto = n;
            sh.phi_lo = sh.phi_hi = phi;
        }
        wave_sync_lds();
    }
    if (k0 < n) {
        bool stopped = false;
        phi_n = wave_seq_sum(term + k0, n - k0, k0 > 0 ? prefix[k0 - 1] : 0.0, cprefix + k0, lane, nullptr, &stopped);
    }
    return ExactPhis{phi, phi_n};
}

// A scripted step's answer in the pinned output (wave 0; system-scope stores): [phi, k, (ray, ptS) x k],
// the changed rays' new t* (the caller holds the model's ptS); k = -1: the whole proposed ptS follows.
// phi: NaN when the answer goes out before phase F (a server's step: the host forms phi_n itself).
__device__ void server_report(double *outp, const Views &v, const Shared &sh, int n, int lane, double phi) {
    long long *out = reinterpret_cast<long long *>(outp);
    auto put = [&](int i, double x) { mb_store(out + i, __double_as_longlong(x)); };
    const int nr = sh.n_rays;
    const bool few = 2 * nr + 2 <= n + 1;
    if (few) {
        for (int i = lane; i < nr; i += 64) {
            const int r = v.ray_at(i);
            put(2 + 2 * i, (double)r);
            put(3 + 2 * i, v.cptS[r]);
        }
    } else {
        for (int r = lane; r < n; r += 64) put(2 + r, v.rflag[r] ? v.cptS[r] : v.ptS[r]);
    }
    if (lane == 0) {
        put(0, phi);
        put(1, few ? (double)nr : -1.0);
    }
}

// SCRIPT: host-given proposals (td_evaluate's incremental path: scripted
// steps, the resident server); a free-running chain's instance has none of
// that code on its path.
// SMALL: the tiles mirrored in LDS (else in HBM, with super-tiles); RLDS: the per-ray arrays and the
// Julia order mirrored too (the 381-ray configs, 8 waves); NTH: 512 threads, or 256 (two chains per CU)
template <bool SMALL, bool SCRIPT, int NTH, bool RLDS = SMALL, bool ROUNDS = false>
__global__ __launch_bounds__(NTH, 2) void k_chain_run(const DevChain *__restrict__ dptr, long long iters,
                                                             ScriptArgs sa) {
    constexpr bool WALK = !SMALL || kSmallWalk;  // chi^2 by the event walk
    constexpr bool kNoBarB = RLDS && !SCRIPT;     // phase B may end without a block barrier (below)
    constexpr int kWv = NTH / 64;  // waves: 8 (one chain per CU), or 4 (rays in HBM: two chains per CU)
    static_assert(!RLDS || SMALL, "rays in LDS only with the tiles in LDS");
    static_assert(NTH == kChainThreads || (!RLDS && !SCRIPT && NTH == kChainThreads / 2),
                  "512 threads, or 256 with the rays in HBM");
    if (sa.pin >= 0) {  // one chain, launched as 8 workgroups: only the one on XCD `pin` runs it
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if ((int)(xcc & 15u) != sa.pin) return;
    }
    const DevChain &d = dptr[sa.pin >= 0 ? 0 : blockIdx.x];  // fields read from memory as needed
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    Shared &sh = *reinterpret_cast<Shared *>(lds);
    const LdsPlan L = lds_plan(d.ntiles, d.n, d.cap, SMALL, kWv, RLDS);
    double(*ray_scratch)[96] = reinterpret_cast<double(*)[96]>(lds + L.scratch);
    tdchain::Draws *draws = reinterpret_cast<tdchain::Draws *>(lds + L.draws);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const tdchain::Params &P = d.params;
    const int n = d.n, NT = d.ntiles;
    const bool prof_on = d.profile != 0;
    const long long t_start = prof_on ? clock64() : 0;  // diagnostic: launch preamble / epilogue (prof[76..79])
    Mailbox *const mb = SCRIPT ? sa.mb : nullptr;  // server mode: resident, steps from the mailbox (iters ignored)
    RoundBox *const rbx = SCRIPT ? nullptr : sa.rb;  // resident tempering rounds (iters ignored)
    // exchange rounds, swaps decided here (ROUNDS instances only: the others carry none of their registers)
    const RoundX *const rxp = (SCRIPT || !ROUNDS) ? nullptr : sa.rx;
    const bool xch = rxp != nullptr;
    const int bchain = sa.pin >= 0 ? 0 : (int)blockIdx.x;
    const int nscript = SCRIPT ? (mb ? 1 : sa.n) : 0;  // > 0: host-given proposals (td_evaluate), iters == nscript

    // ---- views: LDS copies of the tile / ray / order arrays when they fit ----
    Views v;
    v.tlo = d.tile_lo; v.thi = d.tile_hi; v.tmaxd = d.tile_maxd; v.tstart = d.tile_start; v.thit = d.tiles_hit;
    v.ray_off = d.ray_off; v.ptS = d.ptS; v.prefix = d.prefix; v.cptS = d.cand_ptS; v.cprefix = d.cand_prefix;
    v.tS = d.tS; v.sig = d.sig; v.rflag = d.ray_flag; v.rhit = d.rays_hit; v.ord = d.order; v.tray = d.tile_ray;
    v.rhit_g = d.rays_hit;
    v.rhit_cap = 0;
    v.hrec = nullptr;
    v.hrec_cap = 0;
    if (!SMALL && L.lists_lds) {
        v.rhit = reinterpret_cast<int *>(lds + L.rhitl);
        v.rhit_cap = kListLds;
        v.hrec = reinterpret_cast<int4 *>(lds + L.hrec);
        v.hrec_cap = kListLds;
    }
    v.term = d.term;
    v.cterm = d.cand_term;
    v.ctm = v.ctm_g = d.tile_cmax;
    v.ctm_cap = 0;
    if constexpr (SMALL && !RLDS) {  // the tiles only (the rays, the order, the candidate maxima in HBM)
        float *a = reinterpret_cast<float *>(lds + L.tlo), *b = reinterpret_cast<float *>(lds + L.thi);
        double *m = reinterpret_cast<double *>(lds + L.tmaxd);
        int *ts = reinterpret_cast<int *>(lds + L.tstart), *tr = reinterpret_cast<int *>(lds + L.tray);
        {
            constexpr int U = 4;
            CopySeg<float, U, NTH> c0{a, d.tile_lo, 3 * NT}, c1{b, d.tile_hi, 3 * NT};
            CopySeg<double, U, NTH> c2{m, d.tile_maxd, NT};
            CopySeg<int, U, NTH> c7{ts, d.tile_start, NT + 1}, c8{tr, d.tile_ray, NT};
            for (int b0 = tid; b0 < 3 * NT; b0 += U * NTH) {
                c0.load(b0); c1.load(b0); c2.load(b0); c7.load(b0); c8.load(b0);
                c0.store(b0); c1.store(b0); c2.store(b0); c7.store(b0); c8.store(b0);
            }
        }
        v.tlo = a; v.thi = b; v.tmaxd = m; v.tstart = ts; v.tray = tr;
        v.thit = reinterpret_cast<int *>(lds + L.thit);
        v.ctm = reinterpret_cast<double *>(lds + L.ctm);
        v.ctm_cap = kCtmLds;
        __syncthreads();
    }
    if constexpr (RLDS) {
        float *a = reinterpret_cast<float *>(lds + L.tlo), *b = reinterpret_cast<float *>(lds + L.thi);
        double *m = reinterpret_cast<double *>(lds + L.tmaxd);
        int *ts = reinterpret_cast<int *>(lds + L.tstart), *ro = reinterpret_cast<int *>(lds + L.rayoff);
        double *p = reinterpret_cast<double *>(lds + L.ptS), *pf = reinterpret_cast<double *>(lds + L.prefix);
        double *t = reinterpret_cast<double *>(lds + L.tS), *sg = reinterpret_cast<double *>(lds + L.sig);
        int *rf = reinterpret_cast<int *>(lds + L.rflag), *od = reinterpret_cast<int *>(lds + L.ord);
        int *tr = reinterpret_cast<int *>(lds + L.tray);
        v.tray = tr;
        {  // every mirror in one fused copy (positions >= ncells of the order are written before read)
            constexpr int U = 4;
            CopySeg<float, U, NTH> c0{a, d.tile_lo, 3 * NT}, c1{b, d.tile_hi, 3 * NT};
            CopySeg<double, U, NTH> c2{m, d.tile_maxd, NT}, c3{p, d.ptS, n}, c4{pf, d.prefix, n}, c5{t, d.tS, n},
                c6{sg, d.sig, n};
            CopySeg<int, U, NTH> c7{ts, d.tile_start, NT + 1}, c8{tr, d.tile_ray, NT}, c9{ro, d.ray_off, n + 1},
                c10{od, d.order, d.st->ncells};
            const int most = max(max(3 * NT, NT + 1), max(n + 1, c10.n));
            for (int b0 = tid; b0 < most; b0 += U * NTH) {
                c0.load(b0); c1.load(b0); c2.load(b0); c3.load(b0); c4.load(b0); c5.load(b0);
                c6.load(b0); c7.load(b0); c8.load(b0); c9.load(b0); c10.load(b0);
                c0.store(b0); c1.store(b0); c2.store(b0); c3.store(b0); c4.store(b0); c5.store(b0);
                c6.store(b0); c7.store(b0); c8.store(b0); c9.store(b0); c10.store(b0);
            }
        }
        for (int i = tid; i < n; i += NTH) rf[i] = 0;
        v.tlo = a; v.thi = b; v.tmaxd = m; v.tstart = ts; v.ray_off = ro; v.ptS = p; v.prefix = pf; v.tS = t;
        v.sig = sg; v.rflag = rf; v.ord = od;
        v.cptS = reinterpret_cast<double *>(lds + L.cptS);
        v.cprefix = reinterpret_cast<double *>(lds + L.cprefix);
        v.term = reinterpret_cast<double *>(lds + L.term);
        v.cterm = reinterpret_cast<double *>(lds + L.cterm);
        v.thit = reinterpret_cast<int *>(lds + L.thit);
        v.ctm = reinterpret_cast<double *>(lds + L.ctm);
        v.ctm_cap = NT + 1;
        v.rhit = reinterpret_cast<int *>(lds + L.rhit);
        v.rhit_cap = n;
        __syncthreads();  // ptS, tS, sig mirrored
    }
    const long long t_mirror = prof_on ? clock64() : 0;
    // chi^2 term of every ray in the current state (MCsub.jl:171), cached: a
    // proposal recomputes only the terms of the rays it changes
    {
        double part = 0.0;  // (rays in HBM: their sum in any order, the running total of phase F)
        for (int r = tid; r < n; r += NTH) {
            const double df = v.ptS[r] - v.tS[r];
            const double sg = v.sig[r];
            const double t = ((df * df) * 1.0) / (sg * sg);
            v.term[r] = t;
            part = part + t;
        }
        if constexpr (!RLDS) {
            part = wave_sum_f64(part);
            if (lane == 0) sh.wpart[wv] = part;
        }
    }
    if (tid == 0) {
        const ChainScalars &s0 = *d.st;
        sh.iter = s0.iter;
        sh.evaluations = 0;
        sh.bytes = 0;
        sh.cur = 0;
        sh.defer = 0;
        if (!RLDS) sh.dsum = sh.dabs = 0.0;
        sh.grid_fallbacks32 = 0;
        sh.e_done = sh.b_done = 0;
        geo_fill(sh.geo, d);
        for (int a = 0; a < 5; ++a) sh.proposed[a] = sh.accepted[a] = 0;
        sh.phi = s0.phi;
        sh.ncells = s0.ncells;
        for (int k = 0; k < 3; ++k) sh.lnN[k] = d.logN[max(s0.ncells - 1 + k, 0)];
        sh.nslots = s0.nslots;
        sh.nfree = s0.nfree;
        sh.next_stamp = s0.next_stamp;
        sh.g_op = 0;
        sh.grid_ovf = *d.grid_overflow;
        sh.rT = P.temperature;
        sh.rinv2t = P.inv_2t;
        sh.srv_quit = 0;
        sh.rK = 0;
        for (int k = 0; k < kProfSlots; ++k) sh.prof[k] = 0;
        sh.t_last = clock64();
        sh.dseg.nseg = 0;
    }
    __syncthreads();
    const long long t_init = prof_on ? clock64() : 0;
    unsigned long long *smask = reinterpret_cast<unsigned long long *>(lds + L.smask);
    unsigned long long *cmask = reinterpret_cast<unsigned long long *>(lds + L.cmask);
    const int NS = d.nsuper;
    float *slo = reinterpret_cast<float *>(lds + L.slo), *shi = reinterpret_cast<float *>(lds + L.shi);
    float *smax = reinterpret_cast<float *>(lds + L.smax);  // >= the max of its tiles' maxima
    int *shit = reinterpret_cast<int *>(lds + L.shit);
    const bool super_on = !SMALL && L.super_lds;
    if constexpr (WALK) {  // the chi^2 walk's static event words of the current state
        if constexpr (SMALL) __syncthreads();  // the terms above
        delta_marks(v.term, v.prefix, nullptr, n, smask, wv, delta_words(n), kWv, lane);
        for (int w = tid; w < delta_words(n); w += NTH) cmask[w] = 0ull;
    }
    if constexpr (!SMALL) {
        if (super_on) {  // super-tile boxes, and maxima = the max of their tiles' maxima
            for (int i = tid; i < 3 * NS; i += NTH) {
                slo[i] = d.super_lo[i];
                shi[i] = d.super_hi[i];
            }
            for (int S = tid; S < NS; S += NTH) {
                double m = 0.0;
                for (int t = S * kTilePts; t < min(NT, (S + 1) * kTilePts); ++t) m = fmax(m, d.tile_maxd[t]);
                smax[S] = f32_up(m);
            }
            if (tid == 0) sh.n_super[0] = sh.n_super[1] = 0;
        }
        __syncthreads();
    }

    // the draws (and their normal quantiles) of 64 iterations, one lane each:
    // a function of (seed, chain, iteration) only; and the first proposal
    if (wv == 0) {
        if (sa.pre) {  // precomputed (k_draws): one round of loads
            if (lane < iters) draws[lane] = sa.pre[(long long)bchain * sa.pre_stride + lane];
        } else if (!nscript) {
            draws[lane] = tdchain::draw_iteration(d.seed, d.chain, (uint64_t)(sh.iter + lane));
        }
        wave_sync_lds();
        if (mb) {  // the first command (no proposal pending yet)
            if (lane == 0) {
                sh.srv_seq = mb_load(&mb->done);
                sh.srv_quit = 0;
                sh.srv_busy_c = 0;
            }
            wave_sync_lds();
            server_wait(mb, d, v, sh, lane);
        }
        if (rbx) {  // the first round (the last one done is in the slot)
            if (lane == 0) sh.rseq = mb_load(&rbx->slot[bchain].done);
            wave_sync_lds();
            round_wait(rbx, bchain, sh, lane, false, sh.phi);  // (the stored phi is exact)
        }
        if (lane == 0 && iters > 0 && !((mb || rbx) && sh.srv_quit)) {
            if (nscript) {
                sh.step_cur = mb ? sh.srv_step[sh.srv_k++] : sa.step[0];
                script_proposal(sh.ps[0], sh.step_cur, sh.nfree, sh.nslots, d.free_slots,
                                [&](int pos) { return v.ord[pos]; });
            }
            else
                make_proposal(sh.ps[0], P, draws[0], sh.ncells, sh.nfree, sh.nslots, d.free_slots, d.cx, d.cy, d.cz,
                              d.czeta, [&](int pos) { return v.ord[pos]; });
            if (sh.ps[0].p.active) sh.proposed[sh.ps[0].p.action] += 1;
            sh.n_tiles = sh.n_changed = sh.n_orphans = sh.n_rays = 0;
            sh.pts_seen = sh.ray_pts = 0;
            sh.k0 = n;
            sh.gs.accept = 0;
        }
        if (lane == 0) sh.spec_ok = 0;
    }
    __syncthreads();

    // wave 0 lane 0 decides, commits and proposes: the scalars only it changes
    // live in its registers (LDS copies are written, never read back on its path)
    const long long iter0 = sh.iter;
    if (prof_on && tid == 0) {
        const long long t_now = clock64();
        sh.prof[76] += t_now - t_start;  // preamble: mirrors, terms, draws, 1st proposal
#ifdef TD_B_PROBE
        if (false) {
#else
        if (SMALL) {  // its parts (slots of the rays-in-HBM walk diagnostics, unused in this layout)
#endif
            sh.prof[72] += t_mirror - t_start;
            sh.prof[73] += t_init - t_mirror;
            sh.prof[74] += t_now - t_init;
        }
    }
    double phi_r = sh.phi;
    // wave 0: the temperature of the round (tid 0 decides with it) and the round's last iteration
    double inv2t_r = sh.rinv2t;
    long long round_end = rbx ? sh.rK : xch ? (long long)rxp->K : LLONG_MAX;
    int cur_r = 0;
    bool pend_r = false;    // rays in HBM: an accepted proposal's chi^2 partial sums not yet written
    bool pend_sup = false;  // rays in HBM: its super-tiles' maxima not yet refreshed
    int last_action = 0, last_accept = 0;  // tid 0: Model.action / accept of the last iteration
    long long it_done = 0;                 // iterations run (server mode: until QUIT)
    // LDS layout, decisions on bounds (phase F): a proposal accepted on bounds of phi_n leaves its
    // chi^2 partial sums unformed -- prefix[] stays exact below ex_upto only (wave 0), and tid 0
    // keeps phi_r as an estimate inside [phi_lo, phi_hi].  They are made exact again by the next
    // decision the bounds cannot take, at a tempering round's end and at the launch's end.
    if (tid == 0) {
        sh.ex_upto = n;
        sh.phi_lo = sh.phi_hi = phi_r;
        if constexpr (!RLDS) {
            double T = 0.0;
            for (int w = 0; w < kWv; ++w) T = T + sh.wpart[w];
            sh.tsum = T;
            sh.terr = kSumSlack * (double)(n + 1) * fabs(T);  // (any order: within (n - 1) ulps of the exact sum)
        }
    }
    __syncthreads();
    for (long long it = 0; it < iters && !((mb || rbx || xch) && sh.srv_quit); ++it) {
        if (prof_on && tid == 0) sh.t_iter = clock64();
        // rays in HBM: the previous accepted proposal's super-tile maxima (their first round of
        // loads issued here, so it overlaps the partial sums' commit below)
        int sup_n = 0, sup_S = 0, sup_par = 0;
        bool sup_all = false;
        unsigned long long sup_mk = 0ull;
        if constexpr (!SMALL) {
            if (pend_sup) {
                sup_par = (int)((it - 1) & 1);
                const int nsh = sh.n_super[sup_par];
                sup_all = nsh > kListLds;  // the list overflowed: every super-tile
                sup_n = sup_all ? NS : nsh;
                if ((tid >> 4) < sup_n) {
                    sup_S = sup_all ? (tid >> 4) : shit[sup_par * kListLds + (tid >> 4)];
                    const int t = sup_S * kTilePts + (tid & 15);
                    sup_mk = t < NT ? (unsigned long long)__double_as_longlong(d.tile_maxd[t]) : 0ull;
                }
            }
        }
        if constexpr (WALK) {
            // the previous accepted proposal's partial sums (read again only in phase F,
            // after at least one barrier): off its critical path, before this one's tiles
            if (pend_r) delta_commit<SMALL ? 1 : 16>(v.prefix, v.cprefix, n, sh.dseg, tid, NTH);
            pend_r = false;
        }
        if constexpr (!SMALL) {
            if (pend_sup) {  // its hit super-tiles: max of their tiles' new maxima (a tile row each)
                if ((tid >> 4) < sup_n) {  // whole rows: the DPP row max
                    const unsigned long long mk = row_max_u64(sup_mk);
                    if ((tid & 15) == 15) smax[sup_S] = f32_up(__longlong_as_double((long long)mk));
                }
                for (int i = (tid >> 4) + NTH / kTilePts; i < sup_n; i += NTH / kTilePts) {
                    const int S = sup_all ? i : shit[sup_par * kListLds + i], t = S * kTilePts + (tid & 15);
                    unsigned long long mk = t < NT ? (unsigned long long)__double_as_longlong(d.tile_maxd[t]) : 0ull;
                    mk = row_max_u64(mk);
                    if ((tid & 15) == 15) smax[S] = f32_up(__longlong_as_double((long long)mk));
                }
                __syncthreads();
                SKEW(1);
                pend_sup = false;
            }
        }
        bool acc_r = false;
        const PState &cur = sh.ps[sh.cur];
        const Proposal p = cur.p;
        const int action = p.action;
        const int ncells = sh.ncells;
        const int slot_k = cur.slot_k;
        const bool eval = cur.eval != 0;
        const double kx = cur.kx, ky = cur.ky, kz = cur.kz;
        const int new_slot = cur.new_slot;
        const double zeta_killed = cur.zeta_killed;
        double czeta = 0.0, zetanew_death = 0.0;
        STAMP(0);
        // LDS layout: the points of the first kPre hit tiles a wave finds are loaded in
        // phase B (their global round trip overlaps the B barrier and the birth/death
        // query) and judged in phase C
        bool pre_on = false;
        bool nobar = false;  // phase B without its block barrier (block-uniform; below)
        int pre_q = 0, pre_ray = 0, pre_s = 0;
        double pre_bd = 0.0, pre_x = 0.0, pre_y = 0.0, pre_z = 0.0;
        if (p.active) {
            // ============ phase B: tile pass || birth/death Interpolation ============
            // (a scripted step brings its own values: no Interpolation query -- but for a server's death
            // step the reference next asks Interpolation of the proposed model at the killed site
            // (TD_inversion_function.jl:146): the idle query wave answers it here, posted with the report)
            const bool kill_q = SCRIPT && mb && action == tdchain::kDeath && sh.step_cur.decision == kDecideLater;
            const bool query = (!nscript && (action == tdchain::kBirth || action == tdchain::kDeath)) || kill_q;
            // LDS layout, free-running, no birth: phase B ends without a block barrier.  Phase C needs of
            // the tile pass only each wave's own first hit tiles (their points are in its registers) until
            // it walks the whole hit list: each wave counts itself done after its tile pass (a death's
            // query wave before its query, whose answer only the decision reads) and a wave waits for all
            // of them after its own points.  (A birth's marks need the query's answer: the barrier stays.)
            nobar = kNoBarB && action != tdchain::kBirth && p.valid && P.debug_prior != 1;
            if (eval) {
                // tiles whose box can hold a point the proposal changes (the last
                // wave answers the Interpolation query meanwhile)
                const bool q0 = action != tdchain::kBirth;  // old site of the selected cell
                const bool q1 = action == tdchain::kBirth || action == tdchain::kMove;  // new site
                const TileQuery tq0 = tile_query(kx, ky, kz), tq1 = tile_query(p.x, p.y, p.z);
                const int nthr = query ? NTH - 64 : NTH;
                // tiles in flight per thread: LDS latency is short; HBM needs more
                constexpr int TU = SMALL ? 3 : 8;
                if (super_on) {
                    // rays in HBM: the super-tiles (LDS) first, then the tiles of those hit
                    const int par = (int)(it & 1);
                    int *hl = shit + par * kListLds;
                    if (tid < nthr)
                        for (int S0 = tid; S0 < NS; S0 += 4 * nthr) {
                            bool hit[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const int S = min(S0 + u * nthr, NS - 1);
                                const float thr = smax[S] * (1.0f + 0x1p-20f);
                                const bool h0 = tile_may_hit(slo, shi, NS, S, tq0, thr);
                                const bool h1 = tile_may_hit(slo, shi, NS, S, tq1, thr);
                                hit[u] = S0 + u * nthr < NS && ((q0 && h0) || (q1 && h1));
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (hit[u]) {
                                    const int k = atomicAdd(&sh.n_super[par], 1);
                                    if (k < kListLds) hl[k] = S0 + u * nthr;
                                }
                        }
                    __syncthreads();  // (the query wave too: it starts its query after this)
                    SKEW(2);
                    const int nsh = sh.n_super[par];
                    const bool all = nsh > kListLds;  // the list overflowed: every tile
                    const int nitems = all ? NS * kTilePts : nsh * kTilePts;
                    if (tid < nthr)
                        for (int i0 = tid; i0 < nitems; i0 += 4 * nthr) {
                            bool hit[4];
                            int4 rec[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const int i = min(i0 + u * nthr, nitems - 1);
                                const int tu = (all ? (i >> 4) : hl[i >> 4]) * kTilePts + (i & 15);
                                const int t = min(tu, NT - 1);
                                const float thr = tile_thr(v.tmaxd[t]);
                                const bool h0 = tile_may_hit(v.tlo, v.thi, NT, t, tq0, thr);
                                const bool h1 = tile_may_hit(v.tlo, v.thi, NT, t, tq1, thr);
                                rec[u] = int4{t, v.tstart[t], v.tray[t], 0};  // loaded with the box
                                hit[u] = i0 + u * nthr < nitems && tu < NT && ((q0 && h0) || (q1 && h1));
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (hit[u]) {
                                    const int k = atomicAdd(&sh.n_tiles, 1);
                                    v.thit[k] = rec[u].x;
                                    if (k < v.hrec_cap) v.hrec[k] = rec[u];
                                }
                        }
                } else if (SMALL) {
                    const TileQuery2 tr0 = tile_query2(kx, ky, kz), tr1 = tile_query2(p.x, p.y, p.z);
                    if (tid < nthr) {  // wave-uniform
                        int npre = 0;  // preload slots this wave has taken (wave-uniform)
                        int pt[kPre] = {0, 0, 0, 0};  // their tiles (wave-uniform: from the ballots, no LDS)
                        for (int b0 = wv * 64; b0 < NT; b0 += TU * nthr) {  // the same trip count in every lane
                            const int t0 = b0 + lane;
                            bool hit[TU];
                            if constexpr (TD_TILE2) {
                                // every box loaded first (one round of LDS loads), then only the sites the action
                                // has, on scalar branches (the action made wave-uniform for the compiler)
                                TileBox bx[TU];
#pragma unroll
                                for (int u = 0; u < TU; ++u)
                                    bx[u] = tile_box(v.tlo, v.thi, v.tmaxd, NT, min(t0 + u * nthr, NT - 1));
                                const int au = __builtin_amdgcn_readfirstlane(action);
                                const bool s0 = au != tdchain::kBirth, s1 = au == tdchain::kBirth || au == tdchain::kMove;
#pragma unroll
                                for (int u = 0; u < TU; ++u) hit[u] = false;
                                if (s0) {
#pragma unroll
                                    for (int u = 0; u < TU; ++u) hit[u] = tile_may_hit2(bx[u], tr0);
                                }
                                if (s1) {
#pragma unroll
                                    for (int u = 0; u < TU; ++u) hit[u] = hit[u] || tile_may_hit2(bx[u], tr1);
                                }
#pragma unroll
                                for (int u = 0; u < TU; ++u) hit[u] = hit[u] && t0 + u * nthr < NT;
                            } else {
#pragma unroll
                                for (int u = 0; u < TU; ++u) {
                                    const int t = min(t0 + u * nthr, NT - 1);  // clamped: loads stay unconditional
                                    const float thr = tile_thr(v.tmaxd[t]);
                                    const bool h0 = tile_may_hit(v.tlo, v.thi, NT, t, tq0, thr);
                                    const bool h1 = tile_may_hit(v.tlo, v.thi, NT, t, tq1, thr);
                                    hit[u] = t0 + u * nthr < NT && ((q0 && h0) || (q1 && h1));
                                }
                            }
#pragma unroll
                            for (int u = 0; u < TU; ++u) {
                                const unsigned long long m = __ballot(hit[u]);
                                if (m == 0ull) continue;
                                const int first = __builtin_ctzll(m), cnt = __popcll(m);
                                const int rank = __popcll(m & ((1ull << lane) - 1ull));
                                int base = 0;
                                if (lane == first) base = atomicAdd(&sh.n_tiles, cnt);  // one atomic per wave
                                base = __builtin_amdgcn_readlane(base, first);
                                if (hit[u]) {
                                    const int t = t0 + u * nthr, slot = npre + rank;
                                    v.thit[base + rank] = slot < kPre ? (t | INT_MIN) : t;
                                }
                                for (unsigned long long mm = m; mm && npre < kPre; mm &= mm - 1ull) {
                                    const int t = b0 + __builtin_ctzll(mm) + u * nthr;
#pragma unroll
                                    for (int k = 0; k < kPre; ++k) pt[k] = k == npre ? t : pt[k];
                                    ++npre;
                                }
                            }
                        }
                        BPROBE(0);  // (tile pass done)
                        if (npre > 0) {
                            if (lane < kTilePts * npre) {
                                const int g = lane / kTilePts;
                                const int t = g == 0 ? pt[0] : g == 1 ? pt[1] : g == 2 ? pt[2] : pt[3];
                                const int sc = v.tstart[t];
                                if (lane % kTilePts < (sc & 31)) {
                                    const int q = (sc >> 5) + lane % kTilePts;
                                    pre_on = true;
                                    pre_q = q;
                                    pre_ray = v.tray[t];
                                    pre_s = d.best_s[q];  // independent loads: one round trip
                                    pre_bd = d.best_d[q];
                                    pre_x = d.px[q];
                                    pre_y = d.py[q];
                                    pre_z = d.pz[q];
                                }
                            }
                        }
                    }
                } else if (tid < nthr)
                    for (int t0 = tid; t0 < NT; t0 += TU * nthr) {
                        bool hit[TU];
#pragma unroll
                        for (int u = 0; u < TU; ++u) {
                            const int t = min(t0 + u * nthr, NT - 1);  // clamped: loads stay unconditional
                            const float thr = tile_thr(v.tmaxd[t]);
                            const bool h0 = tile_may_hit(v.tlo, v.thi, NT, t, tq0, thr);
                            const bool h1 = tile_may_hit(v.tlo, v.thi, NT, t, tq1, thr);
                            hit[u] = t0 + u * nthr < NT && ((q0 && h0) || (q1 && h1));
                        }
#pragma unroll
                        for (int u = 0; u < TU; ++u)
                            if (hit[u]) {
                                const int k = atomicAdd(&sh.n_tiles, 1), t = t0 + u * nthr;
                                v.thit[k] = t;
                                if (!SMALL && k < v.hrec_cap) v.hrec[k] = int4{t, v.tstart[t], v.tray[t], 0};
                            }
                    }
            }
            BPROBE(1);  // (preload issued)
            if (nobar && !(query && wv == kWv - 1)) {  // (every wave but the query wave: its tile pass is done)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) atomicAdd(&sh.b_done, 1);
                SKEW(3);
            }
            if (RLDS && action == tdchain::kDeath && nscript) {  // deleteat! shift, staged before we know if it is accepted
                const int sthr = query ? NTH - 64 : NTH;  // not the query wave: it starts at once
                // (the order in HBM: no staging -- an accepted death shifts it in phase G)
                if constexpr (RLDS) {
                    if (tid < sthr)
                        for (int j = (int)p.index + 1 + tid; j < ncells; j += sthr) d.order_tmp[j] = v.ord[j];
                }
            }
            if (query && wv == kWv - 1) {  // TD_inversion_function.jl:81 (birth), :146 (death)
                const bool birth = action == tdchain::kBirth;
                if (nobar && lane == 0) atomicAdd(&sh.b_done, 1);  // (a death: nothing in phase C waits for this query)
                const Nearest r = wave_nearest(d, v, sh, lane, birth ? p.x : kx, birth ? p.y : ky, birth ? p.z : kz,
                                               birth ? -1 : slot_k, -1, 0.0, 0.0, 0.0, 0.0);
                if (lane == 0) sh.q_zeta = r.z;
            }
        }
        // Phase B's barrier (tile list complete, query answered) -- taken by an inactive proposal too (a birth
        // at max_cells, a death at min_cells: the reference skips the iteration, nobar stays false).  That one
        // has no phase B-G, and without this barrier nothing would separate the other waves' reads at the
        // loop top (sh.cur, the proposal, sh.srv_quit) from wave 0's writes at this iteration's end (the next
        // proposal goes into ps[cur] when no guess is adopted): a wave still at the loop top would read the
        // NEXT proposal.  So every iteration has a block barrier between the loop top and wave 0's
        // end-of-iteration writes (this one, or C's and F's).  Found by the wave-skew build
        // (tools/skew_probe.py, the 8-cell model at max_cells 12).
        if (!nobar) {
            __syncthreads();
            SKEW(4);
            if (p.active && action == tdchain::kBirth) czeta = sh.q_zeta;
            if (p.active && action == tdchain::kDeath) zetanew_death = sh.q_zeta;
        }
        BPROBE(2);  // (counted / barrier passed)
        Proposal pp = p;
        if (p.active && action == tdchain::kBirth && !nscript) tdchain::birth_zeta(P, pp, czeta);  // every lane, same value
        STAMP(1);
        // the next iteration's proposal can be guessed during phase F if its draws are here
        const bool can_spec = !nscript && it + 1 < iters && ((it + 1) & 63) != 0;
        if (pp.active && pp.valid) {
            const bool fwd = P.debug_prior != 1;
            int no = 0;
            if (fwd) {
                // ================= phase C: affected points =================
                if (!nscript && tid == NTH - 64)  // the decision's phi-free part, off phase F's path
                    sh.ap = tdchain::alpha_parts(P, pp, czeta, zeta_killed,
                                                 nobar && action == tdchain::kDeath ? sh.q_zeta : zetanew_death,
                                                 sh.lnN);  // (nobar: this lane asked the death's query itself)

                const int nt = sh.n_tiles;
                // the selected cell's value, known since the proposal was made: czeta[slot_k] = zeta_killed
                const double zeta_k = slot_k >= 0 ? zeta_killed : 0.0;
                int seen = 0;
                // one candidate point: captured (birth, move), re-valued (change) or orphaned
                // (death, move: its nearest cell is the selected one)
                auto point = [&](int q, int ray, int s, double bd, double qx, double qy, double qz) {
                    if (action == tdchain::kBirth) {  // appended cell: strict capture
                        const double dd = dist2(pp.x, pp.y, pp.z, qx, qy, qz);
                        if (dd < bd) mark(d, v, sh, q, ray, new_slot, dd, pp.zeta);
                    } else if (action == tdchain::kChange) {
                        if (s == slot_k) mark(d, v, sh, q, ray, s, bd, pp.zeta);
                    } else if (s == slot_k) {  // death / move: its points are re-searched
                        const int o = atomicAdd(&sh.n_orphans, 1);
                        d.orphans[o] = q;
                        if (o < kOrphanLds) sh.orph[o] = OrphanRec{qx, qy, qz, q, ray};
                    } else if (action == tdchain::kMove) {
                        const double dd = dist2(pp.x, pp.y, pp.z, qx, qy, qz);
                        // (an exact tie: Julia positions, through the stamps -- loaded only then)
                        if (dd < bd || (dd == bd && s >= 0 && d.stamp[slot_k] < d.stamp[s]))
                            mark(d, v, sh, q, ray, slot_k, dd, zeta_k);
                    }
                };
                if constexpr (SMALL) {
                    if (pre_on) {  // loaded in phase B
                        ++seen;
                        point(pre_q, pre_ray, pre_s, pre_bd, pre_x, pre_y, pre_z);
                    }
                    if (nobar)  // the whole hit list from here on: every wave's tile pass done
                        SPIN_WAIT(__hip_atomic_load(&sh.b_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < kWv, 1);
                    const int nt = sh.n_tiles;
                    for (int item = tid; item < nt * kTilePts; item += NTH) {
                        const int t = v.thit[item / kTilePts];
                        if (t < 0) continue;  // preloaded
                        const int sc = v.tstart[t];  // start << 5 | count
                        if (item % kTilePts >= (sc & 31)) continue;
                        const int q = (sc >> 5) + item % kTilePts;
                        ++seen;
                        // independent loads: one round trip
                        const int s = d.best_s[q];
                        const double bd = d.best_d[q];
                        const double qx = d.px[q], qy = d.py[q], qz = d.pz[q];
                        point(q, v.tray[t], s, bd, qx, qy, qz);
                    }
                } else {
                    constexpr int CU = 4;  // items in flight per thread (rays in HBM: latency)
                    for (int item0 = tid; item0 < nt * kTilePts; item0 += CU * NTH) {
                        int qq[CU], rr[CU], ss[CU];
                        double bb[CU], xx[CU], yy[CU], zz[CU];
#pragma unroll
                        for (int u = 0; u < CU; ++u) {  // every load of the CU items: one round trip
                            const int item = item0 + u * NTH;
                            const int4 rec = v.tile_rec(min(item, nt * kTilePts - 1) / kTilePts);
                            const int sc = rec.y;  // start << 5 | count
                            const bool in = item < nt * kTilePts && item % kTilePts < (sc & 31);
                            const int q = in ? (sc >> 5) + item % kTilePts : 0;
                            qq[u] = in ? q : -1;
                            rr[u] = rec.z;
                            ss[u] = d.best_s[q];
                            bb[u] = d.best_d[q];
                            xx[u] = d.px[q];
                            yy[u] = d.py[q];
                            zz[u] = d.pz[q];
                        }
#pragma unroll
                        for (int u = 0; u < CU; ++u)
                            if (qq[u] >= 0) {
                                ++seen;
                                point(qq[u], rr[u], ss[u], bb[u], xx[u], yy[u], zz[u]);
                            }
                    }
                }
                if (seen) atomicAdd(&sh.pts_seen, seen);
                __syncthreads();
                SKEW(5);
                if (nobar && action == tdchain::kDeath) zetanew_death = sh.q_zeta;  // (the query wave is past it)
                STAMP(2);
                // ========= phase D: re-search orphaned points, one wave each =========
                no = sh.n_orphans;
                const bool death = action == tdchain::kDeath;
                const int skip_s = death ? slot_k : -1, moved_s = death ? -1 : slot_k;
                // the orphans the per-wave search takes: all of them in order, or the batch's unproven ones
                int nlist = no;
                const int *olist = nullptr;
                if constexpr (RLDS) {
                    if (no >= kBatchOrphans && 2 * n >= no && sh.grid_ovf == 0) {  // (block-uniform)
                        // The nearest cell of every orphan, at once: the buckets of the orphans' bucket
                        // box grown by one on each side, their entries staged in LDS (phase E's ray
                        // scratch is idle), then a thread per orphan over all of them, with the moved cell
                        // at its new site.  Proven as the per-wave search proves: a distance strictly
                        // below the region's faces (the region holds every orphan's 3x3x3 block), no tie
                        // at the minimum; else the orphan goes to the per-wave search (its full scan).
                        const CellGrid &G = d.grid;
                        double *ex = reinterpret_cast<double *>(ray_scratch);
                        double *ey = ex + kBatchCand, *ez = ey + kBatchCand;
                        int *es = reinterpret_cast<int *>(ez + kBatchCand);
                        int *fb = reinterpret_cast<int *>(v.cptS);  // (candidate t* of phase E: idle)
                        auto orphan_xyz = [&](int o, double &qx, double &qy, double &qz) {
                            if (o < kOrphanLds) {
                                qx = sh.orph[o].x;
                                qy = sh.orph[o].y;
                                qz = sh.orph[o].z;
                            } else {
                                const int q = d.orphans[o];
                                qx = d.px[q];
                                qy = d.py[q];
                                qz = d.pz[q];
                            }
                        };
                        if (tid == 0) {
                            for (int a3 = 0; a3 < 3; ++a3) {
                                sh.ob_lo[a3] = INT_MAX;
                                sh.ob_hi[a3] = -1;
                            }
                            sh.ob_ncand = sh.ob_nfb = 0;
                        }
                        __syncthreads();
                        SKEW(6);
                        for (int o = tid; o < no; o += NTH) {
                            double qx, qy, qz;
                            orphan_xyz(o, qx, qy, qz);
                            const int bi = grid_axis(qx, G.x0, G.ix, G.gx), bj = grid_axis(qy, G.y0, G.iy, G.gy),
                                      bk = grid_axis(qz, G.z0, G.iz, G.gz);
                            atomicMin(&sh.ob_lo[0], bi);
                            atomicMax(&sh.ob_hi[0], bi);
                            atomicMin(&sh.ob_lo[1], bj);
                            atomicMax(&sh.ob_hi[1], bj);
                            atomicMin(&sh.ob_lo[2], bk);
                            atomicMax(&sh.ob_hi[2], bk);
                        }
                        __syncthreads();
                        SKEW(7);
                        const int i0 = max(sh.ob_lo[0] - 1, 0), i1 = min(sh.ob_hi[0] + 1, G.gx - 1);
                        const int j0 = max(sh.ob_lo[1] - 1, 0), j1 = min(sh.ob_hi[1] + 1, G.gy - 1);
                        const int k0b = max(sh.ob_lo[2] - 1, 0), k1b = min(sh.ob_hi[2] + 1, G.gz - 1);
                        const int nbx = i1 - i0 + 1, nby = j1 - j0 + 1, nbz = k1b - k0b + 1;
                        if (nbx * nby * nbz <= kBatchBuckets) {
                            for (int b = tid; b < nbx * nby * nbz; b += NTH) {
                                const int bucket = ((k0b + b / (nbx * nby)) * G.gy + (j0 + (b / nbx) % nby)) * G.gx +
                                                   (i0 + b % nbx);
                                const int cnt = d.bucket_count[bucket];
                                const int base = cnt > 0 ? atomicAdd(&sh.ob_ncand, cnt) : 0;
                                for (int e = 0; e < cnt && base + e < kBatchCand; ++e) {
                                    const CellEntry &be = d.buckets[bucket * kBucketCap + e];
                                    ex[base + e] = be.x;
                                    ey[base + e] = be.y;
                                    ez[base + e] = be.z;
                                    es[base + e] = d.bslot[bucket * kBucketCap + e];
                                }
                            }
                            __syncthreads();
                            SKEW(8);
                            const int nc = sh.ob_ncand;
                            if (nc <= kBatchCand) {
                                // four lanes per orphan (a quad), each over a quarter of the entries,
                                // then the quad's lexicographic minimum (the loop is wave-uniform)
                                for (int o0 = 0; o0 < no; o0 += NTH / 4) {
                                    const int o = o0 + tid / 4, part = tid & 3;
                                    const bool act = o < no;
                                    double qx = 0.0, qy = 0.0, qz = 0.0;
                                    if (act) orphan_xyz(o, qx, qy, qz);
                                    double bd = kSentinel;
                                    int bs = -1;
                                    bool tie = false;
                                    auto take = [&](double dd, int sl) {
                                        if (dd < bd) {
                                            bd = dd;
                                            bs = sl;
                                            tie = false;
                                        } else if (dd == bd && dd < kSentinel) {
                                            tie = true;
                                        }
                                    };
                                    for (int c = part; c < nc; c += 4) {
                                        const int sl = es[c];
                                        const double dd = dist2(ex[c], ey[c], ez[c], qx, qy, qz);
                                        if (sl != skip_s && sl != moved_s) take(dd, sl);
                                    }
                                    if (moved_s >= 0 && part == 0)  // the moved cell, at its proposed site
                                        take(dist2(pp.x, pp.y, pp.z, qx, qy, qz), moved_s);
#pragma unroll
                                    for (int m = 1; m <= 2; m <<= 1) {  // quad reduction (distinct slots per lane)
                                        const double od = __shfl_xor(bd, m, 4);
                                        const int os = __shfl_xor(bs, m, 4);
                                        const bool ot = __shfl_xor((int)tie, m, 4) != 0;
                                        if (od < bd) {
                                            bd = od;
                                            bs = os;
                                            tie = ot;
                                        } else if (od == bd && od < kSentinel) {
                                            tie = true;
                                        }
                                    }
                                    if (!act || part != 0) continue;
                                    // every cell outside the region lies beyond one of its inner faces
                                    double lb = __builtin_huge_val();
                                    // (and, the grid sealed, its distance to the cells' box: internal.h grid_block_lb)
                                    double o2[3];
                                    grid_out2(G, qx, qy, qz, o2);
                                    auto face = [&lb](double w, double w0, double h, double e, int g, int lo, int hi,
                                                      double other) {
                                        if (lo > 0) {
                                            const double gap = (w - (w0 + (double)lo * h)) - e;
                                            const double f = (gap > 0.0 ? gap * gap : 0.0) + other;
                                            lb = f < lb ? f : lb;
                                        }
                                        if (hi < g - 1) {
                                            const double gap = ((w0 + (double)(hi + 1) * h) - w) - e;
                                            const double f = (gap > 0.0 ? gap * gap : 0.0) + other;
                                            lb = f < lb ? f : lb;
                                        }
                                    };
                                    face(qx, G.x0, G.hx, G.ex, G.gx, i0, i1, o2[1] + o2[2]);
                                    face(qy, G.y0, G.hy, G.ey, G.gy, j0, j1, o2[0] + o2[2]);
                                    face(qz, G.z0, G.hz, G.ez, G.gz, k0b, k1b, o2[0] + o2[1]);
                                    lb = grid_lb_close(lb);
                                    if (bs >= 0 && bd < kSentinel && !tie && bd < lb) {
                                        const int q = o < kOrphanLds ? sh.orph[o].q : d.orphans[o];
                                        const int ray = o < kOrphanLds ? sh.orph[o].ray : d.pt_ray[q];
                                        mark(d, v, sh, q, ray, bs, bd, d.czeta[bs]);
                                    } else {
                                        fb[atomicAdd(&sh.ob_nfb, 1)] = o;
                                    }
                                }
                                __syncthreads();
                                SKEW(9);
                                nlist = sh.ob_nfb;
                                olist = fb;
                            }
                        }
                    }
                }
                for (int k = wv; k < nlist; k += kWv) {  // one wave per orphan, no block barrier
                    const int o = olist ? olist[k] : k;
                    double qx, qy, qz;
                    int q, ray;
                    if (o < kOrphanLds) {
                        qx = sh.orph[o].x;
                        qy = sh.orph[o].y;
                        qz = sh.orph[o].z;
                        q = sh.orph[o].q;
                        ray = sh.orph[o].ray;
                    } else {
                        q = d.orphans[o];
                        qx = d.px[q];
                        qy = d.py[q];
                        qz = d.pz[q];
                        ray = d.pt_ray[q];
                    }
                    const Nearest r =
                        wave_nearest(d, v, sh, lane, qx, qy, qz, skip_s, moved_s, pp.x, pp.y, pp.z, zeta_killed);
                    if (lane == 0) mark(d, v, sh, q, ray, r.s, r.d, r.z);
                }
                if (nlist > 0) __syncthreads();
                SKEW(10);
                STAMP(3);
                // ================= phase E: t* of the rays that changed =================
                const int nr = sh.n_rays;
                const OverlayZeta oz{d.cand_flag, d.cand_z, d.zeta0};
                // the t* of a changed ray and its chi^2 term (MCsub.jl:147-171), kept beside the old
                auto ray_done = [&](int r, double val, double tsr, double sgr, double old_term, int npr) {
                    v.cptS[r] = val;
                    const double df = val - tsr;
                    const double sg = sgr;
                    v.cterm[r] = old_term;                       // kept to undo a rejection
                    const double nterm = ((df * df) * 1.0) / (sg * sg);  // MCsub.jl:171
                    v.term[r] = nterm;
                    if constexpr (!RLDS) {  // (the running total: any order; rays in LDS re-add them all)
                        atomicAdd(&sh.dsum, nterm - old_term);
                        atomicAdd(&sh.dabs, fabs(nterm) + fabs(old_term));
                    }
                    if constexpr (RLDS)  // (the accounting below may run before phase E is over)
                        atomicAdd((unsigned long long *)&sh.bytes, (unsigned long long)npr * 17ull);
                    else
                        atomicAdd(&sh.ray_pts, npr);
                    if constexpr (WALK)  // an event of the walk (scripted steps: the decisions on bounds need none)
                        if (nscript) atomicOr(&cmask[r >> 6], 1ull << (r & 63));
                };
                if constexpr (!SMALL) {
                    // the large geometries (~15 changed rays a proposal, every load from HBM): two rays per
                    // wave at a time, one per half (ray_sum.h half_ray_sum), their loads in one round trip.
                    // Lane l holds the offsets, tS, sigma and old term of the wave's ray of turn l / 2,
                    // half l % 2 (one round of loads before the first sum; past 32 turns: per ray)
                    const int half = lane >> 5, hl = lane & 31;
                    const int mine = 2 * wv + (lane & 1) + 2 * kWv * (lane >> 1);
                    int ra = 0, s0a = 0, e0a = 0;
                    double tsa = 0.0, sga = 0.0, ota = 0.0;
                    if (mine < nr) {
                        ra = v.ray_at(mine);
                        s0a = v.ray_off[ra];
                        e0a = v.ray_off[ra + 1];
                        tsa = v.tS[ra];
                        sga = v.sig[ra];
                        ota = v.term[ra];
                    }
                    double *hs = reinterpret_cast<double *>(lds + L.scratch) + wv * 192 + half * 96;
                    for (int base = 2 * wv, j = 0; base < nr; base += 2 * kWv, ++j) {
                        const int rr = base + half;
                        const bool have = rr < nr;
                        int r = 0, s0 = 0, npr = 0;
                        double tsr = 0.0, sgr = 0.0, old_term = 0.0;
                        if (j < 32) {  // (wave-uniform)
                            const int src = 2 * j + half;
                            r = __shfl(ra, src);
                            s0 = __shfl(s0a, src);
                            npr = __shfl(e0a, src) - s0;
                            tsr = __shfl(tsa, src);
                            sgr = __shfl(sga, src);
                            old_term = __shfl(ota, src);
                        } else if (have) {
                            r = v.ray_at(rr);
                            s0 = v.ray_off[r];
                            npr = v.ray_off[r + 1] - s0;
                            tsr = v.tS[r];
                            sgr = v.sig[r];
                            old_term = v.term[r];
                        }
                        const double val = half_ray_sum(hl, d.w, oz, s0, have ? npr : 0, hs);
                        if (have && hl == 0) ray_done(r, val, tsr, sgr, old_term, npr);
                    }
                } else {
                    // rays in HBM: a wave's rays' offsets, tS, sigma and old terms, one per lane,
                    // in one round of loads before its first sum (the 64 first; more: per ray)
                    int ra = 0, s0a = 0, e0a = 0;
                    double tsa = 0.0, sga = 0.0, ota = 0.0;
                    if (!RLDS && wv + kWv * lane < nr && lane < 64) {
                        ra = v.ray_at(wv + kWv * lane);
                        s0a = v.ray_off[ra];
                        e0a = v.ray_off[ra + 1];
                        tsa = v.tS[ra];
                        sga = v.sig[ra];
                        ota = v.term[ra];
                    }
                    for (int rr = wv, j = 0; rr < nr; rr += kWv, ++j) {
                        int r, s0, npr;
                        double tsr, sgr, old_term;
                        if (!RLDS && j < 64) {
                            r = __builtin_amdgcn_readlane(ra, j);
                            s0 = __builtin_amdgcn_readlane(s0a, j);
                            npr = __builtin_amdgcn_readlane(e0a, j) - s0;
                            tsr = readlane_f64(tsa, j);
                            sgr = readlane_f64(sga, j);
                            old_term = readlane_f64(ota, j);
                        } else {
                            r = v.ray_at(rr);
                            s0 = v.ray_off[r];
                            npr = v.ray_off[r + 1] - s0;
                            tsr = v.tS[r];  // with the offsets
                            sgr = v.sig[r];
                            old_term = v.term[r];
                        }
                        const double val = wave_ray_sum(lane, d.w, oz, s0, npr, ray_scratch[wv]);
                        if (lane == 0) ray_done(r, val, tsr, sgr, old_term, npr);
                    }
                    if constexpr (RLDS) {
                        // no block barrier after phase E: only wave 0's decision reads the new terms, so a
                        // wave that summed rays counts itself done (its LDS writes first) and wave 0 waits
                        // for those (~1.2 rays a proposal: mostly none); the other waves go straight on to
                        // phase F's side work
                        if (wv != 0 && wv < nr) {
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                            if (lane == 0) atomicAdd(&sh.e_done, 1);
                        } else if (wv == 0 && nr > 1) {
                            const int want = min(nr, kWv) - 1;
                            SPIN_WAIT(__hip_atomic_load(&sh.e_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < want,
                                      1000);
                        }
                        SKEW(11);
                    }
                }
                if constexpr (!RLDS) __syncthreads();
                SKEW(12);
                STAMP(4);
            }
            // a server's step decided later: its answer goes out now, before phase F -- the changed rays'
            // new t*, from which the host forms phi_n itself (the sequential sum from the first changed
            // ray on its own partial sums, incremental.cpp), and a death's killed-site Interpolation
            // (phase B); this step's exact sums below then overlap the host's work
            const bool early = SCRIPT && mb && sh.step_cur.decision == kDecideLater;
            // the step's decision, read here, before phase F's barrier: wave 0 writes the next step into
            // step_cur at the iteration's end, which a wave still in phase G must not see
            const int sdec = nscript ? sh.step_cur.decision : 1;
            if (early && wv == 0) {
                server_report(sa.out, v, sh, n, lane, __builtin_nan(""));
                // the answer's system-scope stores acknowledged before done: no system-scope
                // fence, which would write back this XCD's L2 at every call
                __builtin_amdgcn_s_waitcnt(0);
                wave_sync_lds();
                if (lane == 0) {
                    mb_store(&mb->done, sh.srv_seq);
                    if (action == tdchain::kDeath) {  // left in the mailbox under this command's seq
                        mb_store(reinterpret_cast<long long *>(&mb->pq_val), __double_as_longlong(sh.q_zeta));
                        __builtin_amdgcn_s_waitcnt(0);
                        mb_store(&mb->pq_seq, sh.srv_seq);
                    }
                }
            }
            // ==== phase F: chi^2 + decision (wave 0) || next proposal, tile maxima (rays in HBM) ====
            const long long tF = prof_on ? clock64() : 0;  // diagnostic: per-wave time in F
            constexpr bool spec_in_F = true;
            double phi_n = 1.0;  // debug_prior: MCsub.jl:134-136
            int bdec = 0;        // wave 0, LDS layout: 1 rejected / 2 accepted on bounds, 0 on the exact phi_n
            // The proposal's terms summed in any order (decisions on bounds, below): the committed
            // running total plus phase E's changes, Tp, within Ep of the exact real sum (every
            // rounding bounded twice over: the total's own bound, the changes and their magnitudes
            // added in any order, the one add).  When Ep passes 1e-10 of Tp (or is not finite) the
            // sum is formed afresh from all the terms (block-uniform: every lane reads the same LDS).
            // Rays in LDS: the ~400 terms are re-added every time (one wave, one DPP reduction: as
            // cheap as keeping the total).
            const double Tp = RLDS ? 0.0 : sh.tsum + sh.dsum;
            const double Ep = RLDS ? 0.0 : sh.terr + kSumSlack * ((double)(sh.n_rays + 2) * sh.dabs + fabs(Tp));
            const bool anchor = RLDS || !(Ep <= 1e-10 * Tp);
            if constexpr (WALK) {
                // rays in HBM: the whole block adds the proposal's terms afresh in any order --
                // n / 512 global loads per thread, four in flight
                if (!nscript && fwd && sh.k0 < n && anchor) {  // (block-uniform)
                    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
                    int k = tid;
                    for (; k + 3 * NTH < n; k += 4 * NTH) {
                        p0 = p0 + gload(v.term + k);
                        p1 = p1 + gload(v.term + k + NTH);
                        p2 = p2 + gload(v.term + k + 2 * NTH);
                        p3 = p3 + gload(v.term + k + 3 * NTH);
                    }
                    for (; k < n; k += NTH) p0 = p0 + gload(v.term + k);
                    const double wsum = wave_sum_f64((p0 + p1) + (p2 + p3));
                    if (lane == 0) sh.wpart[wv] = wsum;
                    __syncthreads();
                    SKEW(13);
                }
            }
            if (RLDS && !nscript && action == tdchain::kDeath && lane == 0) {  // what phase G's shift overwrites
                if (wv != 0) {
                    int a, b;
                    shift_range((int)p.index, ncells, wv, kWv - 1, a, b);
                    if (b > a) sh.shift_edge[wv] = v.ord[b - 1];
                } else {
                    sh.shift_done = 0;
                }
            }
            if (wv == 0) {
                const int k0 = sh.k0;
                if (fwd) {
                    // the terms added in k order (MCsub.jl:170-172), bit for bit, by this
                    // wave (exact_sum.h); phase E put the changed rays' new terms in place
                    // (the old ones wait in cterm, their sums in prefix).
                    // Rays in LDS: the decision first, on bounds.  The terms are >= 0, so
                    // their sequential sum is within n ulps of any other association: the
                    // sum of ALL the proposal's terms in any order (one DPP reduction,
                    // whatever k0) brackets phi_n within 1e-9; phi_r is exact or likewise
                    // bracketed; the decision is monotone (up in phi, down in phi_n), so
                    // when it is the same at both corners of the brackets it is the one the
                    // exact values give.  A rejection then needs no exact sum; an acceptance
                    // leaves its partial sums unformed (prefix exact below ex_upto, phi_r an
                    // estimate in [phi_lo, phi_hi]) until a decision the brackets cannot
                    // take (phi_n within ~1e-9 of the threshold), a tempering round's end or
                    // the launch's end: then the committed terms from ex_upto and the
                    // proposal's from k0 are added in order, the binade-run scans.
                    // Rays in HBM: the same, the sum of all terms formed by the whole block
                    // (above); a scripted step (exact every time) walks the events instead --
                    // the new sums follow the old ones at a checked constant offset between
                    // events (exact_sum.h delta_walk).
                    if (!WALK || !nscript) {
                        // nothing changed (k0 == n): phi_n IS phi_r, estimate or not (MCsub.jl:169-172
                        // adds the same terms), and phi - phi_n = 0 in the decision either way
                        bool exact = nscript != 0;
                        if (k0 >= n) phi_n = phi_r;
                        if (!exact && k0 < n) {
                            double Sa = Tp, Ea = Ep;
                            if (anchor) {
                                Sa = 0.0;
                                if constexpr (WALK) {
                                    for (int w = 0; w < kWv; ++w) Sa = Sa + sh.wpart[w];
                                } else {
                                    double part = 0.0;
                                    for (int k = lane; k < n; k += 64) part = part + v.term[k];
                                    Sa = wave_sum_f64(part);
                                }
                                Ea = kSumSlack * (double)(n + 1) * fabs(Sa);
                            }
                            if (!RLDS && lane == 0) {  // the running total if the proposal is committed
                                sh.b_T = Sa;
                                sh.b_E = Ea;
                            }
                            // the sequential phi_n lies within (n - 1) ulps of the exact sum, far inside 1e-9
                            const double b_lo = (Sa - Ea) * (1.0 - 1e-9), b_hi = (Sa + Ea) * (1.0 + 1e-9);
                            // most decisions at once from the phi-free part (chain_logic.h decide_sure),
                            // else the two corners side by side: lane 0 (phi_lo, b_hi), lane 1 (phi_hi, b_lo)
                            const int sure = tdchain::decide_sure(sh.ap, pp.log_u, (sh.phi_lo - b_hi) * inv2t_r,
                                                                  (sh.phi_hi - b_lo) * inv2t_r);
                            if (sure != 0) {
                                bdec = sure > 0 ? 2 : 1;
                            } else {
                                const bool lo = lane == 0;
                                const int a = lane < 2 ? (int)tdchain::accept_t(P, inv2t_r, pp, lo ? sh.phi_lo : sh.phi_hi,
                                                                               lo ? b_hi : b_lo, czeta, zeta_killed,
                                                                               zetanew_death, sh.lnN)
                                                       : 0;
                                const int a_min = __builtin_amdgcn_readlane(a, 0), a_max = __builtin_amdgcn_readlane(a, 1);
                                bdec = a_min != a_max ? 0 : a_min ? 2 : 1;
                            }
                            // a tempering round's last iteration publishes phi: decided exactly (and
                            // every sum made exact) whatever the bounds say (testing: every k-th too)
                            if ((rbx || xch) && it + 1 == round_end) bdec = 0;
                            if (d.exact_every > 0 && (it % d.exact_every) == d.exact_every - 1) bdec = 0;
                            exact = bdec == 0;
                            phi_n = Sa;  // (an estimate on a decided proposal)
                            if (bdec == 2 && lane == 0) {  // the accepted terms' sums: unformed
                                sh.ex_upto = min(sh.ex_upto, k0);
                                sh.b_lo = b_lo;
                                sh.b_hi = b_hi;
                            }
                        }
                        if (exact && k0 < n) {  // the committed partial sums and phi_r, then the proposal's
                            const ExactPhis ex = exact_sums(v.term, v.prefix, v.cprefix, v.cterm, v.rflag, sh, n, lane,
                                                            true, k0, phi_r, phi_n);
                            phi_r = ex.phi;
                            phi_n = ex.phi_n;
                            if (prof_on && lane == 0) sh.prof[65] += 1;  // (diagnostic: exact decisions)
                        }
                        if (prof_on && lane == 0 && k0 < n) sh.prof[64] += n - k0;
                    } else {
                        double C = k0 > 0 ? v.prefix[k0 - 1] : 0.0;  // MCsub.jl:169 C = 0
                        if (k0 < n) {  // O(events), not O(tail): exact_sum.h delta_walk
                            C = delta_walk(v.term, v.prefix, v.rflag, k0, n, C, smask, cmask, v.cprefix, sh.dseg, lane,
                                           prof_on ? &sh.prof[72] : nullptr);
                            if (prof_on && lane == 0) sh.prof[64] += n - k0;
                        }
                        phi_n = k0 < n ? C : sh.phi;
                    }
                }
                if (prof_on && lane == 0) sh.prof[66] += clock64() - tF;  // diagnostic: scan done
            }
            if (tid == 0) {
                // Metropolis-Hastings decision (on bounds: the one accept() gives on the exact values);
                // a scripted step's decision is given (kDecideLater: by the server's next command;
                // the grid update below is then staged and applied only if it is a commit)
                const bool acc = nscript ? sh.step_cur.decision == 1
                                 : bdec != 0 ? bdec == 2
                                             : tdchain::accept_t(P, inv2t_r, pp, phi_r, phi_n, czeta, zeta_killed,
                                                                 zetanew_death, sh.lnN);
                acc_r = acc;
                sh.gs = Shared::GSnap{sh.n_changed, sh.n_rays, sh.n_tiles, sh.k0, acc ? 1 : 0};
                sh.defer = bdec == 2 ? 1 : 0;
                sh.phi_n = phi_n;
                if (prof_on) sh.prof[67] += clock64() - tF;  // diagnostic: decision taken
                if (acc || (mb && sh.step_cur.decision == kDecideLater)) {
                    sh.g_op = action == tdchain::kBirth ? 2 : action == tdchain::kDeath ? 1
                              : action == tdchain::kMove ? 3 : 4;
                    sh.g_slot = action == tdchain::kBirth ? new_slot : slot_k;
                    sh.g_ox = kx;
                    sh.g_oy = ky;
                    sh.g_oz = kz;
                    sh.g_nx = pp.x;
                    sh.g_ny = pp.y;
                    sh.g_nz = pp.z;
                    sh.g_nzeta = pp.zeta;
                    if (acc) atomicAdd((unsigned long long *)&sh.accepted[action], 1ull);
                }
                if (prof_on && bdec == 1) atomicAdd((unsigned long long *)&sh.prof[14], 1ull);  // rejected on bounds
            } else if (spec_in_F && tid == 64) {  // the next proposal as if this one were rejected
                if (can_spec) {
                    make_proposal(sh.ps[sh.cur ^ 1], P, draws[(it + 1) & 63], ncells, sh.nfree, sh.nslots, d.free_slots, d.cx,
                                  d.cy, d.cz, d.czeta, [&](int pos) { return v.ord[pos]; });
                    sh.spec_ok = 1;
                }
            } else if (wv == kWv - 1 || (kWv >= 6 && wv == kWv - 2)) {
                // wave kWv - 1: the grid data an accepted update will need; wave kWv - 2 (with 8 waves;
                // with 4 the last wave after its prefetch): accounting and the model-size factors
                if (wv == kWv - 1)
                    grid_prefetch(d, sh, lane, action, action == tdchain::kBirth ? new_slot : slot_k, kx, ky,
                                  kz, pp.x, pp.y, pp.z);
                if (wv == (kWv >= 6 ? kWv - 2 : kWv - 1)) {
                    if (prof_on && lane == 0) {  // diagnostic: work sizes
                        sh.prof[68] += sh.n_tiles;
                        sh.prof[69] += sh.pts_seen;
                        sh.prof[70] += sh.n_changed;
                        sh.prof[71] += sh.n_rays;
                    }
                    if (lane == 0 && fwd) {  // accounting, off wave 0's path
                        atomicAdd((unsigned long long *)&sh.evaluations, 1ull);
                        // bytes this proposal's algorithm must read: tile boxes + maxima (32 B),
                        // candidate points (coords + cached slot/distance, 36 B), grid queries
                        // (27 buckets x 8 entries x 32 B), rays (w, zeta, flag: 17 B per point),
                        // chi^2 tail (ptS, tS, sig, flag: 28 B per ray)
                        atomicAdd((unsigned long long *)&sh.bytes,
                                  (unsigned long long)((super_on ? (long long)NS * 32 +
                                                                      (long long)sh.n_super[it & 1] * kTilePts * 32
                                                                 : (long long)NT * 32) +
                                                       (long long)sh.pts_seen * 36 +
                                                       (long long)(no + (action <= 2 ? 1 : 0)) * 27 * 8 * 32 +
                                                       (RLDS ? 0ll : (long long)sh.ray_pts * 17) + (long long)(n - sh.k0) * 28));
                    }
                    if (lane == 0 && (action == tdchain::kBirth || action == tdchain::kDeath)) {
                        sh.lnN_far[0] = d.logN[max(ncells - 2, 0)];
                        sh.lnN_far[1] = d.logN[ncells + 2];
                    }
                }
            } else if (wv >= 2 && wv <= (kWv >= 6 ? kWv - 3 : 2) && fwd && action != tdchain::kChange) {
                // (waves 2..5 of 8, wave 2 of 4) the hit tiles' maxima if the proposal is accepted (a tile =
                // a DPP row): four items per thread in flight (rays in HBM: ~140 hit tiles, each load a
                // round trip)
                const int nt = sh.n_tiles;
                constexpr int MU = 4, MS = (kWv >= 6 ? kWv - 4 : 1) * 64;
                if constexpr (RLDS) {  // (~8 hit tiles over 4 waves: one item per thread)
                    for (int i = tid - 128; i < nt * kTilePts; i += MS) {
                        const int sc = v.tile_rec(i / kTilePts).y;  // start << 5 | count
                        const int q = (sc >> 5) + (i % kTilePts);
                        unsigned long long mk = 0ull;  // distances are >= 0: max as bit patterns
                        if (i % kTilePts < (sc & 31)) {
                            const double cd = d.cand_d[q], bd = d.best_d[q];
                            mk = (unsigned long long)__double_as_longlong(d.cand_flag[q] ? cd : bd);
                        }
                        mk = row_max_u64(mk);
                        if ((i % kTilePts) == kTilePts - 1) v.ctm_put(i / kTilePts, __longlong_as_double((long long)mk));
                    }
                } else
                for (int i0 = tid - 128; i0 < nt * kTilePts; i0 += MU * MS) {
                    int q[MU];
                    bool in[MU];
#pragma unroll
                    for (int u = 0; u < MU; ++u) {
                        const int i = min(i0 + u * MS, nt * kTilePts - 1);
                        const int sc = v.tile_rec(i / kTilePts).y;  // start << 5 | count
                        in[u] = i0 + u * MS < nt * kTilePts && (i % kTilePts) < (sc & 31);
                        q[u] = in[u] ? (sc >> 5) + (i % kTilePts) : 0;
                    }
                    double cd[MU], bd[MU];
                    unsigned char cf[MU];
#pragma unroll
                    for (int u = 0; u < MU; ++u) {
                        cd[u] = d.cand_d[q[u]];
                        bd[u] = d.best_d[q[u]];
                        cf[u] = d.cand_flag[q[u]];
                    }
#pragma unroll
                    for (int u = 0; u < MU; ++u) {
                        const int i = i0 + u * MS;
                        if (i >= nt * kTilePts) break;  // (whole rows: the same in the 16 lanes of a tile)
                        unsigned long long mk = 0ull;  // distances are >= 0: max as bit patterns
                        if (in[u]) mk = (unsigned long long)__double_as_longlong(cf[u] ? cd[u] : bd[u]);
                        mk = row_max_u64(mk);
                        if ((i % kTilePts) == kTilePts - 1) v.ctm_put(i / kTilePts, __longlong_as_double((long long)mk));
                    }
                }
            }
            if (prof_on && lane == 0)
                atomicAdd((unsigned long long *)&sh.prof[56 + wv], (unsigned long long)(clock64() - tF));
            __syncthreads();
            STAMP(5);
            SKEW(14);
            // ================= phase G: commit (or undo) =================
            const int nc = sh.gs.nc, nr = sh.gs.nr;
            if (nscript && sdec != 1 && !early && wv == 0) server_report(sa.out, v, sh, n, lane, sh.phi_n);
            if (mb && sdec == kDecideLater) {  // answered before phase F; its fate comes with the next command
                if (wv == 0) server_wait(mb, d, v, sh, lane);
                __syncthreads();
                SKEW(15);
                if (tid == 0) acc_r = sh.gs.accept != 0;
            }
            // the changed points' global records (two dependent L2 round trips) and the
            // deleteat! shift go to waves 1.., so wave 0 goes straight to its scalars and
            // the next proposal (kW threads, index w = tid - 64)
            constexpr int kW = NTH - 64;
            const int w = tid - 64;
            if (sh.gs.accept) {
                const int nt = sh.gs.nt, k0 = sh.gs.k0;
                if (wv != 0)
                    for (int c = w; c < nc; c += kW) {
                        if (c < kChgLds) {  // (LDS: stores only)
                            const ChgRec r = sh.chg[c];
                            d.best_s[r.q] = r.s;
                            d.best_d[r.q] = r.d;
                            d.zeta0[r.q] = r.z;
                            d.cand_flag[r.q] = 0;
                        } else {
                            const int q = d.changed[c];
                            d.best_s[q] = d.cand_s[q];
                            d.best_d[q] = d.cand_d[q];
                            d.zeta0[q] = d.cand_z[q];
                            d.cand_flag[q] = 0;
                        }
                    }
                if (fwd && action != tdchain::kChange) {
                    for (int i = tid; i < nt; i += NTH) v.tmaxd[v.tile_rec(i).x] = v.ctm_at(i);
                    pend_sup = super_on;  // their super-tiles' maxima: at the top of the next iteration
                }
                for (int rr = tid; rr < nr; rr += NTH) {
                    const int r = v.ray_at(rr);
                    v.ptS[r] = v.cptS[r];
                    v.rflag[r] = 0;
                }
                if (!WALK || !nscript) {
                    if (!sh.defer)  // (accepted on bounds: its partial sums are left unformed)
                        for (int r = k0 + tid; r < n; r += NTH) v.prefix[r] = v.cprefix[r];
                } else if (fwd && k0 < n) {
                    pend_r = true;  // written at the top of the next iteration
                    if (wv == 1) delta_remark(v.term, v.prefix, v.cprefix, n, sh.dseg, smask, lane);
                }
                if (RLDS && action == tdchain::kDeath && wv != 0 && !nscript) {  // deleteat!, in LDS (shift_range)
                    int a, b;
                    shift_range((int)pp.index, ncells, wv, kWv - 1, a, b);
                    if (b > a) {
                        const int edge = sh.shift_edge[wv];
                        for (int j0 = a; j0 < b; j0 += 64) {
                            const int j = j0 + lane;
                            if (j < b) {
                                const int sl = j == b - 1 ? edge : v.ord[j];
                                v.ord[j - 1] = sl;
                            }
                        }
                    }
                    // this wave's shifted stores, released before its count (wave 0 acquires it below)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) atomicAdd(&sh.shift_done, 1);
                    SKEW(16);
                }
                if (RLDS && action == tdchain::kDeath && wv != 0 && nscript) {  // deleteat!: from the staged copy
                    constexpr int U = 4;                                 // U loads in flight per thread
                    for (int j0 = (int)pp.index + 1 + w; j0 < ncells; j0 += U * kW) {
                        int sl[U];
#pragma unroll
                        for (int u = 0; u < U; ++u) sl[u] = d.order_tmp[min(j0 + u * kW, ncells - 1)];
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const int j = j0 + u * kW;
                            if (j < ncells) v.ord[j - 1] = sl[u];
                        }
                    }
                }
                if (tid == NTH - 64 && sh.g_op) grid_apply(d, sh);
                if (tid == 0) {
                    const int sk = slot_k;
                    if (action == tdchain::kBirth) {  // append!
                        const int s = new_slot;
                        d.cx[s] = pp.x;
                        d.cy[s] = pp.y;
                        d.cz[s] = pp.z;
                        d.czeta[s] = pp.zeta;
                        v.ord[ncells] = s;
                        const long long st_new = sh.next_stamp;  // appended: after every live cell in Julia order
                        d.stamp[s] = st_new;
                        sh.next_stamp = st_new + 1;
                        if (sh.nfree > 0)
                            sh.nfree -= 1;
                        else
                            sh.nslots += 1;
                        sh.ncells = ncells + 1;
                        const double a = sh.lnN[1], b = sh.lnN[2], c = sh.lnN_far[1];
                        sh.lnN[0] = a;
                        sh.lnN[1] = b;
                        sh.lnN[2] = c;
                    } else if (action == tdchain::kDeath) {
                        d.free_slots[sh.nfree] = sk;
                        sh.nfree += 1;
                        d.stamp[sk] = -1;  // a free slot
                        sh.ncells = ncells - 1;
                        const double a = sh.lnN_far[0], b = sh.lnN[0], c = sh.lnN[1];
                        sh.lnN[0] = a;
                        sh.lnN[1] = b;
                        sh.lnN[2] = c;
                    } else if (action == tdchain::kChange) {
                        d.czeta[sk] = pp.zeta;
                    } else {
                        d.cx[sk] = pp.x;
                        d.cy[sk] = pp.y;
                        d.cz[sk] = pp.z;
                    }
                    if (!RLDS && !nscript && fwd && k0 < n) {  // the running total follows the committed terms
                        sh.tsum = sh.b_T;
                        sh.terr = sh.b_E;
                    }
                    if (bdec == 2) {  // an estimate inside the bracket of phase F
                        phi_r = sh.phi_n;
                        sh.phi_lo = sh.b_lo;
                        sh.phi_hi = sh.b_hi;
                    } else if (!(!nscript && fwd && k0 >= n)) {  // (nothing changed: phi_r stays)
                        phi_r = sh.phi_n;
                        sh.phi_lo = sh.phi_hi = phi_r;
                        sh.phi = phi_r;
                    }
                }
                if constexpr (!RLDS) {
                    // the order in HBM, an accepted death (block-uniform): deleteat! in place, the whole
                    // block -- a round's loads, a barrier, its shifted stores (the next round reads
                    // only positions past the ones this one writes); a barrier before wave 0 reads
                    // the shifted order for the next proposal
                    if (action == tdchain::kDeath) {
                        constexpr int U = 8;
                        for (int b0 = (int)pp.index + 1; b0 < ncells; b0 += U * NTH) {
                            int sl[U];
#pragma unroll
                            for (int u = 0; u < U; ++u) sl[u] = gload(v.ord + min(b0 + tid + u * NTH, ncells - 1));
                            __syncthreads();
                            SKEW(18);
#pragma unroll
                            for (int u = 0; u < U; ++u) {
                                const int j = b0 + tid + u * NTH;
                                if (j < ncells) v.ord[j - 1] = sl[u];
                            }
                        }
                        __syncthreads();
                    }
                }
            } else {  // rejected: flags down, the changed rays get their old chi^2 terms back
                if (wv != 0)
                    for (int c = w; c < nc; c += kW) d.cand_flag[c < kChgLds ? sh.chg[c].q : d.changed[c]] = 0;
                for (int rr = tid; rr < nr; rr += NTH) {
                    const int r = v.ray_at(rr);
                    v.term[r] = v.cterm[r];
                    v.rflag[r] = 0;
                }
            }
        }
        last_action = action;
        last_accept = acc_r ? 1 : 0;
        STAMP(12);
        // ===== end of iteration: the next proposal (wave 0; draws refilled every 64) =====
        if (wv == 0) {
            if (prof_on && lane == 0) sh.prof[7 + action] += clock64() - sh.t_iter;  // per-action totals
            if ((rbx || xch) && it + 1 == round_end) {  // a tempering round is done: publish phi, take the next temperature
                {  // (a phase F of this iteration made every sum exact already)
                    phi_r = exact_sums(v.term, v.prefix, v.cprefix, v.cterm, v.rflag, sh, n, lane, false, n, phi_r, 0.0).phi;
                    if (lane == 0) sh.phi = phi_r;
                }
                if (rbx) {
                    round_wait(rbx, bchain, sh, lane, true, phi_r);  // (lane 0 = tid 0 holds phi)
                    round_end = it + 1 + sh.rK;
                } else {
                    const long long Kx = rxp->K;
                    round_exchange(*rxp, bchain, (it + 1) / Kx - 1, sh, lane, phi_r);
                    round_end = it + 1 + Kx;
                }
                inv2t_r = sh.rinv2t;
            }
            if (it + 1 < iters && !((mb || rbx || xch) && sh.srv_quit)) {
                if (((it + 1) & 63) == 0 && !nscript) {
                    wave_sync_lds();
                    if (sa.pre) {
                        if (it + 1 + lane < iters) draws[lane] = sa.pre[(long long)bchain * sa.pre_stride + it + 1 + lane];
                    } else {
                        draws[lane] = tdchain::draw_iteration(d.seed, d.chain, (uint64_t)(iter0 + it + 1 + lane));
                    }
                    wave_sync_lds();
                }
                if (lane == 0) {
                    const bool acc = acc_r;
                    // the guess holds unless an accepted proposal changed what it read
                    const PState &g = sh.ps[cur_r ^ 1];
                    const bool keep = sh.spec_ok && can_spec &&
                                      (!acc || ((action == tdchain::kChange || action == tdchain::kMove) &&
                                                g.slot_k != slot_k));
                    if (keep) {
                        cur_r ^= 1;  // adopt the guess: no copy
                        sh.cur = cur_r;
                    } else {
                        // a just-killed position (LDS layout; in the HBM order phase G has shifted it already):
                        // scripted steps read the staged pre-shift order; a free-running chain the order once
                        // the shifting waves are done
                        const bool killed = RLDS && acc && action == tdchain::kDeath;
                        if (killed && !nscript)
                            SPIN_WAIT(__hip_atomic_load(&sh.shift_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <
                                          kWv - 1,
                                      1000000);
                        auto slot_at = [&](int pos) {
                            return (killed && nscript && pos >= (int)pp.index) ? d.order_tmp[pos + 1] : v.ord[pos];
                        };
                        if (nscript) {
                            sh.step_cur = mb ? sh.srv_step[sh.srv_k++] : sa.step[it + 1];
                            script_proposal(sh.ps[cur_r], sh.step_cur, sh.nfree, sh.nslots, d.free_slots, slot_at);
                        }
                        else
                            make_proposal(sh.ps[cur_r], P, draws[(it + 1) & 63], sh.ncells, sh.nfree, sh.nslots,
                                          d.free_slots, d.cx, d.cy, d.cz, d.czeta, slot_at);
                    }
                    const tdchain::Proposal &np = sh.ps[cur_r].p;
                    if (np.active) atomicAdd((unsigned long long *)&sh.proposed[np.action], 1ull);
                    sh.spec_ok = 0;
                    // the next proposal's counters: no wave reads them after phase F's barrier (phase G reads
                    // the snapshot sh.gs), so they are clear before the iteration-end barrier whatever the skew
                    sh.n_tiles = sh.n_changed = sh.n_orphans = sh.n_rays = 0;
                    if (!RLDS) sh.dsum = sh.dabs = 0.0;
                    sh.n_super[(it + 1) & 1] = 0;  // the other parity's list is refreshed first
                    sh.pts_seen = sh.ray_pts = 0;
                    sh.e_done = sh.b_done = 0;
                    sh.k0 = n;
                }
            }
        }
        STAMP(13);
        it_done = it + 1;
        __syncthreads();
        STAMP(6);
        SKEW(17);
    }

    const long long t_loop_end = prof_on ? clock64() : 0;
    {  // decisions on bounds: the partial sums and phi exact again (the launch leaves them)
        if (wv == 0) {
            phi_r = exact_sums(v.term, v.prefix, v.cprefix, v.cterm, v.rflag, sh, n, lane, false, n, phi_r, 0.0).phi;
            if (lane == 0) sh.phi = phi_r;
        }
        __syncthreads();
    }
    if constexpr (WALK) {
        if (pend_r) delta_commit<SMALL ? 1 : 16>(v.prefix, v.cprefix, n, sh.dseg, tid, NTH);
        if constexpr (SMALL) __syncthreads();  // the LDS sums are written back below
    }
    // ---- leave the LDS copies behind (flags and grid are already clean) ----
    if constexpr (SMALL) {
        for (int i = tid; i < NT; i += NTH) d.tile_maxd[i] = v.tmaxd[i];
        if constexpr (RLDS) {
            for (int i = tid; i < n; i += NTH) {
                d.ptS[i] = v.ptS[i];
                d.prefix[i] = v.prefix[i];
            }
            for (int i = tid; i < sh.ncells; i += NTH) d.order[i] = v.ord[i];
        }
    }
    if (tid == 0) {
        ChainScalars &s = *d.st;
        s.iter = iter0 + it_done;
        s.evaluations += sh.evaluations;
        s.bytes += sh.bytes;
        for (int a = 0; a < 5; ++a) {
            s.proposed[a] += sh.proposed[a];
            s.accepted[a] += sh.accepted[a];
        }
        s.phi = sh.phi;
        s.ncells = sh.ncells;
        s.nslots = sh.nslots;
        s.nfree = sh.nfree;
        s.next_stamp = sh.next_stamp;
        if (iters > 0) {
            s.last_action = last_action;
            s.last_accept = last_accept;
        }
        if (prof_on) {
            sh.prof[77] += clock64() - t_loop_end;  // epilogue (write-backs, scalars) up to here
            sh.prof[78] += 1;                        // launches
        }
        for (int k = 0; k < kProfSlots; ++k) s.prof[k] += sh.prof[k];
        s.prof[15] += sh.grid_fallbacks32;  // diagnostic: unproven grid searches
        if (d.st_host) *d.st_host = s;  // the host's pinned mirror: no copy back per chain
        if (mb) {
            __threadfence_system();
            mb_store(&mb->exited, 1);
        }
        if (rbx) {
            __threadfence_system();
            mb_store(&rbx->slot[bchain].exited, 1);
        }
    }
}

// ------------------------------------------------- one-point queries ----
// Interpolation at one point (MCsub.jl:306-327 with 1-element X/Y/Z, as the
// reference's birth and death queries call it, TD_inversion_function.jl:81,
// 146) against a chain's committed model, or that model plus one edit
// (td_evaluate's pending proposal, incremental.cpp): one wave, the chain's
// bucket grid (full scan when unproven), the same lexicographic (distance,
// Julia position) answer as v_nearest.  out[0] = the value.
__global__ __launch_bounds__(64) void k_chain_query(const DevChain *__restrict__ dptr, double x, double y, double z,
                                                   ScriptStep e, int has_edit, double *out) {
    const DevChain &d = *dptr;
    __shared__ Shared sh;
    const int lane = threadIdx.x;
    if (lane == 0) {
        sh.grid_ovf = *d.grid_overflow;
        sh.nslots = d.st->nslots;
        sh.grid_fallbacks32 = 0;
        geo_fill(sh.geo, d);
    }
    __syncthreads();
    Views v{};
    v.ord = d.order;
    int skip = -1, moved = -1, slot_k = -1;
    if (has_edit && e.action != tdchain::kBirth) slot_k = d.order[e.index];
    if (has_edit && e.action == tdchain::kDeath) skip = slot_k;  // the reduced model (:132-135)
    if (has_edit && e.action == tdchain::kMove) moved = slot_k;  // the cell at its new site
    Nearest r = wave_nearest(d, v, sh, lane, x, y, z, skip, moved, e.x, e.y, e.z, moved >= 0 ? d.czeta[moved] : 0.0);
    double val = r.z;
    if (has_edit && e.action == tdchain::kChange && r.s == slot_k) val = e.zeta;
    if (has_edit && e.action == tdchain::kBirth) {  // the appended cell: last position, wins only strictly
        const double dd = dist2(e.x, e.y, e.z, x, y, z);
        if (dd < r.d && dd < kSentinel) val = e.zeta;
    }
    if (lane == 0) out[0] = val;
}

// ------------------------------------------------------------ full state ----
// chi^2 prefix sums, sequential (MCsub.jl:170-172), and phi.
__global__ __launch_bounds__(256) void k_chi2_prefix(const double *__restrict__ ptS, const double *__restrict__ tS,
                                                     const double *__restrict__ sig, int n,
                                                     double *__restrict__ prefix, ChainScalars *st) {
    __shared__ double t[2048];
    double C = 0.0;
    for (int base = 0; base < n; base += 2048) {
        const int cnt = min(2048, n - base);
        for (int k = threadIdx.x; k < cnt; k += 256) {
            const double df = ptS[base + k] - tS[base + k];
            const double sg = sig[base + k];
            t[k] = ((df * df) * 1.0) / (sg * sg);
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int k = 0; k < cnt; ++k) {
                C = C + t[k];
                prefix[base + k] = C;
            }
        __syncthreads();
    }
    if (threadIdx.x == 0) st->phi = C;
}

__global__ void k_tile_max(const int *__restrict__ tile_start, int ntiles, const double *__restrict__ best_d,
                           double *__restrict__ tile_maxd) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    double mx = -1.0;
    const int sc = tile_start[t];  // start << 5 | count
    for (int q = sc >> 5; q < (sc >> 5) + (sc & 31); ++q) mx = fmax(mx, best_d[q]);
    tile_maxd[t] = mx;
}

// The proposal-time chi^2 of phase F on a caller-given ptS (testing): terms as
// phase E writes them, the one-wave exact scan from k0 = 0 and from k0 = n/2
// (C0 = the sequential prefix[k0 - 1] of k_chi2_prefix).
__global__ __launch_bounds__(64) void k_test_chain_chi2(const double *__restrict__ ptS, const double *__restrict__ tS,
                                                        const double *__restrict__ sig, int n,
                                                        const double *__restrict__ prefix, double *term,
                                                        double *cprefix, double *out) {
    const int lane = threadIdx.x;
    for (int r = lane; r < n; r += 64) {
        const double df = ptS[r] - tS[r];
        const double sg = sig[r];
        term[r] = ((df * df) * 1.0) / (sg * sg);  // MCsub.jl:171
    }
    __syncthreads();
    bool stopped = false;
    const double a = wave_seq_sum(term, n, 0.0, cprefix, lane, nullptr, &stopped);
    const int k0 = n / 2;
    stopped = false;
    const double b = k0 < n ? wave_seq_sum(term + k0, n - k0, k0 > 0 ? prefix[k0 - 1] : 0.0, cprefix + k0, lane, nullptr,
                                           &stopped)
                            : a;
    if (lane == 0) {
        out[0] = a;
        out[1] = b;
    }
}

}  // namespace

hipError_t test_chain_chi2(const double *ptS, const double *tS, const double *sig, int n, int path, double *scratch,
                           double *out, hipStream_t s) {
    if (n < 1 || n > 4096) return hipErrorInvalidValue;
    double *prefix = scratch, *term = scratch + n, *cpre = scratch + 2 * n;
    ChainScalars *st = reinterpret_cast<ChainScalars *>(scratch + 3 * n + 8);  // 16-byte aligned slot
    static_assert(sizeof(ChainScalars) <= 1024, "scratch slot");
    if (path == 2) {
        hipLaunchKernelGGL(k_chi2_prefix, dim3(1), dim3(256), 0, s, ptS, tS, sig, n, prefix, st);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return hipMemcpyAsync(out, &st->phi, sizeof(double), hipMemcpyDeviceToDevice, s);
    }
    hipLaunchKernelGGL(k_chi2_prefix, dim3(1), dim3(256), 0, s, ptS, tS, sig, n, prefix, st);
    hipLaunchKernelGGL(k_test_chain_chi2, dim3(1), dim3(64), 0, s, ptS, tS, sig, n, prefix, term, cpre, out);
    return hipGetLastError();
}

hipError_t chain_full_state(DevChain &d, int ncells, NNWork &work, int num_cus, hipStream_t s) {
    Geometry g;
    g.m = 0;
    g.n = d.n;
    g.P = d.P;
    g.px = const_cast<double *>(d.px);
    g.py = const_cast<double *>(d.py);
    g.pz = const_cast<double *>(d.pz);
    g.w = const_cast<double *>(d.w);
    g.ray_off = const_cast<int *>(d.ray_off);
    g.tS = const_cast<double *>(d.tS);
    g.sig = const_cast<double *>(d.sig);
    // slots 0..ncells-1 hold the cells in order, so nearest index == slot
    hipError_t e = launch_nearest(d.px, d.py, d.pz, d.P, 1, 1, d.cx, d.cap, ncells, work, num_cus, d.best_s,
                                  d.best_d, d.zeta0, s);
    if (e != hipSuccess) return e;
    e = launch_ray_sums(g, d.zeta0, d.ptS, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_chi2_prefix, dim3(1), dim3(256), 0, s, d.ptS, d.tS, d.sig, d.n, d.prefix, d.st);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (d.ntiles > 0) {
        hipLaunchKernelGGL(k_tile_max, dim3((d.ntiles + 255) / 256), dim3(256), 0, s, d.tile_start, d.ntiles,
                           d.best_d, d.tile_maxd);
        e = hipGetLastError();
    }
    return e;
}

// Testing: the latency of a nearest-cell query through the chain's bucket grid, as phases B and D run
// it: one wave answers nq queries back to back, each point offset by 0 * the previous answer (no two
// overlap).  mode 0: wave_nearest; 1: its loads only (the sum of what they bring); 2: its arithmetic only
// (the loads replaced by values made from the lane).  out[0] = cycles, out[1] = unproven queries.
__global__ __launch_bounds__(64) void k_test_query_lat(const DevChain *__restrict__ dptr, const double *__restrict__ pts,
                                                        int nq, int mode, long long *out) {
    __shared__ Shared sh;
    const DevChain &d = *dptr;
    const int lane = threadIdx.x;
    Views v{};
    v.ord = d.order;
    if (lane == 0) {
        sh.grid_ovf = *d.grid_overflow;
        sh.grid_fallbacks32 = 0;
        sh.nslots = d.st->nslots;
        geo_fill(sh.geo, d);
    }
    __syncthreads();
    double acc = 0.0;
    unsigned long long hsh = 0xcbf29ce484222325ull;
    const long long t0 = clock64();
    for (int i = 0; i < nq; ++i) {
        const double k = acc * 0.0;
        const double x = pts[3 * i] + k, y = pts[3 * i + 1] + k, z = pts[3 * i + 2] + k;
        if (mode == 0 || mode == 6) {  // 6: the descriptor-reading search (d.grid), for comparison
            const Nearest r = mode == 0 ? wave_grid_search(sh.geo, sh.grid_ovf != 0, lane, x, y, z, -1, -1, 0.0, 0.0,
                                                           0.0, 0.0)
                                        : wave_grid_search(d, sh.grid_ovf != 0, lane, x, y, z, -1, -1, 0.0, 0.0,
                                                           0.0, 0.0);
            acc = r.z;
            // (a digest of every answer: the two searches must agree)
            hsh = hsh * 0x100000001b3ull ^ (unsigned long long)__double_as_longlong(r.d) ^
                  ((unsigned long long)(unsigned)r.s << 1) ^ (unsigned long long)r.proven;
        } else {
            const CellGrid &G = d.grid;
            const int bi = grid_axis(x, G.x0, G.ix, G.gx), bj = grid_axis(y, G.y0, G.iy, G.gy),
                      bk = grid_axis(z, G.z0, G.iz, G.gz);
            const int nb = lane % 27, grp = lane / 27;
            const int ii = bi + nb % 3 - 1, jj = bj + (nb / 3) % 3 - 1, kk = bk + nb / 9 - 1;
            const bool inb = lane < 54 && ii >= 0 && ii < G.gx && jj >= 0 && jj < G.gy && kk >= 0 && kk < G.gz;
            const int b = inb ? (kk * G.gy + jj) * G.gx + ii : 0;
            double t = 0.0;
            if (mode == 3) {  // the bucket indices alone
                t = (double)(b + grp);
            } else if (mode == 4) {  // the block's face bound alone
                t = grid_block_lb(G, x, y, z, 1);
            } else if (mode == 5) {  // one lexicographic wave minimum alone
                t = (double)wave_min_u64((unsigned long long)(b + lane));
            } else if (mode == 1) {
                const int cnt = gload(d.bucket_count + b);
                double a = 0.0;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const CellEntry *ep = d.buckets + b * kBucketCap + grp * 4 + u;
                    a = a + gload(&ep->x) + gload(&ep->y) + gload(&ep->z) + gload(&ep->zeta) +
                        (double)gload(d.bslot + b * kBucketCap + grp * 4 + u);
                }
                t = a + (double)cnt;
                t = wave_sum_f64(t);
            } else {
                double bd = kSentinel;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double dd = dist2((double)b, (double)u, (double)lane, x, y, z);
                    bd = dd < bd ? dd : bd;
                }
                const double lb = grid_block_lb(G, x, y, z, 1);
                const unsigned long long kmin = wave_min_u64((unsigned long long)__double_as_longlong(bd));
                t = __longlong_as_double((long long)kmin) < lb ? 1.0 : 2.0;
            }
            acc = t;
        }
    }
    const long long t1 = clock64();
    if (lane == 0) {
        out[0] = t1 - t0;
        out[1] = sh.grid_fallbacks32;
        out[2] = __double_as_longlong(acc);
        out[3] = (long long)hsh;
    }
}

// Testing: every query's answer (squared distance, the winning cell's value, proven) from the chain's grid
// search, mode 0 (the LDS GridGeo copy with the global first bound) or 6 (the descriptor-reading form):
// the tests compare the proven ones with an exact scan (tdt_chain_query_answers)
__global__ __launch_bounds__(64) void k_test_query_answers(const DevChain *__restrict__ dptr, const double *__restrict__ pts,
                                                           int nq, int mode, double *out_d, double *out_z, int *out_p) {
    __shared__ Shared sh;
    const DevChain &d = *dptr;
    const int lane = threadIdx.x;
    if (lane == 0) {
        sh.grid_ovf = *d.grid_overflow;
        sh.grid_fallbacks32 = 0;
        geo_fill(sh.geo, d);
    }
    __syncthreads();
    for (int i = 0; i < nq; ++i) {
        const double x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
        const Nearest r = mode == 0 ? wave_grid_search(sh.geo, sh.grid_ovf != 0, lane, x, y, z, -1, -1, 0.0, 0.0, 0.0, 0.0)
                                    : wave_grid_search(d, sh.grid_ovf != 0, lane, x, y, z, -1, -1, 0.0, 0.0, 0.0, 0.0);
        if (lane == 0) {
            out_d[i] = r.d;
            out_z[i] = r.z;
            out_p[i] = r.proven ? 1 : 0;
        }
    }
}

// Testing: the phase-B tile filter on given FP32 boxes (SoA, 3 x nt each), FP64 tile maxima and FP64
// queries: out[q * nt + t] = 1 if the filter lets tile t through for query q (mode 0 tile_may_hit, 1
// tile_may_hit2).  The tests hold it to "never drops a tile holding a point within the maximum".
__global__ void k_test_tile_filter(const float *__restrict__ lo, const float *__restrict__ hi,
                                   const double *__restrict__ maxd, int nt, const double *__restrict__ qs, int nq,
                                   int mode, unsigned char *__restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)nt * nq) return;
    const int t = (int)(i % nt), q = (int)(i / nt);
    const double x = qs[3 * q], y = qs[3 * q + 1], z = qs[3 * q + 2];
    bool h;
    if (mode == 0) {
        h = tile_may_hit(lo, hi, nt, t, tile_query(x, y, z), tile_thr(maxd[t]));
    } else {
        h = tile_may_hit2(tile_box(lo, hi, maxd, nt, t), tile_query2(x, y, z));
    }
    out[i] = h ? 1 : 0;
}

hipError_t test_tile_filter(const float *lo, const float *hi, const double *maxd, int nt, const double *qs, int nq,
                            int mode, unsigned char *out, hipStream_t s) {
    const long long n = (long long)nt * nq;
    hipLaunchKernelGGL(k_test_tile_filter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, lo, hi, maxd, nt, qs,
                       nq, mode, out);
    return hipGetLastError();
}

hipError_t test_query_answers(const DevChain *dev, const double *pts, int nq, int mode, double *out_d, double *out_z,
                              int *out_p, hipStream_t s) {
    hipLaunchKernelGGL(k_test_query_answers, dim3(1), dim3(64), 0, s, dev, pts, nq, mode, out_d, out_z, out_p);
    return hipGetLastError();
}

hipError_t test_query_lat(const DevChain *dev, const double *pts, int nq, int mode, long long *out, hipStream_t s) {
    hipLaunchKernelGGL(k_test_query_lat, dim3(1), dim3(64), 0, s, dev, pts, nq, mode, out);
    return hipGetLastError();
}

hipError_t chain_query(const DevChain *dev, double x, double y, double z, const ScriptStep *edit, double *out,
                       hipStream_t s) {
    ScriptStep e{};
    if (edit) e = *edit;
    hipLaunchKernelGGL(k_chain_query, dim3(1), dim3(64), 0, s, dev, x, y, z, e, edit ? 1 : 0, out);
    return hipGetLastError();
}

void chain_lds_sizes(const DevChain &d, int64_t out[4]) {
    const LdsPlan a = lds_plan(d.ntiles, d.n, d.cap, true), b = lds_plan(d.ntiles, d.n, d.cap, false);
    out[0] = (int64_t)a.total;      // LDS layout (tiles, rays, order mirrored)
    out[1] = (int64_t)b.total;      // HBM layout
    out[2] = b.super_lds ? 1 : 0;   // HBM layout with super-tiles in LDS
    out[3] = (int64_t)(a.total <= kLdsBudget && d.lds_mode != 1);  // the layout a launch takes: 1 = LDS
}

// Every iteration's draws of a launch (a function of seed, chain, iteration: tdchain::draw_iteration),
// one thread each, ahead of k_chain_run: its per-64-iteration refill -- one wave computing 64 draws'
// quantiles and logarithm on the chain's critical path -- becomes one round of loads.
__global__ __launch_bounds__(256) void k_draws(const DevChain *__restrict__ dptr, long long iters,
                                               tdchain::Draws *__restrict__ out) {
    const DevChain &d = dptr[blockIdx.y];
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= iters) return;
    out[(long long)blockIdx.y * iters + i] = tdchain::draw_iteration(d.seed, d.chain, (uint64_t)(d.st->iter + i));
}

hipError_t chain_run(const DevChain *host, const DevChain *dev, int nchains, int64_t iters, hipStream_t s,
                     const ScriptArgs *script, DrawsBuf db, int num_cus) {
    ScriptArgs sa{};
    if (script) sa = *script;
    sa.pin = -1;
    sa.pre = nullptr;
    sa.pre_stride = 0;
    static const bool pre_env = [] {  // diagnostic: TD_PRE_DRAWS=0 keeps the in-kernel draws
        const char *e = std::getenv("TD_PRE_DRAWS");
        return !(e && e[0] == '0');
    }();
    const bool resident = sa.n > 0 || sa.mb != nullptr || sa.rb != nullptr;
    const size_t pre_bytes = sizeof(tdchain::Draws) * (size_t)nchains * (size_t)std::max<int64_t>(iters, 0);
    if (pre_env && db.p && !resident && iters > 0 && pre_bytes <= kDrawsBudget) {
        if (pre_bytes > *db.bytes) {
            if (*db.p) {
                hipError_t e = hipStreamSynchronize(s);
                if (e != hipSuccess) return e;
                (void)hipFree(*db.p);
                *db.p = nullptr;
                *db.bytes = 0;
            }
            hipError_t e = hipMalloc(db.p, pre_bytes);
            if (e != hipSuccess) return e;
            *db.bytes = pre_bytes;
        }
        hipLaunchKernelGGL(k_draws, dim3((unsigned)((iters + 255) / 256), (unsigned)nchains), dim3(256), 0, s, dev,
                           (long long)iters, static_cast<tdchain::Draws *>(*db.p));
        sa.pre = static_cast<const tdchain::Draws *>(*db.p);
        sa.pre_stride = iters;
    }
    static const int pin_env = [] {
        const char *e = std::getenv("TD_XCC_PIN");
        return e ? std::atoi(e) : -1;
    }();
    int grid = nchains;
    if (nchains == 1 && pin_env >= 0) {
        sa.pin = pin_env;
        grid = 8;
    }
    // one LDS size for the whole grid: the largest plan of any chain; the
    // small (LDS-mirrored) variant only if every chain fits
    size_t small = 0, big = 0, half = 0, hyb = 0;
    // packed: every chain asks for two chains per CU (lds_mode 2: the tiles in LDS when they fit; 3, testing:
    // the rays-in-HBM 4-wave kernel)
    bool force_hbm = false, packed = true, tiles_ok = true, all_auto = true;
    for (int b = 0; b < nchains; ++b) {
        const DevChain &d = host[b];
        small = std::max(small, lds_plan(d.ntiles, d.n, d.cap, true).total);
        big = std::max(big, lds_plan(d.ntiles, d.n, d.cap, false).total);
        half = std::max(half, lds_plan(d.ntiles, d.n, d.cap, false, kWaves / 2).total);
        hyb = std::max(hyb, lds_plan(d.ntiles, d.n, d.cap, true, kWaves / 2, false).total);
        force_hbm = force_hbm || d.lds_mode >= 1;
        packed = packed && d.lds_mode >= 2;
        tiles_ok = tiles_ok && d.lds_mode == 2;
        all_auto = all_auto && d.lds_mode == 0;
    }
    const bool scripted = sa.n > 0 || sa.mb != nullptr;
    // More chains than CUs: one chain per CU would run them in rounds of num_cus workgroups; two
    // 4-wave chains per CU run them all at once (1.35x the 8-wave kernel's rate at 512 config-3
    // chains) -- the tiles-in-LDS kernel when it fits, else the all-in-HBM one
    if (all_auto && num_cus > 0 && nchains > num_cus && !scripted && sa.rb == nullptr && sa.rx == nullptr &&
        (hyb <= kLdsBudget / 2 || half <= kLdsBudget / 2)) {
        packed = true;
        tiles_ok = hyb <= kLdsBudget / 2;
        force_hbm = true;
    }
    static bool attr_set = false;  // dynamic LDS above 64 KB needs the attribute (once per kernel)
    if (!attr_set) {
        for (const void *k : {(const void *)k_chain_run<true, false, kChainThreads>,
                              (const void *)k_chain_run<true, true, kChainThreads>,
                              (const void *)k_chain_run<false, false, kChainThreads>,
                              (const void *)k_chain_run<false, true, kChainThreads>,
                              (const void *)k_chain_run<false, false, kChainThreads / 2>,
                              (const void *)k_chain_run<true, false, kChainThreads / 2, false>,
                              (const void *)k_chain_run<true, false, kChainThreads, true, true>,
                              (const void *)k_chain_run<false, false, kChainThreads, false, true>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBudget);
            if (e != hipSuccess) return e;
        }
        attr_set = true;
    }
    if (sa.rx != nullptr) {  // exchange rounds: one 8-wave chain per CU
        if (small <= kLdsBudget && all_auto)
            hipLaunchKernelGGL((k_chain_run<true, false, kChainThreads, true, true>), dim3(grid), dim3(kChainThreads),
                               small, s, dev, (long long)iters, sa);
        else
            hipLaunchKernelGGL((k_chain_run<false, false, kChainThreads, false, true>), dim3(grid),
                               dim3(kChainThreads), big, s, dev, (long long)iters, sa);
    } else if (small <= kLdsBudget && !force_hbm) {
        if (scripted)
            hipLaunchKernelGGL((k_chain_run<true, true, kChainThreads>), dim3(grid), dim3(kChainThreads), small, s,
                               dev, (long long)iters, sa);
        else
            hipLaunchKernelGGL((k_chain_run<true, false, kChainThreads>), dim3(grid), dim3(kChainThreads), small, s,
                               dev, (long long)iters, sa);
    } else if (packed && !scripted && tiles_ok && hyb <= kLdsBudget / 2) {
        // two chains resident per CU (4 waves, <= 80 KB of LDS each): the tiles in LDS, the rays and the
        // order in HBM
        hipLaunchKernelGGL((k_chain_run<true, false, kChainThreads / 2, false>), dim3(grid), dim3(kChainThreads / 2),
                           hyb, s, dev, (long long)iters, sa);
    } else if (packed && !scripted && half <= kLdsBudget / 2) {
        // rays in HBM, 4 waves and <= 80 KB of LDS per chain: two chains resident per CU
        hipLaunchKernelGGL((k_chain_run<false, false, kChainThreads / 2>), dim3(grid), dim3(kChainThreads / 2), half,
                           s, dev, (long long)iters, sa);
    } else {
        if (scripted)
            hipLaunchKernelGGL((k_chain_run<false, true, kChainThreads>), dim3(grid), dim3(kChainThreads), big, s,
                               dev, (long long)iters, sa);
        else
            hipLaunchKernelGGL((k_chain_run<false, false, kChainThreads>), dim3(grid), dim3(kChainThreads), big, s,
                               dev, (long long)iters, sa);
    }
    return hipGetLastError();
}

}  // namespace tdstar
