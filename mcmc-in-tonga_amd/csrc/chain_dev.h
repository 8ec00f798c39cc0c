// chain_dev.h -- device state of one rj-MCMC chain (TD_ENGINE_DEVICE).
//
// Cells live in SLOTS (stable storage); order[pos] = slot keeps the Julia
// order (birth appends, death deleteat!-shifts), which decides nearest-cell
// ties.  Ties compare STAMPS: stamp[slot] = the order the cell entered the
// model (the starting cells 0..N-1, each birth the next number), which is
// Julia position order -- a birth appends after every live cell, a death
// keeps the others' order -- so a death rewrites no per-slot number.  Per ray point the chain caches the exact FP64
// (slot, squared distance, zeta) of its nearest cell -- exactly what a full
// v_nearest scan would give -- so a proposal only touches:
//   birth : points the new cell captures (d < cached d)
//   death : points whose cell is the killed one (re-searched)
//   change: points whose cell is the changed one (zeta only)
//   move  : points of the moved cell (re-searched) + points it captures
// Candidate points are found through 16-point ray tiles whose bounding boxes
// give an exact lower bound of the distance (monotone rounding: lb <= d
// bit-wise).  Re-searches and the birth/death Interpolation queries go
// through a uniform bucket grid over the cells, proven by a lower bound on
// everything outside the 3x3x3 block searched; otherwise (or on an exact
// distance tie, or a full bucket) they scan every slot.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "chain_logic.h"
#include "internal.h"
#include "../../include/tdstar.h"

namespace tdstar {

constexpr int kTilePts = 16;
constexpr int kProfSlots = 80;
constexpr int kChainThreads = 512;  // 8 waves: 256 VGPRs per lane, no spills
constexpr int kBucketCap = 32;
// A bucket entry of the chain's grid: the cell's site and value (its slot in a parallel array), so a
// query's one round of loads brings the value of whichever cell wins.
struct CellEntry {
    double x, y, z, zeta;
};

struct ChainScalars {
    int64_t iter;          // next iteration index
    int64_t evaluations;
    int64_t accepted[5];
    int64_t proposed[5];
    double phi;
    int64_t bytes;         // algorithmic global-memory bytes the proposals needed (roofline)
    int64_t prof[kProfSlots];  // diagnostic (DevChain::profile): cycles per phase [0..13], [14] proven
                               // rejections, [15] grid fallbacks, [16 + 10 (action-1) + j] per-action phases,
                               // [56 + wave] phase F per wave, [64] chi^2 tail terms, [65] chi^2 scan rounds,
                               // [66..67] wave-0 F timeline, [68..71] tiles hit, points seen/changed, rays changed,
                               // [72..75] chi^2 walk (rays in HBM): events, batch-load cycles, event-walk
                               // cycles, terms added one by one
    int ncells;            // cells in the model
    int nslots;            // slot high-water mark
    int nfree;             // free-slot stack depth
    int last_action;       // Model.action / Model.accept of the last iteration (TD_inversion_function.jl:73-74,
    int last_accept;       // 123,179,217,249): the proposal drawn and whether it was accepted
    int pad;
    int64_t next_stamp;    // the next birth's stamp (64-bit: never wraps)
};

// A proposal given by the host instead of drawn (td_evaluate's incremental
// path: the caller's new model is the chain's model with one edit, as the
// reference's proposals are -- TD_inversion_function.jl:85-88 append!, :132-135
// deleteat!, :189 zeta, :234-236 site).  decision: 1 = commit it (the caller
// went on from it), 0 = evaluate it, report phi and ptS, and undo it.
struct ScriptStep {
    int action;      // 1 birth, 2 death, 3 change, 4 move
    int index;       // Julia position (0-based) of the killed / changed / moved cell
    double x, y, z;  // birth site / move target
    double zeta;     // birth / change value
    // death / change / move: the cell at `index` before the step, (x, y, z, zeta) -- from the
    // host's copy of the model, bit-equal to the chain's: the proposal reads no cell array
    double old[4];
    int decision;
    int pad;
};
constexpr int kMaxScript = 2;

struct DevChain {
    // geometry (owned by the td_ctx)
    const double *px, *py, *pz, *w, *tS, *sig;
    const int *ray_off, *pt_ray;
    int P, n;
    // tiles of <= kTilePts consecutive points of one ray
    // tiles in a spatial (Morton) order; super-tile S = tiles [16 S, 16 S + 16)
    const int *tile_start;            // [ntiles] start << 5 | count of the tile's points
    const int *tile_ray;              // [ntiles] ray of each tile
    const float *tile_lo, *tile_hi;   // [3][ntiles] SoA, outward-rounded to FP32
    double *tile_maxd;                // [ntiles] max cached distance of the tile's points
    double *tile_cmax;                // [ntiles] scratch: hit tiles' maxima if accepted
    int ntiles;
    const float *super_lo, *super_hi;  // [3][nsuper] union of the member tiles' boxes
    int nsuper;
    // cells by slot
    double *cx, *cy, *cz, *czeta;  // [cap]
    const double *logN;            // [cap+2] det_log(k), the MH model-size factor
    int *order, *free_slots, *order_tmp;  // [cap]
    long long *stamp;                     // [cap]; -1 = a free slot
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
    double *term, *cand_term;                       // chi^2 term of each ray (MCsub.jl:171)
    int *rays_hit;
    int *ray_flag;
    ChainScalars *st;
    ChainScalars *st_host;  // pinned host mirror (device address), written at the end of a launch
    tdchain::Params params;
    uint64_t seed;
    uint32_t chain;
    int profile;  // diagnostic phase stamps (s_memtime) -- off in measured runs
    int lds_mode;  // 0: mirror tiles/rays/order in LDS when they fit; 1: always work from HBM (testing)
    int exact_every;  // testing: > 0 takes every k-th decision on the exact sums, as an undecided bracket would
    // uniform bucket grid over the cells
    CellGrid grid;
    int *bucket_count;      // [G]
    CellEntry *buckets;     // [G * kBucketCap] a cell's site and value, inline: a grid search reads no cell array
    int *bslot;             // [G * kBucketCap] the entry's slot
    int *grid_overflow;     // sticky: a bucket overflowed -> always scan all cells
};

// Scripted launches (n > 0: iteration k runs step[k] instead of a draw; no
// early rejection, the decision is the step's): a step with decision 0 writes
// [phi_n, ptS_n[0..n)] to out (pinned host memory, device address).  Passed
// by value as a kernel argument: no descriptor copy per call.
// Server mode (mb != nullptr): the launch stays resident and takes its steps
// from a mailbox in pinned host memory (td_evaluate's incremental path,
// incremental.cpp): no launch, no preamble per call.  A step with decision
// kDecideLater is evaluated, reported (out, done = seq) and its fate taken from
// the NEXT command; one-point Interpolation queries are answered while it
// waits.  The kernel returns on QUIT, or by itself after kServerIdleTicks of
// silence (the pending proposal undone) -- no host, no spinning CU.
constexpr int kDecideLater = 2;
enum ServerCmd : int { kCmdEval = 1, kCmdQuery = 2, kCmdQuit = 3 };
constexpr long long kServerIdleTicks = 20000000;  // 200 ms of the 100 MHz wall clock

struct Mailbox {
    // host -> device (seq written last)
    long long seq;
    int type;        // ServerCmd
    int decision;    // kCmdEval: the pending proposal's fate (1 commit, 0 undo)
    int nsteps;      // kCmdEval: steps (the last one kDecideLater)
    int has_edit;    // kCmdQuery: on the committed model plus qedit
    ScriptStep step[kMaxScript];
    double q[3];
    ScriptStep qedit;
    // mailbox_check(seq, words 1 .. check - 1): the kernel polls seq and payload in one read and takes
    // the command only when this matches (a poll may catch the words mid-write)
    unsigned long long check;
    // device -> host
    long long done;    // seq of the last command answered
    long long exited;  // the kernel has returned (its state is written back)
    double qval;
    long long diag[4];  // diagnostic: shader cycles and 100 MHz ticks of the last busy interval, polls
    // a death evaluated with its fate pending: Interpolation of that proposed model at the killed site
    // (TD_inversion_function.jl:146, the host's next call), stored after the answer; pq_seq = its command
    double pq_val;
    long long pq_seq;
};

// The command's words (seq first, check last) and their check: each payload word mixed with its
// position and the seq, xor-combined (the kernel: one word per lane, one DPP reduction).
constexpr int kMailboxCheckWord = (int)(offsetof(Mailbox, check) / sizeof(long long));
__host__ __device__ inline unsigned long long mailbox_word_mix(unsigned long long w, int i, long long seq) {
    return tdchain::swap_mix64(w ^ ((unsigned long long)i * 0x9E3779B97F4A7C15ull) ^
                               ((unsigned long long)seq * 0xD1B54A32D192ED03ull));
}
inline unsigned long long mailbox_check(const Mailbox *m, long long seq) {
    const unsigned long long *w = reinterpret_cast<const unsigned long long *>(m);
    unsigned long long h = 0;
    for (int i = 1; i < kMailboxCheckWord; ++i) h ^= mailbox_word_mix(w[i], i, seq);
    return h;
}

// Resident tempering rounds (td_rounds_*, chain.cpp): a td_chain_run_batch
// launch that stays resident across swap rounds.  Every K proposals each
// workgroup publishes its chain's phi and waits for the next round's
// temperature (parallel tempering, SURVEY 8e: the host gathers the phis,
// decides the swaps and posts the new temperatures) -- no launch per round.
// Pinned host memory; one 64-B slot per chain.
enum RoundCmd : int { kRoundRun = 1, kRoundQuit = 3 };
struct RoundSlot {
    double T, inv_2t;  // host -> device: the chain's temperature for the round (inv_2t = 1/(2T), host-computed)
    long long done;    // device -> host: seq of the last round finished
    double phi;        // the chain's phi after that round
    long long exited;  // the workgroup returned (QUIT, or its idle watchdog at a round boundary)
    // host -> device: 1 = this chain already ran the posted round in a launch that was lost
    // (some other workgroup's watchdog fired as the round was posted): report phi again, run nothing
    long long skip;
    long long idle;  // testing (tdt_rounds_force_exit): > 0 = the idle watchdog of the launch's first wait, ticks
    long long pad;
};
struct RoundBox {
    long long seq;  // host -> device (written last)
    int cmd;        // RoundCmd
    int K;          // proposals in the round
    long long pad[6];
    RoundSlot slot[1];  // [nchains]
};

// Exchange rounds (td_rounds_exchange, chain.cpp): the resident launch runs M
// tempering rounds with no host in the loop.  At the end of round j every
// workgroup puts its chain's exact phi into xin and raises its flag in rdy;
// the phis of all R replicas then arrive in xout -- from an RCCL allgather
// that a second stream issues once workgroup 0 has seen every local flag and
// raised `ready` (the stream waits on it: hipStreamWaitValue64), followed by a
// stream write of `gdone`; or, on one rank, from xin itself once every
// replica's flag is up -- no atomics, only stores and loads -- and
// every workgroup makes the same swap decisions (chain_logic.h swap_accept)
// and takes its chain's new temperature.  Device memory except the logs.
struct RoundX {
    double *xin;                        // [2][local] this rank's phis of round j in row j & 1
    const double *xout;                 // [2][R] every replica's phi, row j & 1 (== xin on one rank)
    unsigned long long *rdy;            // [local] base + j + 1 once workgroup b's phi of round j is in xin
    unsigned long long *ready;          // base + j + 1 once all of this rank's are (workgroup 0; signal memory)
    const unsigned long long *gdone;    // base + j + 1 after round j's allgather (null on one rank)
    unsigned long long ready_base, gdone_base;
    int *lev;                           // [local][R] each workgroup's copy of every replica's level
    const double *temps;                // [R] the ladder
    double *log_phi;                    // [M][R] the gathered phis of every round (pinned; workgroup 0)
    int *log_lev;                       // [M][R] the levels after every round's swaps
    long long *log_t;                   // [M][3] workgroup 0's wall clock (100 MHz): its phi published, this
                                        // rank's phis all in, every phi gathered
    long long *err;                     // pinned: 1 = an exchange never came (watchdog)
    long long rnd0;                     // the ladder's round number of round 0 (its swap parity and draws)
    unsigned long long seed;
    int R, local, rank, M, K;           // R = 0: not an exchange launch
};
constexpr long long kExchangeTicks = 1000000000;  // 10 s of the 100 MHz wall clock without an exchange: give up

struct ScriptArgs {
    const RoundX *rx;  // exchange rounds (device memory), free-running chains
    int n;
    int pin;  // >= 0: the chain runs on the workgroup that lands on this XCD (L2 kept warm across launches)
    ScriptStep step[kMaxScript];
    double *out;
    Mailbox *mb;   // server mode (device address of pinned host memory)
    RoundBox *rb;  // resident tempering rounds (device address of pinned host memory), free-running chains
    // a free-running launch of known length: every iteration's draws precomputed by k_draws
    // (chain b's iteration iter0 + i at pre[b * pre_stride + i]); null: drawn in the kernel
    const tdchain::Draws *pre;
    long long pre_stride;
};

// Device scratch a launch may grow (owned by the context): the precomputed draws.
struct DrawsBuf {
    void **p;
    size_t *bytes;
};

// Build the cache from scratch for the cells currently in slots 0..ncells-1
// (order = rank = identity): nearest search, ray sums, chi^2 prefix, tile maxima.
hipError_t chain_full_state(DevChain &d, int ncells, NNWork &work, int num_cus, hipStream_t s);
// Run `iters` iterations of `nchains` chains, one persistent workgroup each
// (workgroup b runs chain b).  `host` = the descriptors, `dev` = their device
// copy, contiguous (the kernel reads its fields from global memory).
hipError_t chain_run(const DevChain *host, const DevChain *dev, int nchains, int64_t iters, hipStream_t s,
                     const ScriptArgs *script = nullptr, DrawsBuf db = DrawsBuf{nullptr, nullptr},
                     int num_cus = 0);  // > 0: a batch of more chains than CUs packs two per CU
// Testing: the chain's chi^2 code on a caller-given ptS (n <= 4096) --
// path 2: k_chi2_prefix (the starting state's sequential prefix sums, what
// chain_full_state runs), 3: the proposal-time sum (the terms of MCsub.jl:171,
// then the one-wave exact scan of phase F from k0 = 0, and again from
// k0 = n/2 on top of path 2's prefix[k0-1]).  out[0] = phi, out[1] = phi of
// the restart from n/2 (path 3 only).  scratch: 3n + 16 doubles.
hipError_t test_chain_chi2(const double *ptS, const double *tS, const double *sig, int n, int path, double *scratch,
                           double *out, hipStream_t s);
// td_evaluate's incremental path (incremental.cpp): a device chain that never
// draws -- it takes the caller's edits as scripted steps (ScriptStep).
int shadow_chain_create(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                        int64_t ncells, int64_t cap, const double box[6], td_chain **out);
// base_ptS: ptS of the model the last step edits (the report carries the changed rays only);
// *k0_out: the first ray whose t* changed (n: none) -- the caller forms phi_n (incremental.cpp)
int shadow_chain_script(td_chain *ch, const ScriptStep *steps, int nsteps, const double *base_ptS, int64_t *k0_out,
                        double *ptS_out);
int64_t shadow_chain_slots(const td_chain *ch);
int64_t shadow_chain_ncells(const td_chain *ch);
double shadow_chain_phi(const td_chain *ch);
void shadow_chain_destroy(td_chain *ch);
// server mode (a resident launch fed by a mailbox): decision = the pending proposal's fate
bool shadow_server_alive(td_chain *ch);
// the same split: post the command (no wait; one open at a time), then take its answer
int shadow_server_post(td_chain *ch, int decision, const ScriptStep *steps, int nsteps);
int shadow_server_answer(td_chain *ch, const double *base_ptS, int64_t *k0_out, double *ptS_out);
int shadow_server_eval(td_chain *ch, int decision, const ScriptStep *steps, int nsteps, const double *base_ptS,
                       int64_t *k0_out, double *ptS_out);
int shadow_server_query(td_chain *ch, double x, double y, double z, const ScriptStep *edit, double *val);
int shadow_server_query_post(td_chain *ch, double x, double y, double z, const ScriptStep *edit);
int shadow_server_death_query(td_chain *ch, double x, double y, double z, double *val);
int shadow_server_query_answer(td_chain *ch, double *val);
int shadow_server_stop(td_chain *ch);
// Stop every resident server this thread runs except `keep` (nullable): called
// before work on any other stream (chain.cpp t_servers).
void servers_quiesce(const td_chain *keep);
void shadow_server_diag(const td_chain *ch, int64_t out[4]);
int shadow_profile(td_chain *ch, int64_t out[80]);
// One-point Interpolation against the chain's model (edit == NULL) or that
// model plus one edit; *out (device-visible) receives the value.
hipError_t chain_query(const DevChain *dev, double x, double y, double z, const ScriptStep *edit, double *out,
                       hipStream_t s);
int shadow_chain_query(td_chain *ch, double x, double y, double z, const ScriptStep *edit, double *val);
// Testing: cycles of nq back-to-back grid queries by one wave (k_test_query_lat; mode 0 whole, 1 loads, 2 math)
hipError_t test_query_lat(const DevChain *dev, const double *pts, int nq, int mode, long long *out, hipStream_t s);
// Testing: each query's (squared distance, value, proven) from the chain's grid search (k_test_query_answers)
hipError_t test_tile_filter(const float *lo, const float *hi, const double *maxd, int nt, const double *qs, int nq,
                            int mode, unsigned char *out, hipStream_t s);
hipError_t test_query_answers(const DevChain *dev, const double *pts, int nq, int mode, double *out_d, double *out_z,
                              int *out_p, hipStream_t s);
// LDS bytes of the two layouts, whether super-tiles fit, and the layout chain_run takes.
void chain_lds_sizes(const DevChain &d, int64_t out[4]);

}  // namespace tdstar
