/*
 * tdstar_testing.h -- host-only hooks of libtdstar.so that expose the chain's
 * RNG, deterministic math and proposal/acceptance logic (csrc/chain_logic.h)
 * so the CPU test suite can check them without a GPU.  They compute exactly
 * what the device kernel computes (same source, __host__ __device__).
 * Not part of the drop-in boundary; no reference interface is replaced.
 */
#ifndef TDSTAR_TESTING_H
#define TDSTAR_TESTING_H
#include <stdint.h>

#include "tdstar.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Philox4x32-10 block (Salmon et al. 2011; Random123 known-answer vectors). */
void tdt_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double tdt_det_log(double x);
double tdt_det_exp(double x);
/* Wichura AS241 standard-normal quantile. */
double tdt_normal_quantile(double p);
/* The 7 uniforms of one iteration: action, accept, a, b, c, zeta, index. */
void tdt_draws(uint64_t seed, uint32_t chain, uint64_t iter, double out[7]);
/* Proposal of iteration `iter` for the given model (TD_inversion_function.jl:72-236):
 * out = {action, active, valid, index, x, y, z, zeta}; czeta_birth is the
 * Interpolation value at the birth site (needed to draw zetanew). */
int tdt_propose(const td_chain_params *prm, uint64_t iter, int64_t ncells, const double *cx, const double *cy,
                const double *cz, const double *czeta, double czeta_birth, double out[8]);
/* Diagnostic: turn the DEVICE engine's per-phase s_memtime stamps on/off and
 * read the accumulated shader cycles: [0..6] phases A..G of k_chain_run
 * (draw, tiles + birth/death query, points, orphans, ray sums, chi^2 +
 * accept, commit), [8..11] whole proposals by action (birth, death, change,
 * move), [12..13] commit / next proposal, [14] proven early rejections, [15]
 * grid searches that fell back to a full scan, [16 + 10 (action-1) + j] the
 * phases split by action (j: A..F, commit, next proposal, final barrier),
 * [56 + w] phase F of wave w, [64] chi^2 tail terms, [65] chi^2 scan rounds.
 * Never enabled in measured runs. */
int tdt_chain_profile(td_chain *ch, int enable, int64_t out[80]);
/* LDS plan of a device chain: [0] bytes of the LDS layout (tiles, rays and
 * order mirrored), [1] bytes of the HBM layout, [2] 1 if the HBM layout holds
 * its super-tiles in LDS, [3] 1 if runs take the LDS layout. */
int tdt_chain_lds(td_chain *ch, int64_t out[4]);
/* Cycles of nq back-to-back nearest-cell queries through the chain's bucket grid by one wave
 * (pts: nq x {x, y, z}); mode 0: the whole query, 1: its loads only, 2: its arithmetic only.
 * out[0] = cycles, out[1] = unproven queries (full scans). */
int tdt_chain_query_lat(td_chain *ch, const double *pts, int nq, int mode, int64_t out[4]);
/* Each query's answer from the chain's grid search (mode 0: the LDS grid copy with the global first
 * bound; 6: the descriptor-reading form): squared distance, the winning cell's value, proven (1) or
 * left to the full scan (0). */
/* The chain's phase-B tile filter on caller boxes (FP32, SoA: x of every tile, then y, then z), FP64 tile
 * maxima and FP64 queries (x, y, z each): hit[q * nt + t] = 1 if tile t passes for query q.  mode 0: the
 * filter of the HBM layout's super-tiles; 1: the LDS layout's tile pass (tile_may_hit2). */
int tdt_tile_filter(const float *lo, const float *hi, const double *maxd, int nt, const double *queries, int nq,
                    int mode, uint8_t *hit);
int tdt_chain_query_answers(td_chain *ch, const double *pts, int nq, int mode, double *dist, double *value,
                            int32_t *proven);
/* Metropolis-Hastings decision, eqs. 14-17 (:96-97, :151-152, :196, :241). */
int tdt_accept(const td_chain_params *prm, int action, double u_accept, double zeta_new, int64_t ncells, double phi,
               double phi_n, double czeta, double zeta_killed, double zetanew_death);
/* The device chain's decision pre-filter on a bracket of (phi, phi_n) (chain_logic.h decide_sure):
 * 1 = accepted at every point of [phi_lo, phi_hi] x [phin_lo, phin_hi], -1 = rejected at every point,
 * 0 = undecided (the kernel then evaluates the corners with the acceptance rule itself). */
int tdt_decide_sure(const td_chain_params *prm, int action, double u_accept, double zeta_new, int64_t ncells,
                    double phi_lo, double phi_hi, double phin_lo, double phin_hi, double czeta, double zeta_killed,
                    double zetanew_death);
/* Device engine layout: 0 (default) mirrors tiles, rays and the Julia order
 * in LDS when they fit (the 381-ray configs); 1 keeps them in HBM, the path
 * larger geometries take; 2 runs the 4-wave kernel that puts two chains on a
 * CU (td_chain_run_batch of more chains than CUs): the tiles in LDS when they
 * fit in 80 KB, else everything in HBM; 3 (testing) that kernel with
 * everything in HBM.  Same results either way. */
int tdt_chain_set_lds_mode(td_chain *ch, int mode);
/* Device engine, decisions on bounds (DESIGN.md 4.2 phase F): k > 0 takes every
 * k-th decision of a launch on the exact chi^2 sums, as a decision falling
 * inside the brackets would (the committed partial sums made exact again from
 * where accepted proposals left them, with the proposal's terms in place);
 * 0 (default) only where the brackets require it.  Same results either way. */
int tdt_chain_set_exact_every(td_chain *ch, int k);
/* td_evaluate's resident server (incremental.cpp): sleep `ms` between the
 * host's alive check and the post of every command, so the kernel's 200 ms
 * idle watchdog can fire first (the race of a descheduled host thread).  The
 * command must then be re-issued to a new launch with the same results.  0 = off. */
int tdt_set_server_post_delay(int ms);
/* Resident tempering rounds (td_rounds_*): at the next launch the workgroups of
 * the listed chains return at their first wait, before the host posts the
 * round, while the others run it -- the race of a workgroup's idle watchdog
 * firing just as a round is posted.  td_rounds_run must then re-post the round
 * to a new launch in which the chains that ran it only report phi: every chain
 * runs each round once, with the results of an undisturbed launch.  One-shot;
 * ends the running launch. */
int tdt_rounds_force_exit(td_rounds *r, const int32_t *slots, int64_t nslots);
/* Testing: the drop-in path's one-point Interpolation on the host (host_nn.h: MCsub.jl:247-263 over a
 * bucket grid of the committed model).  Builds the grid from the n cells, applies edits[0..nedits) as
 * committed (6 doubles each: action 1 birth / 2 death / 3 change / 4 move, 0-based Julia index, x, y, z,
 * zeta), then answers nq points on that model plus `pending` (6 doubles, or NULL): val_out[k] and, if
 * pos_out, the winner's 0-based Julia position (-1: no cell below the 1e9 sentinel).  Host only. */
int tdt_host_nn_query(const double *x, const double *y, const double *z, const double *zeta, int64_t n,
                      const double *edits, int64_t nedits, const double *pending, const double *qx,
                      const double *qy, const double *qz, int64_t nq, double *val_out, int64_t *pos_out);

/* Diagnostic: the drop-in path's wall time per stage, ns, accumulated on the
 * context (then zeroed if reset): [0] td_evaluate, [1] its model
 * classification (which state the caller's cells are an edit of), [2] its
 * resident server's round trip (post -> answer), [3] td_interpolate of one
 * point, [4] its classification, [5] its server round trip, [6] td_evaluate
 * calls, [7] 1-point td_interpolate calls, [8] full evaluates, [9] a DROPIN
 * chain's modeln copies (the host loop's deepcopy), [10] its iterations'
 * time, [11] its iterations; the full evaluate's host side: [12] cells
 * packed into pinned memory, [13] kernels issued, [14] the wait for them,
 * [15] chi^2 and copy-out; [16] the resident server's busy time by its own
 * clock (command seen -> answered), evaluate commands, [17] queries. */
int tdt_dropin_timing(td_ctx *ctx, int reset, int64_t out[18]);
/* The block-wide exact sequential sum (exact_sum.h, used for chi^2 over long
 * ray lists): prefix[k] = C0 + term[0] + ... + term[k] added strictly left to
 * right in FP64 (MCsub.jl:170-172).  *fast = 1 when the parallel path proved
 * its result (else prefix/C_end are untouched and the kernels take the
 * one-lane loop).  Needs a GPU. */
int tdt_exact_sum(int device, const double *term, int64_t cnt, double C0, double *prefix, double *C_end, int *fast);
/* The one-wave exact sequential sum (exact_sum.h wave_seq_sum, the chain's
 * chi^2 tail): same contract as tdt_exact_sum, always exact; *fallbacks =
 * 256-term chunks that needed the slower binade-by-binade path.  Needs a GPU. */
/* The one-wave sum after a few terms changed (exact_sum.h wave_delta_sum, the
 * chain's chi^2): prefix[k] = C0 + term[0] + ... + term[k] left to right,
 * given old_prefix (the same sums over the old terms) and changed[k] != 0
 * where term[k] differs from the old term.  Needs a GPU. */
int tdt_wave_delta_sum(int device, const double *term, const double *old_prefix, const int *changed, int64_t cnt,
                       double C0, double *prefix, double *C_end);
/* The chain's chi^2 walk (exact_sum.h delta_marks / delta_walk / delta_remark /
 * delta_commit, one 512-thread workgroup): old_prefix[0..n) are the partial
 * sums of term_old (C_{-1} = 0), term[k0..n) the new terms, changed[k] != 0
 * where they differ; prefix = the new partial sums (old ones before k0), C_end
 * = prefix[n-1], events = the terms the walk added one by one, mask_ok = the
 * event words kept across the proposal equal those of the new state.
 * n <= 65536. */
int tdt_block_delta_sum(int device, const double *term, const double *term_old, const double *old_prefix,
                        const int *changed, int64_t k0, int64_t n, double *prefix, double *C_end, int64_t *events,
                        int *mask_ok);
int tdt_wave_seq_sum(int device, const double *term, int64_t cnt, double C0, double *prefix, double *C_end,
                     int *fallbacks);

/* chi^2 (MCsub.jl:169-172) of a caller-given ptS[n] against the context's tS
 * and allSig, through the code that computes it in the product: path 0
 * td_evaluate's (the host adds the terms in k order where the kernel put
 * ptS), 1 the block-wide exact scan of td_misfit (k_chi2), 2 the device
 * chain's starting-state prefix sums (k_chi2_prefix), 3 the chain's
 * proposal-time one-wave scan (from k0 = 0 -> out[0], and restarted at
 * k0 = n/2 on path 2's prefix -> out[1]).  Lets the tests pin the HIP code to
 * the reference's own model.jld phi values.  1 <= n <= 4096.  Needs a GPU. */
int tdt_chi2(td_ctx *ctx, const double *ptS, int path, double out[2]);

/* td_evaluate's incremental path: 0 off (every call a full evaluate), 1 one
 * k_chain_run launch per call, 2 (default) a resident launch fed through a
 * pinned-memory mailbox (it returns by itself after 200 ms without a call).
 * Changing the mode releases the shadow chain. */
int tdt_set_incremental(td_ctx *ctx, int on);

/* Diagnostic of the resident server (mode 2): out = {shader cycles, 100 MHz
 * wall ticks} of its last evaluation (command receipt to answer), the polls of
 * the mailbox before that command arrived, 0. */
int tdt_shadow_diag(td_ctx *ctx, int64_t out[4]);
/* Diagnostic: stop the resident server and read its chain's phase stamps (as
 * tdt_chain_profile; stamps are on only with TD_SHADOW_PROFILE set). */
int tdt_shadow_profile(td_ctx *ctx, int64_t out[80]);

/* Nearest-cell method of td_evaluate / td_interpolate: 0 auto (bucket grid
 * from 256 cells on), 1 brute force (every point x every cell: the one-launch
 * tile search where the points fit a lane each per CU, else the split search),
 * 2 bucket grid, 3 brute force through the split search (k_nn_partial +
 * k_nn_merge) always.  All give the same answer (the lexicographic
 * (distance, index) minimum). */
int tdt_set_nn_method(td_ctx *ctx, int method);

/* Diagnostic: the nearest-cell search alone, `reps` back-to-back launches over
 * the context's ray points on the given cells (method as tdt_set_nn_method,
 * 1..3), timed by two HIP events; *us_out = microseconds per search. */
int tdt_nn_bench(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta, int64_t ncells,
                 int method, int reps, double *us_out);

#ifdef __cplusplus
}
#endif
#endif
