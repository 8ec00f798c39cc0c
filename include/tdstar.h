/*
 * tdstar.h -- C ABI of the MI355X-native t* forward model (libtdstar.so).
 *
 * Drop-in boundary for the per-proposal hot path of the rj-MCMC Voronoi t*
 * tomography in Geronimorz/MCMC-in-Tonga (Julia).  Each entry point names the
 * reference interface it replaces (file:line in the reference tree).  The
 * signatures use plain pointers and sizes only, so a Julia `ccall`, a Python
 * `ctypes` binding or a C/C++ host can call them unchanged.
 *
 * Conventions
 *  - All arrays are FP64 unless noted; ray arrays keep the reference's
 *    DataStruct layout: rayX/rayY/rayZ are m x n COLUMN-MAJOR (ray i = column
 *    i), tail-padded with NaN; rayL/rayU are (m-1) x n (DefStruct.jl:24-28).
 *  - Cell indices crossing the ABI are 0-based (Julia adds 1); -1 = "no cell
 *    closer than the 1e9 sentinel" (MCsub.jl:249-250: v_nearest returns 0.0).
 *  - Every call returns a td_status; on error the message is available from
 *    td_last_error(ctx) (td_last_error(NULL) for td_create failures, per
 *    thread).  No C++ exception crosses the ABI.
 *  - A context is bound to one device, owns one HIP stream, is NOT thread-
 *    safe (one context per Julia worker process, main_inversion.jl:15), and
 *    every call is synchronous: outputs are valid on return.
 *  - Host buffers are owned by the caller and only read/written during the
 *    call.  Ray geometry is copied to device memory once, at td_create.
 */
#ifndef TDSTAR_H
#define TDSTAR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: td_info gained num_cus (its size changed) */
#define TDSTAR_ABI_VERSION 2

typedef struct td_ctx td_ctx;
typedef struct td_chain td_chain;

typedef enum td_status {
    TD_OK = 0,
    TD_ERR_ARG = 1,    /* bad pointer / size / option */
    TD_ERR_LAYOUT = 2, /* NaN padding of rayX and rayL disagree (Julia: DimensionMismatch) */
    TD_ERR_HIP = 3,    /* HIP runtime error (message names the call) */
    TD_ERR_NOMEM = 4,
    TD_ERR_BOUNDS = 5  /* Y/Z shorter than npoints (Julia: BoundsError) */
} td_status;

/* ------------------------------------------------------------------------
 * Context: device-resident copy of DataStruct's hot fields.
 * Replaces the device half of load_data_Tonga.jl:59-81 (rayX/Y/Z, rayL/U,
 * tS, allSig).  Validates the NaN layout: for every ray, the number of
 * leading non-NaN entries of rayL must equal max(npoints-1, 0) where npoints
 * is the number of leading non-NaN entries of rayX (MCsub.jl:150,312-316).
 * n may be 0.  device < 0 selects the current HIP device.
 * ------------------------------------------------------------------------ */
int td_create(td_ctx **out, int device, const double *rayX, const double *rayY, const double *rayZ,
              const double *rayL, const double *rayU, int64_t m, int64_t n, const double *tS,
              const double *allSig);
int td_destroy(td_ctx *ctx);
const char *td_last_error(const td_ctx *ctx);

typedef struct td_info {
    int32_t abi_version;
    int32_t device;
    int64_t m, n;         /* DataStruct.rayX size */
    int64_t npoints;      /* P: valid ray points over all rays */
    int64_t nsegments;    /* S = P - (rays with >= 1 point) */
    double likelihood;    /* the MCsub.jl:179 constant for the current allSig */
    char arch[32];        /* e.g. "gfx950" */
    int32_t num_cus;      /* compute units: td_chain_run_batch packs two chains per CU beyond this many */
} td_info;
int td_get_info(const td_ctx *ctx, td_info *info);

/* Per-kernel device timing with HIP events recorded on the context's stream
 * around every launch (off by default; used by bench.py for the roofline).
 * Kernel names: "nn_partial", "nn_merge", "ray_sums", "chi2", "chain_run".
 * td_timing_get waits for the recorded events and returns the launch count
 * and summed duration since the last reset. */
int td_timing_enable(td_ctx *ctx, int enable);
int td_timing_reset(td_ctx *ctx);
int td_timing_get(td_ctx *ctx, const char *kernel, int64_t *launches, double *total_ms);

/* Replaces DataStruct.allSig (DefStruct.jl:10) for action 5
 * (TD_inversion_function.jl:252-261); n values. */
int td_set_sigma(td_ctx *ctx, const double *allSig);

/* td_evaluate's incremental path (below): 2 (default) = a resident kernel
 * answers every call through a mailbox in pinned host memory; 1 = one launch
 * per call; 0 = every call a full evaluate.  A resident kernel occupies its
 * stream's hardware queue, so one kept alive while the caller runs other GPU
 * work (another context, a collective on another stream) can hold that work
 * back until its 200 ms idle watchdog.  The library stops this thread's
 * resident kernels before any call that launches other work; a caller that
 * interleaves its OWN GPU work with td_evaluate calls (e.g. an allgather
 * between evaluates: a ray-sharded run) should select mode 1. */
int td_set_incremental(td_ctx *ctx, int mode);

/* ------------------------------------------------------------------------
 * evaluate -- replaces MCsub.jl:123-185 `evaluate(model, dataStruct,
 * TD_parameters)` (interp_style 1, MCsub.jl:326-327).
 *   cells: Model.xCell/yCell/zCell/zeta (DefStruct.jl:34-37), nCells long,
 *          in Julia order (tie-breaks follow it).
 *   debug_prior == 1: phi = likelihood = 1, nothing else written
 *          (MCsub.jl:134-136).
 *   ptS_out[n]   -> Model.ptS (MCsub.jl:174)         (nullable)
 *   phi_out      -> Model.phi (MCsub.jl:169-173)     (nullable)
 *   likelihood_out -> Model.likelihood (MCsub.jl:179-182) (nullable)
 *   nearest_out[P] -> 0-based cell chosen for every valid ray point, ray-major
 *          (what v_nearest computes but never returns)  (nullable)
 * phi is the sequential chi^2 of MCsub.jl:170-172 and ptS uses Julia's sum
 * association (oracle/README.md), so both are bit-exact to the CPU oracle.
 * Incremental path: when the cells are the previous call's model (or the model
 * before it) plus ONE reference-shaped edit -- an appended cell (birth,
 * TD_inversion_function.jl:85-88), a deleted one (death, :132-135), one new
 * zeta (change, :189) or one new site (move, :234-236) -- and nearest_out is
 * NULL, the context evaluates only what the edit changes on a device-resident
 * copy of the chain state (the DEVICE engine's algorithm); the results are
 * bit-identical to the full evaluate.  Other calls evaluate in full.
 * ------------------------------------------------------------------------ */
int td_evaluate(td_ctx *ctx, const double *xCell, const double *yCell, const double *zCell,
                const double *zeta, int64_t nCells, int debug_prior, double *ptS_out, double *phi_out,
                double *likelihood_out, int32_t *nearest_out);

/* The chi^2 and likelihood of MCsub.jl:169-182 for a caller-given ptS of n
 * rays (tS, allSig: the n data and errors): phi = the sequential
 * sum_k ((ptS-tS)[k]^2 * 1.0) / allSig[k]^2, computed on the device exactly as
 * td_evaluate's (bit for bit), and likelihood = the a5 constant in Julia's
 * sum association.  The reduction step of a ray-sharded evaluate: every rank
 * td_evaluate's a context over its own ray subset, the ptS are gathered in
 * ray order (one allgather), and phi is this call on the whole vector
 * (mcmc-in-tonga_amd/sharded.py).  tS / allSig are re-uploaded only when
 * they change between calls. */
int td_misfit(td_ctx *ctx, int64_t n, const double *ptS, const double *tS, const double *allSig, double *phi_out,
              double *likelihood_out);

/* Several models at once (independent chains / tempering replicas on one
 * GPU): model k's cells are [cell_off[k], cell_off[k+1]) of the cell arrays.
 * ptS_out is nmodels x n (row k = model k), phi_out/likelihood_out nmodels. */
int td_evaluate_batch(td_ctx *ctx, int64_t nmodels, const int64_t *cell_off, const double *xCell,
                      const double *yCell, const double *zCell, const double *zeta, double *ptS_out,
                      double *phi_out, double *likelihood_out);

/* ------------------------------------------------------------------------
 * Interpolation -- replaces MCsub.jl:306-336 (interp_style 1), as called for
 * the birth/death 1-point queries (TD_inversion_function.jl:81,146) and on
 * grids (MCsub.jl:766-768,800-802).  npoints = leading non-NaN entries of X
 * (MCsub.jl:312-316); ny == 1 / nz == 1 broadcast (MCsub.jl:317-322);
 * otherwise ny, nz must be >= npoints (TD_ERR_BOUNDS).  Writes npoints
 * values to zeta_out (capacity nx) and, if non-NULL, nearest cells to
 * nearest_out and npoints to *npoints_out.
 * ------------------------------------------------------------------------ */
int td_interpolate(td_ctx *ctx, const double *xCell, const double *yCell, const double *zCell,
                   const double *zeta, int64_t nCells, const double *X, int64_t nx, const double *Y,
                   int64_t ny, const double *Z, int64_t nz, double *zeta_out, int32_t *nearest_out,
                   int64_t *npoints_out);

/* Slowness of ray points from a gridded 3-D model: pre_process_data.jl:34
 * `itp.(ix, iy, iz)` with load_3Dvel.jl:32 `interpolate((x, y, z), sn,
 * Gridded(Linear()))`.  Knots strictly increasing (>= 2 per
 * axis); values column-major nx x ny x nz (x fastest, Julia's sn[1,:,:,:]).
 * A point outside the grid (Interpolations.jl: BoundsError) gets NaN and is
 * counted in *n_outside.  Context-free (no ray geometry needed): runs on
 * `device`, synchronous.  td_last_error(NULL) on failure. */
int td_trilinear(int device, const double *xs, int64_t nx, const double *ys, int64_t ny, const double *zs,
                 int64_t nz, const double *values, const double *px, const double *py, const double *pz,
                 int64_t npts, double *out, int64_t *n_outside);

/* ------------------------------------------------------------------------
 * Posterior maps -- the numbers of plot_model_hist (MCsub.jl:753-825), not the
 * plots.  For nq query points (a cross-section: MCsub.jl:765-768 xz at y =
 * ySlice, :799-802 xy at z = zSlice) and nmodels saved models (model k's cells
 * are [cell_off[k], cell_off[k+1]) of the cell arrays, in model_hist order,
 * chain by chain, MCsub.jl:761-763):
 *   values_out[k*nq + q] = v_nearest of model k at point q   (nullable)
 *   mean_out[q] = Statistics.mean over the models            (MCsub.jl:774)
 *   std_out[q]  = Statistics.std (corrected) over the models (MCsub.jl:775)
 * with Julia's sum association for a Vector of matrices (raster.hip).
 * ------------------------------------------------------------------------ */
int td_rasterize(td_ctx *ctx, int64_t nmodels, const int64_t *cell_off, const double *xCell,
                 const double *yCell, const double *zCell, const double *zeta, const double *qx,
                 const double *qy, const double *qz, int64_t nq, double *mean_out, double *std_out,
                 double *values_out);

/* ------------------------------------------------------------------------
 * rj-MCMC chain -- replaces TD_inversion_function.jl:7-305 (one chain) for
 * the three priors of define_TDstructure.jl:15 (1 uniform, the default; 2
 * normal; 3 exponential: TD_inversion_function.jl:91-119, 150-172, 194-212,
 * MCsub.jl:97-108).  The chain
 * state (cells, per-point nearest-cell cache, ptS, phi) lives in device
 * memory; proposals are evaluated incrementally (birth: one new cell vs the
 * cache; death/move: re-search only the points whose cell changed; change:
 * no search) and are bit-identical to a full evaluate of the proposed model.
 * RNG: counter-based Philox4x32-10 keyed by (seed, chain), so runs are
 * reproducible (the reference seeds from the wall clock, :13).
 * ------------------------------------------------------------------------ */
typedef struct td_chain_params {
    /* define_TDstructure.jl:1-44 fields that reach the chain */
    int32_t debug_prior;   /* 1: sample the prior (evaluate returns phi = 1) */
    int32_t sig;           /* percent (10) */
    int32_t zeta_scale;    /* 50 */
    int32_t max_cells;     /* 100 */
    int32_t min_cells;     /* 5 */
    int32_t prior;         /* 1 uniform, 2 normal, 3 exponential (TD_ERR_ARG otherwise) */
    double n_iter, burn_in, keep_each;
    /* xVec/yVec/zVec extents (DataStruct.xVec etc., min(xVec...), max(xVec...)) */
    double xmin, xmax, ymin, ymax, zmin, zmax;
    uint64_t seed;
    int32_t chain;          /* chain id (TD_inversion_function.jl:10) */
    double temperature;     /* tempering: acceptance uses phi / temperature (1 = reference) */
    int32_t engine;         /* TD_ENGINE_DEVICE (default) or TD_ENGINE_HOST */
    int64_t start_iter;     /* first iteration index (resume from a checkpoint); <= 0 means 1 */
} td_chain_params;

/* Engines: DEVICE runs the whole loop (proposal, incremental forward model,
 * accept/reject) inside one persistent GPU workgroup per td_chain_run call;
 * HOST is the reference's structure -- every proposal is a full td_evaluate
 * of the proposed model (TD_inversion_function.jl:93,141,191,238) -- kept as
 * the parity reference for the DEVICE engine. */
#define TD_ENGINE_DEVICE 0
#define TD_ENGINE_HOST 1
/* DROPIN: the host loop of HOST, calling the PUBLIC td_evaluate /
 * td_interpolate exactly as the unchanged Julia host would (td_evaluate's
 * incremental path then follows the chain on the device).  Measures the
 * drop-in boundary; same trajectory as the other two. */
#define TD_ENGINE_DROPIN 2

typedef struct td_chain_stats {
    int64_t iterations;        /* proposals drawn so far */
    int64_t evaluations;       /* forward-model evaluations performed */
    int64_t accepted[5];       /* per action 1..4 (index 0 unused) */
    int64_t proposed[5];
    double phi;                /* current model */
    int64_t ncells;
    int64_t bytes;             /* DEVICE engine: algorithmic global-memory bytes read by the proposals */
    int32_t last_action;       /* Model.action of the last iteration: the drawn action 1..4 (:72-73), 0 before any */
    int32_t last_accept;       /* Model.accept of the last iteration: 1 if its proposal was accepted (:74,123,...) */
} td_chain_stats;

/* Start a chain from the given model (cells may be NULL/0 to draw a starting
 * model as build_starting, MCsub.jl:76-121). */
int td_chain_create(td_chain **out, td_ctx *ctx, const td_chain_params *params, const double *xCell,
                    const double *yCell, const double *zCell, const double *zeta, int64_t nCells);
int td_chain_destroy(td_chain *ch);
/* Run `iterations` proposals (TD_inversion_function.jl:70-274 loop body). */
int td_chain_run(td_chain *ch, int64_t iterations);
/* Run `iterations` proposals on each of `nchains` chains of ONE context in a
 * single launch, one workgroup per chain (independent chains / tempering
 * replicas sharing a GPU: main_inversion.jl:15 pmap over chains).  Device
 * engine: one kernel; host engine: the chains run one after the other.  Each
 * chain's result is identical to td_chain_run(chain, iterations). */
int td_chain_run_batch(td_chain *const *chains, int64_t nchains, int64_t iterations);
int td_chain_stats_get(const td_chain *ch, td_chain_stats *st);
/* Copy the current model out (cells arrays capacity `cap`; *nCells receives
 * the count; ptS_out[n] nullable). */
int td_chain_get_model(const td_chain *ch, double *xCell, double *yCell, double *zCell, double *zeta,
                       int64_t cap, int64_t *nCells, double *phi, double *ptS_out);
/* Tempering: change the temperature between runs (swap step). */
int td_chain_set_temperature(td_chain *ch, double temperature);

/* ------------------------------------------------------------------------
 * Resident tempering rounds (parallel tempering; the reference's
 * chains are independent pmap workers, main_inversion.jl:15, so this is a new
 * capability): DEVICE chains of one context run in ONE launch that stays
 * resident across swap rounds.  td_rounds_run posts a round -- K proposals on
 * every chain at the given temperatures -- and returns each chain's phi after
 * it; the caller gathers the phis (across ranks: an allgather), decides the
 * swaps and passes the new temperatures to the next td_rounds_run.  No
 * launch per round; the launch returns by itself after 200 ms without a
 * round (and is started again by the next one, with identical results).
 * Every chain's trajectory equals td_chain_run of K proposals per round with
 * td_chain_set_temperature between rounds.  Any other call on these chains
 * (or any GPU work of this thread through this library) first ends the
 * launch; td_chain_stats_get's accepted/proposed counts are current after
 * that, phi and iterations after every round. */
typedef struct td_rounds td_rounds;
int td_rounds_create(td_rounds **out, td_chain *const *chains, int64_t nchains);
int td_rounds_run(td_rounds *r, int64_t K, const double *temps, double *phi_out);
int td_rounds_destroy(td_rounds *r);

/* The swap step of parallel tempering (replaces mcmc-in-tonga_amd/tempering.py
 * decide_swaps, the same decision bit for bit): R replicas, phis[g] and
 * levels[g] of replica g (gathered over all ranks), temps[l] the ladder.  In
 * round rnd the level pairs (l, l+1), l = rnd mod 2, 2 + rnd mod 2, ... are
 * tried with u = a SplitMix64 hash of (seed, rnd, l) and accepted when
 * log alpha = (phi_a - phi_b)(1/(2T_l) - 1/(2T_l+1)) >= 0 or log u < log alpha
 * (a at level l, b at l+1).  new_levels[R]; tried/accepted[R-1] are added to
 * (per level pair).  Host-only (no GPU). */
int td_swap_decide(int64_t R, const double *phis, const int64_t *levels, const double *temps, int64_t rnd,
                   uint64_t seed, int64_t *new_levels, int64_t *tried, int64_t *accepted);
/* M rounds of a resident tempering launch whose replicas are all its chains
 * (one process, one GPU: the gather is the identity), the swaps decided
 * between rounds by td_swap_decide -- no return to the caller per round.
 * Round j: K proposals on every chain at temps[levels[k]] (chain k = replica
 * k), then the swap step of round rnd0 + j.  levels[nchains] in/out;
 * phis_out[M x nchains] the phis of each round, levels_out[M x nchains] the
 * levels after it (both nullable); tried/accepted[nchains - 1] added to. */
int td_rounds_temper(td_rounds *r, int64_t M, int64_t K, const double *temps, int64_t *levels, int64_t rnd0,
                     uint64_t seed, double *phis_out, int64_t *levels_out, int64_t *tried, int64_t *accepted);

/* ------------------------------------------------------------------------
 * The exchange across GPUs (one replica per GPU, an RCCL allgather
 * over xGMI for the swap step).  A td_comm is an RCCL communicator of the
 * job's ranks: rank 0 makes the id (td_comm_unique_id) and the caller ships
 * it to every rank (e.g. torch.distributed); td_comm_create blocks until all
 * ranks joined.  td_comm_allgather: count doubles from every rank, host
 * buffers (out[nranks * count], rank order). */
#define TD_COMM_ID_BYTES 128
typedef struct td_comm td_comm;
int td_comm_unique_id(uint8_t *id /* TD_COMM_ID_BYTES */);
int td_comm_create(td_comm **out, int device, int nranks, int rank, const uint8_t *id);
int td_comm_allgather(td_comm *c, const double *in, int64_t count, double *out);
int td_comm_destroy(td_comm *c);
/* M rounds of parallel tempering with no host in the loop: the chains of r
 * (this rank's replicas, replica g = rank * nchains + k; every rank holds as
 * many) run in ONE launch; after every K proposals each publishes its exact
 * phi to device memory, an allgather on the communicator's stream (issued
 * ahead, each waiting on a flag the kernel raises: hipStreamWaitValue64)
 * brings every replica's phi, and every workgroup decides the round's swaps
 * itself (td_swap_decide's rule) and takes its chain's new temperature.
 * comm NULL: one rank holds every replica (the phis meet in device memory, no
 * collective).  Same trace as td_rounds_temper over the same replicas: the
 * host replays every decision on the logged phis and fails (TD_ERR_HIP) if
 * the device's differ.  levels[R] in/out, phis_out / levels_out [M x R],
 * tried / accepted [R-1] added to (all nullable but levels); R <= 64.
 * timing_out[7] (nullable, s): the call, launch issued, exchanges enqueued;
 * per round (means, workgroup 0's wall clock): the exchange (this rank's phis
 * all in -> every phi gathered), the proposals (gathered -> its next phi),
 * the wait for the rank's slowest replica (its phi -> the rank's last); the
 * kernel's span from its first publish to its last gather. */
int td_rounds_exchange(td_rounds *r, td_comm *comm, int64_t M, int64_t K, const double *temps, int64_t *levels,
                       int64_t rnd0, uint64_t seed, double *phis_out, int64_t *levels_out, int64_t *tried,
                       int64_t *accepted, double *timing_out);

#ifdef __cplusplus
}
#endif
#endif /* TDSTAR_H */
