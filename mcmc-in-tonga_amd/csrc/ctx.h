// ctx.h -- the td_ctx object behind the C ABI (include/tdstar.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/tdstar.h"
#include "internal.h"

namespace tdstar {
struct td_shadow;
}

struct td_ctx {
    int device = 0;
    int num_cus = 0;
    std::string arch;
    hipStream_t stream = nullptr;
    tdstar::Geometry g;                 // device-resident ray geometry
    std::vector<int> ray_off_host;      // CSR offsets (host copy)
    std::vector<double> hx, hy, hz;     // CSR points (host copy; chain tiles are built from it)
    std::vector<double> sig_host, tS_host;  // allSig, tS (host copies: td_evaluate's chi^2 is added on the host)
    double likelihood = 0.0;            // MCsub.jl:179 constant for sig_host

    // one cell set (SoA x|y|z|zeta, stride cell_stride <= cell_cap), device + pinned host staging
    double *cells = nullptr;
    int64_t cell_stride = 1;            // SoA stride of the uploaded cells (= their count)
    double *h_cells = nullptr;
    double *h_cells_dev = nullptr;      // the same pinned buffer, as the device addresses it
    const double *cells_stage = nullptr;  // non-null: the device copy is still to be made (from here)
    int64_t cell_cap = 0;

    // per-evaluation outputs / caches
    tdstar::NNWork nn;
    int *best_i = nullptr;
    double *best_d = nullptr;
    double *zeta0 = nullptr;
    double *ptS = nullptr;
    double *phi = nullptr;
    double *h_out = nullptr;            // pinned: [phi, ptS[n]], written by the evaluate kernel
    double *h_out_dev = nullptr;        // the same, as the device addresses it
    int *h_best_i = nullptr;            // pinned [P]

    // query points for td_interpolate
    double *q = nullptr, *h_q = nullptr;
    int64_t q_cap = 0;
    int *q_i = nullptr;
    double *q_z = nullptr;
    int *h_q_i = nullptr;
    double *h_q_z = nullptr;

    tdstar::Timer timer;                // per-kernel HIP-event timing (td_timing_*)
    double *raster = nullptr;           // td_rasterize workspace (doubles)
    size_t raster_cap = 0;
    int *raster_i = nullptr;
    int64_t raster_i_cap = 0;
    int64_t *raster_off = nullptr;      // td_rasterize: the models' cell offsets (batched search)
    int64_t raster_off_cap = 0;
    double *h_raster = nullptr;         // td_rasterize: pinned staging of queries and cells
    size_t h_raster_cap = 0;
    double cell_lo[3] = {0, 0, 0}, cell_hi[3] = {0, 0, 0};  // box of the uploaded cells (NaN skipped)
    int nn_method = 0;                  // 0 auto, 1 brute force, 2 bucket grid (tdt_set_nn_method)
    void *chain_desc = nullptr;         // device array of chain descriptors (td_chain_run_batch)
    size_t chain_desc_bytes = 0;
    void *h_chain_desc = nullptr;       // pinned staging of the same
    void *draws = nullptr;              // k_chain_run: the launch's draws, precomputed (chain_run)
    size_t draws_bytes = 0;
    tdstar::td_shadow *shadow = nullptr;  // td_evaluate's incremental path (incremental.cpp)
    int incremental = 2;                // 0 full evaluates; 1 one launch per call; 2 a resident server (tdt_set_incremental)
    // the drop-in path's time per stage, ns (tdt_dropin_timing): [0] td_evaluate, [1] its model
    // classification, [2] its server round trip (post -> answer), [3] td_interpolate (1 point), [4] its
    // classification, [5] its server round trip, [6] td_evaluate calls, [7] td_interpolate calls, [8] full
    // evaluates, [9] a DROPIN chain's modeln copies, [10] its iterations' time, [11] its iterations;
    // the full evaluate's host side: [12] cells packed into pinned memory, [13] kernels issued, [14] the
    // wait for them, [15] chi^2 and copy-out; [16] server busy, ns (the kernel's own clock), evaluate
    // commands, [17] the same, queries
    int64_t dropin_ns[18] = {};
    // td_misfit: device copies of the last (tS, sig) given and a pinned [ptS | phi] staging area
    double *mf_dev = nullptr;           // [ptS n | tS n | sig n | terms n | phi 1]
    double *mf_host = nullptr;          // pinned [ptS n | phi 1]
    int64_t mf_cap = 0;
    std::vector<double> mf_tS, mf_sig;  // what mf_dev holds
    double mf_likelihood = 0.0;
    std::string err;
};

namespace tdstar {

// Error helpers shared by api.cpp / chain.cpp.
int set_err(td_ctx *ctx, int code, const std::string &msg);
int hip_err(td_ctx *ctx, hipError_t e, const char *what);

// Return the status of a failing HIP call (message names the call).
#define TD_HIP(ctx, call)                                 \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_err(ctx, e_, #call); \
    } while (0)
// Make room for `ncells` cells (device + pinned staging).
int ensure_cells(td_ctx *ctx, int64_t ncells);
// Pack cells into the pinned staging buffer and upload them (async on ctx->stream).
// the bucket-grid search (else brute force) for this many cells
bool uses_grid(const td_ctx *ctx, int64_t ncells);
int upload_cells(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                 int64_t ncells);
// Nearest cell of npts query points against the uploaded cells (brute force
// for small models, the bucket grid otherwise; same answer either way).
hipError_t nearest_uploaded(td_ctx *ctx, const double *qx, const double *qy, const double *qz, int64_t npts,
                            int64_t qy_stride, int64_t qz_stride, int64_t ncells, int *best_i, double *best_d,
                            double *zeta0);
// Julia Base.sum association (see oracle/README.md); used for the likelihood constant.
double julia_sum(const double *a, int64_t n);
double likelihood_constant(const double *sig, int64_t n);
// td_evaluate's full path: nearest search over every point, ray sums, chi^2
// (nearest_out nullable).  The HOST chain engine calls it directly.
double host_chi2(const double *ptS, const double *tS, const double *sig, int64_t n);  // MCsub.jl:169-172
// wall-clock ns (the drop-in breakdown)
int64_t now_ns();
int evaluate_full(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                  int64_t ncells, double *ptS_out, double *phi_out, int32_t *nearest_out = nullptr);
// td_evaluate's incremental path (incremental.cpp): phi and ptS only.
int evaluate_incremental(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                         int64_t ncells, double *ptS_out, double *phi_out);
void shadow_free(td_ctx *ctx);
// The shadow chain of td_evaluate's incremental path (nullptr if none).
td_chain *shadow_chain_of(td_ctx *ctx);
// Stop every resident server this thread runs except `keep` (chain.cpp).
void servers_quiesce(const td_chain *keep);
// td_interpolate of one point on the shadow's model (incremental.cpp); *handled = 0: not applicable.
int interpolate_incremental(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                            int64_t ncells, double qx, double qy, double qz, double *val, int *handled);

}  // namespace tdstar
