// internal.h -- device layout of a td_ctx and the kernel launchers.
//
// HBM layout (one context = one copy of the ray geometry, FP64 throughout):
//   px/py/pz[P]    ray points, ray-major (CSR), the NaN tail padding removed
//   w[P]           rayL*rayU of the segment that starts at point k (0 on the
//                  last point of each ray); load_data_Tonga.jl:66-69 and the
//                  left factor of MCsub.jl:153/159 `rayl .* rayu .* (...)`
//   ray_off[n+1]   int32 CSR offsets
//   tS/sig[n]      DataStruct.tS / allSig
// Per model ("cell set"): SoA x|y|z|zeta, stride = capacity.
// Per evaluation: nearest cell + its FP64 squared distance per point (the
// incremental chain keeps these as its cache), ptS[n], phi.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include <map>
#include <string>
#include <vector>

namespace tdstar {

constexpr double kSentinel = 1e9;  // MCsub.jl:250

// One group step of the brute-force scans (k_nn_tile, k_nn_partial,
// k_raster_brute): the distances dg[k][u] of PPL points to 8 consecutive cells
// base .. base + 7 update each point's running (bd, bi) under v_nearest's
// strict '<' in index order (MCsub.jl:255).  The group minimum is a tree of
// v_min (fmin: a NaN distance never becomes the minimum; the same value as the
// left-to-right chain, with 3 dependent steps instead of 7); every point's
// minimum is formed before ONE branch, taken only when some point improves
// (rare after the first groups), where the first cell reaching the minimum is
// looked up.  A group tie goes to its first cell, a tie with an earlier group
// keeps the earlier cell -- exactly the sequential strict '<' scan.
template <int PPL>
__device__ __forceinline__ void group8_update(const double (&dg)[PPL][8], double (&bd)[PPL], int (&bi)[PPL],
                                              int base) {
    double m[PPL];
    bool any = false;
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const double a = fmin(fmin(dg[k][0], dg[k][1]), fmin(dg[k][2], dg[k][3]));
        const double b = fmin(fmin(dg[k][4], dg[k][5]), fmin(dg[k][6], dg[k][7]));
        m[k] = fmin(a, b);
        any = any || m[k] < bd[k];  // strict: NaN never wins
    }
    if (any) {
#pragma unroll
        for (int k = 0; k < PPL; ++k)
            if (m[k] < bd[k]) {
                int f = 7;
#pragma unroll
                for (int u = 7; u >= 0; --u) f = dg[k][u] == m[k] ? u : f;
                bd[k] = m[k];
                bi[k] = base + f;
            }
    }
}

// Per-kernel timing with HIP events recorded on the launch stream (bench.py's
// roofline numbers).  Disabled: begin()/end() are no-ops.
struct Timer {
    bool on = false;
    struct Pending { std::string name; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> spare;
    std::map<std::string, std::pair<int64_t, double>> acc;  // name -> (launches, ms)
    hipEvent_t begin(hipStream_t s);
    void end(const char *name, hipEvent_t a, hipStream_t s);
    hipError_t collect();  // waits for the recorded events
    void reset();
    void release();
};

// Bucket of a coordinate: clamp(floor((v - v0) * inv), 0, g - 1).  Cells
// outside the box land in the boundary buckets, so "no bucket beyond" really
// means no cell beyond.  Same function on host (build) and device (updates).
struct CellGrid {
    int gx, gy, gz;
    double x0, y0, z0;
    double ix, iy, iz;  // buckets per km
    double hx, hy, hz;  // km per bucket
    // allowance for the rounding of bucket assignment against the faces
    // x0 + i*hx: a cell can sit up to ex on the wrong side of a face
    double ex, ey, ez;
    // sealed != 0: every cell lies inside [lo, hi] on each axis (the evaluate's cells' own box; the
    // device chain's prior box, which every valid proposal stays in) -- a query point outside that box
    // is at least its distance to the box from every cell (grid_block_lb)
    double lo[3], hi[3];
    int sealed;
};

// A uniform grid with about `target` buckets over the box [lo, hi] (degenerate
// axes get one bucket), at most `max_buckets` in all.
CellGrid make_cell_grid(const double lo[3], const double hi[3], double target, int max_dim, int64_t max_buckets);

struct BucketEntry {
    double x, y, z;
    int slot, pad;
};

__host__ __device__ inline int grid_axis(double v, double v0, double inv, int g) {
    const double f = (v - v0) * inv;
    return f >= 0.0 ? (f < (double)g ? (int)f : g - 1) : 0;  // NaN -> 0
}

__host__ __device__ inline int grid_bucket(const CellGrid &G, double x, double y, double z) {
    return (grid_axis(z, G.z0, G.iz, G.gz) * G.gy + grid_axis(y, G.y0, G.iy, G.gy)) * G.gx +
           grid_axis(x, G.x0, G.ix, G.gx);
}

// Squared distance from (x,y,z) in bucket column (i,j,k) to the nearest outer
// face of the block of buckets [i-R, i+R] x [j-R, j+R] x [k-R, k+R], faces on
// the grid boundary excluded (no cell lies beyond them).  Every cell outside
// the block is at least this far away (0 when unknown; +inf when the block
// covers the grid).
//
// A sealed grid also bounds by the point's distance to the cells' box: a cell
// beyond an x face lies inside the box in y and z, so it is at least
// sqrt(gap_x^2 + out_y^2 + out_z^2) away (out_a = the point's distance to the
// box along a, 0 inside).  That proves the nearest cell of a point outside the
// box (the ray ends past the prior box's y range, 3 % of the 381 rays'
// points) from the 3x3x3 block, where the faces alone never could.
__host__ __device__ inline void grid_out2(const CellGrid &G, double x, double y, double z, double o2[3]) {
    const double v[3] = {x, y, z}, e[3] = {G.ex, G.ey, G.ez};
    for (int a = 0; a < 3; ++a) {
        double o = 0.0;
        if (G.sealed) {
            const double below = G.lo[a] - v[a], above = v[a] - G.hi[a];
            o = (below > above ? below : above) - e[a];  // (NaN: not > 0)
        }
        o2[a] = o > 0.0 ? o * o : 0.0;
    }
}
// min over faces of gap^2 + the other axes' out^2, made a strict lower bound of every FP64 dist2 beyond
__host__ __device__ inline double grid_lb_close(double lb) { return lb * (1.0 - 0x1p-40); }
__host__ __device__ inline double grid_block_lb(const CellGrid &G, double x, double y, double z, int R) {
    double lb = __builtin_huge_val();
    double o2[3];
    grid_out2(G, x, y, z, o2);
    auto face = [&lb](double v, double v0, double inv, double h, double e, int g, int R_, double other) {
        const int i = grid_axis(v, v0, inv, g);
        if (i - R_ > 0) {
            const double gap = (v - (v0 + (double)(i - R_) * h)) - e;
            const double f = (gap > 0.0 ? gap * gap : 0.0) + other;
            lb = f < lb ? f : lb;
        }
        if (i + R_ < g - 1) {
            const double gap = ((v0 + (double)(i + R_ + 1) * h) - v) - e;
            const double f = (gap > 0.0 ? gap * gap : 0.0) + other;
            lb = f < lb ? f : lb;
        }
    };
    face(x, G.x0, G.ix, G.hx, G.ex, G.gx, R, o2[1] + o2[2]);
    face(y, G.y0, G.iy, G.hy, G.ey, G.gy, R, o2[0] + o2[2]);
    face(z, G.z0, G.iz, G.hz, G.ez, G.gz, R, o2[0] + o2[1]);
    return grid_lb_close(lb);
}

constexpr int kGridMaxBuckets = 1 << 16;  // bucket grid of the evaluate path
constexpr int kGridCap = 16;               // entries per bucket (a fuller bucket is searched by brute force)
constexpr int kGridMinCells = 256;     // below: the brute force is as fast

// Workspace for the nearest searches (split brute force; bucket grid).
constexpr int kNNAuto = 0;   // brute force: k_nn_tile (every point count up to ~128 M)
constexpr int kNNSplit = 1;  // brute force: always the split search (k_nn_partial + k_nn_merge)

struct NNWork {
    double *part_d = nullptr;  // [chunks][npts]
    int *part_i = nullptr;
    size_t cap = 0;            // elements
    int *g_count = nullptr;        // [2][buckets] cells per bucket: two sets, alternate searches
    BucketEntry *g_ent = nullptr;  // [buckets][kGridCap] entries {x, y, z, cell index}
    size_t g_count_cap = 0, g_ent_cap = 0;  // bytes (g_count: both sets)
    int g_par = 0;                 // the set the next search fills (zero)
    int64_t g_used[2] = {0, 0};    // buckets each set holds counts in (zeroed by the other's search)
    int method = 0;                // brute force: kNNAuto (one-launch tile search where it fits) or kNNSplit
};

struct Geometry {
    int64_t m = 0, n = 0, P = 0;
    double *px = nullptr, *py = nullptr, *pz = nullptr, *w = nullptr;
    int *ray_off = nullptr;
    double *tS = nullptr, *sig = nullptr;
    double *terms = nullptr;  // [n] scratch: chi^2 terms of one evaluation
};

// How a cell set is split over workgroups for the brute-force search.
struct NNPlan {
    int ppl;       // points per lane
    int blocks_x;  // point tiles
    int chunks;    // cell chunks (grid y)
    int chunk;     // cells per chunk (LDS-staged)
};
NNPlan plan_nearest(int64_t npts, int64_t ncells, int num_cus);

// The one-launch brute force (k_nn_tile): tiles of Q points, one workgroup
// per CU taking every gridDim-th tile; a tile's points are checked against
// every cell in S slices of L cells, staged R at a time.
struct TilePlan {
    bool ok = false;  // false: no tile shape fits (the split search)
    int Q = 0, S = 0, L = 0, R = 0, tiles = 0, blocks = 0, ppl = 2;
    size_t lds = 0;
};
TilePlan plan_tile(int64_t npts, int64_t ncells, int num_cus);

// nearest cell of each point (split search + ordered merge).  cells = SoA
// (x at [0], y at [stride], z at [2*stride], zeta at [3*stride]).
// Writes best_i (0-based or -1), best_d (FP64 min distance or 1e9) and
// zeta0 (cell value or 0.0 -- MCsub.jl:249,257).
hipError_t launch_nearest(const double *qx, const double *qy, const double *qz, int64_t npts,
                          int64_t qy_stride, int64_t qz_stride, const double *cells, int64_t stride,
                          int64_t ncells, NNWork &work, int num_cus, int *best_i, double *best_d,
                          double *zeta0, hipStream_t s, Timer *tm = nullptr);

// Same result as launch_nearest through a bucket grid G over the cells (which
// must all lie in G's box; G.gx*G.gy*G.gz <= kGridMaxBuckets, ncells >= 1).
// Cells are ordered by nothing but their index: ties resolve exactly.
// stage (optional): the cells in pinned host memory; the grid build then
// also writes them to `cells` (one pass over PCIe instead of a DMA copy)
hipError_t launch_nearest_grid(const double *qx, const double *qy, const double *qz, int64_t npts,
                               int64_t qy_stride, int64_t qz_stride, double *cells, int64_t stride,
                               int64_t ncells, const CellGrid &G, NNWork &work, int num_cus, int *best_i,
                               double *best_d, double *zeta0, hipStream_t s, Timer *tm = nullptr,
                               const double *stage = nullptr);

// chi^2 of a given ptS (MCsub.jl:169-172, sequential in k, exact): the
// block-wide exact scan of k_chi2.  terms: n doubles of scratch; phi: one
// double (device).
hipError_t launch_chi2(const double *ptS, const double *tS, const double *sig, int n, double *terms, double *phi,
                       hipStream_t s);

// Testing: the block-wide exact sequential sum (exact_sum.h) on device buffers.
hipError_t test_wave_seq_sum(const double *term, int cnt, double C0, double *prefix, double *C_end, int *fallbacks);
hipError_t test_wave_delta_sum(const double *term, const double *old, const int *chg, int cnt, double C0,
                               double *prefix, double *C_end);
hipError_t test_exact_sum(const double *term, int cnt, double C0, double *prefix, double *C_end, int *fast);
// Testing: phi of a caller-given ptS through k_chi2 (td_misfit's chi^2).
hipError_t test_chi2(const double *ptS, const double *tS, const double *sig, int n, double *terms, double *phi,
                     hipStream_t s);
hipError_t test_block_delta(const double *term, const double *term_old, double *old, const int *chg, int k0, int n,
                            double *cprefix, double *C_end, long long *events, int *mask_ok);

// ptS[i] = julia_sum_j w[j] * ((0.5*(z0[j]+z0[j+1])) / 1000) per ray (MCsub.jl:147-159);
// host_out (nullable, device address of pinned memory): a copy of ptS for the host.
hipError_t launch_ray_sums(const Geometry &g, const double *zeta0, double *ptS, hipStream_t s, Timer *tm = nullptr,
                           double *host_out = nullptr);

}  // namespace tdstar
