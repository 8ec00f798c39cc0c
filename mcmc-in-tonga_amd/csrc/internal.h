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

// Workspace for the split-cells nearest search.
struct NNWork {
    double *part_d = nullptr;  // [chunks][npts]
    int *part_i = nullptr;
    size_t cap = 0;            // elements
};

struct Geometry {
    int64_t m = 0, n = 0, P = 0;
    double *px = nullptr, *py = nullptr, *pz = nullptr, *w = nullptr;
    int *ray_off = nullptr;
    double *tS = nullptr, *sig = nullptr;
};

// How a cell set is split over workgroups for the brute-force search.
struct NNPlan {
    int ppl;       // points per lane
    int blocks_x;  // point tiles
    int chunks;    // cell chunks (grid y)
    int chunk;     // cells per chunk (LDS-staged)
};
NNPlan plan_nearest(int64_t npts, int64_t ncells, int num_cus);

// nearest cell of each point (split search + ordered merge).  cells = SoA
// (x at [0], y at [stride], z at [2*stride], zeta at [3*stride]).
// Writes best_i (0-based or -1), best_d (FP64 min distance or 1e9) and
// zeta0 (cell value or 0.0 -- MCsub.jl:249,257).
hipError_t launch_nearest(const double *qx, const double *qy, const double *qz, int64_t npts,
                          int64_t qy_stride, int64_t qz_stride, const double *cells, int64_t stride,
                          int64_t ncells, NNWork &work, int num_cus, int *best_i, double *best_d,
                          double *zeta0, hipStream_t s, Timer *tm = nullptr);

// ptS[i] = julia_sum_j w[j] * ((0.5*(z0[j]+z0[j+1])) / 1000) per ray (MCsub.jl:147-159).
hipError_t launch_ray_sums(const Geometry &g, const double *zeta0, double *ptS, hipStream_t s, Timer *tm = nullptr);

// phi = sequential sum_k ((ptS-tS)^2*1.0)/sig^2 (MCsub.jl:169-172).
hipError_t launch_chi2(const Geometry &g, const double *ptS, double *phi, hipStream_t s, Timer *tm = nullptr);

}  // namespace tdstar
