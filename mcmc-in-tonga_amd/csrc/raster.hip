// raster.hip -- posterior maps of plot_model_hist (MCsub.jl:753-825) without
// the plotting: the nearest-cell value of every saved model at every node of
// a cross-section (v_nearest, MCsub.jl:765-768 / 799-802), then per node the
// mean and the standard deviation over the models (MCsub.jl:774-775) in the
// association Julia's Statistics uses for a Vector of matrices:
//   mean = sum(A) / n          sum: mapreduce(+) -- n < 16 left to right,
//                              else pairwise halves down to <= 1024-element
//                              blocks added left to right (no SIMD
//                              reassociation: the elements are arrays)
//   std  = sqrt.(sum(abs2.(A .- mean)) / (n - 1))      (same association)
// The model sweep reuses the evaluate path's nearest search (bucket grid or
// brute force per model size), one launch group per model.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "ctx.h"

namespace tdstar {

namespace {

// Julia's mapreduce association over k = 0..n-1 of f(k) (n >= 1).
template <class F>
__device__ double julia_mapreduce_seq_blocks(F f, int n) {
    if (n == 1) return f(0);
    if (n < 16) {
        double s = f(0) + f(1);
        for (int k = 2; k < n; ++k) s = s + f(k);
        return s;
    }
    // pairwise: blocks of <= 1024 elements are summed left to right
    int lo_s[40], hi_s[40], st_s[40];
    double vals[40];
    int top = 1, nv = 0;
    lo_s[0] = 0;
    hi_s[0] = n - 1;
    st_s[0] = 0;
    while (top > 0) {
        const int lo = lo_s[top - 1], hi = hi_s[top - 1];
        if (hi - lo < 1024) {
            double s = f(lo) + f(lo + 1);
            for (int k = lo + 2; k <= hi; ++k) s = s + f(k);
            vals[nv++] = s;
            --top;
            continue;
        }
        const int mid = (lo + hi) >> 1;
        if (st_s[top - 1] == 0) {
            st_s[top - 1] = 1;
            lo_s[top] = lo; hi_s[top] = mid; st_s[top] = 0; ++top;
        } else if (st_s[top - 1] == 1) {
            st_s[top - 1] = 2;
            lo_s[top] = mid + 1; hi_s[top] = hi; st_s[top] = 0; ++top;
        } else {
            const double v2 = vals[--nv];
            const double v1 = vals[--nv];
            vals[nv++] = v1 + v2;
            --top;
        }
    }
    return vals[0];
}

// Every model at every node in ONE launch (the section's nodes are few; one
// launch group per model cost ~80 us of launches and host work per model).
// A work item = (model, chunk of kRasterNodes nodes); a 512-thread workgroup
// is 8 waves = 8 slices of the model's cells, each lane 2 nodes of the chunk
// (100 models x 16 chunks x 8 waves: 13 waves per SIMD, no partial last wave).
// The cells a wave reads are the same in every lane, so they come through the
// scalar cache (wave-uniform addresses: s_load, SGPR operands) -- no LDS
// staging, no barrier but the final one.  Each lane keeps its nodes' running
// (distance, index) with v_nearest's strict '<' in index order (MCsub.jl:
// 250-258: the first minimum wins, only distances below the 1e9 sentinel
// count; NaN never wins); groups of 8 cells take one v_min per distance and
// look the index up only when the group beats the running best.  The slices
// are merged in slice order (a tie keeps the lower slice, hence the lower
// index).  The value is zeta of the winner, or 0.0 when none (MCsub.jl:249).
// XCD-aware mapping: the dispatcher deals workgroups round-robin over the 8
// XCDs, so block L runs on XCD L % 8; every chunk of model m is given to a
// block of XCD m % 8, and each model's cells are fetched from HBM into ONE L2.
constexpr int kRasterThreads = 512;
constexpr int kRasterSlices = kRasterThreads / 64;
constexpr int kRasterPPL = 2;
constexpr int kRasterNodes = 64 * kRasterPPL;
constexpr int kXcds = 8;
__global__ __launch_bounds__(kRasterThreads) void k_raster_brute(const int64_t *__restrict__ cell_off,
                                                                 const double *__restrict__ cells, int64_t cs,
                                                                 const double *__restrict__ q, int nq, int nmodels,
                                                                 int nchunks, double *__restrict__ values) {
    __shared__ double md[kRasterSlices][kRasterNodes];
    __shared__ int mi[kRasterSlices][kRasterNodes];
    const int L = blockIdx.x, xcd = L % kXcds, j = L / kXcds;
    const int m = xcd + kXcds * (j / nchunks), chunk = j % nchunks;
    if (m >= nmodels) return;  // the whole workgroup: no barrier reached
    const long a = (long)cell_off[m];
    const int nc = (int)(cell_off[m + 1] - a);
    const int lane = threadIdx.x & 63;
    const int sl = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int per = (nc + kRasterSlices - 1) / kRasterSlices;
    const int c_lo = min(sl * per, nc), c_hi = min(c_lo + per, nc);
    const double *__restrict__ cx = cells + a, *__restrict__ cy = cells + cs + a, *__restrict__ cz = cells + 2 * cs + a;
    double x[kRasterPPL], y[kRasterPPL], z[kRasterPPL], bd[kRasterPPL];
    int bi[kRasterPPL];
#pragma unroll
    for (int k = 0; k < kRasterPPL; ++k) {
        const int nd = min(chunk * kRasterNodes + k * 64 + lane, nq - 1);
        x[k] = q[nd];
        y[k] = q[nq + nd];
        z[k] = q[2 * (long)nq + nd];
        bd[k] = kSentinel;
        bi[k] = -1;
    }
    int c = c_lo;
    // the next group's cells are loaded (scalar loads, wave-uniform) while this group is scanned
    double ux[8], uy[8], uz[8];
    if (c + 8 <= c_hi) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            ux[u] = cx[c + u];
            uy[u] = cy[c + u];
            uz[u] = cz[c + u];
        }
    }
    for (; c + 8 <= c_hi; c += 8) {
        double vx[8], vy[8], vz[8];
        const int cn = c + 8 + 8 <= c_hi ? c + 8 : c;  // (the last group reloads itself: no branch)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            vx[u] = cx[cn + u];
            vy[u] = cy[cn + u];
            vz[u] = cz[cn + u];
        }
        double dg[kRasterPPL][8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
            for (int k = 0; k < kRasterPPL; ++k) {
                // (mx[i]-x)^2 + (my[i]-y)^2 + (mz[i]-z)^2, MCsub.jl:254, left to right, unfused
                const double dx = ux[u] - x[k], dy = uy[u] - y[k], dz = uz[u] - z[k];
                double d = dx * dx;
                d = d + dy * dy;
                d = d + dz * dz;
                dg[k][u] = d;
            }
        }
        group8_update<kRasterPPL>(dg, bd, bi, c);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            ux[u] = vx[u];
            uy[u] = vy[u];
            uz[u] = vz[u];
        }
    }
    for (; c < c_hi; ++c) {
        const double ux = cx[c], uy = cy[c], uz = cz[c];
#pragma unroll
        for (int k = 0; k < kRasterPPL; ++k) {
            const double dx = ux - x[k], dy = uy - y[k], dz = uz - z[k];
            double d = dx * dx;
            d = d + dy * dy;
            d = d + dz * dz;
            if (d < bd[k]) {
                bd[k] = d;
                bi[k] = c;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kRasterPPL; ++k) {
        md[sl][k * 64 + lane] = bd[k];
        mi[sl][k * 64 + lane] = bi[k];
    }
    __syncthreads();
    if (threadIdx.x < kRasterNodes) {
        const int t = threadIdx.x, node = chunk * kRasterNodes + t;
        double d = md[0][t];
        int i = mi[0][t];
#pragma unroll
        for (int s2 = 1; s2 < kRasterSlices; ++s2)
            if (md[s2][t] < d) {  // strict: the lower slice keeps a tie
                d = md[s2][t];
                i = mi[s2][t];
            }
        if (node < nq) values[(long)m * nq + node] = i >= 0 ? cells[3 * cs + a + i] : 0.0;
    }
}

__global__ __launch_bounds__(256) void k_raster_stats(const double *__restrict__ values, int nmodels, int nq,
                                                      double *__restrict__ mean, double *__restrict__ sd) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const double *v = values + q;
    const long st = nq;
    const double m = julia_mapreduce_seq_blocks([&](int k) { return v[k * st]; }, nmodels) / (double)nmodels;
    const double ss = julia_mapreduce_seq_blocks(
        [&](int k) {
            const double d = v[k * st] - m;
            return d * d;  // abs2
        },
        nmodels);
    mean[q] = m;
    sd[q] = sqrt(ss / (double)(nmodels - 1));  // corrected; n == 1 gives 0/0 = NaN as in Julia
}

}  // namespace

}  // namespace tdstar

using namespace tdstar;

extern "C" int td_rasterize(td_ctx *ctx, int64_t nmodels, const int64_t *cell_off, const double *xCell,
                            const double *yCell, const double *zCell, const double *zeta, const double *qx,
                            const double *qy, const double *qz, int64_t nq, double *mean_out, double *std_out,
                            double *values_out) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_rasterize: ctx is NULL");
    if (nmodels < 1 || !cell_off || nq < 0 || (nq > 0 && (!qx || !qy || !qz || !mean_out || !std_out)))
        return set_err(ctx, TD_ERR_ARG, "td_rasterize: bad arguments");
    const int64_t total = cell_off[nmodels];
    if (cell_off[0] != 0 || total < 0 || (total > 0 && (!xCell || !yCell || !zCell || !zeta)))
        return set_err(ctx, TD_ERR_ARG, "td_rasterize: bad cell offsets or arrays");
    for (int64_t k = 0; k < nmodels; ++k)
        if (cell_off[k + 1] < cell_off[k]) return set_err(ctx, TD_ERR_ARG, "td_rasterize: offsets not monotone");
    if (nq == 0) return TD_OK;
    if (nq > 0x7fffffff / std::max<int64_t>(nmodels, 1) || total > 0x7fffffff)
        return set_err(ctx, TD_ERR_ARG, "td_rasterize: too large");
    TD_HIP(ctx, hipSetDevice(ctx->device));
    // one device block: queries (3 nq), all cells SoA (4 total), values (nmodels nq), mean, std (2 nq)
    const size_t nd = 3 * (size_t)nq + 4 * (size_t)std::max<int64_t>(total, 1) + (size_t)nmodels * nq + 2 * (size_t)nq;
    if (nd > ctx->raster_cap) {
        if (ctx->raster) (void)hipFree(ctx->raster);
        ctx->raster = nullptr;
        ctx->raster_cap = 0;
        TD_HIP(ctx, hipMalloc(&ctx->raster, sizeof(double) * nd));
        ctx->raster_cap = nd;
    }
    double *dq = ctx->raster, *dc = dq + 3 * nq, *dv = dc + 4 * std::max<int64_t>(total, 1), *dm = dv + nmodels * nq,
           *ds = dm + nq;
    const int64_t cs = std::max<int64_t>(total, 1);  // SoA stride of the cells
    // packed into a pinned staging block (reused across calls), then one DMA copy: pageable
    // copies of these sizes run at ~1 GB/s here
    const size_t nh = 3 * (size_t)nq + 4 * (size_t)cs;
    if (nh > ctx->h_raster_cap) {
        if (ctx->h_raster) (void)hipHostFree(ctx->h_raster);
        ctx->h_raster = nullptr;
        ctx->h_raster_cap = 0;
        TD_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&ctx->h_raster), sizeof(double) * nh, hipHostMallocDefault));
        ctx->h_raster_cap = nh;
    }
    TD_HIP(ctx, hipStreamSynchronize(ctx->stream));  // the staging block may still feed a previous copy
    double *h = ctx->h_raster;
    std::memcpy(h, qx, sizeof(double) * (size_t)nq);
    std::memcpy(h + nq, qy, sizeof(double) * (size_t)nq);
    std::memcpy(h + 2 * nq, qz, sizeof(double) * (size_t)nq);
    double *hc = h + 3 * nq;
    if (total > 0) {
        std::memcpy(hc, xCell, sizeof(double) * (size_t)total);
        std::memcpy(hc + cs, yCell, sizeof(double) * (size_t)total);
        std::memcpy(hc + 2 * cs, zCell, sizeof(double) * (size_t)total);
        std::memcpy(hc + 3 * cs, zeta, sizeof(double) * (size_t)total);
    }
    TD_HIP(ctx, hipMemcpyAsync(dq, h, sizeof(double) * nh, hipMemcpyHostToDevice, ctx->stream));
    if (nq > ctx->raster_i_cap) {  // nearest-cell indices (not returned)
        if (ctx->raster_i) (void)hipFree(ctx->raster_i);
        ctx->raster_i = nullptr;
        ctx->raster_i_cap = 0;
        TD_HIP(ctx, hipMalloc(&ctx->raster_i, sizeof(int) * (size_t)nq));
        ctx->raster_i_cap = nq;
    }
    Timer *tm = ctx->timer.on ? &ctx->timer : nullptr;
    // a section's few nodes: every model in one brute-force launch; many nodes: per model,
    // the evaluate path's search (the bucket grid from kGridMinCells cells)
    const bool batched = nq * (total / std::max<int64_t>(nmodels, 1)) <= (int64_t)1 << 28 &&
                         (int64_t)kXcds * ((nmodels + kXcds - 1) / kXcds) * ((nq + kRasterNodes - 1) / kRasterNodes) <= INT32_MAX;
    if (batched) {
        if (nmodels + 1 > ctx->raster_off_cap) {
            if (ctx->raster_off) (void)hipFree(ctx->raster_off);
            ctx->raster_off = nullptr;
            ctx->raster_off_cap = 0;
            TD_HIP(ctx, hipMalloc(&ctx->raster_off, sizeof(int64_t) * (size_t)(nmodels + 1)));
            ctx->raster_off_cap = nmodels + 1;
        }
        TD_HIP(ctx, hipMemcpyAsync(ctx->raster_off, cell_off, sizeof(int64_t) * (size_t)(nmodels + 1),
                                   hipMemcpyHostToDevice, ctx->stream));
        hipEvent_t t0 = tm ? tm->begin(ctx->stream) : nullptr;
        const int nchunks = (int)((nq + kRasterNodes - 1) / kRasterNodes);
        const int64_t blocks = (int64_t)kXcds * ((nmodels + kXcds - 1) / kXcds) * nchunks;
        hipLaunchKernelGGL(k_raster_brute, dim3((unsigned)blocks), dim3(kRasterThreads), 0, ctx->stream,
                           ctx->raster_off, dc, cs, dq, (int)nq, (int)nmodels, nchunks, dv);
        if (tm) tm->end("raster_brute", t0, ctx->stream);
        TD_HIP(ctx, hipGetLastError());
    }
    for (int64_t k = 0; k < (batched ? 0 : nmodels); ++k) {
        const int64_t a = cell_off[k], nc = cell_off[k + 1] - a;
        double *out = dv + k * nq;
        hipError_t e;
        if (nc >= kGridMinCells && ctx->nn_method != 1) {
            double lo[3], hi[3];
            const double *src[3] = {xCell + a, yCell + a, zCell + a};
            for (int d = 0; d < 3; ++d) {
                double l = HUGE_VAL, u = -HUGE_VAL;
                for (int64_t i = 0; i < nc; ++i) {
                    l = src[d][i] < l ? src[d][i] : l;
                    u = src[d][i] > u ? src[d][i] : u;
                }
                lo[d] = l <= u ? l : 0.0;
                hi[d] = l <= u ? u : 0.0;
            }
            const CellGrid G = make_cell_grid(lo, hi, (double)nc / 2.0, 4096, kGridMaxBuckets);
            e = launch_nearest_grid(dq, dq + nq, dq + 2 * nq, nq, 1, 1, dc + a, cs, nc, G, ctx->nn, ctx->num_cus,
                                    ctx->raster_i, nullptr, out, ctx->stream, tm);
        } else {
            e = launch_nearest(dq, dq + nq, dq + 2 * nq, nq, 1, 1, dc + a, cs, nc, ctx->nn, ctx->num_cus,
                               ctx->raster_i, nullptr, out, ctx->stream, tm);
        }
        if (e != hipSuccess) return hip_err(ctx, e, "td_rasterize: nearest kernels");
    }
    hipLaunchKernelGGL(k_raster_stats, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, ctx->stream, dv,
                       (int)nmodels, (int)nq, dm, ds);
    TD_HIP(ctx, hipGetLastError());
    TD_HIP(ctx, hipMemcpyAsync(mean_out, dm, sizeof(double) * (size_t)nq, hipMemcpyDeviceToHost, ctx->stream));
    TD_HIP(ctx, hipMemcpyAsync(std_out, ds, sizeof(double) * (size_t)nq, hipMemcpyDeviceToHost, ctx->stream));
    if (values_out)
        TD_HIP(ctx, hipMemcpyAsync(values_out, dv, sizeof(double) * (size_t)nq * nmodels, hipMemcpyDeviceToHost,
                                   ctx->stream));
    TD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return TD_OK;
}
