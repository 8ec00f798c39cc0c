// ingest.hip -- slowness of every ray point from a gridded 3-D velocity model
// (SURVEY.md 8f row 4): pre_process_data.jl:34 `iu = itp.(ix, iy, iz)` with
// load_3Dvel.jl:32 `itp = interpolate((x, y, z), sn, Gridded(Linear()))`.
//
// Interpolations.jl (Gridded(Linear())), per axis: the knot interval
// i = searchsortedlast(knots, x) clamped to [1, n-1] and the weights
// (1 - t, t) with t = (x - k_i) / (k_{i+1} - k_i); a point outside
// [k_1, k_n] on any axis is a BoundsError (no extrapolation).  Interpolations.jl
// is not in the reference tree and the reference pins no version, so the
// association of the 8-corner sum is this build's (x, then y, then z, each
// (1-t)*a + t*b) and the oracle (oracle_np.trilinear) restates the same one:
// parity with the reference is unpinned for the last ulps.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cmath>

#include "ctx.h"

namespace tdstar {

namespace {

// searchsortedlast clamped to [0, n-2] (0-based); -1 when x is outside [k0, kn-1] or NaN
__device__ __forceinline__ int knot_interval(const double *__restrict__ k, int n, double x) {
    if (!(x >= k[0] && x <= k[n - 1])) return -1;
    int lo = 0, hi = n - 1;  // k[lo] <= x, and the answer is < hi or x == k[n-1]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (k[mid] <= x)
            lo = mid;
        else
            hi = mid;
    }
    return lo < n - 1 ? lo : n - 2;
}

// Knots (nx + ny + nz doubles) are staged in LDS when they fit: the three
// binary searches are chains of dependent loads, LDS round trips instead of L2.
constexpr int kTriThreads = 256;
constexpr int kKnotsLds = 4096;  // 32 KB

__global__ __launch_bounds__(kTriThreads) void k_trilinear(const double *__restrict__ knots, int nx, int ny, int nz,
                                                           const double *__restrict__ v,
                                                           const double *__restrict__ px,
                                                           const double *__restrict__ py,
                                                           const double *__restrict__ pz, int npts,
                                                           double *__restrict__ out,
                                                           unsigned long long *__restrict__ outside) {
    __shared__ double kl[kKnotsLds];
    const int ng = nx + ny + nz;
    const bool lds = ng <= kKnotsLds;
    if (lds)
        for (int i = threadIdx.x; i < ng; i += kTriThreads) kl[i] = knots[i];
    __syncthreads();
    const double *k0 = lds ? kl : knots;
    const double *xs = k0, *ys = k0 + nx, *zs = k0 + nx + ny;
    const int p = blockIdx.x * kTriThreads + threadIdx.x;
    if (p >= npts) return;
    const double x = px[p], y = py[p], z = pz[p];
    const int i = knot_interval(xs, nx, x), j = knot_interval(ys, ny, y), k = knot_interval(zs, nz, z);
    if (i < 0 || j < 0 || k < 0) {
        out[p] = __builtin_nan("");
        atomicAdd(outside, 1ull);
        return;
    }
    const double tx = (x - xs[i]) / (xs[i + 1] - xs[i]);
    const double ty = (y - ys[j]) / (ys[j + 1] - ys[j]);
    const double tz = (z - zs[k]) / (zs[k + 1] - zs[k]);
    const double ux = 1.0 - tx, uy = 1.0 - ty, uz = 1.0 - tz;
    // column-major [nx][ny][nz] (Julia's sn[1, :, :, :]): x fastest; the 8 corners loaded at once
    auto at = [&](int a, int b, int c) { return v[((long)c * ny + b) * nx + a]; };
    double cv[2][2][2];
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) cv[dz][dy][dx] = at(i + dx, j + dy, k + dz);
    double c2[2];
#pragma unroll
    for (int dz = 0; dz < 2; ++dz) {
        double c1[2];
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) c1[dy] = ux * cv[dz][dy][0] + tx * cv[dz][dy][1];
        c2[dz] = uy * c1[0] + ty * c1[1];
    }
    out[p] = uz * c2[0] + tz * c2[1];
}

// Device buffers and a stream kept across calls, per thread and device (the
// call is context-free): no hipMalloc / hipFree per call.
struct TriCache {
    int device = -1;
    hipStream_t stream = nullptr;
    void *buf = nullptr;
    size_t cap = 0;
};
thread_local TriCache t_tri;

}  // namespace

}  // namespace tdstar

using namespace tdstar;

extern "C" int td_trilinear(int device, const double *xs, int64_t nx, const double *ys, int64_t ny,
                            const double *zs, int64_t nz, const double *values, const double *px,
                            const double *py, const double *pz, int64_t npts, double *out, int64_t *n_outside) {
    if (nx < 2 || ny < 2 || nz < 2 || npts < 0 || !xs || !ys || !zs || !values || !n_outside ||
        (npts > 0 && (!px || !py || !pz || !out)))
        return set_err(nullptr, TD_ERR_ARG, "td_trilinear: bad arguments (every axis needs >= 2 knots)");
    const double *ax[3] = {xs, ys, zs};
    const int64_t na[3] = {nx, ny, nz};
    for (int a = 0; a < 3; ++a)
        for (int64_t i = 0; i + 1 < na[a]; ++i)
            if (!(ax[a][i] < ax[a][i + 1]))
                return set_err(nullptr, TD_ERR_ARG, "td_trilinear: knots must be strictly increasing");
    if (nx * ny * nz > ((int64_t)1 << 31) || npts > 0x7fffffff)
        return set_err(nullptr, TD_ERR_ARG, "td_trilinear: too large");
    *n_outside = 0;
    if (npts == 0) return TD_OK;
    if (hipSetDevice(device) != hipSuccess) return set_err(nullptr, TD_ERR_HIP, "td_trilinear: hipSetDevice");
    servers_quiesce(nullptr);
    TriCache &c = t_tri;
    hipError_t e = hipSuccess;
    if (c.device != device) {
        if (c.device >= 0) {  // another device: the old one's buffers go
            (void)hipSetDevice(c.device);
            if (c.buf) (void)hipFree(c.buf);
            if (c.stream) (void)hipStreamDestroy(c.stream);
            (void)hipSetDevice(device);
        }
        c = TriCache{};
        e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
        if (e != hipSuccess) return set_err(nullptr, TD_ERR_HIP, "td_trilinear: hipStreamCreate");
        c.device = device;
    }
    const size_t ng = (size_t)(nx + ny + nz), nv = (size_t)(nx * ny * nz), np = (size_t)npts;
    const size_t bytes = sizeof(double) * (ng + nv + 4 * np) + sizeof(unsigned long long);
    if (bytes > c.cap) {
        if (c.buf) (void)hipFree(c.buf);
        c.buf = nullptr;
        c.cap = 0;
        if (hipMalloc(&c.buf, bytes + bytes / 4) != hipSuccess)
            return set_err(nullptr, TD_ERR_NOMEM, "td_trilinear: hipMalloc");
        c.cap = bytes + bytes / 4;
    }
    double *dg = static_cast<double *>(c.buf), *dv = dg + ng, *dp = dv + nv, *dout = dp + 3 * np;
    auto *dcnt = reinterpret_cast<unsigned long long *>(dout + np);
    const struct { void *d; const void *h; size_t b; } up[] = {
        {dg, xs, sizeof(double) * nx}, {dg + nx, ys, sizeof(double) * ny}, {dg + nx + ny, zs, sizeof(double) * nz},
        {dv, values, sizeof(double) * nv}, {dp, px, sizeof(double) * np}, {dp + np, py, sizeof(double) * np},
        {dp + 2 * np, pz, sizeof(double) * np}};
    for (const auto &u : up)
        if (e == hipSuccess) e = hipMemcpyAsync(u.d, u.h, u.b, hipMemcpyHostToDevice, c.stream);
    if (e == hipSuccess) e = hipMemsetAsync(dcnt, 0, sizeof(unsigned long long), c.stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_trilinear, dim3((unsigned)((npts + kTriThreads - 1) / kTriThreads)), dim3(kTriThreads), 0,
                           c.stream, dg, (int)nx, (int)ny, (int)nz, dv, dp, dp + np, dp + 2 * np, (int)npts, dout, dcnt);
        e = hipGetLastError();
    }
    unsigned long long cnt = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(double) * np, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&cnt, dcnt, sizeof cnt, hipMemcpyDeviceToHost, c.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c.stream);
    if (e != hipSuccess) return set_err(nullptr, TD_ERR_HIP, std::string("td_trilinear: ") + hipGetErrorString(e));
    *n_outside = (int64_t)cnt;
    return TD_OK;
}
