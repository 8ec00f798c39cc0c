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

__global__ __launch_bounds__(256) void k_trilinear(const double *__restrict__ xs, int nx,
                                                   const double *__restrict__ ys, int ny,
                                                   const double *__restrict__ zs, int nz,
                                                   const double *__restrict__ v, const double *__restrict__ px,
                                                   const double *__restrict__ py, const double *__restrict__ pz,
                                                   int npts, double *__restrict__ out,
                                                   unsigned long long *__restrict__ outside) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
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
    // column-major [nx][ny][nz] (Julia's sn[1, :, :, :]): x fastest
    auto at = [&](int a, int b, int c) { return v[((long)c * ny + b) * nx + a]; };
    double c2[2];
    for (int dz = 0; dz < 2; ++dz) {
        double c1[2];
        for (int dy = 0; dy < 2; ++dy) c1[dy] = ux * at(i, j + dy, k + dz) + tx * at(i + 1, j + dy, k + dz);
        c2[dz] = uy * c1[0] + ty * c1[1];
    }
    out[p] = uz * c2[0] + tz * c2[1];
}

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
    const size_t ng = (size_t)(nx + ny + nz), nv = (size_t)(nx * ny * nz), np = (size_t)npts;
    void *buf = nullptr;
    const size_t bytes = sizeof(double) * (ng + nv + 4 * np) + sizeof(unsigned long long);
    if (hipMalloc(&buf, bytes) != hipSuccess) return set_err(nullptr, TD_ERR_NOMEM, "td_trilinear: hipMalloc");
    double *dg = static_cast<double *>(buf), *dv = dg + ng, *dp = dv + nv, *dout = dp + 3 * np;
    auto *dcnt = reinterpret_cast<unsigned long long *>(dout + np);
    hipError_t e = hipMemcpy(dg, xs, sizeof(double) * nx, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dg + nx, ys, sizeof(double) * ny, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dg + nx + ny, zs, sizeof(double) * nz, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dv, values, sizeof(double) * nv, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dp, px, sizeof(double) * np, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dp + np, py, sizeof(double) * np, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dp + 2 * np, pz, sizeof(double) * np, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(dcnt, 0, sizeof(unsigned long long));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_trilinear, dim3((unsigned)((npts + 255) / 256)), dim3(256), 0, nullptr, dg, (int)nx,
                           dg + nx, (int)ny, dg + nx + ny, (int)nz, dv, dp, dp + np, dp + 2 * np, (int)npts, dout,
                           dcnt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(double) * np, hipMemcpyDeviceToHost);
    unsigned long long cnt = 0;
    if (e == hipSuccess) e = hipMemcpy(&cnt, dcnt, sizeof cnt, hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    if (e != hipSuccess) return set_err(nullptr, TD_ERR_HIP, std::string("td_trilinear: ") + hipGetErrorString(e));
    *n_outside = (int64_t)cnt;
    return TD_OK;
}
