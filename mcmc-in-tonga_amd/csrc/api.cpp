// api.cpp -- C ABI of libtdstar (include/tdstar.h): context, evaluate,
// interpolate.  Host-side glue only; the arithmetic is in kernels.hip.
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "chain_dev.h"
#include "ctx.h"

namespace {
thread_local std::string g_err;  // td_create failures (no ctx yet)
}

namespace tdstar {

int set_err(td_ctx *ctx, int code, const std::string &msg) {
    if (ctx)
        ctx->err = msg;
    else
        g_err = msg;
    return code;
}

int hip_err(td_ctx *ctx, hipError_t e, const char *what) {
    std::string m = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    return set_err(ctx, TD_ERR_HIP, m);
}


// Julia 1.5 Base.sum(::Vector{Float64}) association: n < 16 sequential;
// otherwise pairwise over 1024-blocks, each block v=a1+a2 then 4 x 8-lane
// accumulators + sequential tail (oracle/README.md for how this was pinned).
static double julia_block(const double *a, int64_t f, int64_t l) {
    if (f == l) return a[f];
    double v = a[f] + a[f + 1];
    const int64_t T = l - f - 1, Q = T >= 32 ? T / 32 : 0;
    int64_t i = f + 2;
    if (Q > 0) {
        double acc[32] = {0.0};
        acc[0] = v;
        for (int64_t q = 0; q < Q; ++q)
            for (int k = 0; k < 32; ++k) acc[k] = acc[k] + a[i + q * 32 + k];
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = acc[j];
        for (int k = 1; k < 4; ++k)
            for (int j = 0; j < 8; ++j) r[j] = acc[k * 8 + j] + r[j];
        for (int h = 4; h >= 1; h >>= 1)
            for (int j = 0; j < h; ++j) r[j] = r[j] + r[j + h];
        v = r[0];
        i += Q * 32;
    }
    for (; i <= l; ++i) v = v + a[i];
    return v;
}
static double julia_pairwise(const double *a, int64_t f, int64_t l) {
    if (l - f < 1024) return julia_block(a, f, l);
    const int64_t mid = f + ((l - f) >> 1);
    const double v1 = julia_pairwise(a, f, mid);
    return v1 + julia_pairwise(a, mid + 1, l);
}
double julia_sum(const double *a, int64_t n) {
    if (n == 0) return 0.0;
    if (n == 1) return a[0];
    if (n < 16) {
        double s = a[0] + a[1];
        for (int64_t i = 2; i < n; ++i) s = s + a[i];
        return s;
    }
    return julia_pairwise(a, 0, n - 1);
}

// MCsub.jl:179: sum(-log.(allSig * sqrt(2 * pi)) * length(tS)).  Line 180 is a
// separate statement in Julia, so the Gaussian term is NOT part of it.
double likelihood_constant(const double *sig, int64_t n) {
    std::vector<double> t((size_t)n);
    const volatile double two_pi = 2.0 * 3.141592653589793;
    const double c = std::sqrt((double)two_pi);
    for (int64_t k = 0; k < n; ++k) t[(size_t)k] = (-std::log(sig[k] * c)) * (double)n;
    return julia_sum(t.data(), n);
}

CellGrid make_cell_grid(const double lo[3], const double hi[3], double target, int max_dim, int64_t max_buckets) {
    double ext[3], prod = 1.0;
    int k = 0;
    for (int a = 0; a < 3; ++a) {
        ext[a] = hi[a] > lo[a] ? hi[a] - lo[a] : 0.0;
        if (ext[a] > 0.0) {
            prod *= ext[a];
            ++k;
        }
    }
    int g[3] = {1, 1, 1};
    if (k > 0 && target > 1.0) {
        const double h = std::pow(prod / target, 1.0 / k);  // edge of a cubic bucket
        for (int a = 0; a < 3; ++a)
            if (ext[a] > 0.0) g[a] = (int)std::min<double>(max_dim, std::max(1.0, std::ceil(ext[a] / h)));
        while ((int64_t)g[0] * g[1] * g[2] > max_buckets) {  // shrink the largest axis
            int a = 0;
            for (int b = 1; b < 3; ++b)
                if (g[b] > g[a]) a = b;
            g[a] = std::max(1, g[a] * 3 / 4);
        }
    }
    CellGrid G{};
    G.gx = g[0]; G.gy = g[1]; G.gz = g[2];
    for (int a = 0; a < 3; ++a) {  // (the callers' boxes hold every cell: sealed; the shadow chain unseals)
        G.lo[a] = lo[a];
        G.hi[a] = hi[a];
    }
    G.sealed = 1;
    G.x0 = lo[0]; G.y0 = lo[1]; G.z0 = lo[2];
    double *inv[3] = {&G.ix, &G.iy, &G.iz}, *h[3] = {&G.hx, &G.hy, &G.hz}, *e[3] = {&G.ex, &G.ey, &G.ez};
    for (int a = 0; a < 3; ++a) {
        *inv[a] = ext[a] > 0.0 ? g[a] / ext[a] : 0.0;
        *h[a] = ext[a] > 0.0 ? ext[a] / g[a] : 0.0;
        // floor((v - v0) * inv) vs v0 + i*h: a few ulps of the box's magnitude
        *e[a] = std::ldexp(std::fabs(lo[a]) + std::fabs(hi[a]) + ext[a], -44);
    }
    return G;
}

int ensure_cells(td_ctx *ctx, int64_t ncells) {
    if (ncells <= ctx->cell_cap && ctx->cells) return TD_OK;
    int64_t cap = ctx->cell_cap > 0 ? ctx->cell_cap : 256;
    while (cap < ncells) cap *= 2;
    if (ctx->cells) (void)hipFree(ctx->cells);
    if (ctx->h_cells) (void)hipHostFree(ctx->h_cells);
    ctx->cells = nullptr;
    ctx->h_cells = nullptr;
    ctx->cell_cap = 0;
    TD_HIP(ctx, hipMalloc(&ctx->cells, sizeof(double) * 4 * (size_t)cap));
    TD_HIP(ctx, hipHostMalloc(&ctx->h_cells, sizeof(double) * 4 * (size_t)cap,
                              hipHostMallocMapped | hipHostMallocNonCoherent));
    TD_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->h_cells_dev), ctx->h_cells, 0));
    ctx->cell_cap = cap;
    return TD_OK;
}

bool uses_grid(const td_ctx *ctx, int64_t ncells) {
    return ncells > 0 && (ctx->nn_method == 2 || (ctx->nn_method == 0 && ncells >= kGridMinCells));
}

// dst[0..n) = src, and the extent of src with NaN skipped (lo = v < lo ? v : lo): the staging of one
// coordinate of the cells and the box the bucket grid is built on, in one pass.  AVX2 when the host
// has it: minpd/maxpd return their second operand unless the first is strictly below/above, which is
// exactly that rule (NaN and +-0 included); the 8 running extents are folded by the same rule.
__attribute__((target("avx2"))) void copy_extent_avx2(const double *src, double *dst, int64_t n, double *lo_out,
                                                      double *hi_out) {
    __m256d l0 = _mm256_set1_pd(HUGE_VAL), l1 = l0, h0 = _mm256_set1_pd(-HUGE_VAL), h1 = h0;
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const __m256d a = _mm256_loadu_pd(src + i), b = _mm256_loadu_pd(src + i + 4);
        _mm256_storeu_pd(dst + i, a);
        _mm256_storeu_pd(dst + i + 4, b);
        l0 = _mm256_min_pd(a, l0);
        l1 = _mm256_min_pd(b, l1);
        h0 = _mm256_max_pd(a, h0);
        h1 = _mm256_max_pd(b, h1);
    }
    double L[8], H[8];
    _mm256_storeu_pd(L, l0);
    _mm256_storeu_pd(L + 4, l1);
    _mm256_storeu_pd(H, h0);
    _mm256_storeu_pd(H + 4, h1);
    double lo = L[0], hi = H[0];
    for (int k = 1; k < 8; ++k) {
        lo = L[k] < lo ? L[k] : lo;
        hi = H[k] > hi ? H[k] : hi;
    }
    for (; i < n; ++i) {
        const double v = src[i];
        dst[i] = v;
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    *lo_out = lo;
    *hi_out = hi;
}

void copy_extent(const double *src, double *dst, int64_t n, double *lo_out, double *hi_out) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) return copy_extent_avx2(src, dst, n, lo_out, hi_out);
    double lo = HUGE_VAL, hi = -HUGE_VAL;
    for (int64_t i = 0; i < n; ++i) {
        const double v = src[i];
        dst[i] = v;
        lo = v < lo ? v : lo;  // NaN compares false: skipped
        hi = v > hi ? v : hi;
    }
    *lo_out = lo;
    *hi_out = hi;
}

int upload_cells(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                 int64_t ncells) {
    int rc = ensure_cells(ctx, ncells);
    if (rc) return rc;
    if (ncells == 0) return TD_OK;
    // packed SoA with stride ncells: one copy over PCIe
    const int64_t s = ncells;
    ctx->cell_stride = s;
    double *h = ctx->h_cells;
    const double *src[3] = {x, y, z};
    for (int a = 0; a < 3; ++a) {  // staged, and the box of the cells for the bucket grid, in one pass
        double lo, hi;
        copy_extent(src[a], h + a * s, ncells, &lo, &hi);
        ctx->cell_lo[a] = lo <= hi ? lo : 0.0;
        ctx->cell_hi[a] = lo <= hi ? hi : 0.0;
    }
    std::memcpy(h + 3 * s, zeta, sizeof(double) * (size_t)ncells);
    if (uses_grid(ctx, ncells)) {  // the grid build reads the staged cells itself (no DMA copy)
        ctx->cells_stage = ctx->h_cells_dev;
        return TD_OK;
    }
    ctx->cells_stage = nullptr;
    TD_HIP(ctx, hipMemcpyAsync(ctx->cells, h, sizeof(double) * 4 * (size_t)ncells, hipMemcpyHostToDevice,
                               ctx->stream));
    return TD_OK;
}

hipError_t nearest_uploaded(td_ctx *ctx, const double *qx, const double *qy, const double *qz, int64_t npts,
                            int64_t qy_stride, int64_t qz_stride, int64_t ncells, int *best_i, double *best_d,
                            double *zeta0) {
    Timer *tm = ctx->timer.on ? &ctx->timer : nullptr;
    if (uses_grid(ctx, ncells)) {
        const CellGrid G = make_cell_grid(ctx->cell_lo, ctx->cell_hi, (double)ncells / 2.0, 4096, kGridMaxBuckets);
        const double *stage = ctx->cells_stage;
        ctx->cells_stage = nullptr;  // copied by this search's grid build
        return launch_nearest_grid(qx, qy, qz, npts, qy_stride, qz_stride, ctx->cells, ctx->cell_stride, ncells, G,
                                   ctx->nn, ctx->num_cus, best_i, best_d, zeta0, ctx->stream, tm, stage);
    }
    return launch_nearest(qx, qy, qz, npts, qy_stride, qz_stride, ctx->cells, ctx->cell_stride, ncells, ctx->nn,
                          ctx->num_cus, best_i, best_d, zeta0, ctx->stream, tm);
}

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// MCsub.jl:169-172: C = 0; for k in 1:n, C += ((ptS - tS)[k]^2 * 1.0) / allSig[k]^2 -- strictly in k
// order, each operation an IEEE double one (no contraction: -ffp-contract=off), as the reference's loop.
double host_chi2(const double *ptS, const double *tS, const double *sig, int64_t n) {
    double C = 0.0;
    for (int64_t k = 0; k < n; ++k) {
        const double d = ptS[k] - tS[k];
        C = C + ((d * d) * 1.0) / (sig[k] * sig[k]);
    }
    return C;
}

int evaluate_full(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                  int64_t ncells, double *ptS_out, double *phi_out, int32_t *nearest_out) {
    const int64_t t0 = now_ns();
    int rc = upload_cells(ctx, x, y, z, zeta, ncells);
    if (rc) return rc;
    const int64_t t1 = now_ns();
    const auto &g = ctx->g;
    Timer *tm = ctx->timer.on ? &ctx->timer : nullptr;
    // (the indices only when asked for, the distances never: td_evaluate needs each point's value)
    hipError_t e = nearest_uploaded(ctx, g.px, g.py, g.pz, g.P, 1, 1, ncells, nearest_out ? ctx->best_i : nullptr,
                                    nullptr, ctx->zeta0);
    if (e != hipSuccess) return hip_err(ctx, e, "nearest kernels");
    // ptS lands in pinned host memory straight from the kernel (no copy back)
    e = launch_ray_sums(g, ctx->zeta0, ctx->ptS, ctx->stream, tm, ctx->h_out_dev + 1);
    if (e != hipSuccess) return hip_err(ctx, e, "ray-sum kernel");
    if (nearest_out && g.P)
        TD_HIP(ctx, hipMemcpyAsync(ctx->h_best_i, ctx->best_i, sizeof(int) * (size_t)g.P, hipMemcpyDeviceToHost,
                                   ctx->stream));
    const int64_t t2 = now_ns();
    TD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int64_t t3 = now_ns();
    // chi^2: the n terms added in k order by the host, where ptS already is (MCsub.jl:169-172)
    const double phi = host_chi2(ctx->h_out + 1, ctx->tS_host.data(), ctx->sig_host.data(), g.n);
    if (phi_out) *phi_out = phi;
    if (ptS_out && g.n) std::memcpy(ptS_out, ctx->h_out + 1, sizeof(double) * (size_t)g.n);
    const int64_t t4 = now_ns();
    ctx->dropin_ns[12] += t1 - t0;
    ctx->dropin_ns[13] += t2 - t1;
    ctx->dropin_ns[14] += t3 - t2;
    ctx->dropin_ns[15] += t4 - t3;
    if (nearest_out && g.P) std::memcpy(nearest_out, ctx->h_best_i, sizeof(int) * (size_t)g.P);
    return TD_OK;
}

}  // namespace tdstar

using namespace tdstar;

namespace {

void free_ctx(td_ctx *c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    shadow_free(c);
    c->timer.release();
    void *dev[] = {c->g.px, c->g.py, c->g.pz, c->g.w, c->g.ray_off, c->g.tS, c->g.sig, c->g.terms, c->cells,
                   c->nn.part_d, c->nn.part_i, c->best_i, c->best_d, c->zeta0, c->phi,
                   c->q, c->q_i, c->q_z, c->chain_desc, c->draws, c->nn.g_count, c->nn.g_ent, c->raster, c->raster_i, c->raster_off,
                   c->mf_dev};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    void *host[] = {c->h_cells, c->h_out, c->h_best_i, c->h_q, c->h_q_i, c->h_q_z, c->h_chain_desc, c->mf_host,
                    c->h_raster};
    for (void *p : host)
        if (p) (void)hipHostFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int64_t leading_non_nan(const double *a, int64_t len) {
    for (int64_t k = 0; k < len; ++k)
        if (std::isnan(a[k])) return k;
    return len;
}

}  // namespace

extern "C" {

const char *td_last_error(const td_ctx *ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int td_create(td_ctx **out, int device, const double *rayX, const double *rayY, const double *rayZ,
              const double *rayL, const double *rayU, int64_t m, int64_t n, const double *tS,
              const double *allSig) {
    if (!out) return set_err(nullptr, TD_ERR_ARG, "td_create: out is NULL");
    *out = nullptr;
    if (m < 1 || n < 0) return set_err(nullptr, TD_ERR_ARG, "td_create: need m >= 1 and n >= 0");
    if (n > 0 && (!rayX || !rayY || !rayZ || !tS || !allSig || (m > 1 && (!rayL || !rayU))))
        return set_err(nullptr, TD_ERR_ARG, "td_create: NULL array");

    // ---- validate the NaN layout and build the CSR geometry on the host ----
    std::vector<int> off((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t np = leading_non_nan(rayX + i * m, m);                    // MCsub.jl:312-316
        const int64_t nl = m > 1 ? leading_non_nan(rayL + i * (m - 1), m - 1) : 0;  // MCsub.jl:150
        const int64_t want = np > 0 ? np - 1 : 0;
        if (nl != want) {
            char buf[200];
            std::snprintf(buf, sizeof buf,
                          "td_create: ray %lld has %lld points but %lld leading non-NaN rayL entries "
                          "(expected %lld; Julia would throw DimensionMismatch)",
                          (long long)(i + 1), (long long)np, (long long)nl, (long long)want);
            return set_err(nullptr, TD_ERR_LAYOUT, buf);
        }
        off[(size_t)i + 1] = off[(size_t)i] + (int)np;
        if ((int64_t)off[(size_t)i + 1] > (int64_t)0x7fffffff)
            return set_err(nullptr, TD_ERR_ARG, "td_create: more than 2^31 points");
    }
    const int64_t P = off[(size_t)n];
    std::vector<double> hx((size_t)P), hy((size_t)P), hz((size_t)P), hw((size_t)P, 0.0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t b = off[(size_t)i], np = off[(size_t)i + 1] - b;
        for (int64_t k = 0; k < np; ++k) {
            hx[(size_t)(b + k)] = rayX[i * m + k];
            hy[(size_t)(b + k)] = rayY[i * m + k];
            hz[(size_t)(b + k)] = rayZ[i * m + k];
            if (k + 1 < np)  // (rayl .* rayu)[k]: first product of MCsub.jl:153/159
                hw[(size_t)(b + k)] = rayL[i * (m - 1) + k] * rayU[i * (m - 1) + k];
        }
    }

    td_ctx *c = new (std::nothrow) td_ctx();
    if (!c) return set_err(nullptr, TD_ERR_NOMEM, "td_create: out of host memory");
    auto fail = [&](int code) {
        g_err = c->err;
        free_ctx(c);
        return code;
    };
    hipError_t e;
    if (device < 0) {
        e = hipGetDevice(&device);
        if (e != hipSuccess) return fail(hip_err(c, e, "hipGetDevice"));
    }
    e = hipSetDevice(device);
    if (e != hipSuccess) return fail(hip_err(c, e, "hipSetDevice"));
    c->device = device;
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return fail(hip_err(c, e, "hipGetDeviceProperties"));
    c->num_cus = prop.multiProcessorCount;
    c->arch = prop.gcnArchName;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) return fail(hip_err(c, e, "hipStreamCreate"));

    c->g.m = m;
    c->g.n = n;
    c->g.P = P;
    c->ray_off_host = off;

    c->hx = hx;
    c->hy = hy;
    c->hz = hz;
    c->sig_host.assign(allSig ? allSig : nullptr, allSig ? allSig + n : nullptr);
    c->tS_host.assign(tS ? tS : nullptr, tS ? tS + n : nullptr);
    c->likelihood = likelihood_constant(c->sig_host.data(), n);

    auto dalloc = [&](void **p, size_t bytes, const char *what) -> int {
        hipError_t er = hipMalloc(p, bytes ? bytes : 8);
        return er == hipSuccess ? TD_OK : hip_err(c, er, what);
    };
    const size_t Pb = sizeof(double) * (size_t)(P > 0 ? P : 1);
    const size_t nb = sizeof(double) * (size_t)(n > 0 ? n : 1);
    int rc = TD_OK;
    rc = rc ? rc : dalloc((void **)&c->g.px, Pb, "hipMalloc(px)");
    rc = rc ? rc : dalloc((void **)&c->g.py, Pb, "hipMalloc(py)");
    rc = rc ? rc : dalloc((void **)&c->g.pz, Pb, "hipMalloc(pz)");
    rc = rc ? rc : dalloc((void **)&c->g.w, Pb, "hipMalloc(w)");
    rc = rc ? rc : dalloc((void **)&c->g.ray_off, sizeof(int) * (size_t)(n + 1), "hipMalloc(ray_off)");
    rc = rc ? rc : dalloc((void **)&c->g.tS, nb, "hipMalloc(tS)");
    rc = rc ? rc : dalloc((void **)&c->g.sig, nb, "hipMalloc(sig)");
    rc = rc ? rc : dalloc((void **)&c->g.terms, nb, "hipMalloc(terms)");
    rc = rc ? rc : dalloc((void **)&c->best_i, sizeof(int) * (size_t)(P > 0 ? P : 1), "hipMalloc(best_i)");
    rc = rc ? rc : dalloc((void **)&c->best_d, Pb, "hipMalloc(best_d)");
    rc = rc ? rc : dalloc((void **)&c->zeta0, Pb, "hipMalloc(zeta0)");
    // [phi, ptS[n]] adjacent: one copy back per evaluate
    rc = rc ? rc : dalloc((void **)&c->phi, sizeof(double) * (size_t)(n + 1), "hipMalloc(phi, ptS)");
    if (!rc) c->ptS = c->phi + 1;
    if (rc) return fail(rc);
    e = hipHostMalloc(&c->h_out, sizeof(double) * (size_t)(n + 1), hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return fail(hip_err(c, e, "hipHostMalloc(out)"));
    e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->h_out_dev), c->h_out, 0);
    if (e != hipSuccess) return fail(hip_err(c, e, "hipHostGetDevicePointer(out)"));
    e = hipHostMalloc(&c->h_best_i, sizeof(int) * (size_t)(P > 0 ? P : 1), hipHostMallocDefault);
    if (e != hipSuccess) return fail(hip_err(c, e, "hipHostMalloc(best_i)"));

    struct Up { void *d; const void *h; size_t b; } ups[] = {
        {c->g.px, hx.data(), sizeof(double) * (size_t)P}, {c->g.py, hy.data(), sizeof(double) * (size_t)P},
        {c->g.pz, hz.data(), sizeof(double) * (size_t)P}, {c->g.w, hw.data(), sizeof(double) * (size_t)P},
        {c->g.ray_off, off.data(), sizeof(int) * (size_t)(n + 1)},
        {c->g.tS, tS, sizeof(double) * (size_t)n}, {c->g.sig, allSig, sizeof(double) * (size_t)n}};
    for (auto &u : ups)
        if (u.b) {
            e = hipMemcpy(u.d, u.h, u.b, hipMemcpyHostToDevice);
            if (e != hipSuccess) return fail(hip_err(c, e, "hipMemcpy(geometry)"));
        }
    rc = ensure_cells(c, 256);
    if (rc) return fail(rc);
    *out = c;
    return TD_OK;
}

int td_destroy(td_ctx *ctx) {
    free_ctx(ctx);
    return TD_OK;
}

int td_get_info(const td_ctx *ctx, td_info *info) {
    if (!ctx || !info) return set_err(const_cast<td_ctx *>(ctx), TD_ERR_ARG, "td_get_info: NULL");
    std::memset(info, 0, sizeof *info);
    info->abi_version = TDSTAR_ABI_VERSION;
    info->device = ctx->device;
    info->m = ctx->g.m;
    info->n = ctx->g.n;
    info->npoints = ctx->g.P;
    int64_t nonempty = 0;
    for (int64_t i = 0; i < ctx->g.n; ++i) nonempty += ctx->ray_off_host[(size_t)i + 1] > ctx->ray_off_host[(size_t)i];
    info->nsegments = ctx->g.P - nonempty;
    info->likelihood = ctx->likelihood;
    std::snprintf(info->arch, sizeof info->arch, "%s", ctx->arch.c_str());
    info->num_cus = ctx->num_cus;
    return TD_OK;
}

int td_set_sigma(td_ctx *ctx, const double *allSig) {
    if (!ctx || (!allSig && ctx->g.n > 0)) return set_err(ctx, TD_ERR_ARG, "td_set_sigma: NULL");
    TD_HIP(ctx, hipSetDevice(ctx->device));
    servers_quiesce(nullptr);
    shadow_free(ctx);  // the shadow chain's chi^2 terms were for the old sigma
    ctx->sig_host.assign(allSig, allSig + ctx->g.n);
    ctx->likelihood = likelihood_constant(allSig, ctx->g.n);
    if (ctx->g.n)
        TD_HIP(ctx, hipMemcpy(ctx->g.sig, allSig, sizeof(double) * (size_t)ctx->g.n, hipMemcpyHostToDevice));
    return TD_OK;
}

int td_misfit(td_ctx *ctx, int64_t n, const double *ptS, const double *tS, const double *allSig, double *phi_out,
              double *likelihood_out) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_misfit: ctx is NULL");
    if (n < 0 || n > 0x7fffffff || (n > 0 && (!ptS || !tS || !allSig)))
        return set_err(ctx, TD_ERR_ARG, "td_misfit: bad arrays");
    if (n == 0) {
        if (phi_out) *phi_out = 0.0;  // MCsub.jl:169 C = 0
        if (likelihood_out) *likelihood_out = 0.0;
        return TD_OK;
    }
    TD_HIP(ctx, hipSetDevice(ctx->device));
    servers_quiesce(nullptr);
    if (n > ctx->mf_cap) {
        if (ctx->mf_dev) (void)hipFree(ctx->mf_dev);
        if (ctx->mf_host) (void)hipHostFree(ctx->mf_host);
        ctx->mf_dev = ctx->mf_host = nullptr;
        ctx->mf_cap = 0;
        ctx->mf_tS.clear();
        ctx->mf_sig.clear();
        TD_HIP(ctx, hipMalloc(&ctx->mf_dev, sizeof(double) * (4 * (size_t)n + 1)));
        TD_HIP(ctx, hipHostMalloc(&ctx->mf_host, sizeof(double) * ((size_t)n + 1)));
        ctx->mf_cap = n;
    }
    double *d_ptS = ctx->mf_dev, *d_tS = d_ptS + n, *d_sig = d_tS + n, *d_terms = d_sig + n, *d_phi = d_terms + n;
    // tS / sigma of a sharded run are the same every call: copied only when they change
    const bool same = (int64_t)ctx->mf_tS.size() == n &&
                      std::memcmp(ctx->mf_tS.data(), tS, sizeof(double) * (size_t)n) == 0 &&
                      std::memcmp(ctx->mf_sig.data(), allSig, sizeof(double) * (size_t)n) == 0;
    if (!same) {
        ctx->mf_tS.assign(tS, tS + n);
        ctx->mf_sig.assign(allSig, allSig + n);
        ctx->mf_likelihood = likelihood_constant(allSig, n);
        TD_HIP(ctx, hipMemcpyAsync(d_tS, tS, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
        TD_HIP(ctx, hipMemcpyAsync(d_sig, allSig, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    }
    std::memcpy(ctx->mf_host, ptS, sizeof(double) * (size_t)n);
    TD_HIP(ctx, hipMemcpyAsync(d_ptS, ctx->mf_host, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    hipError_t e = launch_chi2(d_ptS, d_tS, d_sig, (int)n, d_terms, d_phi, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->mf_host + n, d_phi, sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_err(ctx, e, "td_misfit");
    if (phi_out) *phi_out = ctx->mf_host[n];
    if (likelihood_out) *likelihood_out = ctx->mf_likelihood;  // MCsub.jl:179-182
    return TD_OK;
}

int td_evaluate(td_ctx *ctx, const double *xCell, const double *yCell, const double *zCell,
                const double *zeta, int64_t nCells, int debug_prior, double *ptS_out, double *phi_out,
                double *likelihood_out, int32_t *nearest_out) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_evaluate: ctx is NULL");
    if (debug_prior == 1) {  // MCsub.jl:128-136
        if (phi_out) *phi_out = 1.0;
        if (likelihood_out) *likelihood_out = 1.0;
        return TD_OK;
    }
    if (nCells < 0 || (nCells > 0 && (!xCell || !yCell || !zCell || !zeta)))
        return set_err(ctx, TD_ERR_ARG, "td_evaluate: bad cell arrays");
    if (nCells > 0x7fffffff) return set_err(ctx, TD_ERR_ARG, "td_evaluate: too many cells");
    const int64_t t0 = now_ns();
    TD_HIP(ctx, hipSetDevice(ctx->device));
    servers_quiesce((nearest_out || !ctx->incremental) ? nullptr : shadow_chain_of(ctx));
    int rc = (nearest_out || !ctx->incremental)
                 ? evaluate_full(ctx, xCell, yCell, zCell, zeta, nCells, ptS_out, phi_out, nearest_out)
                 : evaluate_incremental(ctx, xCell, yCell, zCell, zeta, nCells, ptS_out, phi_out);
    ctx->dropin_ns[0] += now_ns() - t0;
    ctx->dropin_ns[6] += 1;
    if (rc) return rc;
    if (likelihood_out) *likelihood_out = ctx->likelihood;  // MCsub.jl:179-182: model-independent
    return TD_OK;
}

int td_evaluate_batch(td_ctx *ctx, int64_t nmodels, const int64_t *cell_off, const double *xCell,
                      const double *yCell, const double *zCell, const double *zeta, double *ptS_out,
                      double *phi_out, double *likelihood_out) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_evaluate_batch: ctx is NULL");
    if (nmodels < 0 || (nmodels > 0 && !cell_off)) return set_err(ctx, TD_ERR_ARG, "td_evaluate_batch: bad offsets");
    for (int64_t k = 0; k < nmodels; ++k) {
        const int64_t a = cell_off[k], b = cell_off[k + 1];
        if (b < a || a < 0) return set_err(ctx, TD_ERR_ARG, "td_evaluate_batch: offsets not monotone");
        if (b > a && (!xCell || !yCell || !zCell || !zeta))
            return set_err(ctx, TD_ERR_ARG, "td_evaluate_batch: bad cell arrays");
        TD_HIP(ctx, hipSetDevice(ctx->device));
        servers_quiesce(nullptr);
        // independent models: the full evaluate (no shadow chain)
        int rc = evaluate_full(ctx, xCell + a, yCell + a, zCell + a, zeta + a, b - a,
                               ptS_out ? ptS_out + k * ctx->g.n : nullptr, phi_out ? phi_out + k : nullptr);
        if (rc) return rc;
        if (likelihood_out) likelihood_out[k] = ctx->likelihood;
    }
    return TD_OK;
}

int td_interpolate(td_ctx *ctx, const double *xCell, const double *yCell, const double *zCell,
                   const double *zeta, int64_t nCells, const double *X, int64_t nx, const double *Y,
                   int64_t ny, const double *Z, int64_t nz, double *zeta_out, int32_t *nearest_out,
                   int64_t *npoints_out) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_interpolate: ctx is NULL");
    if (nx < 0 || (nx > 0 && (!X || !Y || !Z || !zeta_out)) || nCells < 0 ||
        (nCells > 0 && (!xCell || !yCell || !zCell || !zeta)))
        return set_err(ctx, TD_ERR_ARG, "td_interpolate: bad arguments");
    const int64_t np = leading_non_nan(X, nx);  // MCsub.jl:312-316
    if (npoints_out) *npoints_out = np;
    if ((ny != 1 && ny < np) || (nz != 1 && nz < np))
        return set_err(ctx, TD_ERR_BOUNDS, "td_interpolate: Y/Z shorter than npoints (Julia BoundsError)");
    if (np == 0) return TD_OK;
    TD_HIP(ctx, hipSetDevice(ctx->device));
    if (np == 1 && !nearest_out && ctx->incremental && nCells > 0) {  // a chain's 1-point query (:81, :146)
        const int64_t t0 = now_ns();
        servers_quiesce(shadow_chain_of(ctx));
        int handled = 0;
        int rc = interpolate_incremental(ctx, xCell, yCell, zCell, zeta, nCells, X[0], Y[0], Z[0], zeta_out, &handled);
        ctx->dropin_ns[3] += now_ns() - t0;
        ctx->dropin_ns[7] += 1;
        if (rc) return rc;
        if (handled) return TD_OK;
    }
    servers_quiesce(nullptr);
    if (np > ctx->q_cap) {
        void *dev[] = {ctx->q, ctx->q_i, ctx->q_z};
        for (void *p : dev)
            if (p) (void)hipFree(p);
        void *host[] = {ctx->h_q, ctx->h_q_i, ctx->h_q_z};
        for (void *p : host)
            if (p) (void)hipHostFree(p);
        ctx->q = ctx->h_q = ctx->q_z = ctx->h_q_z = nullptr;
        ctx->q_i = ctx->h_q_i = nullptr;
        ctx->q_cap = 0;
        int64_t cap = 64;
        while (cap < np) cap *= 2;
        TD_HIP(ctx, hipMalloc(&ctx->q, sizeof(double) * 3 * (size_t)cap));
        TD_HIP(ctx, hipMalloc(&ctx->q_i, sizeof(int) * (size_t)cap));
        TD_HIP(ctx, hipMalloc(&ctx->q_z, sizeof(double) * (size_t)cap));
        TD_HIP(ctx, hipHostMalloc(&ctx->h_q, sizeof(double) * 3 * (size_t)cap, hipHostMallocDefault));
        TD_HIP(ctx, hipHostMalloc(&ctx->h_q_i, sizeof(int) * (size_t)cap, hipHostMallocDefault));
        TD_HIP(ctx, hipHostMalloc(&ctx->h_q_z, sizeof(double) * (size_t)cap, hipHostMallocDefault));
        ctx->q_cap = cap;
    }
    const int64_t qc = ctx->q_cap;
    std::memcpy(ctx->h_q, X, sizeof(double) * (size_t)np);
    std::memcpy(ctx->h_q + qc, Y, sizeof(double) * (size_t)(ny == 1 ? 1 : np));
    std::memcpy(ctx->h_q + 2 * qc, Z, sizeof(double) * (size_t)(nz == 1 ? 1 : np));
    TD_HIP(ctx, hipMemcpyAsync(ctx->q, ctx->h_q, sizeof(double) * 3 * (size_t)qc, hipMemcpyHostToDevice, ctx->stream));
    int rc = upload_cells(ctx, xCell, yCell, zCell, zeta, nCells);
    if (rc) return rc;
    hipError_t e = nearest_uploaded(ctx, ctx->q, ctx->q + qc, ctx->q + 2 * qc, np, ny == 1 ? 0 : 1,
                                    nz == 1 ? 0 : 1, nCells, ctx->q_i, nullptr, ctx->q_z);
    if (e != hipSuccess) return hip_err(ctx, e, "nearest kernels");
    TD_HIP(ctx, hipMemcpyAsync(ctx->h_q_z, ctx->q_z, sizeof(double) * (size_t)np, hipMemcpyDeviceToHost, ctx->stream));
    if (nearest_out)
        TD_HIP(ctx, hipMemcpyAsync(ctx->h_q_i, ctx->q_i, sizeof(int) * (size_t)np, hipMemcpyDeviceToHost, ctx->stream));
    TD_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(zeta_out, ctx->h_q_z, sizeof(double) * (size_t)np);
    if (nearest_out) std::memcpy(nearest_out, ctx->h_q_i, sizeof(int) * (size_t)np);
    return TD_OK;
}

int tdt_exact_sum(int device, const double *term, int64_t cnt, double C0, double *prefix, double *C_end,
                  int *fast) {
    if (!term || !prefix || !C_end || !fast || cnt < 1 || cnt > (1 << 24)) return TD_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return TD_ERR_HIP;
    const size_t nb = sizeof(double) * (size_t)cnt;
    void *buf = nullptr;
    if (hipMalloc(&buf, 2 * nb + 2 * sizeof(double)) != hipSuccess) return TD_ERR_NOMEM;
    double *dt = static_cast<double *>(buf), *dp = dt + cnt, *de = dp + cnt;
    int *df = reinterpret_cast<int *>(de + 1);
    hipError_t e = hipMemcpy(dt, term, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = test_exact_sum(dt, (int)cnt, C0, dp, de, df);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(fast, df, sizeof(int), hipMemcpyDeviceToHost);
    if (e == hipSuccess && *fast) e = hipMemcpy(prefix, dp, nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess && *fast) e = hipMemcpy(C_end, de, sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    return e == hipSuccess ? TD_OK : TD_ERR_HIP;
}

int tdt_wave_seq_sum(int device, const double *term, int64_t cnt, double C0, double *prefix, double *C_end,
                     int *fallbacks) {
    if (!term || !prefix || !C_end || !fallbacks || cnt < 1 || cnt > (1 << 24)) return TD_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return TD_ERR_HIP;
    const size_t nb = sizeof(double) * (size_t)cnt;
    void *buf = nullptr;
    if (hipMalloc(&buf, 2 * nb + 2 * sizeof(double)) != hipSuccess) return TD_ERR_NOMEM;
    double *dt = static_cast<double *>(buf), *dp = dt + cnt, *de = dp + cnt;
    int *df = reinterpret_cast<int *>(de + 1);
    hipError_t e = hipMemcpy(dt, term, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = test_wave_seq_sum(dt, (int)cnt, C0, dp, de, df);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(prefix, dp, nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(C_end, de, sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(fallbacks, df, sizeof(int), hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    return e == hipSuccess ? TD_OK : TD_ERR_HIP;
}

int tdt_wave_delta_sum(int device, const double *term, const double *old_prefix, const int *changed, int64_t cnt,
                       double C0, double *prefix, double *C_end) {
    if (!term || !old_prefix || !changed || !prefix || !C_end || cnt < 1 || cnt > (1 << 24)) return TD_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return TD_ERR_HIP;
    const size_t nb = sizeof(double) * (size_t)cnt;
    void *buf = nullptr;
    if (hipMalloc(&buf, 3 * nb + sizeof(double) + sizeof(int) * (size_t)cnt) != hipSuccess) return TD_ERR_NOMEM;
    double *dt = static_cast<double *>(buf), *dold = dt + cnt, *dp = dold + cnt, *de = dp + cnt;
    int *dc = reinterpret_cast<int *>(de + 1);
    hipError_t e = hipMemcpy(dt, term, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dold, old_prefix, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dc, changed, sizeof(int) * (size_t)cnt, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = test_wave_delta_sum(dt, dold, dc, (int)cnt, C0, dp, de);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(prefix, dp, nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(C_end, de, sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    return e == hipSuccess ? TD_OK : TD_ERR_HIP;
}

int tdt_block_delta_sum(int device, const double *term, const double *term_old, const double *old_prefix,
                        const int *changed, int64_t k0, int64_t n, double *prefix, double *C_end, int64_t *events,
                        int *mask_ok) {
    if (!term || !term_old || !old_prefix || !changed || !prefix || !C_end || !events || !mask_ok || n < 1 ||
        n > 64 * 1024 || k0 < 0 || k0 > n)
        return TD_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return TD_ERR_HIP;
    const size_t nb = sizeof(double) * (size_t)n;
    void *buf = nullptr;
    if (hipMalloc(&buf, 4 * nb + 3 * sizeof(double) + sizeof(int) * (size_t)n) != hipSuccess) return TD_ERR_NOMEM;
    double *dt = static_cast<double *>(buf), *dto = dt + n, *dold = dto + n, *dcp = dold + n, *de = dcp + n;
    long long *dev = reinterpret_cast<long long *>(de + 1);
    int *dok = reinterpret_cast<int *>(de + 2);
    int *dc = reinterpret_cast<int *>(de + 3);
    hipError_t e = hipMemcpy(dt, term, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dto, term_old, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dold, old_prefix, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dc, changed, sizeof(int) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(dcp, 0xff, nb);  // NaN: a COPY segment that was not written shows
    if (e == hipSuccess) e = test_block_delta(dt, dto, dold, dc, (int)k0, (int)n, dcp, de, dev, dok);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(prefix, dold, nb, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(C_end, de, sizeof(double), hipMemcpyDeviceToHost);
    long long ev = 0;
    if (e == hipSuccess) e = hipMemcpy(&ev, dev, sizeof(long long), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(mask_ok, dok, sizeof(int), hipMemcpyDeviceToHost);
    *events = ev;
    (void)hipFree(buf);
    return e == hipSuccess ? TD_OK : TD_ERR_HIP;
}

int tdt_chi2(td_ctx *ctx, const double *ptS, int path, double out[2]) {
    if (!ctx || !out || (!ptS && ctx->g.n > 0) || path < 0 || path > 3) return set_err(ctx, TD_ERR_ARG, "tdt_chi2");
    const int64_t n = ctx->g.n;
    if (n < 1 || n > 4096) return set_err(ctx, TD_ERR_ARG, "tdt_chi2: n out of range");
    if (path == 0) {  // td_evaluate's: the host's sequential sum
        out[0] = host_chi2(ptS, ctx->tS_host.data(), ctx->sig_host.data(), n);
        out[1] = 0.0;
        return TD_OK;
    }
    TD_HIP(ctx, hipSetDevice(ctx->device));
    double *dp = nullptr, *scratch = nullptr, *dout = nullptr;
    const size_t sn = 3 * (size_t)n + 8 + 1024 / sizeof(double);
    hipError_t e = hipMalloc(&dp, sizeof(double) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&scratch, sizeof(double) * sn);
    if (e == hipSuccess) e = hipMalloc(&dout, sizeof(double) * 2);
    if (e == hipSuccess) e = hipMemsetAsync(dout, 0, sizeof(double) * 2, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dp, ptS, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) {
        if (path == 1)
            e = test_chi2(dp, ctx->g.tS, ctx->g.sig, (int)n, scratch, dout, ctx->stream);
        else
            e = test_chain_chi2(dp, ctx->g.tS, ctx->g.sig, (int)n, path, scratch, dout, ctx->stream);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, sizeof(double) * 2, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (dp) (void)hipFree(dp);
    if (scratch) (void)hipFree(scratch);
    if (dout) (void)hipFree(dout);
    if (e != hipSuccess) return hip_err(ctx, e, "tdt_chi2");
    return TD_OK;
}

int tdt_nn_bench(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta, int64_t ncells,
                 int method, int reps, double *us_out) {
    if (!ctx || !us_out || reps < 1 || method < 1 || method > 3 || ncells < 1)
        return set_err(ctx, TD_ERR_ARG, "tdt_nn_bench");
    TD_HIP(ctx, hipSetDevice(ctx->device));
    const int old_m = ctx->nn_method, old_s = ctx->nn.method;
    ctx->nn_method = method == 2 ? 2 : 1;
    ctx->nn.method = method == 3 ? kNNSplit : kNNAuto;
    int rc = upload_cells(ctx, x, y, z, zeta, ncells);
    const auto &g = ctx->g;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipSuccess;
    if (!rc) {
        e = nearest_uploaded(ctx, g.px, g.py, g.pz, g.P, 1, 1, ncells, ctx->best_i, ctx->best_d, ctx->zeta0);  // warm
        if (e == hipSuccess) e = hipEventCreate(&e0);
        if (e == hipSuccess) e = hipEventCreate(&e1);
        if (e == hipSuccess) e = hipEventRecord(e0, ctx->stream);
        for (int k = 0; k < reps && e == hipSuccess; ++k) {
            if (method == 2) ctx->cells_stage = nullptr;  // grid: rebuilt from the device copy each time
            e = nearest_uploaded(ctx, g.px, g.py, g.pz, g.P, 1, 1, ncells, ctx->best_i, ctx->best_d, ctx->zeta0);
        }
        if (e == hipSuccess) e = hipEventRecord(e1, ctx->stream);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        *us_out = (double)ms * 1e3 / reps;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    ctx->nn_method = old_m;
    ctx->nn.method = old_s;
    if (rc) return rc;
    if (e != hipSuccess) return hip_err(ctx, e, "tdt_nn_bench");
    return TD_OK;
}

int td_set_incremental(td_ctx *ctx, int mode) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_set_incremental: ctx is NULL");
    if (mode < 0 || mode > 2) return set_err(ctx, TD_ERR_ARG, "td_set_incremental: mode must be 0, 1 or 2");
    if (mode != ctx->incremental) shadow_free(ctx);
    ctx->incremental = mode;
    return TD_OK;
}

int tdt_set_incremental(td_ctx *ctx, int on) { return td_set_incremental(ctx, on); }

int tdt_set_nn_method(td_ctx *ctx, int method) {
    if (!ctx || method < 0 || method > 3) return TD_ERR_ARG;
    ctx->nn_method = method == 3 ? 1 : method;  // 3: brute force through the split search
    ctx->nn.method = method == 3 ? kNNSplit : kNNAuto;
    return TD_OK;
}

int td_timing_enable(td_ctx *ctx, int enable) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_timing_enable: ctx is NULL");
    ctx->timer.on = enable != 0;
    return TD_OK;
}

int td_timing_reset(td_ctx *ctx) {
    if (!ctx) return set_err(nullptr, TD_ERR_ARG, "td_timing_reset: ctx is NULL");
    ctx->timer.reset();
    return TD_OK;
}

int td_timing_get(td_ctx *ctx, const char *kernel, int64_t *launches, double *total_ms) {
    if (!ctx || !kernel) return set_err(ctx, TD_ERR_ARG, "td_timing_get: NULL argument");
    hipError_t e = ctx->timer.collect();
    if (e != hipSuccess) return hip_err(ctx, e, "td_timing_get");
    auto it = ctx->timer.acc.find(kernel);
    if (launches) *launches = it == ctx->timer.acc.end() ? 0 : it->second.first;
    if (total_ms) *total_ms = it == ctx->timer.acc.end() ? 0.0 : it->second.second;
    return TD_OK;
}

}  // extern "C"
