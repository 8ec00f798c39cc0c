// nn_grid.hip -- nearest cell of many query points through a uniform bucket
// grid over the cells: the drop-in evaluate / Interpolation path for larger
// models (v_nearest, MCsub.jl:247-263, for every ray point).
//
// The answer is the reference's: the lexicographic minimum of (squared
// distance, cell index) over all cells, among distances below the 1e9
// sentinel -- v_nearest's strict '<' scan in index order keeps the FIRST
// minimum.  The grid only decides where to look:
//   k_grid_fill  one lane per cell: append {x, y, z, index} to its bucket
//                (kGridCap entries, the first two of every bucket side by side
//                -- grid_ent; a fuller bucket is flagged);
//   k_nn_grid    32 lanes per point, one per bucket of the 3x3x3 block
//                around it, DPP reduction; the answer counts only if it is
//                strictly closer than every face of the block
//                (grid_block_lb), i.e. than every cell outside, and no bucket
//                of the block overflowed -- else the 5x5x5 block, else (rare)
//                the same 32 lanes scan every cell;
//   k_nn_grid4   the same search with 4 lanes per point (7 buckets each), for
//                large point sets (>= 65536: the stress geometry, 254 -> 172 us
//                at 584k points x 20k cells); the half-wave form keeps the
//                small sets, where more waves and a wider fallback win.
// Two launches per search: the bucket counts come in two sets used by
// alternate searches, and each search's k_nn_grid zeroes the other set for
// the next one (no memset, no third kernel).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>

#include "internal.h"
#include "wave_ops.h"

namespace tdstar {

namespace {

__device__ __forceinline__ double dist2_q(double cx, double cy, double cz, double x, double y, double z) {
    // (mx-x)^2 + (my-y)^2 + (mz-z)^2, MCsub.jl:254, left to right, unfused
    const double dx = cx - x, dy = cy - y, dz = cz - z;
    double d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

// lexicographic (distance, index) update; distances >= the sentinel never count
__device__ __forceinline__ void take(double d, int i, double &bd, int &bi) {
    if (d < bd || (d == bd && d < kSentinel && i < bi)) {
        bd = d;
        bi = i;
    }
}

// Entry k of bucket b: the first kGridHead entries of every bucket sit together, densely (a bucket
// holds ~2 cells, so a search's one round of loads reads 64 B per bucket and two buckets share a
// 128-B line), the rest in a per-bucket overflow area after them.  nb = the grid's bucket count.
constexpr int kGridHead = 2;
__device__ __forceinline__ long grid_ent(long b, int k, long nb) {
    return k < kGridHead ? b * kGridHead + k : nb * kGridHead + b * kGridCap + k;
}

__global__ __launch_bounds__(256) void k_grid_fill(double *__restrict__ cells, const double *__restrict__ stage,
                                                   int stride, int ncells, CellGrid G, int *__restrict__ count,
                                                   BucketEntry *__restrict__ ent) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncells) return;
    double x, y, z;
    if (stage) {  // the cells straight from pinned host memory, and the device copy on the way
        x = stage[i];
        y = stage[stride + i];
        z = stage[2 * stride + i];
        const double ze = stage[3 * stride + i];
        cells[i] = x;
        cells[stride + i] = y;
        cells[2 * stride + i] = z;
        cells[3 * stride + i] = ze;
    } else {
        x = cells[i];
        y = cells[stride + i];
        z = cells[2 * stride + i];
    }
    const int b = grid_bucket(G, x, y, z);
    const int pos = atomicAdd(&count[b], 1);  // order inside a bucket does not matter
    if (pos < kGridCap) ent[grid_ent(b, pos, (long)G.gx * G.gy * G.gz)] = BucketEntry{x, y, z, i, 0};
}

// lexicographic min of (d, i) over each half-wave (32 lanes), to every lane
__device__ __forceinline__ void half_min(double &d, int &i) {
    unsigned long long k = (unsigned long long)__double_as_longlong(d);
    constexpr unsigned long long I = ~0ull;
    k = umin64(k, dpp_u64<0x111, 0xf>(k, I));
    k = umin64(k, dpp_u64<0x112, 0xf>(k, I));
    k = umin64(k, dpp_u64<0x114, 0xf>(k, I));
    k = umin64(k, dpp_u64<0x118, 0xf>(k, I));
    k = umin64(k, dpp_u64<0x142, 0xa>(k, I));  // row_bcast:15 -> lanes 31, 63: half minima
    const int src = (threadIdx.x & 32) | 31;
    const unsigned long long km = (unsigned long long)__shfl(k, src, 64);
    const bool at = (unsigned long long)__double_as_longlong(d) == km;
    unsigned long long r = at ? (unsigned long long)(unsigned)i : I;
    r = umin64(r, dpp_u64<0x111, 0xf>(r, I));
    r = umin64(r, dpp_u64<0x112, 0xf>(r, I));
    r = umin64(r, dpp_u64<0x114, 0xf>(r, I));
    r = umin64(r, dpp_u64<0x118, 0xf>(r, I));
    r = umin64(r, dpp_u64<0x142, 0xa>(r, I));
    const unsigned long long rm = (unsigned long long)__shfl(r, src, 64);
    d = __longlong_as_double((long long)km);
    i = rm == I ? INT_MAX : (int)rm;
}

__global__ __launch_bounds__(256) void k_nn_grid(const double *__restrict__ qx, const double *__restrict__ qy,
                                                 const double *__restrict__ qz, int npts, int ys, int zs, CellGrid G,
                                                 const int *__restrict__ count, const BucketEntry *__restrict__ ent,
                                                 const double *__restrict__ cells, int stride, int ncells,
                                                 int *__restrict__ best_i, double *__restrict__ best_d,
                                                 double *__restrict__ zeta0, int *__restrict__ other_count,
                                                 int other_nb) {
    // the other set of bucket counts (the previous search's) is zeroed for the next search
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < other_nb; b += gridDim.x * blockDim.x) other_count[b] = 0;
    const int hl = threadIdx.x & 31;                             // lane in the half-wave
    const int p = (blockIdx.x * blockDim.x + threadIdx.x) >> 5;  // one point per half-wave
    const int pc = min(p, npts - 1);                              // whole half-waves stay for the DPP
    const double x = qx[pc], y = qy[(long)pc * ys], z = qz[(long)pc * zs];
    const int bi = grid_axis(x, G.x0, G.ix, G.gx), bj = grid_axis(y, G.y0, G.iy, G.gy),
              bk = grid_axis(z, G.z0, G.iz, G.gz);
    const double *zeta_cells = cells + 3 * (long)stride;
    const long nbk_all = (long)G.gx * G.gy * G.gz;
    double bd = kSentinel;
    int bx = INT_MAX;
    bool proven = false;
    // the 3x3x3 block (one bucket per lane), then the 5x5x5 one (four per lane)
    for (int R = 1; R <= 2 && !proven; ++R) {
        const int W = 2 * R + 1, nbk = W * W * W;
        const double lb = grid_block_lb(G, x, y, z, R);  // independent of the loads: computed while they fly
        bd = kSentinel;
        bx = INT_MAX;
        bool over = false;
        for (int t = hl; t < nbk; t += 32) {
            const int ii = bi + t % W - R, jj = bj + (t / W) % W - R, kk = bk + t / (W * W) - R;
            const bool inb = ii >= 0 && ii < G.gx && jj >= 0 && jj < G.gy && kk >= 0 && kk < G.gz;
            const long b = inb ? ((long)kk * G.gy + jj) * G.gx + ii : 0;
            // one round of loads: the count and the first two entries
            const int cnt = inb ? count[b] : 0;
            const BucketEntry e0 = ent[grid_ent(b, 0, nbk_all)], e1 = ent[grid_ent(b, 1, nbk_all)];
            if (cnt > 0) take(dist2_q(e0.x, e0.y, e0.z, x, y, z), e0.slot, bd, bx);
            if (cnt > 1) take(dist2_q(e1.x, e1.y, e1.z, x, y, z), e1.slot, bd, bx);
            for (int k = 2; k < min(cnt, kGridCap); ++k) {
                const BucketEntry e = ent[grid_ent(b, k, nbk_all)];
                take(dist2_q(e.x, e.y, e.z, x, y, z), e.slot, bd, bx);
            }
            over = over || cnt > kGridCap;
        }
        half_min(bd, bx);
        const unsigned long long ov = __ballot(over);
        const bool any_over = ((ov >> (threadIdx.x & 32)) & 0xffffffffull) != 0ull;
        proven = !any_over && bd < lb;  // nothing outside can tie or win
    }
    if (!proven) {  // rare: every cell, the same half-wave (index order inside each lane)
        bd = kSentinel;
        bx = INT_MAX;
        for (int j = hl; j < ncells; j += 32)
            take(dist2_q(cells[j], cells[stride + j], cells[2 * (long)stride + j], x, y, z), j, bd, bx);
        half_min(bd, bx);
    }
    if (hl == 0 && p < npts) {
        const bool found = bd < kSentinel;
        if (best_i) best_i[p] = found ? bx : -1;
        if (best_d) best_d[p] = bd;
        if (zeta0) zeta0[p] = found ? zeta_cells[bx] : 0.0;  // MCsub.jl:249
    }
}


// lexicographic min of (d, i) over each quad of lanes (4 lanes per point), to every lane of the quad
__device__ __forceinline__ void quad_lexmin(double &d, int &i) {
    constexpr unsigned long long I = ~0ull;
    unsigned long long k = (unsigned long long)__double_as_longlong(d);
    k = umin64(k, dpp_u64<0xB1, 0xf>(k, I));  // quad_perm [1,0,3,2]
    k = umin64(k, dpp_u64<0x4E, 0xf>(k, I));  // quad_perm [2,3,0,1]
    const bool at = (unsigned long long)__double_as_longlong(d) == k;
    unsigned long long r = at ? (unsigned long long)(unsigned)i : I;
    r = umin64(r, dpp_u64<0xB1, 0xf>(r, I));
    r = umin64(r, dpp_u64<0x4E, 0xf>(r, I));
    d = __longlong_as_double((long long)k);
    i = r == I ? INT_MAX : (int)r;
}

// lexicographic min of (d, i) over the wave, to every lane
__device__ __forceinline__ void wave_lexmin(double &d, int &i) {
    const unsigned long long kd = wave_min_u64((unsigned long long)__double_as_longlong(d));
    const bool at = (unsigned long long)__double_as_longlong(d) == kd;
    const unsigned long long ki = wave_min_u64(at ? (unsigned long long)(unsigned)i : ~0ull);
    d = __longlong_as_double((long long)kd);
    i = ki == ~0ull ? INT_MAX : (int)ki;
}

// k_nn_grid with FOUR lanes per point (16 points per wave), for large point
// sets (the stress geometry: the half-wave form spends ~200 wave-instructions
// per point on reductions and the proof, these ~4x fewer).  Lane s of a quad
// takes the buckets s, s + 4, ... of the 3x3x3 block (6 or 7): their counts
// and first entries in one round of loads, then entry k of every bucket
// holding more than k, one round each; then the quad's minimum.  A point the
// block does not prove (rare) is finished by the whole wave, one point at a
// time: the 5x5x5 block (two buckets per lane), else every cell.
constexpr int kGridLpp = 4;
constexpr int64_t kGridQuadMinPts = 65536;  // below: the half-wave kernel (more waves, shorter chains)
__global__ __launch_bounds__(256) void k_nn_grid4(const double *__restrict__ qx, const double *__restrict__ qy,
                                                  const double *__restrict__ qz, int npts, int ys, int zs, CellGrid G,
                                                  const int *__restrict__ count, const BucketEntry *__restrict__ ent,
                                                  const double *__restrict__ cells, int stride, int ncells,
                                                  int *__restrict__ best_i, double *__restrict__ best_d,
                                                  double *__restrict__ zeta0, int *__restrict__ other_count,
                                                  int other_nb) {
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < other_nb; b += gridDim.x * blockDim.x) other_count[b] = 0;
    const int lane = threadIdx.x & 63, sub = threadIdx.x & (kGridLpp - 1);
    const int p = (blockIdx.x * blockDim.x + threadIdx.x) / kGridLpp;  // whole quads stay for the DPP
    const int pc = min(p, npts - 1);
    const double x = qx[pc], y = qy[(long)pc * ys], z = qz[(long)pc * zs];
    const int bi = grid_axis(x, G.x0, G.ix, G.gx), bj = grid_axis(y, G.y0, G.iy, G.gy),
              bk = grid_axis(z, G.z0, G.iz, G.gz);
    constexpr int kMine = (27 + kGridLpp - 1) / kGridLpp;
    const long nbk_all = (long)G.gx * G.gy * G.gz;
    int bb[kMine], cnt[kMine];
    BucketEntry e[kMine];
    bool over = false;
    int most = 0;
#pragma unroll
    for (int u = 0; u < kMine; ++u) {  // counts and first entries: one round of loads
        const int t = sub + u * kGridLpp;
        const int ii = bi + t % 3 - 1, jj = bj + (t / 3) % 3 - 1, kk = bk + t / 9 - 1;
        const bool inb = t < 27 && ii >= 0 && ii < G.gx && jj >= 0 && jj < G.gy && kk >= 0 && kk < G.gz;
        bb[u] = inb ? (kk * G.gy + jj) * G.gx + ii : 0;
        cnt[u] = inb ? count[bb[u]] : 0;
        e[u] = ent[grid_ent(bb[u], 0, nbk_all)];
    }
    const double lb = grid_block_lb(G, x, y, z, 1);  // independent of the loads: computed while they fly
    double bd = kSentinel;
    int bx = INT_MAX;
#pragma unroll
    for (int u = 0; u < kMine; ++u) {
        over = over || cnt[u] > kGridCap;
        cnt[u] = min(cnt[u], kGridCap);
        most = max(most, cnt[u]);
        if (cnt[u] > 0) take(dist2_q(e[u].x, e[u].y, e[u].z, x, y, z), e[u].slot, bd, bx);
    }
    for (int k = 1; k < most; ++k) {  // entry k of each of my buckets: one round of loads
#pragma unroll
        for (int u = 0; u < kMine; ++u)
            if (k < cnt[u]) e[u] = ent[grid_ent(bb[u], k, nbk_all)];
#pragma unroll
        for (int u = 0; u < kMine; ++u)
            if (k < cnt[u]) take(dist2_q(e[u].x, e[u].y, e[u].z, x, y, z), e[u].slot, bd, bx);
    }
    quad_lexmin(bd, bx);
    const int qsh = lane & ~(kGridLpp - 1);  // first lane of my quad
    const bool any_over = ((__ballot(over) >> qsh) & 0xfull) != 0ull;
    const bool proven = p >= npts || (!any_over && bd < lb);
    // points the block does not prove: the whole wave, one at a time
    unsigned long long need = __ballot(!proven && sub == 0);
    while (need) {
        const int src = __builtin_ctzll(need);
        need &= need - 1;
        const double px = readlane_f64(x, src), py = readlane_f64(y, src), pz = readlane_f64(z, src);
        const int ci = __builtin_amdgcn_readlane(bi, src), cj = __builtin_amdgcn_readlane(bj, src),
                  ck = __builtin_amdgcn_readlane(bk, src);
        double d2 = kSentinel;
        int i2 = INT_MAX;
        bool over2 = false;
        for (int t = lane; t < 125; t += 64) {  // the 5x5x5 block
            const int ii = ci + t % 5 - 2, jj = cj + (t / 5) % 5 - 2, kk = ck + t / 25 - 2;
            if (ii < 0 || ii >= G.gx || jj < 0 || jj >= G.gy || kk < 0 || kk >= G.gz) continue;
            const int b = (kk * G.gy + jj) * G.gx + ii;
            const int c = count[b];
            over2 = over2 || c > kGridCap;
            for (int k = 0; k < min(c, kGridCap); ++k) {
                const BucketEntry f = ent[grid_ent(b, k, nbk_all)];
                take(dist2_q(f.x, f.y, f.z, px, py, pz), f.slot, d2, i2);
            }
        }
        wave_lexmin(d2, i2);
        if (__ballot(over2) != 0ull || !(d2 < grid_block_lb(G, px, py, pz, 2))) {  // rare: every cell
            d2 = kSentinel;
            i2 = INT_MAX;
            for (int j = lane; j < ncells; j += 64)
                take(dist2_q(cells[j], cells[stride + j], cells[2 * (long)stride + j], px, py, pz), j, d2, i2);
            wave_lexmin(d2, i2);
        }
        if (qsh == src) {
            bd = d2;
            bx = i2;
        }
    }
    if (sub == 0 && p < npts) {
        const bool found = bd < kSentinel;
        if (best_i) best_i[p] = found ? bx : -1;
        if (best_d) best_d[p] = bd;
        if (zeta0) zeta0[p] = found ? cells[3 * (long)stride + bx] : 0.0;  // MCsub.jl:249
    }
}

}  // namespace

hipError_t launch_nearest_grid(const double *qx, const double *qy, const double *qz, int64_t npts,
                               int64_t qy_stride, int64_t qz_stride, double *cells, int64_t stride,
                               int64_t ncells, const CellGrid &G, NNWork &work, int num_cus, int *best_i,
                               double *best_d, double *zeta0, hipStream_t s, Timer *tm, const double *stage) {
    if (npts <= 0) return hipSuccess;
    const int64_t nb = (int64_t)G.gx * G.gy * G.gz;
    if (nb > kGridMaxBuckets || ncells <= 0) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    auto grow = [&e](void *&ptr, size_t &cap, size_t need) {
        if (e != hipSuccess || need <= cap) return;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
        e = hipMalloc(&ptr, need);
        if (e == hipSuccess) cap = need;
    };
    const size_t had = work.g_count_cap;
    grow(reinterpret_cast<void *&>(work.g_count), work.g_count_cap, 2 * sizeof(int) * (size_t)nb);
    if (e == hipSuccess && work.g_count_cap != had) {  // fresh counters start at zero; later ones are
        e = hipMemsetAsync(work.g_count, 0, work.g_count_cap, s);  // zeroed by the alternate search
        work.g_par = 0;
        work.g_used[0] = work.g_used[1] = 0;
    }
    grow(reinterpret_cast<void *&>(work.g_ent), work.g_ent_cap, sizeof(BucketEntry) * (size_t)nb * (kGridHead + kGridCap));
    if (e != hipSuccess) return e;
    const int64_t half = (int64_t)(work.g_count_cap / (2 * sizeof(int)));
    const int par = work.g_par;
    int *count = work.g_count + par * half, *other = work.g_count + (par ^ 1) * half;
    hipEvent_t t0 = tm ? tm->begin(s) : nullptr;
    hipLaunchKernelGGL(k_grid_fill, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, s, cells, stage,
                       (int)stride, (int)ncells, G, count, work.g_ent);
    if (tm) tm->end("nn_grid_build", t0, s);
    hipEvent_t t1 = tm ? tm->begin(s) : nullptr;
    static const int grid_form = [] {  // diagnostic override: 1 half-wave, 4 quad
        const char *v = std::getenv("TD_NN_GRID_FORM");
        return v ? std::atoi(v) : 0;
    }();
    const bool quad = grid_form ? grid_form == 4 : npts >= kGridQuadMinPts;
    if (!quad)
        hipLaunchKernelGGL(k_nn_grid, dim3((unsigned)((npts + 7) / 8)), dim3(256), 0, s, qx, qy, qz, (int)npts,
                           (int)qy_stride, (int)qz_stride, G, count, work.g_ent, cells, (int)stride, (int)ncells,
                           best_i, best_d, zeta0, other, (int)work.g_used[par ^ 1]);
    else
        hipLaunchKernelGGL(k_nn_grid4, dim3((unsigned)((npts * kGridLpp + 255) / 256)), dim3(256), 0, s, qx, qy, qz,
                           (int)npts, (int)qy_stride, (int)qz_stride, G, count, work.g_ent, cells, (int)stride,
                           (int)ncells, best_i, best_d, zeta0, other, (int)work.g_used[par ^ 1]);
    if (tm) tm->end("nn_grid", t1, s);
    e = hipGetLastError();
    if (e == hipSuccess) {
        work.g_used[par ^ 1] = 0;
        work.g_used[par] = nb;
        work.g_par = par ^ 1;
    }
    return e;
}

}  // namespace tdstar
