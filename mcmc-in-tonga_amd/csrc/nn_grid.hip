// nn_grid.hip -- nearest cell of many query points through a uniform bucket
// grid over the cells: the drop-in evaluate / Interpolation path for larger
// models (v_nearest, MCsub.jl:247-263, for every ray point).
//
// The answer is the reference's: the lexicographic minimum of (squared
// distance, cell index) over all cells, among distances below the 1e9
// sentinel -- v_nearest's strict '<' scan in index order keeps the FIRST
// minimum.  The grid only decides where to look:
//   k_grid_fill  one lane per cell: append {x, y, z, index} to its bucket
//                (kGridCap entries; a fuller bucket is flagged);
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

#include "eval_server.h"
#include "internal.h"
#include "ray_sum.h"
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
    if (pos < kGridCap) ent[(long)b * kGridCap + pos] = BucketEntry{x, y, z, i, 0};
}

__device__ __forceinline__ long long ticks() { return (long long)wall_clock64(); }
// the value v available (its load waited for) before whatever follows: the phase stamps
__device__ __forceinline__ void depend(double v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ int wave_max_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
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
            const BucketEntry e0 = ent[b * kGridCap], e1 = ent[b * kGridCap + 1];
            if (cnt > 0) take(dist2_q(e0.x, e0.y, e0.z, x, y, z), e0.slot, bd, bx);
            if (cnt > 1) take(dist2_q(e1.x, e1.y, e1.z, x, y, z), e1.slot, bd, bx);
            for (int k = 2; k < min(cnt, kGridCap); ++k) {
                const BucketEntry e = ent[b * kGridCap + k];
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
        best_i[p] = found ? bx : -1;
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
// The nearest cell of the lane's point (x, y, z) by its quad (4 lanes; all 64 lanes of the wave
// active): (bd, bx) in every lane of the quad.  valid = false: a padding lane (proven at once).
__device__ __forceinline__ void quad_nearest(double x, double y, double z, bool valid, const CellGrid &G,
                                             const int *__restrict__ count, const BucketEntry *__restrict__ ent,
                                             const double *__restrict__ cells, int stride, int ncells, double &bd,
                                             int &bx, long long *stamp = nullptr) {
    const int lane = threadIdx.x & 63, sub = threadIdx.x & (kGridLpp - 1);
    const int bi = grid_axis(x, G.x0, G.ix, G.gx), bj = grid_axis(y, G.y0, G.iy, G.gy),
              bk = grid_axis(z, G.z0, G.iz, G.gz);
    constexpr int kMine = (27 + kGridLpp - 1) / kGridLpp;
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
        e[u] = ent[(long)bb[u] * kGridCap];
    }
    const double lb = grid_block_lb(G, x, y, z, 1);  // independent of the loads: computed while they fly
    bd = kSentinel;
    bx = INT_MAX;
    if (stamp) {  // (diagnostics: the first round of loads back)
        depend(e[kMine - 1].x + (double)cnt[kMine - 1]);
        stamp[0] = ticks();
    }
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
            if (k < cnt[u]) e[u] = ent[(long)bb[u] * kGridCap + k];
#pragma unroll
        for (int u = 0; u < kMine; ++u)
            if (k < cnt[u]) take(dist2_q(e[u].x, e[u].y, e[u].z, x, y, z), e[u].slot, bd, bx);
    }
    quad_lexmin(bd, bx);
    const int qsh = lane & ~(kGridLpp - 1);  // first lane of my quad
    const bool any_over = ((__ballot(over) >> qsh) & 0xfull) != 0ull;
    const bool proven = !valid || (!any_over && bd < lb);
    // points the block does not prove: the whole wave, one at a time
    unsigned long long need = __ballot(!proven && sub == 0);
    if (stamp) {
        depend(bd);
        stamp[1] = ticks();
        stamp[2] = __popcll(need);
        stamp[3] = __builtin_amdgcn_readfirstlane(wave_max_i(most));
    }
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
                const BucketEntry f = ent[(long)b * kGridCap + k];
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
    if (stamp) {
        depend(bd);
        stamp[4] = ticks();
    }
}

__global__ __launch_bounds__(256) void k_nn_grid4(const double *__restrict__ qx, const double *__restrict__ qy,
                                                  const double *__restrict__ qz, int npts, int ys, int zs, CellGrid G,
                                                  const int *__restrict__ count, const BucketEntry *__restrict__ ent,
                                                  const double *__restrict__ cells, int stride, int ncells,
                                                  int *__restrict__ best_i, double *__restrict__ best_d,
                                                  double *__restrict__ zeta0, int *__restrict__ other_count,
                                                  int other_nb) {
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < other_nb; b += gridDim.x * blockDim.x) other_count[b] = 0;
    const int sub = threadIdx.x & (kGridLpp - 1);
    const int p = (blockIdx.x * blockDim.x + threadIdx.x) / kGridLpp;  // whole quads stay for the DPP
    const int pc = min(p, npts - 1);
    const double x = qx[pc], y = qy[(long)pc * ys], z = qz[(long)pc * zs];
    double bd;
    int bx;
    quad_nearest(x, y, z, p < npts, G, count, ent, cells, stride, ncells, bd, bx);
    if (sub == 0 && p < npts) {
        const bool found = bd < kSentinel;
        best_i[p] = found ? bx : -1;
        if (best_d) best_d[p] = bd;
        if (zeta0) zeta0[p] = found ? cells[3 * (long)stride + bx] : 0.0;  // MCsub.jl:249
    }
}

// ---- td_evaluate's full path as one resident launch (eval_server.h) ----

// pinned host memory: system-scope atomics (coherent, never served from a stale cache line)
__device__ __forceinline__ long long sys_load(const long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(long long *p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ long long readlane_i64(long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(unsigned long long)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)v >> 32), l);
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ int sgpr_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double sgpr_d(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the workgroup's points' zeta0 in LDS, addressed by global point index
struct LdsZeta {
    const double *z;
    int p0;
    __device__ __forceinline__ double operator()(int k) const { return z[k - p0]; }
};

enum : int { kEvalGo = 0, kEvalStop = 1, kEvalFail = 2 };

// Wave 0 of each workgroup: the next command into cmd (LDS, EvalCmd's bytes); the outcome in *state.
// Workgroup 0 polls the mailbox (every word in one round trip, taken when its check matches) and
// forwards the words as {word, tag} granules: 8-byte agent-scope atomics, each whole or not at all,
// so a reader that sees every granule with the new tag has the whole command with no further
// ordering.  The others poll the granules.  Workgroup 0 alone quits on silence: it marks the launch
// exited (the host then knows it took nothing more), then forwards a QUIT.
__device__ __forceinline__ void eval_take(const EvalArgs &A, long long last, unsigned *cmd, int *state, int lane,
                                          long long *t_take) {
    constexpr int W = kEvalCmdWords, G2 = 2 * kEvalCmdWords;
    const long long t0 = ticks();
    if (blockIdx.x == 0) {
        while (true) {
            const long long w = lane < W ? sys_load(reinterpret_cast<const long long *>(A.mb) + lane) : 0;
            const long long sq = readlane_i64(w, 0);
            bool fresh = sq != last;
            if (fresh) {  // (a poll that caught the host between its words: polled again)
                const unsigned long long h = wave_xor_u64(
                    lane >= 1 && lane < W - 1 ? eval_mix((unsigned long long)w, lane, sq) : 0ull);
                fresh = h == (unsigned long long)readlane_i64(w, W - 1);
            }
            const bool idle = !fresh && ticks() - t0 > A.idle_ticks;
            if (fresh || idle) {
                long long v = w;
                if (idle) {  // the QUIT forwarded to the others: seq last + 1, type kEvalQuit
                    v = lane == 0 ? last + 1 : (lane == 1 ? (long long)kEvalQuit : 0);
                    if (lane == 0) sys_store(&A.ctl->exited, 1);
                }
                const unsigned long long tag = (unsigned long long)eval_tag(readlane_i64(v, 0)) << 32;
                if (lane < W) {
                    __hip_atomic_store(&A.bcast[2 * lane], tag | (unsigned)(unsigned long long)v, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&A.bcast[2 * lane + 1], tag | (unsigned)((unsigned long long)v >> 32),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    cmd[2 * lane] = (unsigned)(unsigned long long)v;
                    cmd[2 * lane + 1] = (unsigned)((unsigned long long)v >> 32);
                }
                if (lane == 0) {
                    *t_take = ticks();
                    if (fresh) sys_store(&A.ctl->t_take, *t_take);
                    *state = idle ? kEvalStop : (readlane_i64(v, 1) & 0xffffffff) == kEvalRun ? kEvalGo : kEvalStop;
                }
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    const unsigned expect = eval_tag(last + 1);
    while (true) {
        const unsigned long long g =
            lane < G2 ? __hip_atomic_load(&A.bcast[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : (unsigned long long)expect << 32;
        if (__ballot((unsigned)(g >> 32) != expect) == 0ull) {
            if (lane < G2) cmd[lane] = (unsigned)g;
            const int type = __builtin_amdgcn_readlane((int)(unsigned)g, 2);  // word 1's low half
            if (lane == 0) {
                *t_take = ticks();
                *state = type == kEvalRun ? kEvalGo : kEvalStop;
            }
            return;
        }
        // workgroup 0 gone without a QUIT reaching this one (it failed): leave after twice its watchdog
        if (ticks() - t0 > 2 * A.idle_ticks + A.guard_ticks) {
            if (lane == 0) *state = kEvalStop;
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__global__ __launch_bounds__(kEvalThreads) void k_eval_server(const EvalArgs A) {
    extern __shared__ double zsh[];  // [lds_pts]: the zeta0 of this workgroup's points
    __shared__ double scratch[kEvalThreads / 64][96];
    __shared__ __attribute__((aligned(16))) unsigned cmd[2 * kEvalCmdWords];
    __shared__ int state;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wg = blockIdx.x;
    const int r0 = A.wg_ray[wg], r1 = A.wg_ray[wg + 1];
    const int p0 = A.ray_off[r0], p1 = A.ray_off[r1];
    const int shard = wg & 7;
    const unsigned in_shard = (unsigned)((A.nwg - shard + 7) / 8);  // workgroups w with w % 8 == shard
    unsigned *fin = A.arrive + 8 * 32;                               // the finish shards, after the arrival ones
    long long last = A.seq0;
    unsigned k = 0;  // commands run by this launch (the grid barrier's target is k * nwg arrivals)
    long long st[15] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // phase stamps (tid 0; EvalStamps)
    while (true) {
        if (wv == 0) eval_take(A, last, cmd, &state, lane, &st[0]);
        __syncthreads();
        if (state != kEvalGo) break;
        const EvalCmd &c = *reinterpret_cast<const EvalCmd *>(cmd);
        const long long seq = readlane_i64(c.seq, 0);
        const int ncells = sgpr_i(c.ncells), stride = sgpr_i(c.stride), par = sgpr_i(c.par);
        const int other_nb = sgpr_i(c.other_nb), diag = sgpr_i(c.diag);
        // (through address space 1: global_ loads and stores, not flat_ ones, which LDS waits would count)
        using gdouble = __attribute__((address_space(1))) double;
        double *cells = (double *)(gdouble *)readlane_i64(reinterpret_cast<long long>(c.cells), 0);
        const double *stage = (const double *)(const gdouble *)readlane_i64(reinterpret_cast<long long>(c.stage), 0);
        CellGrid G;
        G.gx = sgpr_i(c.G.gx), G.gy = sgpr_i(c.G.gy), G.gz = sgpr_i(c.G.gz);
        G.x0 = sgpr_d(c.G.x0), G.y0 = sgpr_d(c.G.y0), G.z0 = sgpr_d(c.G.z0);
        G.ix = sgpr_d(c.G.ix), G.iy = sgpr_d(c.G.iy), G.iz = sgpr_d(c.G.iz);
        G.hx = sgpr_d(c.G.hx), G.hy = sgpr_d(c.G.hy), G.hz = sgpr_d(c.G.hz);
        G.ex = sgpr_d(c.G.ex), G.ey = sgpr_d(c.G.ey), G.ez = sgpr_d(c.G.ez);
        for (int a = 0; a < 3; ++a) {
            G.lo[a] = sgpr_d(c.G.lo[a]);
            G.hi[a] = sgpr_d(c.G.hi[a]);
        }
        G.sealed = sgpr_i(c.G.sealed);
        last = seq;
        ++k;
        int *count = A.count + (long)par * kGridMaxBuckets;
        int *other = A.count + (long)(par ^ 1) * kGridMaxBuckets;
        // ---- fill: this workgroup's share of the cells into their buckets (k_grid_fill) ----
        const int per = (ncells + A.nwg - 1) / A.nwg;
        const int c1 = min(ncells, (wg + 1) * per);
#ifndef TD_EVS_STAGE
#define TD_EVS_STAGE 0
#endif
#if TD_EVS_STAGE == 1
        if (wg * per < c1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (system scope: stale staged lines out)
#endif
        for (int i = wg * per + tid; i < c1; i += kEvalThreads) {
#if TD_EVS_STAGE == 0
            const double x = __longlong_as_double(sys_load(reinterpret_cast<const long long *>(stage + i)));
            const double y = __longlong_as_double(sys_load(reinterpret_cast<const long long *>(stage + stride + i)));
            const double z =
                __longlong_as_double(sys_load(reinterpret_cast<const long long *>(stage + 2 * (long)stride + i)));
            const double ze =
                __longlong_as_double(sys_load(reinterpret_cast<const long long *>(stage + 3 * (long)stride + i)));
#else
            const double x = stage[i], y = stage[stride + i], z = stage[2 * (long)stride + i],
                         ze = stage[3 * (long)stride + i];
#endif
            if (diag && tid == 0) {
                depend(x + y + z + ze);
                st[1] = ticks();
            }
            cells[i] = x;
            cells[stride + i] = y;
            cells[2 * (long)stride + i] = z;
            cells[3 * (long)stride + i] = ze;
            const int b = grid_bucket(G, x, y, z);
            const int pos = atomicAdd(&count[b], 1);  // order inside a bucket does not matter
            if (diag && tid == 0) {
                depend((double)pos);
                st[2] = ticks();
            }
            if (pos < kGridCap) A.ent[(long)b * kGridCap + pos] = BucketEntry{x, y, z, i, 0};
        }
        // the previous evaluate's counts zeroed for the next one (ordered before it by this barrier)
        const int zper = (other_nb + A.nwg - 1) / A.nwg;
        const int z1 = min(other_nb, (wg + 1) * zper);
        for (int b = wg * zper + tid; b < z1; b += kEvalThreads) other[b] = 0;
        // ---- grid barrier: every store above, from every workgroup, before any search ----
        // (cdna_hip_programming.md Guideline 16: stores drained, workgroup barrier, one agent release,
        // drained again, then the arrival; the waiter's one agent acquire before the workgroup barrier)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            st[3] = ticks();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st[4] = ticks();
            __hip_atomic_fetch_add(&A.arrive[shard * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (wv == 0) {
            const unsigned target = k * (unsigned)A.nwg;
            const long long t0 = ticks();
            bool fail = false;
            while (true) {
                const unsigned v =
                    lane < 8 ? __hip_atomic_load(&A.arrive[lane * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                unsigned s = 0;
#pragma unroll
                for (int l = 0; l < 8; ++l) s += (unsigned)__builtin_amdgcn_readlane((int)v, l);
                if ((int)(s - target) >= 0) break;  // (wraps with the counters)
                if (ticks() - t0 > A.guard_ticks) {
                    fail = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0 && fail) state = kEvalFail;
        }
        __syncthreads();
        if (tid == 0) st[5] = ticks();
        if (state == kEvalFail) {  // abandoned: the host takes the launches (and this launch ends)
            if (tid == 0) {
                sys_store(&A.ctl->failed, seq);
                if (wg == 0) sys_store(&A.ctl->exited, 1);
            }
            break;
        }
        // ---- search: the points of this workgroup's rays, 16 per wave (k_nn_grid4's quads) ----
        for (int base = p0 + wv * 16; base < p1; base += kEvalThreads / 4) {
            const int p = base + (lane >> 2);
            const int pc = min(p, p1 - 1);
            double bd;
            int bx;
            quad_nearest(A.px[pc], A.py[pc], A.pz[pc], p < p1, G, count, A.ent, cells, stride, ncells, bd, bx,
                         diag && wv == 0 && base == p0 ? &st[10] : nullptr);
            const double zv = bd < kSentinel ? cells[3 * (long)stride + bx] : 0.0;  // MCsub.jl:249
            if ((lane & 3) == 0 && p < p1) zsh[p - p0] = zv;
            if (diag && tid == 0 && base == p0) {
                depend(zv);
                st[6] = ticks();
            }
        }
        __syncthreads();
        if (tid == 0) st[7] = ticks();
        // ---- ray sums: one wave per ray (ray_sum.h), ptS straight into pinned memory ----
        for (int r = r0 + wv; r < r1; r += kEvalThreads / 64) {
            const int s0 = A.ray_off[r];
            const double v = wave_ray_sum(lane, A.w, LdsZeta{zsh, p0}, s0, A.ray_off[r + 1] - s0, scratch[wv]);
            if (lane == 0) {
                A.ptS[r] = v;
                sys_store(reinterpret_cast<long long *>(A.ptS_host + r), __double_as_longlong(v));
            }
        }
        if (tid == 0) st[8] = ticks();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every reply word acknowledged before done
        __syncthreads();
        if (tid == 0) {
            st[9] = ticks();
            if (diag) {
                for (int j = 0; j < 15; ++j) sys_store(&A.stamps[wg].t[j], st[j]);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // the shard's last workgroup (its add returns the shard's full count) tells the host
            const unsigned old = __hip_atomic_fetch_add(&fin[shard * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1u == k * in_shard) {
                sys_store(&A.ctl->t_end[shard], ticks());
                sys_store(&A.ctl->done[shard], seq);
            }
        }
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
    grow(reinterpret_cast<void *&>(work.g_ent), work.g_ent_cap, sizeof(BucketEntry) * (size_t)nb * kGridCap);
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

namespace tdstar {

hipError_t launch_eval_server(const EvalArgs &a, hipStream_t s) {
    if (a.nwg <= 0 || a.lds_pts <= 0 || a.lds_pts > kEvalMaxLdsPts) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_eval_server, dim3((unsigned)a.nwg), dim3(kEvalThreads), sizeof(double) * (size_t)a.lds_pts,
                       s, a);
    return hipGetLastError();
}

}  // namespace tdstar
