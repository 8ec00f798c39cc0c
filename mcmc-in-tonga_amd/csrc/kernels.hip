// kernels.hip -- FP64 forward-model kernels for gfx950 (CDNA4).
//
// The three stages of MCsub.jl:123-185 `evaluate`:
//   1. nearest cell per ray point (v_nearest, MCsub.jl:247-263) -- brute force
//      over every cell, the only heavy stage (P x N distance evaluations).
//      Cells are split into chunks staged in LDS (grid.y), points are spread
//      over lanes (grid.x, PPL points per lane), and the per-chunk partial
//      minima are merged in chunk order so the FIRST minimum index wins,
//      exactly as the reference's sequential strict '<' scan.
//   2. per-ray t* integral (MCsub.jl:147-159) in Julia's Base.sum association
//      (oracle/README.md: VF=8 x IC=4 accumulators + sequential tail).
//   3. chi^2 (MCsub.jl:169-172), strictly sequential in k.
//
// Numerics: the whole TU is compiled with -ffp-contract=off (and the pragma
// below) so no a*b+c is fused -- the reference's FP64 rounding is reproduced
// operation for operation, and nearest indices are bit-exact.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "internal.h"
#include "exact_sum.h"
#include "ray_sum.h"

namespace tdstar {

namespace {

constexpr int kNNThreads = 256;
constexpr int kMaxChunk = 2048;  // cells per LDS chunk (64 KiB as double4)
constexpr int kMinChunk = 64;

// ---------------------------------------------------------------------------
// Stage 1a: partial nearest over one chunk of cells.
//   grid.x = point tiles of 256*PPL points, grid.y = cell chunks.
//   Cells of the chunk are staged as {x,y,z,-} double4 in LDS; every lane
//   reads the same cell (LDS broadcast, conflict-free) and updates PPL
//   independent (min distance, first index) pairs.
// ---------------------------------------------------------------------------
template <int PPL>
__global__ __launch_bounds__(kNNThreads) void k_nn_partial(
    const double *__restrict__ qx, const double *__restrict__ qy, const double *__restrict__ qz,
    int npts, int ys, int zs, const double *__restrict__ cells, int stride, int ncells, int chunk,
    double *__restrict__ part_d, int *__restrict__ part_i) {
    extern __shared__ double4 sc[];
    const int c0 = blockIdx.y * chunk;
    const int nc = min(chunk, ncells - c0);
    for (int j = threadIdx.x; j < nc; j += kNNThreads)
        sc[j] = make_double4(cells[c0 + j], cells[stride + c0 + j], cells[2 * stride + c0 + j], 0.0);

    double x[PPL], y[PPL], z[PPL], bd[PPL];
    int bi[PPL];
    const int base = blockIdx.x * (kNNThreads * PPL) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int p = min(base + k * kNNThreads, npts - 1);
        x[k] = qx[p];
        y[k] = qy[(long)p * ys];
        z[k] = qz[(long)p * zs];
        bd[k] = kSentinel;
        bi[k] = -1;
    }
    __syncthreads();

    // groups of kGroup cells: the group minimum takes one v_min per distance
    // (instead of compare + three selects); only when it beats the running
    // best is the first cell reaching it looked up (group8_update, internal.h)
    constexpr int kGroup = 8;
    int j = 0;
    for (; j + kGroup <= nc; j += kGroup) {
        double dg[PPL][kGroup];
#pragma unroll
        for (int u = 0; u < kGroup; ++u) {
            const double4 c = sc[j + u];
#pragma unroll
            for (int k = 0; k < PPL; ++k) {
                // (mx[i]-x)^2 + (my[i]-y)^2 + (mz[i]-z)^2, MCsub.jl:254, left to right, unfused
                const double dx = c.x - x[k], dy = c.y - y[k], dz = c.z - z[k];
                double d = dx * dx;
                d = d + dy * dy;
                d = d + dz * dz;
                dg[k][u] = d;
            }
        }
        group8_update<PPL>(dg, bd, bi, c0 + j);
    }
    for (; j < nc; ++j) {  // the tail, one cell at a time
        const double4 c = sc[j];
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
            const double dx = c.x - x[k], dy = c.y - y[k], dz = c.z - z[k];
            double d = dx * dx;
            d = d + dy * dy;
            d = d + dz * dz;
            const bool lt = d < bd[k];  // MCsub.jl:255 strict: NaN never wins
            bd[k] = lt ? d : bd[k];
            bi[k] = lt ? c0 + j : bi[k];
        }
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int p = base + k * kNNThreads;
        if (p < npts) {
            part_d[(long)blockIdx.y * npts + p] = bd[k];
            part_i[(long)blockIdx.y * npts + p] = bi[k];
        }
    }
}

// ---------------------------------------------------------------------------
// Stage 1 (one launch, no partials): k_nn_tile.  The points are cut into
// equal tiles of Q points; one 1024-thread workgroup per CU (grid = min(tiles,
// CUs)) takes tiles blockIdx.x, blockIdx.x + gridDim.x, ... and scans EVERY
// cell for each, so nothing but the answer leaves the CU and the chip is
// balanced to within one tile (the planner picks Q so every CU holds about the
// same number of tiles: one tile per CU up to 2048 points per CU, several for
// the stress geometry's 584k points).  Lane t takes point group t % Qg and
// cell slice t / Qg (S slices of L cells, S * Qg <= 1024): the slices are
// merged in LDS in slice order at the end of a tile, so the lowest cell index
// wins a tie exactly as in the sequential scan.  Cells are staged in rounds of
// R per slice, SoA with an odd stride (R + 1 doubles: two slices read by one
// lane group never share a bank), double buffered with one barrier per round;
// the next round's global loads are in flight while the current round is
// scanned.  The tail of a round is padded with NaN cells: fmin and the strict
// '<' never pick them.  Traffic: the points once, the cells once per XCD (L2),
// the answers once -- no per-chunk partials, no merge launch.
// ---------------------------------------------------------------------------
constexpr int kTileThreads = 1024;

template <int PPL>
__global__ __launch_bounds__(kTileThreads) void k_nn_tile(
    const double *__restrict__ qx, const double *__restrict__ qy, const double *__restrict__ qz,
    int npts, int ys, int zs, const double *__restrict__ cells, int stride, int ncells, int Q, int S, int L,
    int R, int ntiles, int *__restrict__ best_i, double *__restrict__ best_d, double *__restrict__ zeta0) {
    extern __shared__ double lds[];  // [2 buffers][3 fields: x, y, z][S][R + 1]; the merge reuses it
    const int RS = R + 1;
    const int buf_sz = 3 * S * RS;
    const int t = threadIdx.x;
    const int Qg = (Q + PPL - 1) / PPL;  // point groups: lane g takes points g, g + Qg, ... of the tile
    const int g = t % Qg, s = t / Qg;
    const int rounds = (L + R - 1) / R;
    const int nstage = S * R;  // cells staged per round
    const bool active = s < S;

    // one cell of round r for staging element e (slice e / R, offset e % R), NaN past the slice / cell set
    auto fetch = [&](int r, int e, double &cx, double &cy, double &cz) {
        const int ss = e / R, j = e - ss * R;
        const int off = r * R + j;
        const int c = ss * L + off;
        if (off < L && c < ncells) {
            cx = cells[c];
            cy = cells[stride + c];
            cz = cells[2 * stride + c];
        } else {
            cx = cy = cz = __builtin_nan("");
        }
    };
    auto put = [&](double *buf, int e, double cx, double cy, double cz) {
        const int ss = e / R, j = e - ss * R;
        buf[(0 * S + ss) * RS + j] = cx;
        buf[(1 * S + ss) * RS + j] = cy;
        buf[(2 * S + ss) * RS + j] = cz;
    };
    constexpr int kStageMax = 2;  // staging elements per thread (S * R <= 2048)
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int p0 = tile * Q;
        double sx[kStageMax], sy[kStageMax], sz[kStageMax];
#pragma unroll
        for (int k = 0; k < kStageMax; ++k) {  // round 0's cells and the points: one round trip
            const int e = t + k * kTileThreads;
            if (e < nstage) fetch(0, e, sx[k], sy[k], sz[k]);
        }
        double x[PPL], y[PPL], z[PPL], bd[PPL];
        int bi[PPL];
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
            const int p = min(p0 + min(g + k * Qg, Q - 1), npts - 1);
            x[k] = qx[p];
            y[k] = qy[(long)p * ys];
            z[k] = qz[(long)p * zs];
            bd[k] = kSentinel;
            bi[k] = -1;
        }
        __syncthreads();  // the previous tile's merge has read the LDS
#pragma unroll
        for (int k = 0; k < kStageMax; ++k) {
            const int e = t + k * kTileThreads;
            if (e < nstage) put(lds, e, sx[k], sy[k], sz[k]);
        }
        __syncthreads();
        for (int r = 0; r < rounds; ++r) {
            const bool more = r + 1 < rounds;
            if (more) {
#pragma unroll
                for (int k = 0; k < kStageMax; ++k) {
                    const int e = t + k * kTileThreads;
                    if (e < nstage) fetch(r + 1, e, sx[k], sy[k], sz[k]);
                }
            }
            if (active) {
                const double *bx = lds + (r & 1) * buf_sz + s * RS;
                const double *by = bx + S * RS;
                const double *bz = by + S * RS;
                const int cbase = s * L + r * R;
                // groups of 8: one v_min per distance; the first cell reaching a new best is looked up only
                // when the group beats it (MCsub.jl:255 strict '<' in index order; group8_update)
                for (int j = 0; j < R; j += 8) {
                    double dg[PPL][8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const double cx = bx[j + u], cy = by[j + u], cz = bz[j + u];
#pragma unroll
                        for (int k = 0; k < PPL; ++k) {
                            // (mx[i]-x)^2 + (my[i]-y)^2 + (mz[i]-z)^2, MCsub.jl:254, left to right, unfused
                            const double dx = cx - x[k], dy = cy - y[k], dz = cz - z[k];
                            double d = dx * dx;
                            d = d + dy * dy;
                            d = d + dz * dz;
                            dg[k][u] = d;
                        }
                    }
                    group8_update<PPL>(dg, bd, bi, cbase + j);
                }
            }
            if (more) {
                double *nb = lds + ((r + 1) & 1) * buf_sz;
#pragma unroll
                for (int k = 0; k < kStageMax; ++k) {
                    const int e = t + k * kTileThreads;
                    if (e < nstage) put(nb, e, sx[k], sy[k], sz[k]);
                }
            }
            __syncthreads();
        }
        // merge the slices in slice order (strict '<': the lower slice, hence the lower index, keeps a tie)
        double *md = lds;                                // [S][Q]
        int *mi = reinterpret_cast<int *>(lds + S * Q);  // [S][Q]
        if (active) {
#pragma unroll
            for (int k = 0; k < PPL; ++k) {
                const int qq = g + k * Qg;
                if (qq < Q) {
                    md[s * Q + qq] = bd[k];
                    mi[s * Q + qq] = bi[k];
                }
            }
        }
        __syncthreads();
        for (int qq = t; qq < Q && p0 + qq < npts; qq += kTileThreads) {
            double d = md[qq];
            int ks = 0;
            for (int k0 = 1; k0 < S; k0 += 8) {  // eight slices' distances in flight, then compared in order
                double dk[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) dk[u] = k0 + u < S ? md[(k0 + u) * Q + qq] : kSentinel;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (dk[u] < d) {
                        d = dk[u];
                        ks = k0 + u;
                    }
            }
            const int pp = p0 + qq, i = mi[ks * Q + qq];
            if (best_i) best_i[pp] = i;
            if (best_d) best_d[pp] = d;
            if (zeta0) zeta0[pp] = i >= 0 ? cells[3 * stride + i] : 0.0;  // MCsub.jl:249 v = 0 when nothing < 1e9
        }
    }
}

// Stage 1b: merge the chunk minima in chunk order (strict '<': the lowest
// chunk, hence the lowest cell index, wins a tie) and gather zeta.
__global__ __launch_bounds__(256) void k_nn_merge(const double *__restrict__ part_d,
                                                  const int *__restrict__ part_i, int npts, int chunks,
                                                  const double *__restrict__ zeta_cells,
                                                  int *__restrict__ best_i, double *__restrict__ best_d,
                                                  double *__restrict__ zeta0) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npts) return;
    double d = kSentinel;
    int i = -1;
    for (int c = 0; c < chunks; ++c) {
        const double dc = part_d[(long)c * npts + p];
        if (dc < d) {
            d = dc;
            i = part_i[(long)c * npts + p];
        }
    }
    if (best_i) best_i[p] = i;
    if (best_d) best_d[p] = d;
    if (zeta0) zeta0[p] = (i >= 0) ? zeta_cells[i] : 0.0;  // MCsub.jl:249 v = 0 when nothing < 1e9
}

// ---------------------------------------------------------------------------
// Stage 2: per-ray t*.  One 64-lane wave per ray, 4 rays per workgroup
// (ray_sum.h: Julia's sum association, bit-exact to the oracle).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ray_sums(const int *__restrict__ ray_off, int n,
                                                  const double *__restrict__ w,
                                                  const double *__restrict__ z0, double *__restrict__ ptS,
                                                  double *host_out) {
    __shared__ double scratch[4][96];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ray = blockIdx.x * 4 + wv;
    if (ray >= n) return;  // wave-uniform; no block barrier below
    const int s0 = ray_off[ray];
    const int np = ray_off[ray + 1] - s0;
    const double r = wave_ray_sum(lane, w, PlainZeta{z0}, s0, np, scratch[wv]);
    if (lane == 0) {
        ptS[ray] = r;
        if (host_out) host_out[ray] = r;  // pinned host memory (td_evaluate: no copy back)
    }
}

// ---------------------------------------------------------------------------
// Stage 3: chi^2, MCsub.jl:169-172, strictly sequential in k, reproduced
// exactly with binade-segmented integer scans (exact_sum.h): k_chi2, a
// 1024-thread launch (the block-wide scan, the one-wave sum if its guess
// fails) -- td_misfit's chi^2 of gathered ray shards.  td_evaluate's ptS land
// in pinned host memory, where the host adds the n terms in k order itself
// (api.cpp host_chi2): shorter than any launch.
// ---------------------------------------------------------------------------
constexpr int kChi2Threads = 1024;

__global__ __launch_bounds__(kChi2Threads) void k_chi2(const double *__restrict__ ptS,
                                                       const double *__restrict__ tS,
                                                       const double *__restrict__ sig, int n,
                                                       double *__restrict__ terms, double *__restrict__ phi,
                                                       double *host_out) {
    __shared__ ExactSumLds w;
    for (int k = threadIdx.x; k < n; k += kChi2Threads) {
        const double d = ptS[k] - tS[k];
        const double s = sig[k];
        terms[k] = ((d * d) * 1.0) / (s * s);  // MCsub.jl:171
    }
    __syncthreads();
    double C = 0.0;
    const bool done = block_exact_sum<kChi2Threads>(terms, n, 0.0, nullptr, &C, w);
    if (!done && threadIdx.x < 64) {
        bool stopped = false;
        C = wave_seq_sum(terms, n, 0.0, nullptr, (int)threadIdx.x, nullptr, &stopped);
    }
    if (threadIdx.x == 0) {
        *phi = C;
        if (host_out) host_out[0] = C;
        __threadfence_system();
    }
}

__global__ __launch_bounds__(kChi2Threads) void k_test_exact_sum(const double *__restrict__ term, int cnt, double C0,
                                                                double *__restrict__ prefix, double *C_end,
                                                                int *fast) {
    __shared__ ExactSumLds w;
    double C = 0.0;
    const bool ok = block_exact_sum<kChi2Threads>(term, cnt, C0, prefix, &C, w);
    if (threadIdx.x == 0) {
        *fast = ok ? 1 : 0;
        if (ok) *C_end = C;
    }
}

__global__ __launch_bounds__(64) void k_test_wave_seq_sum(const double *__restrict__ term, int cnt, double C0,
                                                          double *__restrict__ prefix, double *C_end,
                                                          int *fallbacks) {
    bool stopped = false;
    const double C = wave_seq_sum(term, cnt, C0, prefix, (int)threadIdx.x, nullptr, &stopped);
    if (threadIdx.x == 0) {
        *C_end = C;
        *fallbacks = 0;
    }
}

__global__ __launch_bounds__(64) void k_test_wave_delta_sum(const double *__restrict__ term,
                                                            const double *__restrict__ old,
                                                            const int *__restrict__ chg, int cnt, double C0,
                                                            double *__restrict__ prefix, double *C_end) {
    bool stopped = false;
    const double C = wave_delta_sum(term, old, chg, cnt, C0, prefix, (int)threadIdx.x, nullptr, &stopped);
    if (threadIdx.x == 0) *C_end = C;
}

// The chain's chi^2 walk (exact_sum.h) on its own, as the chain uses it:
// static event words of the OLD state kept across proposals, the changed terms
// in their own words, the walk, the re-marking and the commit; then the kept
// words are checked against words computed from scratch for the new state.
__global__ __launch_bounds__(512) void k_test_block_delta(const double *__restrict__ term,
                                                          const double *__restrict__ term_old, double *old,
                                                          const int *__restrict__ chg, int k0, int n, double *cprefix,
                                                          double *C_end, long long *events, int *mask_ok) {
    __shared__ DeltaSegs sg;
    __shared__ unsigned long long smask[1024], cmask[1024], check[1024];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int W = delta_words(n);
    delta_marks(term_old, old, nullptr, n, smask, wv, W, 8, lane);
    for (int w = wv; w < W; w += 8) {
        const unsigned long long m = __ballot(64 * w + lane < n && chg[min(64 * w + lane, n - 1)] != 0);
        if (lane == 0) cmask[w] = m;
    }
    __syncthreads();
    if (wv == 0) {
        const double C0 = k0 > 0 ? old[k0 - 1] : 0.0;
        long long diag[4] = {0, 0, 0, 0};
        double C = C0;
        if (k0 < n) C = delta_walk(term, old, chg, k0, n, C0, smask, cmask, cprefix, sg, lane, diag);
        else if (lane == 0) sg.nseg = 0;
        const long long ev = diag[0] + diag[3];
        if (lane == 0) {
            *C_end = C;
            *events = ev;
        }
        wave_sync_lds();
        delta_remark(term, old, cprefix, n, sg, smask, lane);
    }
    __syncthreads();
    delta_commit<4>(old, cprefix, n, sg, tid, 512);
    __syncthreads();
    delta_marks(term, old, nullptr, n, check, wv, W, 8, lane);
    __syncthreads();
    if (tid == 0) {
        int ok = 1;
        for (int w = 0; w < W; ++w) ok &= (check[w] == smask[w]) & (cmask[w] == 0ull);
        *mask_ok = ok;
    }
}

}  // namespace

hipError_t test_block_delta(const double *term, const double *term_old, double *old, const int *chg, int k0, int n,
                            double *cprefix, double *C_end, long long *events, int *mask_ok) {
    if (n > 64 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_test_block_delta, dim3(1), dim3(512), 0, nullptr, term, term_old, old, chg, k0, n, cprefix,
                       C_end, events, mask_ok);
    return hipGetLastError();
}

hipError_t test_wave_delta_sum(const double *term, const double *old, const int *chg, int cnt, double C0,
                               double *prefix, double *C_end) {
    hipLaunchKernelGGL(k_test_wave_delta_sum, dim3(1), dim3(64), 0, nullptr, term, old, chg, cnt, C0, prefix, C_end);
    return hipGetLastError();
}

hipError_t test_wave_seq_sum(const double *term, int cnt, double C0, double *prefix, double *C_end, int *fallbacks) {
    hipLaunchKernelGGL(k_test_wave_seq_sum, dim3(1), dim3(64), 0, nullptr, term, cnt, C0, prefix, C_end, fallbacks);
    return hipGetLastError();
}

hipError_t test_chi2(const double *ptS, const double *tS, const double *sig, int n, double *terms, double *phi,
                     hipStream_t s) {
    hipLaunchKernelGGL(k_chi2, dim3(1), dim3(kChi2Threads), 0, s, ptS, tS, sig, n, terms, phi, nullptr);
    return hipGetLastError();
}

hipError_t launch_chi2(const double *ptS, const double *tS, const double *sig, int n, double *terms, double *phi,
                       hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(phi, 0, sizeof(double), s);  // MCsub.jl:169 C = 0
    return test_chi2(ptS, tS, sig, n, terms, phi, s);
}

hipError_t test_exact_sum(const double *term, int cnt, double C0, double *prefix, double *C_end, int *fast) {
    hipLaunchKernelGGL(k_test_exact_sum, dim3(1), dim3(kChi2Threads), 0, nullptr, term, cnt, C0, prefix, C_end, fast);
    return hipGetLastError();
}

NNPlan plan_nearest(int64_t npts, int64_t ncells, int num_cus) {
    NNPlan p{};
    p.ppl = npts >= 65536 ? 4 : 2;  // more points per lane once there are blocks enough for every CU
    const int64_t per_block = (int64_t)kNNThreads * p.ppl;
    p.blocks_x = (int)std::max<int64_t>(1, (npts + per_block - 1) / per_block);
    if (ncells <= 0) {
        p.chunks = 0;
        p.chunk = 0;
        return p;
    }
    const int64_t target = (int64_t)std::max(num_cus, 1) * 4;  // ~4 workgroups (16 waves) per CU
    int64_t chunks = (target + p.blocks_x - 1) / p.blocks_x;
    chunks = std::min<int64_t>(chunks, (ncells + kMinChunk - 1) / kMinChunk);
    chunks = std::max<int64_t>(chunks, (ncells + kMaxChunk - 1) / kMaxChunk);
    chunks = std::max<int64_t>(chunks, 1);
    p.chunk = (int)((ncells + chunks - 1) / chunks);
    p.chunks = (int)((ncells + p.chunk - 1) / p.chunk);
    return p;
}

TilePlan plan_tile(int64_t npts, int64_t ncells, int num_cus) {
    TilePlan best{};
    const int64_t G = std::max(num_cus, 1);
    if (npts <= 0 || ncells <= 0) return best;
    constexpr int ppl = 2;  // points per lane (measured against 1: tools/nn_bench2.py)
    constexpr int fields = 3;
    // tiles per CU m = 1, 2, ...: a tile of Q points is S * Qg lanes (Qg = Q / ppl point groups, S
    // cell slices of L cells); estimated cycles per CU = its tiles x (the busiest SIMD's waves x the
    // distances a lane computes x ~40 cycles each + a tile's fixed cost: first round trip, slice merge)
    double best_cost = 0.0;
    for (int64_t m = 1; m <= 256; ++m) {
        const int64_t Q = (npts + G * m - 1) / (G * m);
        const int64_t Qg = (Q + ppl - 1) / ppl;
        if (Qg > kTileThreads) continue;
        int64_t S = std::min<int64_t>(kTileThreads / Qg, 256);  // <= 256 slices: S * 8 <= 2048 staged cells
        S = std::min<int64_t>(S, (ncells + 7) / 8);              // >= 8 cells per slice
        S = std::max<int64_t>(S, 1);
        const int64_t L = (ncells + S - 1) / S;
        S = (ncells + L - 1) / L;  // no empty slice
        const int64_t tiles = (npts + Q - 1) / Q;
        const int64_t per_cu = (tiles + G - 1) / G;
        const int64_t waves = (Qg * S + 63) / 64;
        const double cost = (double)per_cu * ((double)((waves + 3) / 4) * ppl * (double)L * 40.0 + 12000.0);
        if (best.ok && cost >= best_cost) {
            if (Q < 64) break;  // tiles only get smaller and dearer from here
            continue;
        }
        // rounds: as many cells as the staging registers (2 per thread) and the LDS (double buffered) hold
        int64_t rmax = std::min<int64_t>(64, (2048 / S) / 8 * 8);
        rmax = std::min<int64_t>(rmax, ((int64_t)(150 * 1024) / (2 * fields * 8 * S) - 1) / 8 * 8);
        rmax = std::max<int64_t>(rmax, 8);
        const int64_t rounds = (L + rmax - 1) / rmax;
        const int64_t R = ((L + rounds - 1) / rounds + 7) / 8 * 8;
        const size_t lds = std::max<size_t>((size_t)2 * fields * S * (R + 1) * sizeof(double),
                                            (size_t)S * Q * (sizeof(double) + sizeof(int)));
        if (lds > 160 * 1024) continue;
        TilePlan t{};
        t.ok = true;
        t.Q = (int)Q;
        t.S = (int)S;
        t.L = (int)L;
        t.R = (int)R;
        t.ppl = ppl;
        t.tiles = (int)tiles;
        t.blocks = (int)std::min<int64_t>(tiles, G);
        // more than half the CU's LDS: one workgroup per CU, never two on one CU while another idles
        t.lds = std::max<size_t>(lds, 81 * 1024);
        best = t;
        best_cost = cost;
    }
    return best;
}

hipError_t launch_nearest(const double *qx, const double *qy, const double *qz, int64_t npts,
                          int64_t qy_stride, int64_t qz_stride, const double *cells, int64_t stride,
                          int64_t ncells, NNWork &work, int num_cus, int *best_i, double *best_d,
                          double *zeta0, hipStream_t s, Timer *tm) {
    if (npts <= 0) return hipSuccess;
    if (work.method != kNNSplit) {
        const TilePlan tp = plan_tile(npts, ncells, num_cus);
        if (tp.ok) {
            hipEvent_t t0 = tm ? tm->begin(s) : nullptr;
            auto kern = k_nn_tile<2>;
            static bool attr_set = false;  // dynamic LDS above 64 KB needs the attribute
            if (!attr_set) {
                hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   160 * 1024);
                if (e != hipSuccess) return e;
                attr_set = true;
            }
            hipLaunchKernelGGL(kern, dim3((unsigned)tp.blocks), dim3(kTileThreads), tp.lds, s, qx, qy, qz,
                               (int)npts, (int)qy_stride, (int)qz_stride, cells, (int)stride, (int)ncells, tp.Q, tp.S,
                               tp.L, tp.R, tp.tiles, best_i, best_d, zeta0);
            if (tm) tm->end("nn_tile", t0, s);
            return hipGetLastError();
        }
    }
    const NNPlan p = plan_nearest(npts, ncells, num_cus);
    const size_t need = (size_t)p.chunks * (size_t)npts;
    if (need > work.cap) {
        if (work.part_d) (void)hipFree(work.part_d);
        if (work.part_i) (void)hipFree(work.part_i);
        work.part_d = nullptr;
        work.part_i = nullptr;
        work.cap = 0;
        hipError_t e = hipMalloc(&work.part_d, need * sizeof(double));
        if (e != hipSuccess) return e;
        e = hipMalloc(&work.part_i, need * sizeof(int));
        if (e != hipSuccess) return e;
        work.cap = need;
    }
    if (p.chunks > 0) {
        dim3 grid(p.blocks_x, p.chunks);
        const size_t lds = (size_t)p.chunk * sizeof(double4);
        hipEvent_t t0 = tm ? tm->begin(s) : nullptr;
        if (p.ppl == 4)
            hipLaunchKernelGGL(k_nn_partial<4>, grid, dim3(kNNThreads), lds, s, qx, qy, qz, (int)npts,
                               (int)qy_stride, (int)qz_stride, cells, (int)stride, (int)ncells, p.chunk,
                               work.part_d, work.part_i);
        else
            hipLaunchKernelGGL(k_nn_partial<2>, grid, dim3(kNNThreads), lds, s, qx, qy, qz, (int)npts,
                               (int)qy_stride, (int)qz_stride, cells, (int)stride, (int)ncells, p.chunk,
                               work.part_d, work.part_i);
        if (tm) tm->end("nn_partial", t0, s);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipEvent_t t1 = tm ? tm->begin(s) : nullptr;
    hipLaunchKernelGGL(k_nn_merge, dim3((unsigned)((npts + 255) / 256)), dim3(256), 0, s, work.part_d,
                       work.part_i, (int)npts, p.chunks, cells + 3 * stride, best_i, best_d, zeta0);
    if (tm) tm->end("nn_merge", t1, s);
    return hipGetLastError();
}

hipError_t launch_ray_sums(const Geometry &g, const double *zeta0, double *ptS, hipStream_t s, Timer *tm,
                           double *host_out) {
    if (g.n <= 0) return hipSuccess;
    hipEvent_t t0 = tm ? tm->begin(s) : nullptr;
    hipLaunchKernelGGL(k_ray_sums, dim3((unsigned)((g.n + 3) / 4)), dim3(256), 0, s, g.ray_off, (int)g.n, g.w,
                       zeta0, ptS, host_out);
    if (tm) tm->end("ray_sums", t0, s);
    return hipGetLastError();
}

// ------------------------------------------------------------------ Timer ----
hipEvent_t Timer::begin(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t e = nullptr;
    if (!spare.empty()) {
        e = spare.back();
        spare.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        return nullptr;
    }
    (void)hipEventRecord(e, s);
    return e;
}

void Timer::end(const char *name, hipEvent_t a, hipStream_t s) {
    if (!on || !a) return;
    hipEvent_t b = nullptr;
    if (!spare.empty()) {
        b = spare.back();
        spare.pop_back();
    } else if (hipEventCreate(&b) != hipSuccess) {
        spare.push_back(a);
        return;
    }
    (void)hipEventRecord(b, s);
    pending.push_back(Pending{name, a, b});
}

hipError_t Timer::collect() {
    for (auto &p : pending) {
        hipError_t e = hipEventSynchronize(p.b);
        if (e != hipSuccess) return e;
        float ms = 0.f;
        e = hipEventElapsedTime(&ms, p.a, p.b);
        if (e != hipSuccess) return e;
        auto &slot = acc[p.name];
        slot.first += 1;
        slot.second += ms;
        spare.push_back(p.a);
        spare.push_back(p.b);
    }
    pending.clear();
    return hipSuccess;
}

void Timer::reset() {
    (void)collect();
    acc.clear();
}

void Timer::release() {
    for (auto &p : pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    pending.clear();
    for (auto e : spare) (void)hipEventDestroy(e);
    spare.clear();
}

}  // namespace tdstar
