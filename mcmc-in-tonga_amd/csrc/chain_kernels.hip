// chain_kernels.hip -- the device-resident rj-MCMC chain (TD_ENGINE_DEVICE).
//
// One persistent 1024-thread workgroup runs `iters` iterations of
// TD_inversion_function.jl:70-274 without returning to the host: draw the
// proposal (chain_logic.h, shared with the host engine), evaluate it
// incrementally against the cached per-point nearest cells (chain_dev.h),
// recompute t* only for the rays whose points changed (Julia sum order,
// ray_sum.h) and chi^2 only from the first changed ray on (the cached
// prefix sums ARE the reference's sequential partial sums), then accept or
// reject.  Every phi it produces is bit-identical to a full evaluate of the
// proposed model (tests/test_gpu_chain.py checks it against the host engine).
//
// Why one workgroup: a proposal touches ~P/N points and a few rays, i.e.
// microseconds of work; a grid-wide barrier costs 4-10 us on MI355X
// (MI355X_MICROARCH.md, barrier-xcd), a kernel boundary ~1.5 us.  One CU keeps
// the loop free of both; the ~1 MB of geometry + cache stays in its XCD's L2.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <climits>

#include "chain_dev.h"
#include "internal.h"
#include "ray_sum.h"

namespace tdstar {

namespace {

using tdchain::Proposal;

__device__ __forceinline__ double dist2(double cx, double cy, double cz, double x, double y, double z) {
    // (mx-x)^2 + (my-y)^2 + (mz-z)^2, MCsub.jl:254 -- same ops as k_nn_partial
    const double dx = cx - x, dy = cy - y, dz = cz - z;
    double d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

// Lower bound of dist2(q, p) over every point p of a tile, computed with the
// same rounded operations (rounding is monotone, so lb2 <= dist2 bit-wise).
__device__ __forceinline__ double tile_lb2(const DevChain &d, int t, double qx, double qy, double qz) {
    const int nt = d.ntiles;
    auto gap = [](double q, double lo, double hi) { return q < lo ? lo - q : (q > hi ? q - hi : 0.0); };
    const double gx = gap(qx, d.tile_lo[t], d.tile_hi[t]);
    const double gy = gap(qy, d.tile_lo[nt + t], d.tile_hi[nt + t]);
    const double gz = gap(qz, d.tile_lo[2 * nt + t], d.tile_hi[2 * nt + t]);
    double s = gx * gx;
    s = s + gy * gy;
    s = s + gz * gz;
    return s;
}

struct OverlayZeta {
    const unsigned char *flag;
    const double *cand, *cur;
    __device__ __forceinline__ double operator()(int k) const { return flag[k] ? cand[k] : cur[k]; }
};

// lexicographic (distance, position) minimum across a wave
__device__ __forceinline__ void wave_min_dj(double &dd, int &jj) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double od = __shfl_xor(dd, off, 64);
        const int oj = __shfl_xor(jj, off, 64);
        if (od < dd || (od == dd && oj < jj)) {
            dd = od;
            jj = oj;
        }
    }
}

struct Shared {
    Proposal p;
    double czeta, zeta_killed, zetanew_death, kx, ky, kz, phi_n;
    int slot_k, new_slot, ncells, accept;
    int n_tiles, n_changed, n_orphans, n_rays, k0;
    int pts_seen, ray_pts;  // roofline accounting
    double red_d[kChainThreads / 64];
    int red_j[kChainThreads / 64];
};

__device__ __forceinline__ void mark(const DevChain &d, Shared &sh, int p, int s, double dd, double z) {
    d.cand_s[p] = s;
    d.cand_d[p] = dd;
    d.cand_z[p] = z;
    d.cand_flag[p] = 1;
    d.changed[atomicAdd(&sh.n_changed, 1)] = p;
}

// Interpolation (MCsub.jl:306-327) of ONE point over the current cells by the
// whole workgroup; cell at position `skip` is left out (the model after a
// death).  Returns on all threads after a barrier: sh.red_j[0] = position.
__device__ void block_nearest(const DevChain &d, Shared &sh, int ncells, int skip, double qx, double qy,
                              double qz) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double bd = kSentinel;
    int bj = INT_MAX;
    for (int j = tid; j < ncells; j += kChainThreads) {
        if (j == skip) continue;
        const int s = d.order[j];
        const double dd = dist2(d.cx[s], d.cy[s], d.cz[s], qx, qy, qz);
        if (dd < bd) {  // per thread j increases: first minimum kept
            bd = dd;
            bj = j;
        }
    }
    wave_min_dj(bd, bj);
    if (lane == 0) {
        sh.red_d[wv] = bd;
        sh.red_j[wv] = bj;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kChainThreads / 64; ++w)
            if (sh.red_d[w] < bd || (sh.red_d[w] == bd && sh.red_j[w] < bj)) {
                bd = sh.red_d[w];
                bj = sh.red_j[w];
            }
        sh.red_d[0] = bd;
        sh.red_j[0] = bj;
    }
    __syncthreads();
}

__global__ __launch_bounds__(kChainThreads) void k_chain_run(DevChain d, long long iters) {
    __shared__ Shared sh;
    __shared__ double ray_scratch[kChainThreads / 64][96];
    __shared__ double chi_t[2048];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int kWaves = kChainThreads / 64;
    const tdchain::Params &P = d.params;
    ChainScalars *st = d.st;

    for (long long it = 0; it < iters; ++it) {
        // ---------------- draw the proposal (one lane) ----------------
        if (tid == 0) {
            const int ncells = st->ncells;
            const tdchain::Draws dr = tdchain::draw_iteration(d.seed, d.chain, (uint64_t)st->iter);
            Proposal p = tdchain::propose(P, dr, ncells);
            sh.slot_k = -1;
            sh.new_slot = -1;
            if (p.active && p.action != tdchain::kBirth) {
                const int s = d.order[p.index];
                sh.slot_k = s;
                sh.kx = d.cx[s];
                sh.ky = d.cy[s];
                sh.kz = d.cz[s];
                sh.zeta_killed = d.czeta[s];
                tdchain::complete_proposal(P, dr, p, d.cx[s], d.cy[s], d.cz[s], d.czeta[s]);
            }
            if (p.active && p.action == tdchain::kBirth)
                sh.new_slot = st->nfree > 0 ? d.free_slots[st->nfree - 1] : st->nslots;
            if (p.active) st->proposed[p.action] += 1;
            sh.p = p;
            sh.ncells = ncells;
            sh.n_tiles = sh.n_changed = sh.n_orphans = sh.n_rays = 0;
            sh.pts_seen = sh.ray_pts = 0;
            sh.k0 = d.n;
            sh.accept = 0;
        }
        __syncthreads();
        const int action = sh.p.action;
        const int ncells = sh.ncells;
        if (sh.p.active) {
            // -------- 1-point Interpolations of the birth/death branches --------
            if (action == tdchain::kBirth || action == tdchain::kDeath) {
                const bool birth = action == tdchain::kBirth;
                block_nearest(d, sh, ncells, birth ? -1 : (int)sh.p.index, birth ? sh.p.x : sh.kx,
                              birth ? sh.p.y : sh.ky, birth ? sh.p.z : sh.kz);
                if (tid == 0) {
                    st->bytes += (int64_t)ncells * 28;  // order + coordinates of every cell
                    const int j = sh.red_j[0];
                    const double v = (j != INT_MAX) ? d.czeta[d.order[j]] : 0.0;
                    if (birth) {
                        sh.czeta = v;  // TD_inversion_function.jl:81
                        tdchain::birth_zeta(P, sh.p, v);
                    } else {
                        sh.zetanew_death = v;  // :146
                    }
                }
                __syncthreads();
            }
            if (sh.p.valid) {
                if (P.debug_prior == 1) {
                    if (tid == 0) sh.phi_n = 1.0;  // MCsub.jl:134-136
                } else {
                    const Proposal p = sh.p;
                    const int slot_k = sh.slot_k;
                    const bool q0 = action != tdchain::kBirth;  // old site of the selected cell
                    const bool q1 = action == tdchain::kBirth || action == tdchain::kMove;  // new site
                    // ---------------- tiles that may hold affected points ----------------
                    for (int t = tid; t < d.ntiles; t += kChainThreads) {
                        const double mx = d.tile_maxd[t];
                        bool hit = false;
                        if (q0) hit = tile_lb2(d, t, sh.kx, sh.ky, sh.kz) <= mx;
                        if (q1 && !hit) hit = tile_lb2(d, t, p.x, p.y, p.z) <= mx;
                        if (hit) d.tiles_hit[atomicAdd(&sh.n_tiles, 1)] = t;
                    }
                    __syncthreads();
                    // ---------------- affected points ----------------
                    const int nt = sh.n_tiles;
                    const int rank_k = slot_k >= 0 ? d.rank[slot_k] : 0;
                    int seen = 0;
                    for (int item = tid; item < nt * kTilePts; item += kChainThreads) {
                        const int t = d.tiles_hit[item / kTilePts];
                        const int q = d.tile_start[t] + item % kTilePts;
                        if (q >= d.tile_start[t + 1]) continue;
                        ++seen;
                        const int s = d.best_s[q];
                        const double bd = d.best_d[q];
                        if (action == tdchain::kBirth) {  // appended cell: strict capture
                            const double dd = dist2(p.x, p.y, p.z, d.px[q], d.py[q], d.pz[q]);
                            if (dd < bd) mark(d, sh, q, sh.new_slot, dd, p.zeta);
                        } else if (action == tdchain::kChange) {
                            if (s == slot_k) mark(d, sh, q, s, bd, p.zeta);
                        } else if (s == slot_k) {  // death / move: its points are re-searched
                            d.orphans[atomicAdd(&sh.n_orphans, 1)] = q;
                        } else if (action == tdchain::kMove) {
                            const double dd = dist2(p.x, p.y, p.z, d.px[q], d.py[q], d.pz[q]);
                            if (dd < bd || (dd == bd && s >= 0 && rank_k < d.rank[s]))
                                mark(d, sh, q, slot_k, dd, d.czeta[slot_k]);
                        }
                    }
                    if (seen) atomicAdd(&sh.pts_seen, seen);
                    __syncthreads();
                    // ---------------- re-search orphaned points, one wave each ----------------
                    const int no = sh.n_orphans;
                    const bool death = action == tdchain::kDeath;
                    for (int o = wv; o < no; o += kWaves) {
                        const int q = d.orphans[o];
                        const double x = d.px[q], y = d.py[q], z = d.pz[q];
                        double bd = kSentinel;
                        int bj = INT_MAX;
                        for (int j = lane; j < ncells; j += 64) {
                            if (death && j == (int)p.index) continue;
                            const int s = d.order[j];
                            double dd;
                            if (s == slot_k)  // the moved cell at its proposed site
                                dd = dist2(p.x, p.y, p.z, x, y, z);
                            else
                                dd = dist2(d.cx[s], d.cy[s], d.cz[s], x, y, z);
                            if (dd < bd) {
                                bd = dd;
                                bj = j;
                            }
                        }
                        wave_min_dj(bd, bj);
                        if (lane == 0) {
                            if (bj != INT_MAX) {
                                const int s = d.order[bj];
                                mark(d, sh, q, s, bd, d.czeta[s]);
                            } else {
                                mark(d, sh, q, -1, kSentinel, 0.0);
                            }
                        }
                    }
                    __syncthreads();
                    // ---------------- rays holding changed points ----------------
                    const int nc = sh.n_changed;
                    for (int c = tid; c < nc; c += kChainThreads) {
                        const int r = d.pt_ray[d.changed[c]];
                        if (atomicExch(&d.ray_flag[r], 1) == 0) {
                            d.rays_hit[atomicAdd(&sh.n_rays, 1)] = r;
                            atomicMin(&sh.k0, r);
                        }
                    }
                    __syncthreads();
                    const int nr = sh.n_rays;
                    const OverlayZeta oz{d.cand_flag, d.cand_z, d.zeta0};
                    for (int rr = wv; rr < nr; rr += kWaves) {
                        const int r = d.rays_hit[rr];
                        const int s0 = d.ray_off[r];
                        const double v = wave_ray_sum(lane, d.w, oz, s0, d.ray_off[r + 1] - s0, ray_scratch[wv]);
                        if (lane == 0) {
                            d.cand_ptS[r] = v;
                            atomicAdd(&sh.ray_pts, d.ray_off[r + 1] - s0);
                        }
                    }
                    __syncthreads();
                    // ---------------- chi^2 from the first changed ray on ----------------
                    const int k0 = sh.k0;
                    double C = k0 > 0 ? d.prefix[k0 - 1] : 0.0;  // MCsub.jl:169 C = 0
                    for (int base = k0; base < d.n; base += 2048) {
                        const int cnt = min(2048, d.n - base);
                        for (int k = tid; k < cnt; k += kChainThreads) {
                            const int r = base + k;
                            const double pt = d.ray_flag[r] ? d.cand_ptS[r] : d.ptS[r];
                            const double df = pt - d.tS[r];
                            const double sg = d.sig[r];
                            chi_t[k] = ((df * df) * 1.0) / (sg * sg);  // MCsub.jl:171
                        }
                        __syncthreads();
                        if (tid == 0)
                            for (int k = 0; k < cnt; ++k) {
                                C = C + chi_t[k];
                                d.cand_prefix[base + k] = C;
                            }
                        __syncthreads();
                    }
                    if (tid == 0) {
                        sh.phi_n = k0 < d.n ? C : st->phi;
                        st->evaluations += 1;
                        // bytes this proposal's algorithm must read: tile boxes + maxima (56 B),
                        // candidate points (coords + cached slot/distance, 36 B), orphan scans
                        // (order + coords per cell, 28 B), rays (w, zeta, flag: 17 B per point),
                        // chi^2 tail (ptS, tS, sig, flag: 28 B per ray)
                        st->bytes += (int64_t)d.ntiles * 56 + (int64_t)sh.pts_seen * 36 +
                                     (int64_t)sh.n_orphans * ncells * 28 + (int64_t)sh.ray_pts * 17 +
                                     (int64_t)(d.n - k0) * 28;
                    }
                }
                __syncthreads();
                // ---------------- Metropolis-Hastings decision ----------------
                if (tid == 0) {
                    const bool acc = tdchain::accept(P, sh.p, ncells, st->phi, sh.phi_n, sh.czeta, sh.zeta_killed,
                                                     sh.zetanew_death);
                    sh.accept = acc ? 1 : 0;
                    if (acc) st->accepted[action] += 1;
                }
                __syncthreads();
                const int nc = sh.n_changed, nr = sh.n_rays, nt = sh.n_tiles;
                if (sh.accept) {
                    // -------- commit: points, rays, chi^2 prefix, cells --------
                    for (int c = tid; c < nc; c += kChainThreads) {
                        const int q = d.changed[c];
                        d.best_s[q] = d.cand_s[q];
                        d.best_d[q] = d.cand_d[q];
                        d.zeta0[q] = d.cand_z[q];
                        d.cand_flag[q] = 0;
                    }
                    for (int rr = tid; rr < nr; rr += kChainThreads) {
                        const int r = d.rays_hit[rr];
                        d.ptS[r] = d.cand_ptS[r];
                        d.ray_flag[r] = 0;
                    }
                    for (int r = sh.k0 + tid; r < d.n; r += kChainThreads) d.prefix[r] = d.cand_prefix[r];
                    const Proposal p = sh.p;
                    if (action == tdchain::kDeath) {  // deleteat!: positions after the killed one shift down
                        for (int j = (int)p.index + 1 + tid; j < ncells; j += kChainThreads) d.order_tmp[j] = d.order[j];
                        __syncthreads();
                        for (int j = (int)p.index + 1 + tid; j < ncells; j += kChainThreads) {
                            const int s = d.order_tmp[j];
                            d.order[j - 1] = s;
                            d.rank[s] = j - 1;
                        }
                    }
                    if (tid == 0) {
                        const int sk = sh.slot_k;
                        if (action == tdchain::kBirth) {  // append!
                            const int s = sh.new_slot;
                            d.cx[s] = p.x;
                            d.cy[s] = p.y;
                            d.cz[s] = p.z;
                            d.czeta[s] = p.zeta;
                            d.order[ncells] = s;
                            d.rank[s] = ncells;
                            if (st->nfree > 0)
                                st->nfree -= 1;
                            else
                                st->nslots += 1;
                            st->ncells = ncells + 1;
                        } else if (action == tdchain::kDeath) {
                            d.free_slots[st->nfree] = sk;
                            st->nfree += 1;
                            d.rank[sk] = -1;
                            st->ncells = ncells - 1;
                        } else if (action == tdchain::kChange) {
                            d.czeta[sk] = p.zeta;
                        } else {
                            d.cx[sk] = p.x;
                            d.cy[sk] = p.y;
                            d.cz[sk] = p.z;
                        }
                        st->phi = sh.phi_n;
                    }
                    __syncthreads();
                    // tile maxima of the committed distances (changed points lie in hit tiles)
                    if (P.debug_prior != 1)
                        for (int i = tid; i < nt; i += kChainThreads) {
                            const int t = d.tiles_hit[i];
                            double mx = -1.0;
                            for (int q = d.tile_start[t]; q < d.tile_start[t + 1]; ++q) mx = fmax(mx, d.best_d[q]);
                            d.tile_maxd[t] = mx;
                        }
                } else {
                    for (int c = tid; c < nc; c += kChainThreads) d.cand_flag[d.changed[c]] = 0;
                    for (int rr = tid; rr < nr; rr += kChainThreads) d.ray_flag[d.rays_hit[rr]] = 0;
                }
            }
        }
        __syncthreads();
        if (tid == 0) st->iter += 1;
        __syncthreads();
    }
}

// ------------------------------------------------------------ full state ----
// chi^2 prefix sums, sequential (MCsub.jl:170-172), and phi.
__global__ __launch_bounds__(256) void k_chi2_prefix(const double *__restrict__ ptS, const double *__restrict__ tS,
                                                     const double *__restrict__ sig, int n,
                                                     double *__restrict__ prefix, ChainScalars *st) {
    __shared__ double t[2048];
    double C = 0.0;
    for (int base = 0; base < n; base += 2048) {
        const int cnt = min(2048, n - base);
        for (int k = threadIdx.x; k < cnt; k += 256) {
            const double df = ptS[base + k] - tS[base + k];
            const double sg = sig[base + k];
            t[k] = ((df * df) * 1.0) / (sg * sg);
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int k = 0; k < cnt; ++k) {
                C = C + t[k];
                prefix[base + k] = C;
            }
        __syncthreads();
    }
    if (threadIdx.x == 0) st->phi = C;
}

__global__ void k_tile_max(const int *__restrict__ tile_start, int ntiles, const double *__restrict__ best_d,
                           double *__restrict__ tile_maxd) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    double mx = -1.0;
    for (int q = tile_start[t]; q < tile_start[t + 1]; ++q) mx = fmax(mx, best_d[q]);
    tile_maxd[t] = mx;
}

}  // namespace

hipError_t chain_full_state(DevChain &d, int ncells, NNWork &work, int num_cus, hipStream_t s) {
    Geometry g;
    g.m = 0;
    g.n = d.n;
    g.P = d.P;
    g.px = const_cast<double *>(d.px);
    g.py = const_cast<double *>(d.py);
    g.pz = const_cast<double *>(d.pz);
    g.w = const_cast<double *>(d.w);
    g.ray_off = const_cast<int *>(d.ray_off);
    g.tS = const_cast<double *>(d.tS);
    g.sig = const_cast<double *>(d.sig);
    // slots 0..ncells-1 hold the cells in order, so nearest index == slot
    hipError_t e = launch_nearest(d.px, d.py, d.pz, d.P, 1, 1, d.cx, d.cap, ncells, work, num_cus, d.best_s,
                                  d.best_d, d.zeta0, s);
    if (e != hipSuccess) return e;
    e = launch_ray_sums(g, d.zeta0, d.ptS, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_chi2_prefix, dim3(1), dim3(256), 0, s, d.ptS, d.tS, d.sig, d.n, d.prefix, d.st);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (d.ntiles > 0) {
        hipLaunchKernelGGL(k_tile_max, dim3((d.ntiles + 255) / 256), dim3(256), 0, s, d.tile_start, d.ntiles,
                           d.best_d, d.tile_maxd);
        e = hipGetLastError();
    }
    return e;
}

hipError_t chain_run(const DevChain &d, int64_t iters, hipStream_t s) {
    hipLaunchKernelGGL(k_chain_run, dim3(1), dim3(kChainThreads), 0, s, d, (long long)iters);
    return hipGetLastError();
}

}  // namespace tdstar
