// ray_sum.h -- one ray's predicted t* computed by ONE 64-lane wave, in the
// association Julia's Base.sum uses (oracle/README.md):
//   term(k) = (rayL*rayU)[k] * ((0.5*(zeta0[k]+zeta0[k+1])) / 1000)   MCsub.jl:147,153
//   L < 16        : strictly sequential            (reduce.jl _mapreduce)
//   16 <= L <= 1024: t0+t1, then 32 lane-parallel accumulators (8 lanes x 4
//                   interleaved parts of the @simd loop), folded
//                   part3+(part2+(part1+part0)), halving tree, sequential tail
//   L > 1024      : pairwise split (mapreduce_impl), one lane
// `zeta(k)` returns zeta0 of point k (a functor, so the chain kernel can
// overlay candidate values).  Scratch: 96 doubles of LDS owned by this wave.
#pragma once
#include <hip/hip_runtime.h>

#include "wave_ops.h"

namespace tdstar {


template <class Z>
__device__ __forceinline__ double seg_term_z(const double *__restrict__ w, const Z &zeta, int k) {
    const double rz = 0.5 * (zeta(k) + zeta(k + 1));
    return w[k] * (rz / 1000.0);
}

template <class Z>
__device__ __attribute__((noinline)) double julia_block_lane(const double *__restrict__ w, const Z zeta, int s0, int f, int l) {
    if (f == l) return seg_term_z(w, zeta, s0 + f);
    double v = seg_term_z(w, zeta, s0 + f) + seg_term_z(w, zeta, s0 + f + 1);
    const int T = l - f - 1;
    const int Q = T >= 32 ? T / 32 : 0;
    int i = f + 2;
    if (Q > 0) {
        double acc[32];
        for (int a = 0; a < 32; ++a) acc[a] = 0.0;
        acc[0] = v;
        for (int q = 0; q < Q; ++q)
            for (int a = 0; a < 32; ++a) acc[a] = acc[a] + seg_term_z(w, zeta, s0 + i + q * 32 + a);
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = acc[j];
        for (int k = 1; k < 4; ++k)
            for (int j = 0; j < 8; ++j) r[j] = acc[k * 8 + j] + r[j];
        for (int h = 4; h >= 1; h >>= 1)
            for (int j = 0; j < h; ++j) r[j] = r[j] + r[j + h];
        v = r[0];
        i += Q * 32;
    }
    for (; i <= l; ++i) v = v + seg_term_z(w, zeta, s0 + i);
    return v;
}

template <class Z>
__device__ __attribute__((noinline)) double julia_pairwise_lane(const double *__restrict__ w, const Z zeta, int s0, int L) {
    int ff[48], ll[48], st[48];
    double vals[48];
    int top = 1, nv = 0;
    ff[0] = 0;
    ll[0] = L - 1;
    st[0] = 0;
    while (top > 0) {
        const int f = ff[top - 1], l = ll[top - 1];
        if (l - f < 1024) {
            vals[nv++] = julia_block_lane(w, zeta, s0, f, l);
            --top;
            continue;
        }
        const int mid = f + ((l - f) >> 1);
        if (st[top - 1] == 0) {
            st[top - 1] = 1;
            ff[top] = f; ll[top] = mid; st[top] = 0; ++top;
        } else if (st[top - 1] == 1) {
            st[top - 1] = 2;
            ff[top] = mid + 1; ll[top] = l; st[top] = 0; ++top;
        } else {
            const double v2 = vals[--nv];
            const double v1 = vals[--nv];
            vals[nv++] = v1 + v2;
            --top;
        }
    }
    return vals[0];
}

// Returns the ray's t* on lane 0 (other lanes: unspecified).  s0 = first point
// of the ray, np = its valid points.  scratch: 96 doubles (this wave only).
template <class Z>
__device__ double wave_ray_sum(int lane, const double *__restrict__ w, const Z &zeta, int s0, int np,
                               double *scratch) {
    double *acc_sh = scratch;       // 32
    double *seq_sh = scratch + 32;  // 64
    const int L = np > 0 ? np - 1 : 0;
    double res = 0.0;  // sum over an empty array
    if (L == 1) {
        res = seg_term_z(w, zeta, s0);
    } else if (L >= 2 && L < 16) {
        if (lane < L) seq_sh[lane] = seg_term_z(w, zeta, s0 + lane);
        wave_sync_lds();
        if (lane == 0) {
            double s = seq_sh[0] + seq_sh[1];
            for (int a = 2; a < L; ++a) s = s + seq_sh[a];
            res = s;
        }
    } else if (L >= 16 && L <= 1024) {
        const int T = L - 2;
        const int Q = T >= 32 ? T / 32 : 0;
        const int tail0 = 2 + 32 * Q;
        const int ntail = L - tail0;  // <= 31
        if (Q > 0 && lane < 32) {
            double acc = 0.0;
            if (lane == 0) acc = seg_term_z(w, zeta, s0) + seg_term_z(w, zeta, s0 + 1);
            // four accumulator steps' terms loaded before any is added (one round of loads for
            // a ray of up to 130 segments), then added in q order: the same association
            for (int q0 = 0; q0 < Q; q0 += 4) {
                double t[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    t[u] = q0 + u < Q ? seg_term_z(w, zeta, s0 + 2 + 32 * (q0 + u) + lane) : 0.0;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (q0 + u < Q) acc = acc + t[u];
            }
            acc_sh[lane] = acc;
        }
        if (lane < ntail) seq_sh[lane] = seg_term_z(w, zeta, s0 + tail0 + lane);
        wave_sync_lds();
        if (lane == 0) {
            double v;
            if (Q > 0) {
                double r[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = acc_sh[j];
#pragma unroll
                for (int k = 1; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < 8; ++j) r[j] = acc_sh[k * 8 + j] + r[j];
                r[0] = r[0] + r[4];
                r[1] = r[1] + r[5];
                r[2] = r[2] + r[6];
                r[3] = r[3] + r[7];
                r[0] = r[0] + r[2];
                r[1] = r[1] + r[3];
                v = r[0] + r[1];
            } else {
                v = seg_term_z(w, zeta, s0) + seg_term_z(w, zeta, s0 + 1);
            }
            for (int a = 0; a < ntail; ++a) v = v + seq_sh[a];
            res = v;
        }
    } else if (L > 1024) {
        if (lane == 0) res = julia_pairwise_lane(w, zeta, s0, L);
    }
    wave_sync_lds();  // scratch may be reused by this wave right after
    return res;
}

// wave_ray_sum on HALF a wave: lanes 0..31 sum one ray and lanes 32..63 another, in the same
// instructions -- two rays' loads in one round trip (the rays in HBM, where a ray's loads are
// the phase's latency).  hl = lane % 32; the half's result on its lane hl == 0.  The same terms
// in the same association as wave_ray_sum (a 32-lane accumulator step is what it uses too).
// scratch: 96 doubles per half.  np = 0: nothing (the half has no ray).
template <class Z>
__device__ double half_ray_sum(int hl, const double *__restrict__ w, const Z &zeta, int s0, int np, double *scratch) {
    double *acc_sh = scratch;       // 32
    double *seq_sh = scratch + 32;  // 64
    const int L = np > 0 ? np - 1 : 0;
    double res = 0.0;  // sum over an empty array
    if (L == 1) {
        res = seg_term_z(w, zeta, s0);
    } else if (L >= 2 && L < 16) {
        if (hl < L) seq_sh[hl] = seg_term_z(w, zeta, s0 + hl);
        wave_sync_lds();
        if (hl == 0) {
            double s = seq_sh[0] + seq_sh[1];
            for (int a = 2; a < L; ++a) s = s + seq_sh[a];
            res = s;
        }
    } else if (L >= 16 && L <= 1024) {
        const int T = L - 2;
        const int Q = T >= 32 ? T / 32 : 0;
        const int tail0 = 2 + 32 * Q;
        const int ntail = L - tail0;  // <= 31
        if (Q > 0) {
            double acc = 0.0;
            if (hl == 0) acc = seg_term_z(w, zeta, s0) + seg_term_z(w, zeta, s0 + 1);
            for (int q0 = 0; q0 < Q; q0 += 4) {
                double t[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    t[u] = q0 + u < Q ? seg_term_z(w, zeta, s0 + 2 + 32 * (q0 + u) + hl) : 0.0;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (q0 + u < Q) acc = acc + t[u];
            }
            acc_sh[hl] = acc;
        }
        if (hl < ntail) seq_sh[hl] = seg_term_z(w, zeta, s0 + tail0 + hl);
        wave_sync_lds();
        if (hl == 0) {
            double v;
            if (Q > 0) {
                double r[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = acc_sh[j];
#pragma unroll
                for (int k = 1; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < 8; ++j) r[j] = acc_sh[k * 8 + j] + r[j];
                r[0] = r[0] + r[4];
                r[1] = r[1] + r[5];
                r[2] = r[2] + r[6];
                r[3] = r[3] + r[7];
                r[0] = r[0] + r[2];
                r[1] = r[1] + r[3];
                v = r[0] + r[1];
            } else {
                v = seg_term_z(w, zeta, s0) + seg_term_z(w, zeta, s0 + 1);
            }
            for (int a = 0; a < ntail; ++a) v = v + seq_sh[a];
            res = v;
        }
    } else if (L > 1024) {
        if (hl == 0) res = julia_pairwise_lane(w, zeta, s0, L);
    }
    wave_sync_lds();  // scratch may be reused by this wave right after
    return res;
}

struct PlainZeta {
    const double *z;
    __device__ __forceinline__ double operator()(int k) const { return z[k]; }
};

}  // namespace tdstar
