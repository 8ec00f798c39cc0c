// exact_sum.h -- the sequential sum of MCsub.jl:169-172
//     C = C0;  for k in 1:n  C += term[k]  end
// reproduced bit for bit by a whole workgroup, for long sums (the 10k-ray
// stress geometry: one lane needs ~10k dependent FP64 adds, ~90 us).
//
// All terms are >= 0, so the partial sums never decrease.  While C stays in
// one binade [2^b, 2^(b+1)) every partial sum is M*u with u = 2^(b-52) and
// 2^52 <= M < 2^53, and one rounded step C + t is an integer step on M:
//     x = t/u (exact);  f = floor(x);  frac < 1/2: M += f;  > 1/2: M += f+1;
//     == 1/2: M becomes the even one of M+f, M+f+1   (ties-to-even)
// i.e. M -> M + D[M mod 2] with two integers D, a class closed under
// composition.  So a run of terms inside one binade is a SCAN.  The block:
//   A. sums its chunks and scans the chunk sums (any association) to label
//      every partial sum with a binade guess; a change of label starts a
//      segment;
//   B. turns each term into its step for its label's unit and scans the steps
//      (segmented: a segment's first term is not a step, see C);
//   C. thread 0 walks the segments in order: the first term of a segment is
//      added with an ordinary FP64 add (the reference's own operation), the
//      rest of the segment is its composed step;
//   D. checks every guess (each segment's first sum lies in its binade, its
//      last one below the top) and reports failure otherwise: the caller then
//      runs the one-lane loop.  The result is always the sequential sum.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "wave_ops.h"

namespace tdstar {

constexpr int kExactMaxSeg = 128;  // binade segments (more: the caller's loop)

struct ExactSumLds {
    double wsum[16];                  // per-wave totals of the approximate scan
    unsigned long long wd0[16], wd1[16];
    int wreset[16], wcnt[16];
    int first_start[1025];            // does thread j's first term start a segment (+1 sentinel)
    int last_b[1024];                 // label of thread j's last term
    int seg_b[kExactMaxSeg];
    double seg_t[kExactMaxSeg];
    unsigned long long seg_d0[kExactMaxSeg], seg_d1[kExactMaxSeg], seg_base[kExactMaxSeg];
    double C_end;
    int nseg, ok;
};

namespace exact_detail {

__device__ __forceinline__ int binade(double x) {  // x > 0 normal: floor(log2 x)
    return (int)(((unsigned long long)__double_as_longlong(x) >> 52) & 0x7ff) - 1023;
}
__device__ __forceinline__ double pow2(int e) {  // 2^e, -1022 <= e <= 1023
    return __longlong_as_double((long long)((unsigned long long)(e + 1023) << 52));
}

// M -> M + d[M & 1]; `reset`: a segment's first term (identity step; scans restart there)
struct Step {
    unsigned long long d0, d1;
    int reset;
};
__device__ __forceinline__ Step then(const Step &a, const Step &b) {  // a first, then b
    if (b.reset) return b;
    Step r;
    r.d0 = a.d0 + ((a.d0 & 1ull) ? b.d1 : b.d0);
    r.d1 = a.d1 + ((a.d1 & 1ull) ? b.d0 : b.d1);
    r.reset = a.reset;
    return r;
}
// the step of term t in a segment of binade b (not its first term); bad: not representable
__device__ __forceinline__ Step step_of(double t, int b, bool &bad) {
    Step e{0ull, 0ull, 0};
    const double x = t * pow2(52 - b);  // exact: a power-of-two scaling
    if (!(x < 9007199254740992.0)) {    // >= 2^53 (or NaN): the sum leaves the binade
        bad = true;
        return e;
    }
    const double f = floor(x);
    const double r = x - f;  // exact
    const unsigned long long fi = (unsigned long long)f;
    if (r < 0.5) {
        e.d0 = e.d1 = fi;
    } else if (r > 0.5) {
        e.d0 = e.d1 = fi + 1ull;
    } else {                                 // halfway: land on the even integer
        e.d0 = fi + (fi & 1ull);             // M even: M + f is even iff f is
        e.d1 = fi + ((fi & 1ull) ^ 1ull);    // M odd:  M + f is even iff f is odd
    }
    return e;
}
__device__ __forceinline__ unsigned long long apply(const Step &s, unsigned long long M) {
    return M + ((M & 1ull) ? s.d1 : s.d0);
}

// exclusive block scans through the wave shuffles + one LDS round (T threads)
template <int T>
__device__ double block_excl_f64(double v, ExactSumLds &w) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(incl, o, 64);
        if (lane >= o) incl = incl + u;
    }
    if (lane == 63) w.wsum[wv] = incl;
    __syncthreads();
    double base = 0.0;
    for (int k = 0; k < wv; ++k) base = base + w.wsum[k];
    __syncthreads();
    return base + (incl - v);
}
template <int T>
__device__ Step block_excl_step(const Step &v, ExactSumLds &w) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    Step incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        Step u;
        u.d0 = __shfl_up(incl.d0, o, 64);
        u.d1 = __shfl_up(incl.d1, o, 64);
        u.reset = __shfl_up(incl.reset, o, 64);
        if (lane >= o) incl = then(u, incl);
    }
    Step ex;
    ex.d0 = __shfl_up(incl.d0, 1, 64);
    ex.d1 = __shfl_up(incl.d1, 1, 64);
    ex.reset = __shfl_up(incl.reset, 1, 64);
    if (lane == 0) ex = Step{0ull, 0ull, 0};
    if (lane == 63) {
        w.wd0[wv] = incl.d0;
        w.wd1[wv] = incl.d1;
        w.wreset[wv] = incl.reset;
    }
    __syncthreads();
    Step base{0ull, 0ull, 0};
    for (int k = 0; k < wv; ++k) base = then(base, Step{w.wd0[k], w.wd1[k], w.wreset[k]});
    __syncthreads();
    return then(base, ex);
}
template <int T>
__device__ int block_excl_int(int v, int &total, ExactSumLds &w) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) w.wcnt[wv] = incl;
    __syncthreads();
    int base = 0;
    total = 0;
    for (int k = 0; k < T / 64; ++k) {
        if (k < wv) base += w.wcnt[k];
        total += w.wcnt[k];
    }
    __syncthreads();
    return base + incl - v;
}

}  // namespace exact_detail

// The block's T threads (all of them must call) sum term[0..cnt) after C0.
// On success: *C_end (every thread), prefix[k] = C after term k if prefix is
// non-null; returns true.  On failure (a guess did not hold) returns false and
// writes nothing: the caller adds the terms one by one.
template <int T>
__device__ bool block_exact_sum(const double *term, int cnt, double C0, double *prefix, double *C_end,
                                ExactSumLds &w) {
    using namespace exact_detail;
    static_assert(T <= 1024 && T % 64 == 0, "block size");
    const int tid = threadIdx.x;
    const int E = (cnt + T - 1) / T;
    const int lo = min(cnt, tid * E), hi = min(cnt, lo + E);
    // ---- A: approximate partial sums -> a binade label per term ----
    double S = 0.0;
    for (int k = lo; k < hi; ++k) S = S + term[k];
    const double run0 = C0 + block_excl_f64<T>(S, w);
    bool bad = !(C0 >= 0.0);
    {
        double run = run0;
        int lb = 0;
        for (int k = lo; k < hi; ++k) {
            const double t = term[k];
            run = run + t;
            const int b = binade(run);
            if (!(t >= 0.0) || !(run > 0.0) || !(run < 1e300) || b < -960) bad = true;
            lb = b;
        }
        w.last_b[tid] = lb;
    }
    __syncthreads();
    // ---- B: steps, segment starts, local composition ----
    auto label_before = [&](int j) { return w.last_b[j]; };
    Step loc{0ull, 0ull, 0};
    int nstart = 0;
    {
        double run = run0;
        int pb = 0;
        // the last label of the nearest earlier thread that owns terms
        for (int j = tid - 1; j >= 0 && lo > 0; --j) {
            if (min(cnt, j * E) < min(cnt, j * E + E)) {
                pb = label_before(j);
                break;
            }
        }
        for (int k = lo; k < hi; ++k) {
            const double t = term[k];
            run = run + t;
            const int b = binade(run);
            const bool st = k == 0 || b != pb;
            Step e{0ull, 0ull, st ? 1 : 0};
            if (!st) e = step_of(t, b, bad);
            if (k == lo) w.first_start[tid] = st ? 1 : 0;
            loc = then(loc, e);
            nstart += st ? 1 : 0;
            pb = b;
        }
        if (lo >= hi) w.first_start[tid] = 0;
        if (tid == 0) w.first_start[T] = 1;  // past the end
    }
    w.ok = 1;
    __syncthreads();
    if (bad) w.ok = 0;
    int nseg = 0;
    const int soff = block_excl_int<T>(nstart, nseg, w);  // also a barrier: w.ok is final
    const Step ex = block_excl_step<T>(loc, w);
    if (!w.ok || nseg > kExactMaxSeg || nseg < 1) return false;
    // ---- per segment: binade, first term, composed step of the rest ----
    {
        double run = run0;
        int s = soff - 1, pb = 0;
        for (int j = tid - 1; j >= 0 && lo > 0; --j)
            if (min(cnt, j * E) < min(cnt, j * E + E)) {
                pb = w.last_b[j];
                break;
            }
        Step acc = ex;
        for (int k = lo; k < hi; ++k) {
            const double t = term[k];
            run = run + t;
            const int b = binade(run);
            const bool st = k == 0 || b != pb;
            bool dummy = false;
            const Step e = st ? Step{0ull, 0ull, 1} : step_of(t, b, dummy);
            acc = then(acc, e);
            if (st) {
                ++s;
                w.seg_b[s] = b;
                w.seg_t[s] = t;
            }
            // the segment ends here if the next term starts one
            bool next_st;
            if (k + 1 < hi) {
                const double r2 = run + term[k + 1];
                next_st = binade(r2) != b;
            } else {
                int jn = tid + 1;  // the next thread that owns terms
                while (jn < T && min(cnt, jn * E) >= min(cnt, jn * E + E)) ++jn;
                next_st = jn >= T || w.first_start[jn] != 0;
            }
            if (next_st) {
                w.seg_d0[s] = acc.d0;
                w.seg_d1[s] = acc.d1;
            }
            pb = b;
        }
    }
    __syncthreads();
    // ---- C: the segments in order, one thread ----
    if (tid == 0) {
        int ok = 1;
        double C = C0;
        for (int g = 0; g < nseg && ok; ++g) {
            if (g > 0) {  // the previous segment's last sum
                const unsigned long long M0 = w.seg_base[g - 1];
                const unsigned long long M = M0 + ((M0 & 1ull) ? w.seg_d1[g - 1] : w.seg_d0[g - 1]);
                if (M >= (1ull << 53)) ok = 0;
                C = (double)M * pow2(w.seg_b[g - 1] - 52);
            }
            C = C + w.seg_t[g];  // the reference's own rounded add
            if (!(C > 0.0) || binade(C) != w.seg_b[g]) ok = 0;
            w.seg_base[g] = ok ? (unsigned long long)(C * pow2(52 - w.seg_b[g])) : 0ull;
        }
        if (ok) {
            const unsigned long long M0 = w.seg_base[nseg - 1];
            const unsigned long long M = M0 + ((M0 & 1ull) ? w.seg_d1[nseg - 1] : w.seg_d0[nseg - 1]);
            if (M >= (1ull << 53)) ok = 0;
            w.C_end = (double)M * pow2(w.seg_b[nseg - 1] - 52);
        }
        w.ok = ok;
    }
    __syncthreads();
    if (!w.ok) return false;
    *C_end = w.C_end;
    // ---- D: every partial sum: its segment's first sum with the step so far ----
    if (prefix) {
        double run = run0;
        int s = soff - 1, pb = 0;
        for (int j = tid - 1; j >= 0 && lo > 0; --j)
            if (min(cnt, j * E) < min(cnt, j * E + E)) {
                pb = w.last_b[j];
                break;
            }
        Step acc = ex;
        for (int k = lo; k < hi; ++k) {
            const double t = term[k];
            run = run + t;
            const int b = binade(run);
            const bool st = k == 0 || b != pb;
            bool dummy = false;
            const Step e = st ? Step{0ull, 0ull, 1} : step_of(t, b, dummy);
            acc = then(acc, e);
            if (st) ++s;
            prefix[k] = (double)apply(acc, w.seg_base[s]) * pow2(w.seg_b[s] - 52);
            pb = b;
        }
    }
    return true;
}

// ---- one wave: the sequential sum of a short tail (the chain's chi^2) ----
// out[k] = C_k with C_k = C_{k-1} + t[k] (C_{-1} = C), k = 0..cnt-1, FP64 left
// to right -- the loop of MCsub.jl:170-172 bit for bit; returns C_{cnt-1}.
// The binade argument above without its general tie handling: while C stays
// in [2^b, 2^(b+1)) and no t/u is a tie, every step adds the integer rint(t/u)
// to M, and integers < 2^53 add exactly in any order, so a run of terms is a
// DPP scan; a tie (t/u = k + 1/2) steps by k or k + 1 whichever makes M even,
// settled tie by tie in order after the scan.  A round scans the next 64 terms
// at the unit of C's binade, keeps the values up to the first term that leaves
// the binade or is not >= 0, adds that term with an ordinary FP64 add (the
// reference's own operation) and starts the next round after it.  One wave is latency-bound:
// a round costs ~500 cycles, the one-lane loop ~30 per term (more rows per
// round were measured slower: tools/sum_bench.hip).  Every lane of the wave
// calls it with the same arguments; out may be null (only the total is
// wanted); *stop (if given) is polled once per round: when set, the sum is
// abandoned and *stopped set.
namespace wseq {
__device__ __forceinline__ int expo(double x) {  // biased exponent (sign set: >= 2048)
    return (int)((unsigned long long)__double_as_longlong(x) >> 52);
}
__device__ __forceinline__ double p2(int biased) {  // 2^(biased - 1023), 1 <= biased <= 2046
    return __longlong_as_double((long long)((unsigned long long)biased << 52));
}
}  // namespace wseq

__device__ __forceinline__ double wave_seq_sum(const double *t, int cnt, double C, double *out, int lane,
                                               const int *stop, bool *stopped, long long *rounds = nullptr) {
    using namespace wseq;
    int pos = 0;
    double tv = lane < cnt ? t[lane] : 0.0;  // the window [pos, pos + 64)
    while (pos < cnt) {
        if (rounds && lane == 0) *rounds += 1;  // diagnostic
        const int lim = min(64, cnt - pos);
        // the next window, if this round keeps all 64 terms
        const double tn = pos + 64 + lane < cnt ? t[pos + 64 + lane] : 0.0;
        if (stop && __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            *stopped = true;
            return C;
        }
        const int eb = expo(C);
        int f;  // first term off the run
        double Ci = C;
        if (eb < 64 || eb > 2000) {  // 0, tiny, huge, inf, NaN or negative: one plain step
            f = 0;
        } else {
            const double u = p2(eb - 52), top = p2(eb + 1);
            const bool act = lane < lim;  // (bitwise & |: no branches)
            const double x = act ? tv * p2(2098 - eb) : 0.0;  // t/u, exact
            const double fl = __builtin_floor(x);
            const bool tie = act & (x - fl == 0.5);
            // ties step by floor(x) first; each is then rounded to even in order below
            Ci = C + wave_scan_f64(tie ? fl : __builtin_rint(x)) * u;  // exact below top
            unsigned long long ties = __ballot(tie);
            while (ties) {  // (M + k) + 1/2 rounds to the even one of M + k, M + k + 1
                const int l = __builtin_ctzll(ties);
                ties &= ties - 1;
                const unsigned lo32 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)__double_as_longlong(Ci), l);
                if (lo32 & 1u) Ci = lane >= l ? Ci + u : Ci;  // odd: one unit up from lane l on
            }
            const unsigned long long bad = __ballot(act & (!(tv >= 0.0) | !(Ci < top)));
            f = bad ? __builtin_ctzll(bad) : lim;
            if (out && lane < f) out[pos + lane] = Ci;
        }
        if (f < lim) {
            C = (f > 0 ? readlane_f64(Ci, f - 1) : C) + readlane_f64(tv, f);  // the reference's add
            if (out && lane == 0) out[pos + f] = C;
            pos += f + 1;
            if (f < 16 && pos + 16 <= cnt) {  // short runs (small sums cross binades often): plain adds
                double tt[16], cc[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) tt[u] = t[pos + u];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    C = C + tt[u];
                    cc[u] = C;
                }
                if (out && lane < 16) {
                    double o = cc[0];
#pragma unroll
                    for (int u = 1; u < 16; ++u) o = lane == u ? cc[u] : o;
                    out[pos + lane] = o;
                }
                pos += 16;
            }
            tv = pos + lane < cnt ? t[pos + lane] : 0.0;
        } else {
            C = readlane_f64(Ci, lim - 1);
            pos += lim;
            tv = tn;
        }
    }
    return C;
}

// ---- one wave: the sequential sum again after a few of its terms changed ----
// out[k] = C_k, C_k = C_{k-1} + t[k] (C_{-1} = C, the same value before and
// after the change), given the OLD partial sums old[k] (the same recurrence
// over the old terms) and chg[k] != 0 where t[k] changed.  Between changed
// terms the new sum follows the old one at a constant offset D: if old[k-1]
// and old[k] lie in one binade [2^b, 2^(b+1)), old[k-1] + D and old[k] + D in
// the same one, and t[k]/u is not a tie (or D/u is even: the same parity), both
// sums take the same rounded step, so C_k = old[k] + D exactly.  A term where
// that does not hold, or that changed, is added with an ordinary FP64 add (the
// reference's operation) and D is re-derived (and checked exact).  Each round
// checks 64 terms with a few VALU ops and a ballot -- no scan -- so a long tail
// with few changed terms (the chain after one proposal) costs little more than
// reading it.  Every lane of the wave calls it with the same arguments; *stop
// (if given) is polled once per round.
namespace wdelta {
__device__ __forceinline__ double shr1_f64(double v, double first) {  // lane l: v of lane l-1; lane 0: first
    const unsigned long long b = (unsigned long long)__double_as_longlong(v),
                             f = (unsigned long long)__double_as_longlong(first);
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)f, (int)(unsigned)b, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(f >> 32), (int)(unsigned)(b >> 32), 0x138, 0xf, 0xf,
                                               false);  // wave_shr:1
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
}  // namespace wdelta

// wave_delta_run: the same from different sums before the first term
// (prev_old = old[-1], prev_new = the new sum there); wave_delta_sum starts
// both at C.
__device__ __forceinline__ double wave_delta_run(const double *t, const double *old, const int *chg, int cnt,
                                                 double prev_old, double prev_new, double *out, int lane,
                                                 const int *stop, bool *stopped, long long *rounds = nullptr) {
    using namespace wseq;
    double D = prev_new - prev_old;  // new - old at the last settled position
    bool dexact = (prev_old + D == prev_new) && (prev_new - D == prev_old);
    // 64-term windows, the next one in flight
    auto ld = [&](int p, double &tv, double &ov, int &cv) {
        const bool in = p + lane < cnt;
        tv = in ? t[p + lane] : 0.0;
        ov = in ? old[p + lane] : 0.0;
        cv = in ? chg[p + lane] : 0;
    };
    double tv, ov, tn, on;
    int cv, cn;
    ld(0, tv, ov, cv);
    ld(64, tn, on, cn);
    for (int base = 0; base < cnt; base += 64) {
        const int lim = min(64, cnt - base);
        if (stop && __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            *stopped = true;
            return prev_new;
        }
        const double op = wdelta::shr1_f64(ov, prev_old);  // old[k - 1] (lane 0: the window's predecessor)
        const int bo = expo(op), eo = expo(ov);
        const double inv_u = p2(2098 - min(max(bo, 64), 2000));
        const double x = tv * inv_u;  // t/u (exact: power-of-two scaling)
        const bool tie = x - __builtin_floor(x) == 0.5;
        // what does not depend on the offset (bitwise & |: no branches)
        const int fixed = (int)(cv == 0) & (int)(bo >= 64) & (int)(bo <= 2000) & (int)(eo == bo) & (int)(tv >= 0.0);
        int lo = 0;
        while (true) {  // settle runs at offset D; a failing term is added plainly, D re-derived
            if (rounds && lane == 0) *rounds += 1;  // diagnostic
            const double np = op + D, nk = ov + D;  // the new sums at k - 1 and k, if the offset holds
            const double dq = D * inv_u;            // D/u (exact)
            const bool dodd = dq - 2.0 * __builtin_floor(dq * 0.5) != 0.0;
            const bool ok = (fixed & (int)dexact & (int)(expo(np) == bo) & (int)(expo(nk) == bo) &
                             (int)!(tie && dodd)) != 0;
            const bool mine = lane >= lo && lane < lim;
            const unsigned long long bad = __ballot(mine && !ok);
            const int f = bad ? __builtin_ctzll(bad) : lim;
            if (out && mine && lane < f) out[base + lane] = nk;
            if (f == lim) {
                prev_old = readlane_f64(ov, lim - 1);
                prev_new = readlane_f64(nk, lim - 1);
                break;
            }
            const double cnm1 = f > lo ? readlane_f64(nk, f - 1) : prev_new;
            const double cnew = cnm1 + readlane_f64(tv, f);  // the reference's add
            const double cold = readlane_f64(ov, f);
            if (out && lane == 0) out[base + f] = cnew;
            D = cnew - cold;
            dexact = (cold + D == cnew) && (cnew - D == cold);
            prev_old = cold;
            prev_new = cnew;
            lo = f + 1;
            if (lo >= lim) break;
        }
        tv = tn;
        ov = on;
        cv = cn;
        ld(base + 128, tn, on, cn);
    }
    return prev_new;
}

__device__ __forceinline__ double wave_delta_sum(const double *t, const double *old, const int *chg, int cnt,
                                                 double C, double *out, int lane, const int *stop, bool *stopped,
                                                 long long *rounds = nullptr) {
    return wave_delta_run(t, old, chg, cnt, C, C, out, lane, stop, stopped, rounds);
}

// ---- the whole block: the sequential sum again, walking only its events ----
// The same problem as wave_delta_sum (new terms t, OLD partial sums old),
// split so its cost follows the number of changed terms rather than the length
// of the tail.  A term k is an EVENT when its step cannot be inferred from the
// old sums whatever the offset: it changed, it is not >= 0, old[k-1] and
// old[k] lie in different binades (or outside [2^-959, 2^977]), or t/u is a
// tie.  Between two events every old partial sum lies in ONE binade b, so a
// constant offset D = new - old (a multiple of u = 2^(b-52), checked exact)
// carries over the whole run exactly when the run's first and last shifted
// sums stay in binade b (the shifted sums are monotone): two checks per run
// instead of one per term.  An event is added with an ordinary FP64 add (the
// reference's operation, MCsub.jl:172) and re-derives D.  A run that fails its
// checks (rare: the new sum crosses a binade the old one does not) is handed
// to wave_delta_run, term by term.
//   delta_marks : the STATIC event bits (everything but "changed") of 64-term
//                 words; the chain keeps them across proposals (delta_remark);
//   delta_walk  : one wave walks the events in order (64 at a time: their
//                 positions from the words OR the changed-term words, their
//                 old sums and terms in one round of loads) and records the
//                 new sums as segments: OFFSET (old + D), VALUE (one event's
//                 sum) or COPY (written to out by wave_delta_run);
//   delta_remark: after an accepted proposal, the static bits that can change:
//                 around VALUE events and inside COPY segments (an OFFSET run
//                 stays in its binade, so its bits stand);
//   delta_commit: the block applies the segments to old in place.
constexpr int kDeltaSegCap = 128;
constexpr int kSegOffset = 0, kSegValue = 1, kSegCopy = 2;
constexpr int kSegPosMask = (1 << 29) - 1;

struct DeltaSegs {
    int sm[kDeltaSegCap];  // start | mode << 29
    double v[kDeltaSegCap];  // OFFSET: D, VALUE: the sum
    int evbuf[64];           // event positions of the batch being walked
    int nseg, k0;
};

__host__ __device__ __forceinline__ int delta_words(int n) { return (n + 63) >> 6; }

// the static event bit of term k: t = t[k], pm = old[k-1] (0 for k = 0), pk = old[k]
__device__ __forceinline__ bool delta_static_event(double t, double pm, double pk) {
    using namespace wseq;
    const int bo = expo(pm), eo = expo(pk);
    const double x = t * p2(2098 - min(max(bo, 64), 2000));  // t/u (exact)
    const bool tie = x - __builtin_floor(x) == 0.5;
    return !((t >= 0.0) & (bo == eo) & (bo >= 64) & (bo <= 2000) & !tie);
}

// Event words w_first, w_first + w_step, ... below w_end (one wave per call);
// chg (nullable) adds the changed terms.
__device__ __forceinline__ void delta_marks(const double *t, const double *old, const int *chg, int n,
                                            unsigned long long *mask, int w_first, int w_end, int w_step, int lane) {
    constexpr int U = 4;  // words in flight
    for (int w0 = w_first; w0 < w_end; w0 += U * w_step) {
        double tv[U], ov[U], pv[U];
        int cv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = min(64 * (w0 + u * w_step) + lane, n - 1);  // clamped: loads stay unconditional
            tv[u] = t[k];
            ov[u] = old[k];
            pv[u] = old[max(k - 1, 0)];
            cv[u] = chg ? chg[k] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int w = w0 + u * w_step;
            const int k = 64 * w + lane;
            const bool ev = delta_static_event(tv[u], k > 0 ? pv[u] : 0.0, ov[u]) | (cv[u] != 0);
            const unsigned long long m = __ballot(k < n && ev);
            if (w < w_end && lane == 0) mask[w] = m;
        }
    }
}

// One wave, every lane with the same arguments; C0 = the sum before k0 (old
// and new alike); the events are the bits of smask | cmask from k0 on (cmask
// nullable; its words are cleared as they are read).  Returns the new sum
// through n-1; sg holds the segments.
__device__ double delta_walk(const double *t, const double *old, const int *chg, int k0, int n, double C0,
                             const unsigned long long *smask, unsigned long long *cmask, double *out, DeltaSegs &sg,
                             int lane, long long *diag = nullptr) {
    // diag (diagnostic, nullable): [0] events, [1] cycles in batch loads, [2] cycles walking
    // events, [3] terms added by wave_delta_run
    using namespace wseq;
    const int w0 = k0 >> 6, W = delta_words(n);
    double prev_old = C0, prev_new = C0;  // the sums just before p
    int p = k0, nseg = 0;
    bool mat = false;  // the segment table is full: the rest goes to out
    auto seg = [&](int start, int mode, double v) -> bool {  // false: write out[] instead
        if (mat) return false;
        if (nseg == kDeltaSegCap - 1) {
            mat = true;
            mode = kSegCopy;
        }
        if (lane == 0) {
            sg.sm[nseg] = start | (mode << 29);
            sg.v[nseg] = v;
        }
        ++nseg;
        return !mat;
    };
    auto offset_run = [&](int e, double D) {  // [p, e) at offset D
        if (!seg(p, kSegOffset, D))
            for (int k = p + lane; k < e; k += 64) out[k] = old[k] + D;
    };
    auto run = [&](int s, double cend) {  // the run [p, s), old[s-1] = cend
        const int b = expo(cend);         // every old sum of the run lies in binade b
        while (p < s) {
            const double D = prev_new - prev_old;
            const bool dex = (prev_old + D == prev_new) && (prev_new - D == prev_old);
            const int bn = expo(prev_new);
            if (dex && bn == b && expo(cend + D) == b) {  // the whole rest at offset D
                offset_run(s, D);
                prev_new = cend + D;
                prev_old = cend;
                p = s;
                return;
            }
            if (dex && bn == b) {
                // the new sums leave binade b before the old ones (D > 0): the offset
                // holds up to the first k with old[k] + D outside b, the rest of the
                // run is added term by term (one window of loads)
                const int k = s - 64 + lane;
                const double ow = old[max(k, 0)], tw = t[max(k, 0)];
                const unsigned long long bad = __ballot(k >= p && expo(ow + D) != b);
                const int fl = __builtin_ctzll(bad);  // lane 63 (k = s - 1) fails
                const int f = s - 64 + fl;
                if (fl > 0 || f == p) {
                    double C = prev_new;
                    if (f > p) {
                        offset_run(f, D);
                        C = readlane_f64(ow, fl - 1) + D;
                    }
                    seg(f, kSegCopy, 0.0);
                    if (diag && lane == 0) diag[3] += s - f;
                    for (int i = fl; i < 64; ++i) {
                        C = C + readlane_f64(tw, i);  // the reference's add
                        if (lane == 0) out[s - 64 + i] = C;
                    }
                    prev_new = C;
                    prev_old = cend;
                    p = s;
                    return;
                }
            } else if (dex && bn < b && prev_new >= 0.0) {
                // the new sum has not reached binade b yet (D < 0): term by term until it
                // does (one window of loads per 64 terms), then the offset again
                const int cnt = min(64, s - p);
                const int k = min(p + lane, s - 1);
                const double ow = old[k], tw = t[k];
                seg(p, kSegCopy, 0.0);
                double C = prev_new, O = prev_old;
                int i = 0;
                for (; i < cnt; ++i) {
                    C = C + readlane_f64(tw, i);  // the reference's add
                    O = readlane_f64(ow, i);
                    if (lane == 0) out[p + i] = C;
                    if (expo(C) >= b) break;
                }
                const int used = i < cnt ? i + 1 : cnt;
                if (diag && lane == 0) diag[3] += used;
                prev_new = C;
                prev_old = O;
                p += used;
                continue;
            }
            // anything else (rare): term by term to the end of the run
            seg(p, kSegCopy, 0.0);
            if (diag && lane == 0) diag[3] += s - p;
            prev_new = wave_delta_run(t + p, old + p, chg + p, s - p, prev_old, prev_new, out + p, lane, nullptr,
                                      nullptr);
            prev_old = cend;
            p = s;
        }
    };
    auto event = [&](int s, double os, double ts) {
        const double cnew = prev_new + ts;  // the reference's add
        if (!seg(s, kSegValue, cnew) && lane == 0) out[s] = cnew;
        prev_old = os;
        prev_new = cnew;
        p = s + 1;
    };
    for (int wb = w0; wb < W; wb += 64) {  // 64 words = 4096 terms at a time
        const int wi = wb + lane;
        unsigned long long m = 0ull;
        if (wi < W) {
            m = smask[wi];
            if (cmask) {
                m |= cmask[wi];
                cmask[wi] = 0ull;
            }
            if (wi == w0) m &= ~0ull << (k0 & 63);
        }
        const int pc = __popcll(m);
        const int incl = (int)wave_scan_f64((double)pc);
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        if (tot == 0) continue;
        if (tot <= 64) {
            int e = incl - pc;
            for (unsigned long long mm = m; mm; mm &= mm - 1) sg.evbuf[e++] = 64 * wi + __builtin_ctzll(mm);
            wave_sync_lds();
            const long long c0 = diag ? clock64() : 0;
            const int sl = lane < tot ? sg.evbuf[lane] : k0;
            const double os = old[sl], om = old[max(sl - 1, 0)], ts = t[sl];  // one round of loads
            wave_sync_lds();  // evbuf read before the next batch rewrites it
            long long c1 = 0;
            if (diag) {
                const double probe = os + om + ts;  // wait for the loads
                c1 = clock64();
                if (lane == 0) {
                    diag[0] += tot;
                    diag[1] += c1 - c0 + (probe == 1.2345e300 ? 1 : 0);
                }
            }
            // Speculative pass: every run at its offset (3 dependent adds per event),
            // lane j keeping what event j saw; then all runs checked at once; the
            // events before the first failed check stand, the rest go the slow way.
            double pnv = 0.0, pov = 0.0, cv = 0.0;
            int hasv = 0;
            {
                double pn = prev_new, po = prev_old;
                int pp = p;
                for (int j = 0; j < tot; ++j) {
                    const int sj = __builtin_amdgcn_readlane(sl, j);
                    const double omj = readlane_f64(om, j), tsj = readlane_f64(ts, j), osj = readlane_f64(os, j);
                    const bool has = sj > pp;
                    const double pr = has ? omj + (pn - po) : pn;  // new sum at s - 1
                    const double c = pr + tsj;                     // the reference's add
                    if (lane == j) {
                        pnv = pn;
                        pov = po;
                        cv = c;
                        hasv = has;
                    }
                    po = osj;
                    pn = c;
                    pp = sj + 1;
                }
            }
            const double Dv = pnv - pov;
            const int bj = expo(om);
            const bool okj = !hasv || ((pov + Dv == pnv) && (pnv - Dv == pov) && expo(pnv) == bj &&
                                       expo(om + Dv) == bj);
            const unsigned long long badm = __ballot(lane < tot && !okj);
            const int f = badm ? __builtin_ctzll(badm) : tot;
            // segments of the confirmed events: [run at its offset,] the event's sum
            const int cnt_j = lane < f ? hasv + 1 : 0;
            const int seg_incl = (int)wave_scan_f64((double)cnt_j);
            const int nnew = __builtin_amdgcn_readlane(seg_incl, 63);
            int j0 = 0;
            if (f > 0 && !mat && nseg + nnew < kDeltaSegCap - 1) {
                const int prev_s = __shfl_up(sl, 1);
                const int start = lane == 0 ? p : prev_s + 1;
                int o = nseg + seg_incl - cnt_j;
                if (lane < f) {
                    if (hasv) {
                        sg.sm[o] = start | (kSegOffset << 29);
                        sg.v[o] = Dv;
                        ++o;
                    }
                    sg.sm[o] = sl | (kSegValue << 29);
                    sg.v[o] = cv;
                }
                nseg += nnew;
                prev_new = readlane_f64(cv, f - 1);
                prev_old = readlane_f64(os, f - 1);
                p = __builtin_amdgcn_readlane(sl, f - 1) + 1;
                j0 = f;
            }
            for (int j = j0; j < tot; ++j) {
                const int s = __builtin_amdgcn_readlane(sl, j);
                run(s, readlane_f64(om, j));
                event(s, readlane_f64(os, j), readlane_f64(ts, j));
            }
            if (diag && lane == 0) diag[2] += clock64() - c1;
        } else {  // dense events (tiny sums, or every term changed): term by term
            const int e = min(n, 64 * (wb + 64));
            if (diag && lane == 0) diag[3] += e - p;
            seg(p, kSegCopy, 0.0);
            prev_new = wave_delta_run(t + p, old + p, chg + p, e - p, prev_old, prev_new, out + p, lane, nullptr,
                                      nullptr);
            prev_old = old[e - 1];
            p = e;
        }
    }
    if (p < n) run(n, old[n - 1]);
    if (lane == 0) {
        sg.nseg = nseg;
        sg.k0 = k0;
    }
    return prev_new;
}

// The new partial sum at k (k0 - 1 <= k < n) from the segments: k lies in
// segment i (i = -1: before the tail, unchanged).
__device__ __forceinline__ double delta_new_at(const double *old, const double *out, const DeltaSegs &sg, int i,
                                               int k) {
    if (k < 0) return 0.0;
    if (i < 0) return old[k];
    const int mode = sg.sm[i] >> 29;
    return mode == kSegOffset ? old[k] + sg.v[i] : mode == kSegValue ? sg.v[i] : out[k];
}

// After an accepted proposal (before delta_commit): the static event bits of
// the new state (t = the new terms) where they can differ from the old ones.
// One wave.
__device__ void delta_remark(const double *t, const double *old, const double *out, int n, const DeltaSegs &sg,
                             unsigned long long *smask, int lane) {
    const int nseg = sg.nseg;
    auto set_bit = [&](int k, bool ev) {
        const unsigned long long b = 1ull << (k & 63);
        if (ev) atomicOr(&smask[k >> 6], b);
        else atomicAnd(&smask[k >> 6], ~b);
    };
    // VALUE events, one per lane: the bits at s and s + 1
    for (int i0 = 0; i0 < nseg; i0 += 64) {
        const int i = i0 + lane;
        const int sm = i < nseg ? sg.sm[i] : 0;
        if (i < nseg && (sm >> 29) == kSegValue) {
            const int s = sm & kSegPosMask;
            const double pm = delta_new_at(old, out, sg, i - 1, s - 1);
            const double ps = sg.v[i];
            set_bit(s, delta_static_event(t[s], pm, ps));
            if (s + 1 < n) set_bit(s + 1, delta_static_event(t[s + 1], ps, delta_new_at(old, out, sg, i + 1, s + 1)));
        }
    }
    // COPY segments (rare): every bit of [a, b], b the next segment's start
    for (int i = 0; i < nseg; ++i) {
        const int sm = sg.sm[i];
        if ((sm >> 29) != kSegCopy) continue;
        const int a = sm & kSegPosMask, b = i + 1 < nseg ? (sg.sm[i + 1] & kSegPosMask) : n;
        for (int k = a + lane; k <= min(b, n - 1); k += 64) {
            const double pm = k == a ? delta_new_at(old, out, sg, i - 1, k - 1) : out[k - 1];
            const double pk = k == b ? delta_new_at(old, out, sg, i + 1, k) : out[k];
            set_bit(k, delta_static_event(t[k], pm, pk));
        }
    }
}

// An accepted proposal: old[k0..n) becomes the new partial sums (whole block;
// every thread calls it after a barrier that follows delta_walk).  U = the
// positions each thread has in flight.
template <int U>
__device__ __forceinline__ void delta_commit(double *old, const double *out, int n, const DeltaSegs &sg, int tid,
                                             int nthreads) {
    const int nseg = sg.nseg, k0 = sg.k0;
    if (nseg == 0 || k0 + tid >= n) return;
    // the segment of this thread's first position (binary search), then forward
    int lo = 0, hi = nseg - 1;
    const int k1 = k0 + tid;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((sg.sm[mid] & kSegPosMask) <= k1) lo = mid;
        else hi = mid - 1;
    }
    int i = lo;
    int nxt = i + 1 < nseg ? (sg.sm[i + 1] & kSegPosMask) : INT_MAX;
    for (int kb = k1; kb < n; kb += U * nthreads) {
        double src[U], val[U];
        int mode[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * nthreads;
            while (k >= nxt) {
                ++i;
                nxt = i + 1 < nseg ? (sg.sm[i + 1] & kSegPosMask) : INT_MAX;
            }
            mode[u] = sg.sm[i] >> 29;
            val[u] = sg.v[i];
            const int kc = min(k, n - 1);
            src[u] = mode[u] == kSegCopy ? out[kc] : old[kc];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + u * nthreads;
            if (k < n) old[k] = mode[u] == kSegOffset ? src[u] + val[u] : mode[u] == kSegValue ? val[u] : src[u];
        }
    }
}

}  // namespace tdstar
