// chain_logic.h -- rj-MCMC proposal logic shared by the host chain and the
// device-resident chain kernel (TD_inversion_function.jl:70-274; priors 1
// uniform, 2 normal, 3 exponential, define_TDstructure.jl:15).
//
// Everything here is __host__ __device__ and uses only IEEE +,-,*,/ and
// sqrt (all correctly rounded on both sides, the TUs are compiled with
// -ffp-contract=off), so a chain driven from the host and the same chain run
// inside a GPU kernel draw bit-identical proposals and make identical
// accept/reject decisions.  That is what the chain parity tests check.
//
// RNG: Philox4x32-10 (Salmon et al., SC'11), counter = (iteration, slot,
// chain), key = seed.  Counter-based, so a proposal's draws depend only on
// (seed, chain, iteration) -- reproducible, unlike the reference's
// wall-clock seed (TD_inversion_function.jl:13).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#if defined(__HIP_DEVICE_COMPILE__)
#define TD_HD __host__ __device__ __forceinline__
#else
#define TD_HD __host__ __device__ inline
#endif

namespace tdchain {

// ------------------------------------------------------------------ RNG ----
struct U4 {
    uint32_t x, y, z, w;
};

TD_HD void mulhilo(uint32_t a, uint32_t b, uint32_t &hi, uint32_t &lo) {
    const uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
}

TD_HD U4 philox(U4 c, uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(0xD2511F53u, c.x, hi0, lo0);
        mulhilo(0xCD9E8D57u, c.z, hi1, lo1);
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Uniform in (0,1): (k + 0.5) / 2^52 for a 52-bit k -- k + 0.5 is exact in
// FP64, so u lies in [2^-53, 1 - 2^-53], never 0 or 1 (with a 53-bit k the
// sum rounds to 2^53 for the top values: u = 1 and an infinite normal
// quantile; found by the host sanitizer driver, oracle/san).
TD_HD double u01(uint32_t a, uint32_t b) {
    const uint64_t k = (((uint64_t)a << 20) ^ (uint64_t)(b >> 12)) & ((1ull << 52) - 1);
    return ((double)k + 0.5) * (1.0 / 4503599627370496.0);
}

// Draw slots of one iteration: each slot is one Philox block = 2 uniforms.
enum Slot : uint32_t { kSlotAction = 0, kSlotXY = 1, kSlotZZeta = 2, kSlotIndex = 3 };

struct Draws {
    double u_action, u_accept, u_a, u_b, u_c, u_zeta, u_index;
    double z_a, z_b, z_c, z_zeta;  // standard-normal quantiles of u_a, u_b, u_c, u_zeta
    double log_u;                  // log(u_accept): only for the early-rejection bound (reject_bound)
};

TD_HD double normal_quantile(double p);
TD_HD double det_log(double x);

TD_HD Draws draw_iteration(uint64_t seed, uint32_t chain, uint64_t iter) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const uint32_t i0 = (uint32_t)iter, i1 = (uint32_t)(iter >> 32);
    const U4 a = philox(U4{i0, i1, kSlotAction, chain}, k0, k1);
    const U4 b = philox(U4{i0, i1, kSlotXY, chain}, k0, k1);
    const U4 c = philox(U4{i0, i1, kSlotZZeta, chain}, k0, k1);
    const U4 d = philox(U4{i0, i1, kSlotIndex, chain}, k0, k1);
    Draws r;
    r.u_action = u01(a.x, a.y);
    r.u_accept = u01(a.z, a.w);
    r.u_a = u01(b.x, b.y);
    r.u_b = u01(b.z, b.w);
    r.u_c = u01(c.x, c.y);
    r.u_zeta = u01(c.z, c.w);
    r.u_index = u01(d.x, d.y);
    // the normals every branch may need, drawn up front: a pure function of the
    // uniforms, so the device can precompute them for many iterations at once
    r.z_a = normal_quantile(r.u_a);
    r.z_b = normal_quantile(r.u_b);
    r.z_c = normal_quantile(r.u_c);
    r.z_zeta = normal_quantile(r.u_zeta);
    r.log_u = r.u_accept > 0.0 ? det_log(r.u_accept) : -__builtin_huge_val();
    return r;
}

// ------------------------------------------------- deterministic math ----
TD_HD uint64_t dbits(double x) {
    union { double d; uint64_t u; } v;
    v.d = x;
    return v.u;
}
TD_HD double bitsd(uint64_t u) {
    union { double d; uint64_t u; } v;
    v.u = u;
    return v.d;
}

// natural log for finite x > 0 (atanh series around 1 after exponent split).
TD_HD double det_log(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -__builtin_huge_val() : __builtin_nan("");
    if (x == __builtin_huge_val()) return x;
    uint64_t u = dbits(x);
    int e = (int)((u >> 52) & 0x7ff);
    if (e == 0) {  // subnormal: scale up by 2^54
        x = x * 18014398509481984.0;
        u = dbits(x);
        e = (int)((u >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = bitsd((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);  // [1,2)
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    // 2*(s + s^3/3 + ... + s^23/23), |s| < 0.1716
    double p = 1.0 / 23.0;
    p = p * s2 + 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    p = p * s2 + 1.0;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    return (double)e * ln2_hi + (2.0 * s * p + (double)e * ln2_lo);
}

TD_HD double det_exp(double x) {
    if (x != x) return x;
    if (x > 709.78) return __builtin_huge_val();
    if (x < -745.2) return 0.0;
    const double inv_ln2 = 1.4426950408889634;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    double kd = x * inv_ln2;
    kd = kd >= 0.0 ? (double)(int64_t)(kd + 0.5) : -(double)(int64_t)(-kd + 0.5);
    const double r = (x - kd * ln2_hi) - kd * ln2_lo;
    // Taylor to r^13, |r| <= 0.35
    double p = 1.0 / 6227020800.0;
    p = p * r + 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    int k = (int)kd;
    // scale by 2^k in two steps to stay in range
    const int k1 = k / 2, k2 = k - k1;
    p = p * bitsd((uint64_t)(1023 + k1) << 52);
    return p * bitsd((uint64_t)(1023 + k2) << 52);
}

// Standard normal quantile, Wichura AS241 (PPND16), u in (0,1).
TD_HD double normal_quantile(double p) {
    const double q = p - 0.5;
    if ((q < 0 ? -q : q) <= 0.425) {
        const double r = 0.180625 - q * q;
        return q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                         45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                      133.14166789178437745) * r + 3.387132872796366608) /
               (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                    21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
                 42.313330701600911252) * r + 1.0);
    }
    double r = q < 0 ? p : 1.0 - p;
    r = __builtin_sqrt(-det_log(r));
    double val;
    if (r <= 5.0) {
        r -= 1.6;
        val = (((((((r * 7.7454501427834140764e-4 + 0.0227238449892691845833) * r + 0.24178072517745061177) * r +
                   1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
                4.6303378461565452959) * r + 1.42343711074968357734) /
              (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + 0.0151986665636164571966) * r +
                   0.14810397642748007459) * r + 0.68976733498510000455) * r + 1.6763848301838038494) * r +
                2.05319162663775882187) * r + 1.0);
    } else {
        r -= 5.0;
        val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + 0.0012426609473880784386) * r +
                   0.026532189526576123093) * r + 0.29656057182850489123) * r + 1.7848265399172913358) * r +
                5.4637849111641143699) * r + 6.6579046435011037772) /
              (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
                   7.868691311456132591e-4) * r + 0.0148753612908506148525) * r + 0.13692988092273580531) * r +
                0.59983220655588793769) * r + 1.0);
    }
    return q < 0 ? -val : val;
}

// ------------------------------------------------------ the proposal ----
enum Action : int { kBirth = 1, kDeath = 2, kChange = 3, kMove = 4 };

enum Prior : int { kUniform = 1, kNormal = 2, kExponential = 3 };

struct Params {
    int debug_prior, max_cells, min_cells;
    int prior;                             // define_TDstructure.jl:15 (1 uniform, 2 normal, 3 exponential)
    double zeta_scale, sig_zeta;           // sig_zeta = zeta_scale*sig/100 (TD_inversion_function.jl:22)
    double xmin, xmax, ymin, ymax, zmin, zmax;
    double xr, yr, zr;                     // (sig/100)*(max-min), :30-32
    double temperature;
    // log of the constant prior factors of the birth / death ratios (:96-97,
    // :151-152), and 1/(2T), 1/(2 sig_zeta^2): computed once on the host (libm),
    // the same numbers in both engines
    double log_prior_birth, log_prior_death;
    double inv_2t, inv_2sig2;
    double inv_zs, inv_zs2, inv_2zs2;      // 1/zeta_scale, 1/zeta_scale^2, 1/(2 zeta_scale^2): priors 2, 3
};

// the derived constants of Params (after any change of temperature or sig_zeta)
inline void params_derived(Params &P) {
    P.inv_2t = 1.0 / (2.0 * P.temperature);
    P.inv_2sig2 = 1.0 / (2.0 * P.sig_zeta * P.sig_zeta);
    P.inv_zs = 1.0 / P.zeta_scale;
    P.inv_zs2 = 1.0 / (P.zeta_scale * P.zeta_scale);
    P.inv_2zs2 = 1.0 / (2.0 * (P.zeta_scale * P.zeta_scale));
}

// Is a proposed zeta inside the prior's support?  Birth (:92, :111) and change
// (:195, :206): uniform (0, zeta_scale); normal: always (no check at :105-109,
// :201-204); exponential: > 0.  (Death's exponential check is on the
// Interpolation value at the killed site, :165: see accept().)
TD_HD int prior_valid(const Params &P, double zeta) {
    if (P.prior == kNormal) return 1;
    if (P.prior == kExponential) return zeta > 0.0 ? 1 : 0;
    return (zeta > 0.0 && zeta < P.zeta_scale) ? 1 : 0;
}

// What the iteration proposes, before any forward-model evaluation.
struct Proposal {
    int action;       // 1..4
    int active;       // 0: branch skipped (nCells at max / min)
    int valid;        // 0: invalid, no evaluation, rejected
    int64_t index;    // kill / change / move cell (0-based)
    double x, y, z;   // birth location / move target
    double zeta;      // change: new value (birth: filled after czeta is known)
    double z_zeta;    // birth: standard normal for zetanew ~ Normal(czeta, sig_zeta)
    double u_accept;
    double log_u;     // log(u_accept), for reject_bound
};

// TD_inversion_function.jl:72 (action = rand(1:4)) and the draws of each
// branch that do not depend on the selected cell.
TD_HD Proposal propose(const Params &P, const Draws &d, int64_t ncells) {
    Proposal p{};
    p.action = 1 + (int)(d.u_action * 4.0);
    if (p.action > 4) p.action = 4;
    p.u_accept = d.u_accept;
    p.log_u = d.log_u;
    p.z_zeta = d.z_zeta;
    p.valid = 1;
    p.active = 1;
    switch (p.action) {
        case kBirth:  // :77-80
            if (ncells >= P.max_cells) { p.active = 0; p.valid = 0; break; }
            p.x = d.u_a * (P.xmax - P.xmin) + P.xmin;
            p.y = d.u_b * (P.ymax - P.ymin) + P.ymin;
            p.z = d.u_c * (P.zmax - P.zmin) + P.zmin;
            break;
        case kDeath:  // :127-128 kill = rand(1:nCells)
            if (ncells <= P.min_cells) { p.active = 0; p.valid = 0; break; }
            break;
        case kChange:  // :184 (always active)
        case kMove:    // :221
            if (ncells <= 0) { p.active = 0; p.valid = 0; break; }
            break;
    }
    if (p.active && p.action != kBirth) {
        p.index = (int64_t)(d.u_index * (double)ncells);
        if (p.index >= ncells) p.index = ncells - 1;
    }
    return p;
}

// The parts that need the selected cell (position p.index): change draws the
// new zeta (:188, validity :195), move draws the new site (:226-232).
TD_HD void complete_proposal(const Params &P, const Draws &d, Proposal &p, double cx, double cy, double cz,
                             double czeta) {
    if (!p.active) return;
    if (p.action == kChange) {
        p.zeta = czeta + P.sig_zeta * d.z_zeta;
        p.valid = prior_valid(P, p.zeta);
    } else if (p.action == kMove) {
        p.x = cx + P.xr * d.z_a;
        p.y = cy + P.yr * d.z_b;
        p.z = cz + P.zr * d.z_c;
        p.zeta = czeta;
        p.valid = (p.x >= P.xmin && p.x <= P.xmax && p.y >= P.ymin && p.y <= P.ymax && p.z >= P.zmin &&
                   p.z <= P.zmax) ? 1 : 0;
    }
}

// Birth, once czeta = Interpolation(model, xNew, yNew, zNew) is known (:81-82, :92).
TD_HD void birth_zeta(const Params &P, Proposal &p, double czeta) {
    p.zeta = czeta + P.sig_zeta * p.z_zeta;
    p.valid = prior_valid(P, p.zeta);
}

// {log(N-1), log(N), log(N+1)} for log_alpha (the device engine reads the same
// det_log values from a table built on the host)
inline void log_window(double out[3], int64_t N) {
    for (int k = 0; k < 3; ++k) out[k] = det_log((double)(N - 1 + k));
}

// The Metropolis-Hastings decision: rand < min(1, alpha) with alpha of
// eqs. 14-17, decided in the log domain:
//     log u < log alpha = log f + h + (phi - phi_n)/(2T)
// (u < 1, so the min(1, .) never matters; the same decision as comparing u
// with alpha, without an exp on the critical path).  log f = the model-size
// factor lnN[1] - lnN[1 +- 1] (det_log) plus the constant prior ratio (host
// libm log); h = the exponent's zeta terms, per prior:
//   birth  (:96-97 / :107-108 / :113-114, eq. 16), dz = czeta - zetanew:
//     uniform dz^2/2s^2, normal -zn^2/zs^2 + dz^2/2s^2 (zs^2, not 2 zs^2, as
//     the reference writes it), exponential -zn/zs + dz^2/2s^2
//   death  (:151-152 / :160-162 / :166-168, eq. 17), dz = zeta_killed -
//     zetanew, zetanew = Interpolation(modeln, killed site) (:146):
//     uniform -dz^2/2s^2, normal zk^2/2zs^2 - dz^2/2s^2, exponential zk/zs - dz^2/2s^2
//   change (:196 / :202-203 / :207-208, eq. 15), zo = the old value (passed
//     as zeta_killed): uniform 0, normal (zo^2 - zn^2)/2zs^2, exponential (zo - zn)/zs
//   move   (:241, eq. 14): 0.
// T = 1 is the reference; a tempered replica divides only the misfit term.
// Written as one if-chain into one variable: a `switch` with a `return -x`
// default was miscompiled for gfx950 (the default path returned a stale
// register; tools/repro_accept.hip).
// inv_2t = 1/(2T) of the chain's current temperature (P.inv_2t; a resident
// tempering launch keeps its own, set between rounds)
TD_HD double log_alpha_t(const Params &P, double inv_2t, const Proposal &p, double phi, double phi_n, double czeta,
                         double zeta_killed, double zetanew_death, const double *lnN) {
    // (multiplications by precomputed reciprocals: no division on the device's decision path)
    const double g = (phi - phi_n) * inv_2t;
    double la = g;
    if (p.action == kBirth) {
        const double dz = czeta - p.zeta;
        double h = (dz * dz) * P.inv_2sig2;
        if (P.prior == kNormal) h = -(p.zeta * p.zeta) * P.inv_zs2 + h;
        else if (P.prior == kExponential) h = -p.zeta * P.inv_zs + h;
        la = ((lnN[1] - lnN[2]) + P.log_prior_birth) + (h + g);
    } else if (p.action == kDeath) {
        const double dz = zeta_killed - zetanew_death;
        double h = -((dz * dz) * P.inv_2sig2);
        if (P.prior == kNormal) h = (zeta_killed * zeta_killed) * P.inv_2zs2 + h;
        else if (P.prior == kExponential) h = zeta_killed * P.inv_zs + h;
        la = ((lnN[1] - lnN[0]) + P.log_prior_death) + (h + g);
    } else if (p.action == kChange) {
        if (P.prior == kNormal) la = (zeta_killed * zeta_killed - p.zeta * p.zeta) * P.inv_2zs2 + g;
        else if (P.prior == kExponential) la = (zeta_killed - p.zeta) * P.inv_zs + g;
    }
    return la;
}
TD_HD double log_alpha(const Params &P, const Proposal &p, double phi, double phi_n, double czeta,
                       double zeta_killed, double zetanew_death, const double *lnN) {
    return log_alpha_t(P, P.inv_2t, p, phi, phi_n, czeta, zeta_killed, zetanew_death, lnN);
}
TD_HD bool accept_t(const Params &P, double inv_2t, const Proposal &p, double phi, double phi_n, double czeta,
                    double zeta_killed, double zetanew_death, const double *lnN) {
    if (!p.active || !p.valid) return false;  // rand(1)[1] < alpha && valid == 1
    // exponential death: valid only when the reduced model's value at the killed site is > 0 (:165, :171)
    if (p.action == kDeath && P.prior == kExponential && !(zetanew_death > 0.0)) return false;
    return p.log_u < log_alpha_t(P, inv_2t, p, phi, phi_n, czeta, zeta_killed, zetanew_death, lnN);
}
TD_HD bool accept(const Params &P, const Proposal &p, double phi, double phi_n, double czeta, double zeta_killed,
                  double zetanew_death, const double *lnN) {
    return accept_t(P, P.inv_2t, p, phi, phi_n, czeta, zeta_killed, zetanew_death, lnN);
}

// The decision's phi-free part, for deciding a bracket of (phi, phi_n) with one add and two compares:
// log_alpha_t is la = A + (H + g) (birth, death) or A + g (change) or g (move), g = (phi - phi_n) * inv_2t;
// la0 = la at g = 0, as log_alpha_t forms it, and mag = |A| + 2|H| bound the rounding:
//     |la_fp(g) - (la0 + g)| <= 3u (|la0| + mag + 2|g|)     (u = 2^-53)
// so decide_sure() answers only where log_u < la_fp at every point of the bracket (1: accept) or at
// none (-1: reject), with a margin of 2^-45 relative -- else 0, and the caller evaluates the bracket's
// corners with accept_t.  (la_fp is monotone in g and g in phi, phi_n: each IEEE step is.)
struct AlphaParts {
    double la0, mag;
    int reject;  // accept_t rejects whatever phi, phi_n (an invalid proposal; an exponential death at zetanew <= 0)
};
TD_HD AlphaParts alpha_parts(const Params &P, const Proposal &p, double czeta, double zeta_killed,
                             double zetanew_death, const double *lnN) {
    AlphaParts r;
    r.reject = !p.active || !p.valid || (p.action == kDeath && P.prior == kExponential && !(zetanew_death > 0.0));
    r.la0 = log_alpha_t(P, 1.0, p, 0.0, 0.0, czeta, zeta_killed, zetanew_death, lnN);  // g = 0
    double A = 0.0, H = 0.0;
    if (p.action == kBirth) {
        const double dz = czeta - p.zeta;
        H = (dz * dz) * P.inv_2sig2;
        if (P.prior == kNormal) H = -(p.zeta * p.zeta) * P.inv_zs2 + H;
        else if (P.prior == kExponential) H = -p.zeta * P.inv_zs + H;
        A = (lnN[1] - lnN[2]) + P.log_prior_birth;
    } else if (p.action == kDeath) {
        const double dz = zeta_killed - zetanew_death;
        H = -((dz * dz) * P.inv_2sig2);
        if (P.prior == kNormal) H = (zeta_killed * zeta_killed) * P.inv_2zs2 + H;
        else if (P.prior == kExponential) H = zeta_killed * P.inv_zs + H;
        A = (lnN[1] - lnN[0]) + P.log_prior_death;
    } else {
        A = r.la0;  // change: A + g; move: g (la0 = 0)
    }
    r.mag = fabs(A) + 2.0 * fabs(H);
    return r;
}
// 1: accept_t accepts for every g >= g_lo; -1: for no g <= g_hi; 0: undecided (g_lo <= g_hi)
TD_HD int decide_sure(const AlphaParts &a, double log_u, double g_lo, double g_hi) {
    if (a.reject) return -1;
    const double lo = a.la0 + g_lo, hi = a.la0 + g_hi;
    const double tl = 0x1p-45 * (fabs(a.la0) + a.mag + 2.0 * fabs(g_lo) + fabs(lo) + fabs(log_u));
    const double th = 0x1p-45 * (fabs(a.la0) + a.mag + 2.0 * fabs(g_hi) + fabs(hi) + fabs(log_u));
    if (lo - tl > log_u) return 1;  // (NaN, infinities: every comparison false -> undecided)
    if (hi + th < log_u) return -1;
    return 0;
}

// The phi_n from which accept() rejects: log_alpha is dphi-affine, so
//     reject  <=>  phi_n >= phi + 2T (log f + g - log u)
// (f, g as in log_alpha).  For deciding before phi_n is known exactly (the
// chi^2 partial sums only grow); the caller adds a margin far above every
// rounding involved, so the outcome is the one accept() gives on the exact
// phi_n.  +inf when no finite bound exists (u == 0).
TD_HD double reject_bound_t(const Params &P, double temperature, double inv_2t, const Proposal &p, double phi,
                            double czeta, double zeta_killed, double zetanew_death, const double *lnN) {
    if (!(p.u_accept > 0.0)) return __builtin_huge_val();
    const double lf = log_alpha_t(P, inv_2t, p, phi, phi, czeta, zeta_killed, zetanew_death, lnN);  // dphi = 0
    return phi + 2.0 * temperature * (lf - p.log_u);  // (a bound: its own rounding is covered by the margin)
}
TD_HD double reject_bound(const Params &P, const Proposal &p, double phi, double czeta, double zeta_killed,
                          double zetanew_death, const double *lnN) {
    return reject_bound_t(P, P.temperature, P.inv_2t, p, phi, czeta, zeta_killed, zetanew_death, lnN);
}

// ------------------------------------------------ parallel-tempering swap ----
// (the reference's chains are independent, main_inversion.jl:15.)
// Round rnd tries the level pairs (l, l+1), l = rnd mod 2, 2 + rnd mod 2, ...
// -- disjoint, so each is decided alone: a at level l, b at l+1 swap when
// log alpha = (phi_a - phi_b)(1/(2T_l) - 1/(2T_l+1)) >= 0 or log u < log alpha,
// u a SplitMix64 hash of (seed, rnd, l).  The same function on the host
// (td_swap_decide, tempering.decide_swaps) and inside the resident kernel that
// decides the swaps itself (td_rounds_exchange): det_log, not a libm log.
TD_HD uint64_t swap_mix64(uint64_t x) {  // SplitMix64's finaliser
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
TD_HD double swap_uniform(uint64_t seed, uint64_t rnd, uint64_t level) {
    uint64_t x = swap_mix64(seed * 0x9E3779B97F4A7C15ull + rnd);
    x = swap_mix64(x + level * 0xD1B54A32D192ED03ull + 1ull);
    return ((double)(x >> 12) + 0.5) / 4503599627370496.0;  // (k + 1/2) / 2^52: in (0, 1), exact
}
TD_HD bool swap_accept(double phi_a, double phi_b, double t_lo, double t_hi, uint64_t seed, uint64_t rnd,
                       uint64_t level) {
    const double la = (phi_a - phi_b) * (1.0 / (2.0 * t_lo) - 1.0 / (2.0 * t_hi));
    return la >= 0.0 || det_log(swap_uniform(seed, rnd, level)) < la;
}

}  // namespace tdchain
