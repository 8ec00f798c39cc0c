// chain.cpp -- rj-MCMC chain behind the C ABI (td_chain_*), both engines,
// plus the host-only testing hooks of include/tdstar_testing.h.
//
// TD_ENGINE_HOST mirrors TD_inversion_function.jl:70-274 literally: every
// proposal builds the proposed model on the host and calls td_evaluate /
// td_interpolate (the drop-in boundary).  TD_ENGINE_DEVICE runs the same
// iterations inside k_chain_run (chain_kernels.hip).  Both draw from the same
// counter-based RNG and share chain_logic.h, so their trajectories agree bit
// for bit; the HOST engine is the parity reference for the DEVICE one.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/tdstar_testing.h"
#include "chain_dev.h"
#include "chain_logic.h"
#include "comm.h"
#include "ctx.h"

using namespace tdstar;

struct td_chain {
    td_ctx *ctx = nullptr;
    td_chain_params prm{};
    tdchain::Params P{};
    int engine = TD_ENGINE_DEVICE;
    // host engine state (also the device engine's mirror after get_model)
    std::vector<double> x, y, z, zeta;
    double phi = 0.0;
    std::vector<double> ptS;
    int64_t iter = 1;  // Julia: for iter in iter_ind:n_iter, iter_ind = 1
    td_chain_stats stats{};
    // device engine
    DevChain dev{};
    DevChain *dev_ptr = nullptr;  // device copy the kernel reads
    void *dev_block = nullptr;  // one allocation for every device array
    ChainScalars *st_dev = nullptr;
    ChainScalars *st_host = nullptr;  // pinned
    NNWork nn;
    double *script_host = nullptr;  // pinned, mapped: [phi_n, ptS_n] of a scripted step (shadow chains)
    double *script_dev = nullptr;   // the same, as the device addresses it
    bool desc_dirty = true;         // dev changed on the host since the device copy was made
    // server mode (shadow chains): the resident launch and its mailbox
    Mailbox *mb_host = nullptr, *mb_dev = nullptr;
    hipStream_t srv_stream = nullptr;
    bool srv_running = false;
    std::chrono::steady_clock::time_point srv_last{};
    ScriptStep srv_pending{};     // the step the server holds undecided (kDecideLater), if any
    bool srv_has_pending = false;
    // a command posted and not yet answered (shadow_server_post / shadow_server_answer)
    bool post_open = false;
    int post_decision = 0, post_nsteps = 0;
    ScriptStep post_steps[kMaxScript]{};
    ScriptStep post_held{};
    bool post_had = false;
    long long post_seq = 0;
    int64_t post_t0 = 0;
    long long pq_expect = -1;  // the death evaluate whose killed-site query the kernel answers ahead (pq_seq)
    td_rounds *rounds = nullptr;  // a resident tempering launch holds this chain (td_rounds_*)
};

// A resident tempering launch over chains of one context (chain_dev.h RoundBox).
struct td_rounds {
    std::vector<td_chain *> chains;
    td_ctx *ctx = nullptr;
    RoundBox *rb_host = nullptr, *rb_dev = nullptr;  // pinned, mapped
    DevChain *desc_dev = nullptr, *desc_host = nullptr;
    hipStream_t stream = nullptr;
    bool running = false;
    long long seq = 0;
    double tr_first = 0.0, tr_last = 0.0;  // diagnostic (TD_ROUNDS_TRACE): summed arrival times, rounds
    long long tr_n = 0;
    std::vector<char> force_exit;  // testing (tdt_rounds_force_exit): one-shot, per chain
    // exchange rounds (td_rounds_exchange, chain_dev.h RoundX): buffers made on first use
    int x_R = 0;                  // replicas the buffers are sized for
    double *x_in = nullptr, *x_out = nullptr, *x_temps = nullptr;  // device; x_in [2][local], x_out [2][R] by round parity
    long long *x_bar = nullptr;   // device: the entry barrier's and the failure vote's word (multi-rank)
    unsigned long long *x_rdy = nullptr, *x_gdone = nullptr;       // device
    unsigned long long *x_ready = nullptr;                         // signal memory (or pinned, host trigger)
    bool x_ready_pinned = false;
    int *x_lev = nullptr;                                          // device [local][R]
    double *x_log_phi = nullptr;                                   // pinned [M][R]
    int *x_log_lev = nullptr;                                      // pinned [M][R]
    long long *x_log_t = nullptr;                                  // pinned [M][3]
    long long *x_err = nullptr;                                    // pinned
    int64_t x_log_cap = 0;        // rounds the logs hold
    RoundX x_host{};              // the launch's exchange descriptor, and its device copy
    RoundX *x_desc = nullptr;
    unsigned long long x_tag = 0, x_gtag = 0;  // rounds exchanged so far (the flags' bases)
};

namespace {

bool rounds_trace() {
    static const bool on = [] {
        const char *e = std::getenv("TD_ROUNDS_TRACE");
        return e && e[0] == '1';
    }();
    return on;
}

int chain_err(td_chain *ch, int code, const std::string &m) { return set_err(ch ? ch->ctx : nullptr, code, m); }

tdchain::Params make_params(const td_chain_params &p) {
    tdchain::Params P{};
    P.debug_prior = p.debug_prior;
    P.max_cells = p.max_cells;
    P.min_cells = p.min_cells;
    P.prior = p.prior;
    P.zeta_scale = (double)p.zeta_scale;
    // TD_inversion_function.jl:22: zeta_scale * sig / 100 (Int*Int, then /)
    P.sig_zeta = (double)(p.zeta_scale * p.sig) / 100.0;
    P.xmin = p.xmin; P.xmax = p.xmax;
    P.ymin = p.ymin; P.ymax = p.ymax;
    P.zmin = p.zmin; P.zmax = p.zmax;
    // :30-32: (sig / 100) * (max - min)
    P.xr = ((double)p.sig / 100.0) * (p.xmax - p.xmin);
    P.yr = ((double)p.sig / 100.0) * (p.ymax - p.ymin);
    P.zr = ((double)p.sig / 100.0) * (p.zmax - p.zmin);
    P.temperature = p.temperature > 0.0 ? p.temperature : 1.0;
    const double two_pi_sqrt = 2.5066282746310002;
    if (p.prior == tdchain::kNormal) {  // :107, :160
        P.log_prior_birth = std::log(P.sig_zeta / P.zeta_scale);
        P.log_prior_death = std::log(P.zeta_scale / P.sig_zeta);
    } else if (p.prior == tdchain::kExponential) {  // :113, :166
        P.log_prior_birth = std::log((two_pi_sqrt * P.sig_zeta) / P.zeta_scale);
        P.log_prior_death = std::log(P.zeta_scale / (two_pi_sqrt * P.sig_zeta));
    } else {  // uniform :96, :151
        P.log_prior_birth = std::log((P.sig_zeta * two_pi_sqrt) / P.zeta_scale);
        P.log_prior_death = std::log(P.zeta_scale / (P.sig_zeta * two_pi_sqrt));
    }
    tdchain::params_derived(P);
    return P;
}

// build_starting (MCsub.jl:76-121) with the chain's counter-based RNG in a
// counter range the iterations never use (iteration index 0).
void build_starting(td_chain *ch) {
    const tdchain::Params &P = ch->P;
    const tdchain::Draws d0 = tdchain::draw_iteration(ch->prm.seed, (uint32_t)ch->prm.chain, 0);
    // :86-87 floor(exp(rand * log(max/min) + log(min)))
    const double lr = tdchain::det_log((double)P.max_cells / (double)P.min_cells);
    const int64_t n = (int64_t)std::floor(tdchain::det_exp(d0.u_action * lr + tdchain::det_log((double)P.min_cells)));
    ch->x.resize((size_t)n);
    ch->y.resize((size_t)n);
    ch->z.resize((size_t)n);
    ch->zeta.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        // slots (2^31 + i) of iteration 0: never drawn by propose()
        const tdchain::Draws d = tdchain::draw_iteration(ch->prm.seed ^ 0x5bd1e995ull, (uint32_t)ch->prm.chain,
                                                         (uint64_t)i);
        ch->x[(size_t)i] = P.xmin + (P.xmax - P.xmin) * d.u_a;  // :92-94
        ch->y[(size_t)i] = P.ymin + (P.ymax - P.ymin) * d.u_b;
        ch->z[(size_t)i] = P.zmin + (P.zmax - P.zmin) * d.u_c;
        if (P.prior == tdchain::kNormal)  // :104 rand(Normal(0, zeta_scale))
            ch->zeta[(size_t)i] = 0.0 + P.zeta_scale * d.z_zeta;
        else if (P.prior == tdchain::kExponential)  // :107 -log(rand) * zeta_scale
            ch->zeta[(size_t)i] = -tdchain::det_log(d.u_zeta) * P.zeta_scale;
        else  // :100 rand * zeta_scale
            ch->zeta[(size_t)i] = d.u_zeta * P.zeta_scale;
    }
}

// HOST: the full evaluate of every proposed model (the parity reference);
// DROPIN: the public td_evaluate, i.e. what an unchanged Julia host calls
// (its incremental path follows the chain on the device, incremental.cpp)
int host_evaluate(td_chain *ch, const std::vector<double> &x, const std::vector<double> &y,
                  const std::vector<double> &z, const std::vector<double> &zeta, double *phi, double *ptS) {
    if (ch->engine == TD_ENGINE_DROPIN || ch->prm.debug_prior == 1)
        return td_evaluate(ch->ctx, x.data(), y.data(), z.data(), zeta.data(), (int64_t)x.size(),
                           ch->prm.debug_prior, ptS, phi, nullptr, nullptr);
    TD_HIP(ch->ctx, hipSetDevice(ch->ctx->device));
    return evaluate_full(ch->ctx, x.data(), y.data(), z.data(), zeta.data(), (int64_t)x.size(), ptS, phi);
}

int host_interp1(td_chain *ch, const std::vector<double> &x, const std::vector<double> &y,
                 const std::vector<double> &z, const std::vector<double> &zeta, double qx, double qy, double qz,
                 double *val) {
    int64_t np = 0;
    return td_interpolate(ch->ctx, x.data(), y.data(), z.data(), zeta.data(), (int64_t)x.size(), &qx, 1, &qy, 1,
                          &qz, 1, val, nullptr, &np);
}

// One iteration of TD_inversion_function.jl:70-274 on the host engine.
int host_iteration(td_chain *ch) {
    const tdchain::Params &P = ch->P;
    const tdchain::Draws dr = tdchain::draw_iteration(ch->prm.seed, (uint32_t)ch->prm.chain, (uint64_t)ch->iter);
    const int64_t N = (int64_t)ch->x.size();
    tdchain::Proposal p = tdchain::propose(P, dr, N);
    ch->iter += 1;
    ch->stats.iterations += 1;
    ch->stats.last_action = p.action;  // model.action = action; model.accept = 0 (:73-74)
    ch->stats.last_accept = 0;
    if (!p.active) return TD_OK;
    ch->stats.proposed[p.action] += 1;
    double czeta = 0.0, zeta_killed = 0.0, zetanew = 0.0;
    const size_t k = (size_t)p.index;
    if (p.action != tdchain::kBirth) {
        zeta_killed = ch->zeta[k];
        tdchain::complete_proposal(P, dr, p, ch->x[k], ch->y[k], ch->z[k], ch->zeta[k]);
    } else {
        int rc = host_interp1(ch, ch->x, ch->y, ch->z, ch->zeta, p.x, p.y, p.z, &czeta);  // :81
        if (rc) return rc;
        tdchain::birth_zeta(P, p, czeta);
    }
    if (!p.valid) return TD_OK;
    const int64_t tcopy = now_ns();
    std::vector<double> nx = ch->x, ny = ch->y, nz = ch->z, nzeta = ch->zeta;  // modeln = deepcopy(model)
    switch (p.action) {
        case tdchain::kBirth:  // :85-88 append!
            nx.push_back(p.x); ny.push_back(p.y); nz.push_back(p.z); nzeta.push_back(p.zeta);
            break;
        case tdchain::kDeath:  // :132-135 deleteat!
            nx.erase(nx.begin() + (long)k); ny.erase(ny.begin() + (long)k);
            nz.erase(nz.begin() + (long)k); nzeta.erase(nzeta.begin() + (long)k);
            break;
        case tdchain::kChange: nzeta[k] = p.zeta; break;  // :189
        case tdchain::kMove: nx[k] = p.x; ny[k] = p.y; nz[k] = p.z; break;  // :234-236
    }
    ch->ctx->dropin_ns[9] += now_ns() - tcopy;
    double phi_n = 0.0;
    std::vector<double> ptS_n(ch->ptS.size());
    int rc = host_evaluate(ch, nx, ny, nz, nzeta, &phi_n, ptS_n.data());
    if (rc) return rc;
    ch->stats.evaluations += 1;
    if (p.action == tdchain::kDeath) {  // :146 zetanew = Interpolation(modeln, killed site)
        rc = host_interp1(ch, nx, ny, nz, nzeta, ch->x[k], ch->y[k], ch->z[k], &zetanew);
        if (rc) return rc;
    }
    double lnN[3];
    tdchain::log_window(lnN, N);
    if (tdchain::accept(P, p, ch->phi, phi_n, czeta, zeta_killed, zetanew, lnN)) {
        ch->x.swap(nx); ch->y.swap(ny); ch->z.swap(nz); ch->zeta.swap(nzeta);
        ch->phi = phi_n;
        ch->ptS.swap(ptS_n);
        ch->stats.accepted[p.action] += 1;
        ch->stats.last_accept = 1;
    }
    return TD_OK;
}

// ---------------------------------------------------------------- device ----
template <class T>
T *carve(char *&cur, size_t count) {
    T *p = reinterpret_cast<T *>(cur);
    cur += ((count * sizeof(T) + 255) / 256) * 256;
    return p;
}

int device_setup(td_chain *ch) {
    td_ctx *c = ch->ctx;
    const int64_t P = c->g.P, n = c->g.n;
    if (P >= (int64_t)1 << 26)  // tile_start packs start << 5 | count
        return set_err(c, TD_ERR_ARG, "td_chain_create: more than 2^26 ray points");
    // ---- tiles: <= kTilePts consecutive points of one ray; bounding boxes
    //      rounded OUTWARD to FP32 (the lower bound stays valid, LDS holds them) ----
    std::vector<int> tstart, tray, pt_ray((size_t)P);
    for (int64_t r = 0; r < n; ++r) {
        const int a = c->ray_off_host[(size_t)r], b = c->ray_off_host[(size_t)r + 1];
        for (int q = a; q < b; ++q) pt_ray[(size_t)q] = (int)r;
        for (int q = a; q < b; q += kTilePts) {
            tstart.push_back(q);
            tray.push_back((int)r);
        }
    }
    const int ntiles = (int)tstart.size();
    tstart.push_back((int)P);
    std::vector<float> lo(3 * (size_t)ntiles), hi(3 * (size_t)ntiles);
    std::vector<int> tcount((size_t)ntiles);
    for (int t = 0; t < ntiles; ++t) tcount[(size_t)t] = tstart[(size_t)t + 1] - tstart[(size_t)t];
    for (int t = 0; t < ntiles; ++t) {
        double l[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, h[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        for (int q = tstart[(size_t)t]; q < tstart[(size_t)t + 1]; ++q) {
            const double v[3] = {c->hx[(size_t)q], c->hy[(size_t)q], c->hz[(size_t)q]};
            for (int a = 0; a < 3; ++a)
                if (!std::isnan(v[a])) {
                    l[a] = std::min(l[a], v[a]);
                    h[a] = std::max(h[a], v[a]);
                }
        }
        for (int a = 0; a < 3; ++a) {
            float fl = (float)l[a], fh = (float)h[a];
            if ((double)fl > l[a]) fl = std::nextafter(fl, -HUGE_VALF);
            if ((double)fh < h[a]) fh = std::nextafter(fh, HUGE_VALF);
            lo[(size_t)a * ntiles + t] = fl;
            hi[(size_t)a * ntiles + t] = fh;
        }
    }
    // ---- tiles in a spatial order (Morton code of the box centre) so that 16
    //      consecutive tiles form a compact SUPER-TILE; its box is the union of
    //      theirs.  Rays in HBM test super-tiles first (chain_kernels.hip phase B).
    //      A tile's points: tile_sc[t] = start << 5 | count ----
    std::vector<int> torder((size_t)ntiles);
    {
        double gl[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, gh[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        for (int t = 0; t < ntiles; ++t)
            for (int a = 0; a < 3; ++a) {
                gl[a] = std::min(gl[a], (double)lo[(size_t)a * ntiles + t]);
                gh[a] = std::max(gh[a], (double)hi[(size_t)a * ntiles + t]);
            }
        std::vector<uint64_t> key((size_t)ntiles);
        for (int t = 0; t < ntiles; ++t) {
            uint64_t k = 0;
            uint32_t c3[3];
            for (int a = 0; a < 3; ++a) {
                const double ctr = 0.5 * ((double)lo[(size_t)a * ntiles + t] + (double)hi[(size_t)a * ntiles + t]);
                const double u = gh[a] > gl[a] ? (ctr - gl[a]) / (gh[a] - gl[a]) : 0.0;
                c3[a] = (uint32_t)std::min(1023.0, std::max(0.0, std::floor(u * 1024.0)));
            }
            for (int bit = 9; bit >= 0; --bit)
                for (int a = 0; a < 3; ++a) k = (k << 1) | ((c3[a] >> bit) & 1u);
            key[(size_t)t] = k;
            torder[(size_t)t] = t;
        }
        std::stable_sort(torder.begin(), torder.end(), [&](int a, int b) { return key[(size_t)a] < key[(size_t)b]; });
    }
    {
        // The LDS layout's tile pass gives each wave runs of 64 consecutive tiles, and a wave
        // preloads the points of only the first kPre tiles it finds (phase B).  The tiles one
        // proposal hits are Morton neighbours: dealt round-robin over the 8 waves instead
        // (Morton rank J*512 + r -> J*512 + (r % 8) * 64 + r / 8, whole rounds of 512), each wave
        // finds one or two and phase C reads no point of its own.  The HBM layout keeps the
        // Morton order: its super-tiles are 16 consecutive tiles.
        DevChain probe{};
        probe.ntiles = ntiles;
        probe.n = (int)n;
        probe.cap = std::max<int>(ch->prm.max_cells, (int)ch->x.size()) + 1;
        int64_t sz[4];
        chain_lds_sizes(probe, sz);
        if (sz[0] <= 160 * 1024) {
            constexpr int kRound = kChainThreads, kW = kChainThreads / 64;
            std::vector<int> dealt(torder);
            for (int J = 0; (J + 1) * kRound <= ntiles; ++J)
                for (int r = 0; r < kRound; ++r)
                    dealt[(size_t)J * kRound + (size_t)(r % kW) * 64 + (size_t)(r / kW)] = torder[(size_t)J * kRound + r];
            torder.swap(dealt);
        }
    }
    std::vector<int> tsc((size_t)ntiles + 1, 0), tray2((size_t)ntiles);
    std::vector<float> lo2(lo.size()), hi2(hi.size());
    for (int i = 0; i < ntiles; ++i) {
        const int t = torder[(size_t)i];
        tsc[(size_t)i] = (tstart[(size_t)t] << 5) | tcount[(size_t)t];
        tray2[(size_t)i] = tray[(size_t)t];
        for (int a = 0; a < 3; ++a) {
            lo2[(size_t)a * ntiles + i] = lo[(size_t)a * ntiles + t];
            hi2[(size_t)a * ntiles + i] = hi[(size_t)a * ntiles + t];
        }
    }
    const int nsuper = (ntiles + kTilePts - 1) / kTilePts;
    std::vector<float> slo(3 * (size_t)std::max(nsuper, 1)), shi(3 * (size_t)std::max(nsuper, 1));
    for (int S = 0; S < nsuper; ++S)
        for (int a = 0; a < 3; ++a) {
            float l = HUGE_VALF, h = -HUGE_VALF;
            for (int i = S * kTilePts; i < std::min(ntiles, (S + 1) * kTilePts); ++i) {
                l = std::min(l, lo2[(size_t)a * ntiles + i]);
                h = std::max(h, hi2[(size_t)a * ntiles + i]);
            }
            slo[(size_t)a * nsuper + S] = l;
            shi[(size_t)a * nsuper + S] = h;
        }
    const int cap = std::max<int>(ch->prm.max_cells, (int)ch->x.size()) + 1;
    // ---- bucket grid over the cells: ~2 cells per bucket at the starting size ----
    // the prior box (every valid birth and move stays in it, TD_inversion_function.jl:77-80,226-232) and the
    // starting cells: the grid is sealed -- no cell ever lies outside it (internal.h grid_block_lb)
    double glo[3] = {ch->P.xmin, ch->P.ymin, ch->P.zmin}, ghi[3] = {ch->P.xmax, ch->P.ymax, ch->P.zmax};
    {
        const std::vector<double> *cv[3] = {&ch->x, &ch->y, &ch->z};
        for (int a = 0; a < 3; ++a) {
            for (double v : *cv[a])
                if (v == v) glo[a] = std::min(glo[a], v), ghi[a] = std::max(ghi[a], v);
            const double pad = std::ldexp(std::fabs(glo[a]) + std::fabs(ghi[a]) + 1.0, -40);  // a birth's rounding
            glo[a] -= pad;
            ghi[a] += pad;
        }
    }
    const CellGrid G = make_cell_grid(glo, ghi, std::max<double>((double)ch->x.size(), 16.0) / 2.0, 256, 1 << 24);
    const size_t nbuckets = (size_t)G.gx * G.gy * G.gz;
    std::vector<int> bcount(nbuckets, 0);
    std::vector<CellEntry> bent(nbuckets * kBucketCap, CellEntry{0.0, 0.0, 0.0, 0.0});
    std::vector<int> bslot(nbuckets * kBucketCap, 0);
    int overflow = 0;
    for (size_t i = 0; i < ch->x.size(); ++i) {
        const int b = grid_bucket(G, ch->x[i], ch->y[i], ch->z[i]);
        if (bcount[(size_t)b] < kBucketCap) {
            bslot[(size_t)b * kBucketCap + bcount[(size_t)b]] = (int)i;
            bent[(size_t)b * kBucketCap + bcount[(size_t)b]++] = CellEntry{ch->x[i], ch->y[i], ch->z[i], ch->zeta[i]};
        }
        else
            overflow = 1;
    }
    // ---- one device block for everything the chain owns ----
    size_t bytes = 0;
    auto add = [&](size_t b) { bytes += ((b + 255) / 256) * 256; };
    const size_t Pn = (size_t)std::max<int64_t>(P, 1), nn = (size_t)std::max<int64_t>(n, 1);
    add(sizeof(int) * (ntiles + 1)); add(sizeof(int) * (ntiles + 1)); add(sizeof(int) * Pn);
    add(sizeof(float) * 3 * ntiles); add(sizeof(float) * 3 * ntiles); add(sizeof(double) * (ntiles + 1)); add(sizeof(double) * (ntiles + 1));
    add(sizeof(float) * 3 * std::max(nsuper, 1)); add(sizeof(float) * 3 * std::max(nsuper, 1));
    add(sizeof(double) * 4 * cap); add(sizeof(double) * (cap + 2)); for (int i = 0; i < 3; ++i) add(sizeof(int) * cap); add(sizeof(long long) * cap);
    add(sizeof(int) * Pn); add(sizeof(double) * Pn); add(sizeof(double) * Pn);
    add(sizeof(int) * Pn); add(sizeof(double) * Pn); add(sizeof(double) * Pn); add(Pn);
    add(sizeof(int) * Pn); add(sizeof(int) * Pn); add(sizeof(int) * (ntiles + 1));
    for (int i = 0; i < 6; ++i) add(sizeof(double) * nn);
    add(sizeof(int) * nn); add(sizeof(int) * nn); add(sizeof(ChainScalars));
    add(sizeof(int) * nbuckets); add(sizeof(CellEntry) * nbuckets * kBucketCap); add(sizeof(int) * nbuckets * kBucketCap); add(sizeof(int));
    add(sizeof(DevChain));
    hipError_t e = hipMalloc(&ch->dev_block, bytes);
    if (e != hipSuccess) return hip_err(c, e, "hipMalloc(chain state)");
    e = hipMemsetAsync(ch->dev_block, 0, bytes, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "hipMemset(chain state)");
    char *cur = (char *)ch->dev_block;
    DevChain &d = ch->dev;
    d.px = c->g.px; d.py = c->g.py; d.pz = c->g.pz; d.w = c->g.w; d.tS = c->g.tS; d.sig = c->g.sig;
    d.ray_off = c->g.ray_off;
    d.P = (int)P;
    d.n = (int)n;
    int *tile_start = carve<int>(cur, ntiles + 1);
    int *tile_ray_d = carve<int>(cur, ntiles + 1);
    int *pt_ray_d = carve<int>(cur, Pn);
    float *tlo = carve<float>(cur, 3 * (size_t)ntiles);
    float *thi = carve<float>(cur, 3 * (size_t)ntiles);
    d.tile_start = tile_start; d.tile_ray = tile_ray_d; d.pt_ray = pt_ray_d; d.tile_lo = tlo; d.tile_hi = thi;
    d.tile_maxd = carve<double>(cur, ntiles + 1);
    d.tile_cmax = carve<double>(cur, ntiles + 1);
    d.ntiles = ntiles;
    float *slo_d = carve<float>(cur, 3 * (size_t)std::max(nsuper, 1));
    float *shi_d = carve<float>(cur, 3 * (size_t)std::max(nsuper, 1));
    d.super_lo = slo_d; d.super_hi = shi_d; d.nsuper = nsuper;
    double *cells = carve<double>(cur, 4 * (size_t)cap);
    d.cx = cells; d.cy = cells + cap; d.cz = cells + 2 * cap; d.czeta = cells + 3 * cap;
    double *logN_d = carve<double>(cur, (size_t)cap + 2);
    d.logN = logN_d;
    d.order = carve<int>(cur, cap); d.stamp = carve<long long>(cur, cap);
    d.free_slots = carve<int>(cur, cap); d.order_tmp = carve<int>(cur, cap);
    d.cap = cap;
    d.best_s = carve<int>(cur, Pn); d.best_d = carve<double>(cur, Pn); d.zeta0 = carve<double>(cur, Pn);
    d.cand_s = carve<int>(cur, Pn); d.cand_d = carve<double>(cur, Pn); d.cand_z = carve<double>(cur, Pn);
    d.cand_flag = carve<unsigned char>(cur, Pn);
    d.changed = carve<int>(cur, Pn); d.orphans = carve<int>(cur, Pn); d.tiles_hit = carve<int>(cur, ntiles + 1);
    d.ptS = carve<double>(cur, nn); d.cand_ptS = carve<double>(cur, nn);
    d.prefix = carve<double>(cur, nn); d.cand_prefix = carve<double>(cur, nn);
    d.term = carve<double>(cur, nn); d.cand_term = carve<double>(cur, nn);
    d.rays_hit = carve<int>(cur, nn); d.ray_flag = carve<int>(cur, nn);
    d.st = carve<ChainScalars>(cur, 1);
    d.grid = G;
    d.bucket_count = carve<int>(cur, nbuckets);
    d.buckets = carve<CellEntry>(cur, nbuckets * kBucketCap);
    d.bslot = carve<int>(cur, nbuckets * kBucketCap);
    d.grid_overflow = carve<int>(cur, 1);
    ch->dev_ptr = carve<DevChain>(cur, 1);
    ch->st_dev = d.st;
    d.params = ch->P;
    d.seed = ch->prm.seed;
    d.chain = (uint32_t)ch->prm.chain;

    // pinned, mapped and coherent: k_chain_run writes its scalars here at the end of a launch
    e = hipHostMalloc(&ch->st_host, sizeof(ChainScalars), hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return hip_err(c, e, "hipHostMalloc(chain scalars)");
    e = hipHostGetDevicePointer(reinterpret_cast<void **>(&d.st_host), ch->st_host, 0);
    if (e != hipSuccess) return hip_err(c, e, "hipHostGetDevicePointer(chain scalars)");
    // ---- uploads ----
    const int N = (int)ch->x.size();
    std::vector<int> ident((size_t)cap);
    std::vector<long long> rank0((size_t)cap, -1);  // stamps: slots >= N are free
    for (int i = 0; i < cap; ++i) ident[(size_t)i] = i;
    for (int i = 0; i < N; ++i) rank0[(size_t)i] = i;
    std::vector<double> hc(4 * (size_t)cap, 0.0);
    std::copy(ch->x.begin(), ch->x.end(), hc.begin());
    std::copy(ch->y.begin(), ch->y.end(), hc.begin() + cap);
    std::copy(ch->z.begin(), ch->z.end(), hc.begin() + 2 * cap);
    std::copy(ch->zeta.begin(), ch->zeta.end(), hc.begin() + 3 * cap);
    ChainScalars s0{};
    s0.iter = ch->iter;
    s0.ncells = N;
    s0.nslots = N;
    s0.nfree = 0;
    s0.next_stamp = N;  // stamps 0..N-1: the starting cells in Julia order
    s0.phi = 1.0;  // debug_prior: evaluate returns phi = 1 (MCsub.jl:131)
    std::vector<double> logN((size_t)cap + 2);  // logN[k] = det_log(k): the MH model-size factor
    for (size_t k = 0; k < logN.size(); ++k) logN[k] = tdchain::det_log((double)k);
    struct Up { void *d; const void *h; size_t b; } ups[] = {
        {logN_d, logN.data(), sizeof(double) * logN.size()},
        {tile_start, tsc.data(), sizeof(int) * tsc.size()},
        {tile_ray_d, tray2.data(), sizeof(int) * tray2.size()},
        {pt_ray_d, pt_ray.data(), sizeof(int) * (size_t)P},
        {tlo, lo2.data(), sizeof(float) * lo2.size()},
        {thi, hi2.data(), sizeof(float) * hi2.size()},
        {slo_d, slo.data(), sizeof(float) * slo.size()},
        {shi_d, shi.data(), sizeof(float) * shi.size()},
        {cells, hc.data(), sizeof(double) * hc.size()},
        {d.order, ident.data(), sizeof(int) * (size_t)cap},
        {d.stamp, rank0.data(), sizeof(long long) * (size_t)cap},
        {d.bucket_count, bcount.data(), sizeof(int) * nbuckets},
        {d.buckets, bent.data(), sizeof(CellEntry) * bent.size()},
        {d.bslot, bslot.data(), sizeof(int) * bslot.size()},
        {d.grid_overflow, &overflow, sizeof(int)},
        {d.st, &s0, sizeof s0}};
    for (auto &u : ups)
        if (u.b) {
            e = hipMemcpyAsync(u.d, u.h, u.b, hipMemcpyHostToDevice, c->stream);
            if (e != hipSuccess) return hip_err(c, e, "hipMemcpy(chain setup)");
        }
    if (ch->prm.debug_prior != 1) {
        e = chain_full_state(d, N, ch->nn, c->num_cus, c->stream);
        if (e != hipSuccess) return hip_err(c, e, "chain initial evaluate");
    }
    e = hipStreamSynchronize(c->stream);  // the host vectors above die here
    if (e != hipSuccess) return hip_err(c, e, "chain setup sync");
    return TD_OK;
}

// the chain's scalars from its pinned mirror (written by k_chain_run at the end
// of every launch, or copied by device_pull_scalars)
void adopt_scalars(td_chain *ch) {
    const ChainScalars &s = *ch->st_host;
    ch->iter = s.iter;
    ch->phi = s.phi;
    ch->stats.evaluations = s.evaluations;
    for (int a = 0; a < 5; ++a) {
        ch->stats.accepted[a] = s.accepted[a];
        ch->stats.proposed[a] = s.proposed[a];
    }
    ch->stats.ncells = s.ncells;
    ch->stats.phi = s.phi;
    ch->stats.bytes = s.bytes;
    ch->stats.last_action = s.last_action;
    ch->stats.last_accept = s.last_accept;
}

int device_pull_scalars(td_chain *ch) {
    td_ctx *c = ch->ctx;
    hipError_t e = hipMemcpyAsync(ch->st_host, ch->st_dev, sizeof(ChainScalars), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "chain scalars");
    adopt_scalars(ch);
    return TD_OK;
}

int server_stop(td_chain *ch);

// The resident servers this thread started.  A resident kernel occupies its
// stream's hardware queue; HIP maps streams onto GPU_MAX_HW_QUEUES (4 on the
// box) queues, so work on any other stream -- another context's, this
// context's own, torch's, RCCL's -- may sit behind it until its watchdog.
// servers_quiesce stops them before such work (include/tdstar.h, contexts).
// One registry for the process, each entry tagged with the thread that started
// it: a thread quiesces its own launches, and a launch stopped or freed on any
// thread (a Python finaliser may run anywhere) leaves no entry behind.
struct Resident {
    td_chain *srv;    // a td_evaluate shadow server, or
    td_rounds *rnd;   // a resident tempering launch
    std::thread::id owner;
};
std::mutex g_res_mu;
std::vector<Resident> g_res;
int rounds_stop(td_rounds *r);

void servers_register(td_chain *ch) {
    std::lock_guard<std::mutex> g(g_res_mu);
    g_res.push_back(Resident{ch, nullptr, std::this_thread::get_id()});
}
void servers_unregister(td_chain *ch) {
    std::lock_guard<std::mutex> g(g_res_mu);
    g_res.erase(std::remove_if(g_res.begin(), g_res.end(), [&](const Resident &e) { return e.srv == ch; }),
                g_res.end());
}
void rounds_register(td_rounds *r) {
    std::lock_guard<std::mutex> g(g_res_mu);
    g_res.push_back(Resident{nullptr, r, std::this_thread::get_id()});
}
void rounds_unregister(td_rounds *r) {
    std::lock_guard<std::mutex> g(g_res_mu);
    g_res.erase(std::remove_if(g_res.begin(), g_res.end(), [&](const Resident &e) { return e.rnd == r; }),
                g_res.end());
}

}  // namespace

namespace tdstar {
void servers_quiesce(const td_chain *keep) {
    std::vector<Resident> mine;
    {
        std::lock_guard<std::mutex> g(g_res_mu);
        for (const Resident &e : g_res)
            if (e.owner == std::this_thread::get_id()) mine.push_back(e);
    }
    for (const Resident &e : mine) {
        if (e.srv && e.srv != keep) (void)server_stop(e.srv);
        if (e.rnd) (void)rounds_stop(e.rnd);
    }
}
}  // namespace tdstar

namespace {

void free_chain(td_chain *ch) {
    if (!ch) return;
    if (ch->rounds) (void)rounds_stop(ch->rounds);
    if (ch->rounds) {  // the rounds object outlives the chain: forget it
        auto &v = ch->rounds->chains;
        v.erase(std::remove(v.begin(), v.end(), ch), v.end());
    }
    (void)server_stop(ch);
    if (ch->srv_stream) (void)hipStreamDestroy(ch->srv_stream);
    if (ch->mb_host) (void)hipHostFree(ch->mb_host);
    if (ch->ctx && ch->ctx->stream) (void)hipStreamSynchronize(ch->ctx->stream);
    if (ch->dev_block) (void)hipFree(ch->dev_block);
    if (ch->st_host) (void)hipHostFree(ch->st_host);
    if (ch->script_host) (void)hipHostFree(ch->script_host);
    if (ch->nn.part_d) (void)hipFree(ch->nn.part_d);
    if (ch->nn.part_i) (void)hipFree(ch->nn.part_i);
    delete ch;
}

// ---- server mode: one resident k_chain_run per shadow chain, fed through a
//      mailbox in pinned host memory (chain_dev.h Mailbox) ----
volatile long long *vol(long long *p) { return p; }

// testing hook (tdt_set_server_post_delay): sleep between the alive check and the
// post, so the kernel's idle watchdog fires first (the race of a descheduled host)
std::atomic<int> g_post_delay_ms{0};
constexpr int kExitedEarly = -1;  // server_post: the kernel returned before answering

// Publish the command written into the mailbox: its check, then seq (the kernel reads them all
// in one poll and takes the command only when the check matches)
void post_seq(Mailbox *m, long long sq) {
    m->check = mailbox_check(m, sq);
    std::atomic_thread_fence(std::memory_order_release);
    *vol(&m->seq) = sq;
}

int server_stop(td_chain *ch) {
    if (!ch || !ch->srv_running) return TD_OK;
    Mailbox *m = ch->mb_host;
    if (!*vol(&m->exited)) {
        m->type = kCmdQuit;
        post_seq(m, m->seq + 1);
    }
    hipError_t e = hipStreamSynchronize(ch->srv_stream);  // the kernel returns (QUIT, or its idle watchdog)
    ch->srv_running = false;
    ch->srv_has_pending = false;  // the kernel undid it
    servers_unregister(ch);
    if (e != hipSuccess) return hip_err(ch->ctx, e, "chain server exit");
    adopt_scalars(ch);
    return TD_OK;
}

int server_start(td_chain *ch) {
    if (ch->srv_running) return TD_OK;
    servers_quiesce(ch);  // one resident kernel per thread
    td_ctx *c = ch->ctx;
    Mailbox *m = ch->mb_host;
    m->exited = 0;
    m->done = m->seq;
    m->pq_seq = -1;
    ch->pq_expect = -1;
    std::atomic_thread_fence(std::memory_order_release);
    hipError_t e = hipSuccess;
    if (ch->desc_dirty) {
        e = hipMemcpyAsync(ch->dev_ptr, &ch->dev, sizeof(DevChain), hipMemcpyHostToDevice, ch->srv_stream);
        if (e != hipSuccess) return hip_err(c, e, "server descriptor upload");
        ch->desc_dirty = false;
    }
    ScriptArgs sa{};
    sa.out = ch->script_dev;
    sa.mb = ch->mb_dev;
    e = chain_run(&ch->dev, ch->dev_ptr, 1, LLONG_MAX, ch->srv_stream, &sa);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_run launch (server)");
    ch->srv_running = true;
    ch->srv_last = std::chrono::steady_clock::now();
    servers_register(ch);
    return TD_OK;
}

// Wait for the answer to command `sq`.  kExitedEarly: the kernel had returned
// (idle watchdog) before it read the command -- its pending proposal undone,
// its state written back, nothing of the command done; the caller re-issues it
// to a new launch.
int server_wait(td_chain *ch, long long sq) {
    Mailbox *m = ch->mb_host;
    const auto t0 = std::chrono::steady_clock::now();
    for (long long spin = 0;; ++spin) {
        if (*vol(&m->done) == sq) break;
        if (*vol(&m->exited)) {  // returned before answering (it was idle past its watchdog)
            const hipError_t e = hipStreamSynchronize(ch->srv_stream);
            ch->srv_running = false;
            ch->srv_has_pending = false;
            servers_unregister(ch);
            if (e != hipSuccess) return hip_err(ch->ctx, e, "chain server exit");
            adopt_scalars(ch);
            return kExitedEarly;
        }
        if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20))
            return set_err(ch->ctx, TD_ERR_HIP, "chain server: no answer in 20 s");
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    ch->srv_last = std::chrono::steady_clock::now();
    return TD_OK;
}


// ---- resident tempering rounds ----
int rounds_stop(td_rounds *r) {
    if (!r || !r->running) return TD_OK;
    RoundBox *b = r->rb_host;
    b->cmd = kRoundQuit;
    b->K = 0;
    std::atomic_thread_fence(std::memory_order_release);
    *vol(&b->seq) = ++r->seq;
    const hipError_t e = hipStreamSynchronize(r->stream);  // every workgroup returns (QUIT or its watchdog)
    r->running = false;
    rounds_unregister(r);
    if (e != hipSuccess) return hip_err(r->ctx, e, "tempering rounds exit");
    for (td_chain *ch : r->chains) adopt_scalars(ch);
    return TD_OK;
}

int rounds_start(td_rounds *r) {
    if (r->running) return TD_OK;
    td_ctx *c = r->ctx;
    servers_quiesce(nullptr);  // (stops every other resident launch of this thread)
    RoundBox *b = r->rb_host;
    const int nc = (int)r->chains.size();
    for (int k = 0; k < nc; ++k) {
        b->slot[k].done = r->seq;  // the workgroup waits for a seq past this
        b->slot[k].exited = 0;
        r->desc_host[k] = r->chains[(size_t)k]->dev;
        r->chains[(size_t)k]->desc_dirty = true;  // (its own descriptor copy is refreshed on its next run)
    }
    b->seq = r->seq;
    std::atomic_thread_fence(std::memory_order_release);
    hipError_t e = hipMemcpyAsync(r->desc_dev, r->desc_host, sizeof(DevChain) * (size_t)nc, hipMemcpyHostToDevice,
                                  r->stream);
    if (e != hipSuccess) return hip_err(c, e, "tempering rounds descriptors");
    ScriptArgs sa{};
    sa.rb = r->rb_dev;
    e = chain_run(r->desc_host, r->desc_dev, nc, LLONG_MAX, r->stream, &sa);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_run launch (tempering rounds)");
    r->running = true;
    rounds_register(r);
    return TD_OK;
}

}  // namespace

extern "C" {

int td_rounds_create(td_rounds **out, td_chain *const *chains, int64_t nchains) {
    if (!out || !chains || nchains <= 0 || nchains > 65536) return set_err(nullptr, TD_ERR_ARG, "td_rounds_create");
    *out = nullptr;
    td_ctx *c = chains[0] ? chains[0]->ctx : nullptr;
    if (!c) return set_err(nullptr, TD_ERR_ARG, "td_rounds_create: NULL chain");
    for (int64_t b = 0; b < nchains; ++b) {
        if (!chains[b] || chains[b]->ctx != c || chains[b]->engine != TD_ENGINE_DEVICE || chains[b]->rounds)
            return set_err(c, TD_ERR_ARG, "td_rounds_create: DEVICE chains of one context, each in one td_rounds");
        for (int64_t k = 0; k < b; ++k)
            if (chains[k] == chains[b]) return set_err(c, TD_ERR_ARG, "td_rounds_create: a chain appears twice");
    }
    // every workgroup must be resident at once (each waits for the host between rounds): one per CU
    if (nchains > c->num_cus)
        return set_err(c, TD_ERR_ARG, "td_rounds_create: more chains than compute units (one resident workgroup each)");
    td_rounds *r = new (std::nothrow) td_rounds();
    if (!r) return set_err(c, TD_ERR_NOMEM, "td_rounds_create");
    r->ctx = c;
    r->chains.assign(chains, chains + nchains);
    const size_t bytes = sizeof(RoundBox) + sizeof(RoundSlot) * (size_t)nchains;
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipHostMalloc(&r->rb_host, bytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        std::memset(r->rb_host, 0, bytes);
        e = hipHostGetDevicePointer(reinterpret_cast<void **>(&r->rb_dev), r->rb_host, 0);
    }
    if (e == hipSuccess) e = hipMalloc(&r->desc_dev, sizeof(DevChain) * (size_t)nchains);
    if (e == hipSuccess) e = hipHostMalloc(&r->desc_host, sizeof(DevChain) * (size_t)nchains, hipHostMallocDefault);
    // the resident launch on a hardware queue of its own: it must not hold back other streams
    // (torch's, RCCL's exchange stream) that HIP would otherwise deal onto its queue
    if (e == hipSuccess) e = rounds_stream(&r->stream, c->device);
    if (e != hipSuccess) {
        (void)td_rounds_destroy(r);
        return hip_err(c, e, "td_rounds_create");
    }
    for (td_chain *ch : r->chains) ch->rounds = r;
    *out = r;
    return TD_OK;
}

int td_rounds_run(td_rounds *r, int64_t K, const double *temps, double *phi_out) {
    if (!r || K <= 0 || K > INT32_MAX || !temps) return set_err(r ? r->ctx : nullptr, TD_ERR_ARG, "td_rounds_run");
    const int nc = (int)r->chains.size();
    if (nc == 0) return set_err(r->ctx, TD_ERR_ARG, "td_rounds_run: its chains were destroyed");
    for (int k = 0; k < nc; ++k)
        if (!(temps[k] > 0.0)) return set_err(r->ctx, TD_ERR_ARG, "td_rounds_run: need T > 0");
    TD_HIP(r->ctx, hipSetDevice(r->ctx->device));
    // ran[k]: chain k ran this round in a launch that was lost (another workgroup's idle watchdog
    // fired as the round was posted); the retry asks it only to report phi again (RoundSlot::skip)
    std::vector<char> ran((size_t)nc, 0);
    RoundBox *b = r->rb_host;
    for (int attempt = 0;; ++attempt) {
        const bool forcing = !r->force_exit.empty();  // testing: tdt_rounds_force_exit
        for (int k = 0; k < nc; ++k) b->slot[k].idle = (forcing && r->force_exit[(size_t)k]) ? 1 : 0;
        int rc = rounds_start(r);
        if (rc) return rc;
        if (forcing) {  // the forced workgroups return at their first wait, before the round is posted
            const auto tf = std::chrono::steady_clock::now();
            for (int k = 0; k < nc; ++k)
                while (r->force_exit[(size_t)k] && !*vol(&b->slot[k].exited))
                    if (std::chrono::steady_clock::now() - tf > std::chrono::seconds(20))
                        return set_err(r->ctx, TD_ERR_HIP, "tempering rounds: forced exit never came");
            r->force_exit.clear();
            for (int k = 0; k < nc; ++k) b->slot[k].idle = 0;
        }
        for (int k = 0; k < nc; ++k) {  // the chain's temperature: its host params too (td_chain_set_temperature)
            td_chain *ch = r->chains[(size_t)k];
            ch->prm.temperature = temps[k];
            ch->P.temperature = temps[k];
            tdchain::params_derived(ch->P);
            ch->dev.params = ch->P;
            b->slot[k].T = ch->P.temperature;
            b->slot[k].inv_2t = ch->P.inv_2t;
            b->slot[k].skip = ran[(size_t)k];
        }
        b->cmd = kRoundRun;
        b->K = (int)K;
        std::atomic_thread_fence(std::memory_order_release);
        const long long sq = ++r->seq;
        *vol(&b->seq) = sq;
        bool lost = false;
        const auto t0 = std::chrono::steady_clock::now();
        if (rounds_trace()) {  // diagnostic: when each replica's round ends, from the post (TD_ROUNDS_TRACE)
            double first = -1.0, last = 0.0;
            int left = nc;
            std::vector<char> seen((size_t)nc, 0);
            for (long long spin = 0; left > 0 && !lost; ++spin) {
                for (int k = 0; k < nc; ++k) {
                    if (seen[(size_t)k]) continue;
                    if (*vol(&b->slot[k].done) == sq) {
                        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                        if (first < 0.0) first = us;
                        last = us;
                        seen[(size_t)k] = 1;
                        --left;
                    } else if (*vol(&b->slot[k].exited)) {
                        lost = true;
                    }
                }
                if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
                    return set_err(r->ctx, TD_ERR_HIP, "tempering rounds: no answer in 60 s");
            }
            if (!lost) {
                r->tr_first += first;
                r->tr_last += last;
                r->tr_n += 1;
            }
        }
        for (int k = 0; k < nc && !lost; ++k)
            for (long long spin = 0;; ++spin) {
                if (*vol(&b->slot[k].done) == sq) break;
                if (*vol(&b->slot[k].exited)) {  // its watchdog fired before this round was posted
                    lost = true;
                    break;
                }
                if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
                    return set_err(r->ctx, TD_ERR_HIP, "tempering rounds: no answer in 60 s");
            }
        if (!lost) break;
        // Some workgroup returned at the round boundary before it saw this round (its idle
        // watchdog), while others may have run it.  End the launch (QUIT for the ones still
        // waiting; every state is consistent between rounds), note who ran the round, and post it
        // again to a new launch: the chains that ran it only report phi (skip).
        b->cmd = kRoundQuit;
        b->K = 0;
        std::atomic_thread_fence(std::memory_order_release);
        *vol(&b->seq) = ++r->seq;
        const hipError_t e = hipStreamSynchronize(r->stream);
        r->running = false;
        rounds_unregister(r);
        if (e != hipSuccess) return hip_err(r->ctx, e, "tempering rounds exit");
        for (td_chain *ch : r->chains) adopt_scalars(ch);
        for (int k = 0; k < nc; ++k)
            if (*vol(&b->slot[k].done) == sq) ran[(size_t)k] = 1;
        if (attempt > 2) return set_err(r->ctx, TD_ERR_HIP, "tempering rounds: the launch keeps returning");
    }
    for (int k = 0; k < nc; ++k) b->slot[k].skip = 0;
    std::atomic_thread_fence(std::memory_order_acquire);
    for (int k = 0; k < nc; ++k) {
        td_chain *ch = r->chains[(size_t)k];
        const double phi = *reinterpret_cast<volatile double *>(&r->rb_host->slot[k].phi);
        ch->phi = phi;
        ch->stats.phi = phi;
        ch->stats.iterations += K;
        if (phi_out) phi_out[k] = phi;
    }
    return TD_OK;
}

int td_swap_decide(int64_t R, const double *phis, const int64_t *levels, const double *temps, int64_t rnd,
                   uint64_t seed, int64_t *new_levels, int64_t *tried, int64_t *accepted) {
    if (R < 1 || !phis || !levels || !temps || !new_levels || rnd < 0) return TD_ERR_ARG;
    std::vector<int64_t> owner((size_t)R, -1);
    for (int64_t g = 0; g < R; ++g) {
        if (levels[g] < 0 || levels[g] >= R || owner[(size_t)levels[g]] >= 0) return TD_ERR_ARG;  // a permutation
        owner[(size_t)levels[g]] = g;
        new_levels[g] = levels[g];
    }
    for (int64_t l = rnd % 2; l < R - 1; l += 2) {
        const int64_t a = owner[(size_t)l], b = owner[(size_t)l + 1];
        if (tried) tried[l] += 1;
        // chain_logic.h swap_accept: what the exchange kernel decides with (no contraction: -ffp-contract=off)
        if (tdchain::swap_accept(phis[a], phis[b], temps[l], temps[l + 1], seed, (uint64_t)rnd, (uint64_t)l)) {
            new_levels[a] = l + 1;
            new_levels[b] = l;
            owner[(size_t)l] = b;
            owner[(size_t)l + 1] = a;
            if (accepted) accepted[l] += 1;
        }
    }
    return TD_OK;
}

int td_rounds_temper(td_rounds *r, int64_t M, int64_t K, const double *temps, int64_t *levels, int64_t rnd0,
                     uint64_t seed, double *phis_out, int64_t *levels_out, int64_t *tried, int64_t *accepted) {
    if (!r || M < 0 || K <= 0 || !temps || !levels || rnd0 < 0)
        return set_err(r ? r->ctx : nullptr, TD_ERR_ARG, "td_rounds_temper");
    const int64_t R = (int64_t)r->chains.size();
    std::vector<double> T((size_t)R), phi((size_t)R);
    std::vector<int64_t> nl((size_t)R);
    {  // levels must be a permutation of 0..R-1 before any round runs (td_swap_decide keeps it one)
        std::vector<char> seen((size_t)R, 0);
        for (int64_t k = 0; k < R; ++k) {
            if (levels[k] < 0 || levels[k] >= R || seen[(size_t)levels[k]])
                return set_err(r->ctx, TD_ERR_ARG, "td_rounds_temper: levels are not a permutation");
            seen[(size_t)levels[k]] = 1;
        }
    }
    for (int64_t j = 0; j < M; ++j) {
        for (int64_t k = 0; k < R; ++k) T[(size_t)k] = temps[levels[k]];
        const int rc = td_rounds_run(r, K, T.data(), phi.data());
        if (rc) return rc;
        if (td_swap_decide(R, phi.data(), levels, temps, rnd0 + j, seed, nl.data(), tried, accepted))
            return set_err(r->ctx, TD_ERR_ARG, "td_rounds_temper: levels are not a permutation");
        for (int64_t k = 0; k < R; ++k) levels[k] = nl[(size_t)k];
        if (phis_out) std::memcpy(phis_out + j * R, phi.data(), sizeof(double) * (size_t)R);
        if (levels_out) std::memcpy(levels_out + j * R, levels, sizeof(int64_t) * (size_t)R);
    }
    return TD_OK;
}

}  // extern "C"

namespace {

void exchange_free(td_rounds *r) {
    for (void *p : {(void *)r->x_in, (void *)r->x_out, (void *)r->x_temps, (void *)r->x_rdy, (void *)r->x_gdone,
                    (void *)r->x_lev, (void *)r->x_desc, (void *)r->x_bar})
        if (p) (void)hipFree(p);
    if (r->x_ready) (void)(r->x_ready_pinned ? hipHostFree(r->x_ready) : hipFree(r->x_ready));
    for (void *p : {(void *)r->x_log_phi, (void *)r->x_log_lev, (void *)r->x_log_t, (void *)r->x_err})
        if (p) (void)hipHostFree(p);
    r->x_in = r->x_out = r->x_temps = nullptr;
    r->x_bar = nullptr;
    r->x_rdy = r->x_gdone = r->x_ready = nullptr;
    r->x_lev = nullptr;
    r->x_desc = nullptr;
    r->x_log_phi = nullptr;
    r->x_log_lev = nullptr;
    r->x_log_t = nullptr;
    r->x_err = nullptr;
    r->x_R = 0;
    r->x_log_cap = 0;
    r->x_tag = r->x_gtag = 0;
}

// TD_EXCHANGE_TRIGGER=host: the host watches `ready` (pinned memory) and issues each allgather itself,
// instead of the exchange stream waiting on it (hipStreamWaitValue64) -- a diagnostic alternative
bool exchange_host_trigger() {
    static const bool on = [] {
        const char *e = std::getenv("TD_EXCHANGE_TRIGGER");
        return e && std::strcmp(e, "host") == 0;
    }();
    return on;
}

int exchange_alloc(td_rounds *r, int R, int64_t M) {
    td_ctx *c = r->ctx;
    const int local = (int)r->chains.size();
    if (r->x_R != R) {
        exchange_free(r);
        // double-buffered by round parity: a workgroup still reading round j's gathered phis cannot see a
        // faster one's round j+1 phi (on one rank x_out is x_in)
        TD_HIP(c, hipMalloc(&r->x_in, sizeof(double) * 2 * (size_t)local));
        TD_HIP(c, hipMalloc(&r->x_out, sizeof(double) * 2 * (size_t)R));
        TD_HIP(c, hipMalloc(&r->x_bar, sizeof(long long)));
        TD_HIP(c, hipMalloc(&r->x_temps, sizeof(double) * (size_t)R));
        TD_HIP(c, hipMalloc(&r->x_rdy, sizeof(unsigned long long) * (size_t)local));
        TD_HIP(c, hipMalloc(&r->x_gdone, sizeof(unsigned long long)));
        TD_HIP(c, hipMalloc(&r->x_lev, sizeof(int) * (size_t)local * (size_t)R));
        TD_HIP(c, hipMalloc(&r->x_desc, sizeof(RoundX)));
        TD_HIP(c, hipMemset(r->x_rdy, 0, sizeof(unsigned long long) * (size_t)local));
        TD_HIP(c, hipMemset(r->x_gdone, 0, sizeof(unsigned long long)));
        r->x_ready_pinned = exchange_host_trigger();
        if (r->x_ready_pinned) {
            TD_HIP(c, hipHostMalloc(&r->x_ready, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent));
        } else {  // what hipStreamWaitValue64 waits on
            TD_HIP(c, hipExtMallocWithFlags(reinterpret_cast<void **>(&r->x_ready), sizeof(unsigned long long),
                                            hipMallocSignalMemory));
        }
        *reinterpret_cast<volatile unsigned long long *>(r->x_ready) = 0;  // (host-visible either way)
        TD_HIP(c, hipHostMalloc(&r->x_err, sizeof(long long), hipHostMallocMapped | hipHostMallocCoherent));
        r->x_R = R;
        r->x_tag = r->x_gtag = 0;
    }
    if (M > r->x_log_cap) {
        if (r->x_log_phi) (void)hipHostFree(r->x_log_phi);
        if (r->x_log_lev) (void)hipHostFree(r->x_log_lev);
        if (r->x_log_t) (void)hipHostFree(r->x_log_t);
        r->x_log_phi = nullptr;
        r->x_log_lev = nullptr;
        r->x_log_t = nullptr;
        r->x_log_cap = 0;
        TD_HIP(c, hipHostMalloc(&r->x_log_phi, sizeof(double) * (size_t)M * (size_t)R, hipHostMallocMapped));
        TD_HIP(c, hipHostMalloc(&r->x_log_lev, sizeof(int) * (size_t)M * (size_t)R, hipHostMallocMapped));
        TD_HIP(c, hipHostMalloc(&r->x_log_t, sizeof(long long) * 3 * (size_t)M, hipHostMallocMapped));
        r->x_log_cap = M;
    }
    return TD_OK;
}

// One-word max all-reduce over the communicator, host-synchronized: with vote 0 it is a barrier (every rank
// has reached it when it returns); *out = the maximum vote over the ranks.
int comm_vote(td_ctx *c, td_comm *comm, long long *word, long long vote, long long *out) {
    TD_HIP(c, hipMemcpyAsync(word, &vote, sizeof(long long), hipMemcpyHostToDevice, comm->stream));
    const ncclResult_t nr = ncclAllReduce(word, word, 1, ncclInt64, ncclMax, comm->comm, comm->stream);
    if (nr != ncclSuccess) return set_err(c, TD_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(nr));
    long long v = 0;
    TD_HIP(c, hipMemcpyAsync(&v, word, sizeof(long long), hipMemcpyDeviceToHost, comm->stream));
    TD_HIP(c, hipStreamSynchronize(comm->stream));
    if (out) *out = v;
    return TD_OK;
}

template <class T>
T *dev_addr(T *host) {  // the device address of mapped pinned memory
    void *d = nullptr;
    return hipHostGetDevicePointer(&d, host, 0) == hipSuccess ? static_cast<T *>(d) : nullptr;
}

}  // namespace

extern "C" {

int td_rounds_exchange(td_rounds *r, td_comm *comm, int64_t M, int64_t K, const double *temps, int64_t *levels,
                       int64_t rnd0, uint64_t seed, double *phis_out, int64_t *levels_out, int64_t *tried,
                       int64_t *accepted, double *timing_out) {
    if (!r || M < 0 || K <= 0 || K > INT32_MAX || M * K > ((int64_t)1 << 40) || !temps || !levels || rnd0 < 0)
        return set_err(r ? r->ctx : nullptr, TD_ERR_ARG, "td_rounds_exchange");
    td_ctx *c = r->ctx;
    const int local = (int)r->chains.size();
    if (local == 0) return set_err(c, TD_ERR_ARG, "td_rounds_exchange: its chains were destroyed");
    const int nranks = comm ? comm->nranks : 1, rank = comm ? comm->rank : 0;
    const int64_t R = (int64_t)local * nranks;
    if (R > 64) return set_err(c, TD_ERR_ARG, "td_rounds_exchange: at most 64 replicas (one lane each)");
    if (comm && comm->device != c->device)
        return set_err(c, TD_ERR_ARG, "td_rounds_exchange: the communicator is on another device");
    {
        std::vector<char> seen((size_t)R, 0);
        for (int64_t g = 0; g < R; ++g) {
            if (levels[g] < 0 || levels[g] >= R || seen[(size_t)levels[g]])
                return set_err(c, TD_ERR_ARG, "td_rounds_exchange: levels are not a permutation");
            seen[(size_t)levels[g]] = 1;
        }
        for (int64_t l = 0; l < R; ++l)
            if (!(temps[l] > 0.0)) return set_err(c, TD_ERR_ARG, "td_rounds_exchange: need T > 0");
    }
    if (M == 0) return TD_OK;
    const auto t_call = std::chrono::steady_clock::now();
    TD_HIP(c, hipSetDevice(c->device));
    servers_quiesce(nullptr);
    int rc = rounds_stop(r);  // this launch's host-posted rounds, whichever thread posted them
    if (rc) return rc;
    rc = exchange_alloc(r, (int)R, M);
    if (rc) return rc;
    if (comm) {  // entry barrier: every rank is here before any kernel's exchange watchdog starts
        rc = comm_vote(c, comm, r->x_bar, 0, nullptr);
        if (rc) return rc;
    }
    // every chain starts at its level's temperature; the kernel's workgroups each keep all levels
    std::vector<int> lev0((size_t)local * (size_t)R);
    std::vector<int64_t> iter0((size_t)local);
    for (int k = 0; k < local; ++k) {
        iter0[(size_t)k] = r->chains[(size_t)k]->iter;
        td_chain *ch = r->chains[(size_t)k];
        ch->prm.temperature = temps[levels[rank * local + k]];
        ch->P.temperature = ch->prm.temperature;
        tdchain::params_derived(ch->P);
        ch->dev.params = ch->P;
        r->desc_host[k] = ch->dev;
        ch->desc_dirty = true;  // (its own descriptor copy is refreshed on its next run)
        for (int64_t g = 0; g < R; ++g) lev0[(size_t)k * (size_t)R + (size_t)g] = (int)levels[g];
    }
    *reinterpret_cast<volatile long long *>(r->x_err) = 0;
    TD_HIP(c, hipMemcpyAsync(r->x_lev, lev0.data(), sizeof(int) * lev0.size(), hipMemcpyHostToDevice, r->stream));
    TD_HIP(c, hipMemcpyAsync(r->x_temps, temps, sizeof(double) * (size_t)R, hipMemcpyHostToDevice, r->stream));
    TD_HIP(c, hipMemcpyAsync(r->desc_dev, r->desc_host, sizeof(DevChain) * (size_t)local, hipMemcpyHostToDevice,
                             r->stream));
    RoundX &x = r->x_host;
    x = RoundX{};
    x.xin = r->x_in;
    x.xout = comm ? r->x_out : r->x_in;
    x.rdy = r->x_rdy;
    x.ready = r->x_ready_pinned ? dev_addr(r->x_ready) : r->x_ready;
    x.gdone = comm ? r->x_gdone : nullptr;
    x.ready_base = r->x_tag;
    x.gdone_base = r->x_gtag;
    x.lev = r->x_lev;
    x.temps = r->x_temps;
    x.log_phi = dev_addr(r->x_log_phi);
    x.log_lev = dev_addr(r->x_log_lev);
    x.log_t = dev_addr(r->x_log_t);
    x.err = dev_addr(r->x_err);
    x.rnd0 = rnd0;
    x.seed = seed;
    x.R = (int)R;
    x.local = local;
    x.rank = rank;
    x.M = (int)M;
    x.K = (int)K;
    if (!x.ready || !x.log_phi || !x.log_lev || !x.log_t || !x.err)
        return set_err(c, TD_ERR_HIP, "td_rounds_exchange: pinned memory without a device address");
    TD_HIP(c, hipMemcpyAsync(r->x_desc, &r->x_host, sizeof(RoundX), hipMemcpyHostToDevice, r->stream));
    ScriptArgs sa{};
    sa.rx = r->x_desc;
    hipError_t e = chain_run(r->desc_host, r->desc_dev, local, M * K, r->stream, &sa,
                             DrawsBuf{&c->draws, &c->draws_bytes});
    if (e != hipSuccess) return hip_err(c, e, "k_chain_run launch (exchange rounds)");
    const auto t_launched = std::chrono::steady_clock::now();
    // the exchanges: each allgather on the exchange stream once this rank's phis of the round are in
    bool stuck = false;
    if (comm) {
        for (int64_t j = 0; j < M && !stuck; ++j) {
            const unsigned long long tag = r->x_tag + (unsigned long long)j + 1ull;
            if (r->x_ready_pinned) {  // host trigger
                const auto t0 = std::chrono::steady_clock::now();
                for (long long spin = 0; *reinterpret_cast<volatile unsigned long long *>(r->x_ready) < tag; ++spin)
                    if ((spin & 1023) == 1023 &&
                        (*reinterpret_cast<volatile long long *>(r->x_err) ||
                         std::chrono::steady_clock::now() - t0 > std::chrono::seconds(12))) {
                        stuck = true;
                        break;
                    }
                if (stuck) {  // still post this rank's remaining allgathers, so that no peer waits on them forever
                    for (int64_t q = j; q < M; ++q) {
                        const ncclResult_t nq = ncclAllGather(r->x_in + (q & 1) * local, r->x_out + (q & 1) * R,
                                                              (size_t)local, ncclFloat64, comm->comm, comm->stream);
                        if (nq != ncclSuccess)
                            return set_err(c, TD_ERR_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(nq));
                    }
                    break;
                }
            } else {
                e = hipStreamWaitValue64(comm->stream, r->x_ready, tag, hipStreamWaitValueGte);
                if (e != hipSuccess) return hip_err(c, e, "hipStreamWaitValue64");
            }
            const ncclResult_t nr = ncclAllGather(r->x_in + (j & 1) * local, r->x_out + (j & 1) * R, (size_t)local,
                                                  ncclFloat64, comm->comm, comm->stream);
            if (nr != ncclSuccess) return set_err(c, TD_ERR_HIP, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
            e = hipStreamWriteValue64(comm->stream, r->x_gdone, r->x_gtag + (unsigned long long)j + 1ull, 0);
            if (e != hipSuccess) return hip_err(c, e, "hipStreamWriteValue64");
        }
    }
    const auto t_enqueued = std::chrono::steady_clock::now();
    e = hipStreamSynchronize(r->stream);  // (the kernel gives up after 10 s without an exchange)
    if (e != hipSuccess) return hip_err(c, e, "exchange rounds");
    bool failed = *reinterpret_cast<volatile long long *>(r->x_err) != 0 || stuck;
    if (comm) {
        if (failed && !r->x_ready_pinned) {  // release the exchange stream's waits, then drain it
            e = hipStreamWriteValue64(r->stream, r->x_ready, ~0ull >> 1, 0);
            if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
        }
        e = hipStreamSynchronize(comm->stream);
        if (e != hipSuccess) return hip_err(c, e, "exchange stream");
        // the ranks agree on the outcome: levels are committed only when no rank failed
        long long any = 0;
        rc = comm_vote(c, comm, r->x_bar, failed ? 1 : 0, &any);
        if (rc) return rc;
        failed = any != 0;
    }
    const auto t_done = std::chrono::steady_clock::now();
    for (int k = 0; k < local; ++k) {
        td_chain *ch = r->chains[(size_t)k];
        adopt_scalars(ch);
        ch->stats.iterations += ch->iter - iter0[(size_t)k];
    }
    if (failed) {
        exchange_free(r);  // (fresh flags next time)
        return set_err(c, TD_ERR_HIP, "td_rounds_exchange: an exchange never came (10 s) on this or another rank");
    }
    // the host replays every round's decisions on the logged phis: the device's levels must be its
    std::vector<int64_t> lv(levels, levels + R), nl((size_t)R);
    for (int64_t j = 0; j < M; ++j) {
        const double *ph = r->x_log_phi + j * R;
        if (td_swap_decide(R, ph, lv.data(), temps, rnd0 + j, seed, nl.data(), tried, accepted))
            return set_err(c, TD_ERR_ARG, "td_rounds_exchange: levels");
        for (int64_t g = 0; g < R; ++g)
            if (nl[(size_t)g] != r->x_log_lev[j * R + g])
                return set_err(c, TD_ERR_HIP, "td_rounds_exchange: the device's swap decisions differ from the host's");
        lv = nl;
        if (phis_out) std::memcpy(phis_out + j * R, ph, sizeof(double) * (size_t)R);
        if (levels_out) std::memcpy(levels_out + j * R, lv.data(), sizeof(int64_t) * (size_t)R);
    }
    for (int64_t g = 0; g < R; ++g) levels[g] = lv[(size_t)g];
    for (int k = 0; k < local; ++k) {  // each chain leaves at its final level's temperature
        td_chain *ch = r->chains[(size_t)k];
        const double phi = r->x_log_phi[(M - 1) * R + rank * local + k];
        if (phi != ch->phi) return set_err(c, TD_ERR_HIP, "td_rounds_exchange: a published phi is not the chain's");
        ch->prm.temperature = temps[lv[(size_t)(rank * local + k)]];
        ch->P.temperature = ch->prm.temperature;
        tdchain::params_derived(ch->P);
        ch->dev.params = ch->P;
        ch->desc_dirty = true;
    }
    r->x_tag += (unsigned long long)M;
    r->x_gtag += (unsigned long long)M;
    if (timing_out) {
        // [0] the call, s; [1] launch issued, s; [2] exchanges enqueued, s; [3] mean time from this rank's phis
        // all in (workgroup 0 saw every local flag) to every phi gathered: the exchange; [4] mean time from
        // the phis gathered to workgroup 0's next phi (its proposals); [5] mean time from workgroup 0's phi to
        // the rank's last (waiting for the slowest local replica); [6] the kernel's first publish to its last
        // gather, s
        double ex = 0.0, pr = 0.0, lw = 0.0;
        const long long *t = r->x_log_t;
        for (int64_t j = 0; j < M; ++j) {
            ex += (double)(t[3 * j + 2] - t[3 * j + 1]);
            lw += (double)(t[3 * j + 1] - t[3 * j]);
            if (j > 0) pr += (double)(t[3 * j] - t[3 * j - 1]);
        }
        const double tick = 1e-8;  // the 100 MHz wall clock
        timing_out[0] = std::chrono::duration<double>(t_done - t_call).count();
        timing_out[1] = std::chrono::duration<double>(t_launched - t_call).count();
        timing_out[2] = std::chrono::duration<double>(t_enqueued - t_call).count();
        timing_out[3] = ex / (double)M * tick;
        timing_out[4] = M > 1 ? pr / (double)(M - 1) * tick : 0.0;
        timing_out[5] = lw / (double)M * tick;
        timing_out[6] = (double)(t[3 * (M - 1) + 2] - t[0]) * tick;
    }
    return TD_OK;
}

int td_rounds_destroy(td_rounds *r) {
    if (!r) return TD_OK;
    if (rounds_trace() && r->tr_n > 0)
        std::fprintf(stderr, "[rounds_trace] %d replicas, %lld rounds: first done %.2f us, last done %.2f us after the post\n",
                     (int)r->chains.size(), (long long)r->tr_n, r->tr_first / r->tr_n, r->tr_last / r->tr_n);
    exchange_free(r);
    int rc = rounds_stop(r);
    for (td_chain *ch : r->chains) ch->rounds = nullptr;
    if (r->stream) (void)hipStreamSynchronize(r->stream);  // (the process's rounds stream: kept)
    if (r->rb_host) (void)hipHostFree(r->rb_host);
    if (r->desc_dev) (void)hipFree(r->desc_dev);
    if (r->desc_host) (void)hipHostFree(r->desc_host);
    delete r;
    return rc;
}

int td_chain_create(td_chain **out, td_ctx *ctx, const td_chain_params *params, const double *xCell,
                    const double *yCell, const double *zCell, const double *zeta, int64_t nCells) {
    if (!out || !ctx || !params) return set_err(ctx, TD_ERR_ARG, "td_chain_create: NULL argument");
    *out = nullptr;
    const td_chain_params &p = *params;
    if (p.prior < 1 || p.prior > 3)
        return set_err(ctx, TD_ERR_ARG, "td_chain_create: prior must be 1 (uniform), 2 (normal) or 3 (exponential)");
    if (p.min_cells < 1 || p.max_cells < p.min_cells || p.sig <= 0 || p.zeta_scale <= 0)
        return set_err(ctx, TD_ERR_ARG, "td_chain_create: bad cell bounds / sig / zeta_scale");
    if (!(p.xmax >= p.xmin && p.ymax >= p.ymin && p.zmax >= p.zmin))
        return set_err(ctx, TD_ERR_ARG, "td_chain_create: empty box");
    if (p.engine != TD_ENGINE_DEVICE && p.engine != TD_ENGINE_HOST && p.engine != TD_ENGINE_DROPIN)
        return set_err(ctx, TD_ERR_ARG, "td_chain_create: unknown engine");
    if (nCells < 0 || (nCells > 0 && (!xCell || !yCell || !zCell || !zeta)))
        return set_err(ctx, TD_ERR_ARG, "td_chain_create: bad cell arrays");
    td_chain *ch = new (std::nothrow) td_chain();
    if (!ch) return set_err(ctx, TD_ERR_NOMEM, "td_chain_create: out of memory");
    servers_quiesce(nullptr);
    ch->ctx = ctx;
    ch->prm = p;
    ch->P = make_params(p);
    ch->engine = p.engine;
    ch->iter = p.start_iter > 0 ? p.start_iter : 1;
    if (nCells > 0) {
        ch->x.assign(xCell, xCell + nCells);
        ch->y.assign(yCell, yCell + nCells);
        ch->z.assign(zCell, zCell + nCells);
        ch->zeta.assign(zeta, zeta + nCells);
    } else {
        build_starting(ch);
    }
    ch->ptS.assign((size_t)ctx->g.n, 0.0);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) {
        int rc = hip_err(ctx, e, "hipSetDevice");
        free_chain(ch);
        return rc;
    }
    int rc = TD_OK;
    if (ch->engine != TD_ENGINE_DEVICE) {
        rc = host_evaluate(ch, ch->x, ch->y, ch->z, ch->zeta, &ch->phi, ch->ptS.data());  // build_starting :118
        if (!rc) ch->stats.evaluations = 1;
    } else {
        rc = device_setup(ch);
        if (!rc) rc = device_pull_scalars(ch);
        if (!rc) ch->stats.evaluations = 1;
    }
    if (rc) {
        free_chain(ch);
        return rc;
    }
    ch->stats.phi = ch->phi;
    ch->stats.ncells = (int64_t)ch->x.size();
    *out = ch;
    return TD_OK;
}

int td_chain_destroy(td_chain *ch) {
    free_chain(ch);
    return TD_OK;
}

int td_chain_run(td_chain *ch, int64_t iterations) {
    if (!ch || iterations < 0) return chain_err(ch, TD_ERR_ARG, "td_chain_run: bad arguments");
    if (iterations == 0) return TD_OK;
    hipError_t e = hipSetDevice(ch->ctx->device);
    if (e != hipSuccess) return hip_err(ch->ctx, e, "hipSetDevice");
    if (ch->engine != TD_ENGINE_DROPIN) servers_quiesce(nullptr);  // DROPIN's td_evaluate keeps its own
    if (ch->engine != TD_ENGINE_DEVICE) {
        const int64_t t0 = now_ns();
        for (int64_t i = 0; i < iterations; ++i) {
            int rc = host_iteration(ch);
            if (rc) return rc;
        }
        ch->ctx->dropin_ns[10] += now_ns() - t0;
        ch->ctx->dropin_ns[11] += iterations;
        ch->stats.phi = ch->phi;
        ch->stats.ncells = (int64_t)ch->x.size();
        return TD_OK;
    }
    Timer *tm = ch->ctx->timer.on ? &ch->ctx->timer : nullptr;
    hipEvent_t t0 = tm ? tm->begin(ch->ctx->stream) : nullptr;
    if (ch->desc_dirty) {  // the device copy of the descriptor is current otherwise
        e = hipMemcpyAsync(ch->dev_ptr, &ch->dev, sizeof(DevChain), hipMemcpyHostToDevice, ch->ctx->stream);
        if (e != hipSuccess) return hip_err(ch->ctx, e, "chain descriptor upload");
        ch->desc_dirty = false;
    }
    e = chain_run(&ch->dev, ch->dev_ptr, 1, iterations, ch->ctx->stream, nullptr,
                  DrawsBuf{&ch->ctx->draws, &ch->ctx->draws_bytes});
    if (tm) tm->end("chain_run", t0, ch->ctx->stream);
    if (e != hipSuccess) return hip_err(ch->ctx, e, "k_chain_run launch");
    e = hipStreamSynchronize(ch->ctx->stream);  // the kernel wrote the scalars to st_host
    if (e != hipSuccess) return hip_err(ch->ctx, e, "k_chain_run");
    adopt_scalars(ch);
    ch->stats.iterations += iterations;
    return TD_OK;
}

int td_chain_run_batch(td_chain *const *chains, int64_t nchains, int64_t iterations) {
    if (!chains || nchains <= 0 || iterations < 0 || nchains > INT32_MAX) return TD_ERR_ARG;
    td_ctx *c = chains[0] ? chains[0]->ctx : nullptr;
    if (!c) return TD_ERR_ARG;
    bool host = false;
    for (int64_t b = 0; b < nchains; ++b) {
        if (!chains[b] || chains[b]->ctx != c)
            return set_err(c, TD_ERR_ARG, "td_chain_run_batch: every chain must be non-NULL and share one context");
        host |= chains[b]->engine != TD_ENGINE_DEVICE;
        for (int64_t k = 0; k < b; ++k)
            if (chains[k] == chains[b]) return set_err(c, TD_ERR_ARG, "td_chain_run_batch: a chain appears twice");
    }
    if (iterations == 0) return TD_OK;
    if (!host) servers_quiesce(nullptr);
    if (host || nchains == 1) {  // the host engine is the sequential parity twin
        for (int64_t b = 0; b < nchains; ++b) {
            int rc = td_chain_run(chains[b], iterations);
            if (rc) return rc;
        }
        return TD_OK;
    }
    TD_HIP(c, hipSetDevice(c->device));
    const size_t bytes = sizeof(DevChain) * (size_t)nchains;
    if (bytes > c->chain_desc_bytes) {
        TD_HIP(c, hipStreamSynchronize(c->stream));
        if (c->chain_desc) (void)hipFree(c->chain_desc);
        if (c->h_chain_desc) (void)hipHostFree(c->h_chain_desc);
        c->chain_desc = c->h_chain_desc = nullptr;
        c->chain_desc_bytes = 0;
        TD_HIP(c, hipMalloc(&c->chain_desc, bytes));
        TD_HIP(c, hipHostMalloc(&c->h_chain_desc, bytes, hipHostMallocDefault));
        c->chain_desc_bytes = bytes;
    }
    TD_HIP(c, hipStreamSynchronize(c->stream));  // the pinned staging may still feed a previous copy
    DevChain *hd = static_cast<DevChain *>(c->h_chain_desc);
    for (int64_t b = 0; b < nchains; ++b) hd[b] = chains[b]->dev;
    Timer *tm = c->timer.on ? &c->timer : nullptr;
    hipEvent_t t0 = tm ? tm->begin(c->stream) : nullptr;
    TD_HIP(c, hipMemcpyAsync(c->chain_desc, hd, bytes, hipMemcpyHostToDevice, c->stream));
    hipError_t e = chain_run(hd, static_cast<const DevChain *>(c->chain_desc), (int)nchains, iterations, c->stream,
                             nullptr, DrawsBuf{&c->draws, &c->draws_bytes}, c->num_cus);
    if (tm) tm->end("chain_run", t0, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_run launch (batch)");
    TD_HIP(c, hipStreamSynchronize(c->stream));  // every chain wrote its scalars to its st_host
    for (int64_t b = 0; b < nchains; ++b) {
        adopt_scalars(chains[b]);
        chains[b]->stats.iterations += iterations;
    }
    return TD_OK;
}

int td_chain_stats_get(const td_chain *ch, td_chain_stats *st) {
    if (!ch || !st) return TD_ERR_ARG;
    if (ch->rounds && ch->rounds->running) {  // the counts are the launch's until it returns
        int rc = rounds_stop(ch->rounds);
        if (rc) return rc;
    }
    *st = ch->stats;
    return TD_OK;
}

int td_chain_get_model(const td_chain *chc, double *xCell, double *yCell, double *zCell, double *zeta, int64_t cap,
                       int64_t *nCells, double *phi, double *ptS_out) {
    td_chain *ch = const_cast<td_chain *>(chc);
    if (!ch) return TD_ERR_ARG;
    td_ctx *c = ch->ctx;
    if (ch->engine == TD_ENGINE_DEVICE) {
        servers_quiesce(nullptr);
        int rc = device_pull_scalars(ch);
        if (rc) return rc;
        const int N = ch->st_host->ncells, cp = ch->dev.cap;
        std::vector<double> hc(4 * (size_t)cp);
        std::vector<int> order((size_t)std::max(N, 1));
        hipError_t e = hipMemcpy(hc.data(), ch->dev.cx, sizeof(double) * hc.size(), hipMemcpyDeviceToHost);
        if (e == hipSuccess && N > 0)
            e = hipMemcpy(order.data(), ch->dev.order, sizeof(int) * (size_t)N, hipMemcpyDeviceToHost);
        if (e == hipSuccess && ptS_out && c->g.n)
            e = hipMemcpy(ch->ptS.data(), ch->dev.ptS, sizeof(double) * (size_t)c->g.n, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_err(c, e, "td_chain_get_model");
        ch->x.resize((size_t)N); ch->y.resize((size_t)N); ch->z.resize((size_t)N); ch->zeta.resize((size_t)N);
        for (int j = 0; j < N; ++j) {
            const int s = order[(size_t)j];
            ch->x[(size_t)j] = hc[(size_t)s];
            ch->y[(size_t)j] = hc[(size_t)cp + s];
            ch->z[(size_t)j] = hc[2 * (size_t)cp + s];
            ch->zeta[(size_t)j] = hc[3 * (size_t)cp + s];
        }
    }
    const int64_t N = (int64_t)ch->x.size();
    if (nCells) *nCells = N;
    if (phi) *phi = ch->phi;
    if (cap < N) return set_err(c, TD_ERR_ARG, "td_chain_get_model: capacity smaller than nCells");
    if (xCell) std::copy(ch->x.begin(), ch->x.end(), xCell);
    if (yCell) std::copy(ch->y.begin(), ch->y.end(), yCell);
    if (zCell) std::copy(ch->z.begin(), ch->z.end(), zCell);
    if (zeta) std::copy(ch->zeta.begin(), ch->zeta.end(), zeta);
    if (ptS_out) std::copy(ch->ptS.begin(), ch->ptS.end(), ptS_out);
    return TD_OK;
}

int td_chain_set_temperature(td_chain *ch, double temperature) {
    if (!ch || !(temperature > 0.0)) return chain_err(ch, TD_ERR_ARG, "td_chain_set_temperature: need T > 0");
    ch->prm.temperature = temperature;
    ch->P.temperature = temperature;
    tdchain::params_derived(ch->P);
    ch->dev.params = ch->P;
    ch->desc_dirty = true;
    return TD_OK;
}

}  // extern "C"

// ------------------------------------------------ td_evaluate's shadow ----
namespace tdstar {

int shadow_chain_create(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                        int64_t ncells, int64_t cap, const double box[6], td_chain **out) {
    *out = nullptr;
    td_chain_params p{};
    p.debug_prior = 0;
    p.sig = 10;
    p.zeta_scale = 50;
    p.max_cells = (int32_t)std::max<int64_t>(cap - 1, ncells);
    p.min_cells = 1;
    p.prior = 1;
    p.n_iter = p.burn_in = p.keep_each = 1.0;
    p.xmin = box[0]; p.xmax = box[1]; p.ymin = box[2]; p.ymax = box[3]; p.zmin = box[4]; p.zmax = box[5];
    p.temperature = 1.0;
    p.engine = TD_ENGINE_DEVICE;
    td_chain *ch = nullptr;
    int rc = td_chain_create(&ch, ctx, &p, x, y, z, zeta, ncells);
    if (rc) return rc;
    ch->dev.grid.sealed = 0;  // the caller's edits may put a cell anywhere: bounds from the faces only
    ch->desc_dirty = true;
    hipError_t e = hipHostMalloc(&ch->script_host, sizeof(double) * ((size_t)ctx->g.n + 2),
                                 hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&ch->script_dev), ch->script_host, 0);
    if (e == hipSuccess)
        e = hipHostMalloc(&ch->mb_host, sizeof(Mailbox), hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        std::memset(ch->mb_host, 0, sizeof(Mailbox));
        e = hipHostGetDevicePointer(reinterpret_cast<void **>(&ch->mb_dev), ch->mb_host, 0);
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ch->srv_stream, hipStreamNonBlocking);
    if (std::getenv("TD_SHADOW_PROFILE")) ch->dev.profile = 1;  // diagnostic phase stamps (tdt_shadow_profile)
    if (e != hipSuccess) {
        free_chain(ch);
        return hip_err(ctx, e, "hipHostMalloc(shadow output)");
    }
    *out = ch;
    return TD_OK;
}

int64_t shadow_chain_slots(const td_chain *ch) { return ch->dev.cap; }
int64_t shadow_chain_ncells(const td_chain *ch) { return ch->stats.ncells; }
double shadow_chain_phi(const td_chain *ch) { return ch->phi; }

// The kernel's report [phi, k, (ray, ptS) x k] (k = -1: the whole ptS
// follows) over the model's ptS `base` -> phi, the proposed model's ptS.
int64_t unpack_report(const double *buf, int64_t n, const double *base, double *ptS) {
    if (n == 0) return 0;
    const long long k = (long long)buf[1];
    if (k < 0) {
        std::memcpy(ptS, buf + 2, sizeof(double) * (size_t)n);
        return 0;
    }
    std::memcpy(ptS, base, sizeof(double) * (size_t)n);
    int64_t k0 = n;
    for (long long i = 0; i < k; ++i) {
        const int64_t r = (int64_t)buf[2 + 2 * i];
        ptS[(size_t)r] = buf[3 + 2 * i];
        k0 = std::min(k0, r);
    }
    return k0;
}

// Run 1..kMaxScript host-given steps in one k_chain_run launch; the step with
// decision 0 (the last) leaves [phi_n, ptS_n] in the pinned output.
int shadow_chain_script(td_chain *ch, const ScriptStep *steps, int nsteps, const double *base_ptS, int64_t *k0_out,
                        double *ptS_out) {
    td_ctx *c = ch->ctx;
    if (nsteps < 1 || nsteps > kMaxScript) return set_err(c, TD_ERR_ARG, "shadow script");
    ScriptArgs sa{};
    sa.n = nsteps;
    for (int k = 0; k < nsteps; ++k) sa.step[k] = steps[k];
    sa.out = ch->script_dev;
    Timer *tm = c->timer.on ? &c->timer : nullptr;
    hipEvent_t t0 = tm ? tm->begin(c->stream) : nullptr;
    hipError_t e = hipSuccess;
    if (ch->desc_dirty) {
        e = hipMemcpyAsync(ch->dev_ptr, &ch->dev, sizeof(DevChain), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) return hip_err(c, e, "shadow descriptor upload");
        ch->desc_dirty = false;
    }
    e = chain_run(&ch->dev, ch->dev_ptr, 1, nsteps, c->stream, &sa);
    if (tm) tm->end("chain_script", t0, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_run launch (script)");
    e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_run (script)");
    adopt_scalars(ch);
    if (steps[nsteps - 1].decision == 0) {
        *k0_out = unpack_report(ch->script_host, c->g.n, base_ptS, ptS_out);
    }
    return TD_OK;
}

int shadow_chain_query(td_chain *ch, double x, double y, double z, const ScriptStep *edit, double *val) {
    td_ctx *c = ch->ctx;
    hipError_t e = hipSuccess;
    if (ch->desc_dirty) {
        e = hipMemcpyAsync(ch->dev_ptr, &ch->dev, sizeof(DevChain), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) return hip_err(c, e, "shadow descriptor upload");
        ch->desc_dirty = false;
    }
    Timer *tm = c->timer.on ? &c->timer : nullptr;
    hipEvent_t t0 = tm ? tm->begin(c->stream) : nullptr;
    e = chain_query(ch->dev_ptr, x, y, z, edit, ch->script_dev, c->stream);
    if (tm) tm->end("chain_query", t0, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_query launch");
    e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "k_chain_query");
    *val = ch->script_host[0];
    return TD_OK;
}

void shadow_chain_destroy(td_chain *ch) { free_chain(ch); }

// Server mode.  Alive: running and used recently (the kernel's own watchdog is
// 200 ms of silence; past 100 ms the host stops it first, so no command races
// the watchdog); a stopped server leaves no proposal pending.
bool shadow_server_alive(td_chain *ch) {
    if (!ch->srv_running) return false;
    if (*vol(&ch->mb_host->exited) ||
        std::chrono::steady_clock::now() - ch->srv_last > std::chrono::milliseconds(100)) {
        (void)server_stop(ch);
        return false;
    }
    return true;
}

// Server mode, split so the caller can work while the device evaluates: post an evaluate command
// (its steps, the fate of the pending proposal), and later take its answer.  One command open at a time.
namespace {
int server_post_eval(td_chain *ch, int decision, const ScriptStep *steps, int nsteps, bool reissue) {
    if (nsteps < 1 || nsteps > kMaxScript || ch->post_open) return set_err(ch->ctx, TD_ERR_ARG, "server steps");
    int rc = server_start(ch);
    if (rc) return rc;
    if (!reissue && g_post_delay_ms.load() > 0)  // (testing: the host descheduled before its post)
        std::this_thread::sleep_for(std::chrono::milliseconds(g_post_delay_ms.load()));
    Mailbox *m = ch->mb_host;
    m->type = kCmdEval;
    m->decision = decision;
    m->nsteps = nsteps;
    for (int k = 0; k < nsteps; ++k) m->step[k] = ch->post_steps[k] = steps[k];
    ch->post_decision = decision;
    ch->post_nsteps = nsteps;
    ch->post_held = ch->srv_pending;
    ch->post_had = ch->srv_has_pending;
    ch->post_t0 = now_ns();
    ch->post_seq = m->seq + 1;
    post_seq(m, ch->post_seq);
    ch->post_open = true;
    return TD_OK;
}
}  // namespace

int shadow_server_post(td_chain *ch, int decision, const ScriptStep *steps, int nsteps) {
    return server_post_eval(ch, decision, steps, nsteps, false);
}

int shadow_server_answer(td_chain *ch, const double *base_ptS, int64_t *k0_out, double *ptS_out) {
    if (!ch->post_open) return set_err(ch->ctx, TD_ERR_ARG, "server: no command posted");
    ch->post_open = false;
    int rc = server_wait(ch, ch->post_seq);
    ch->ctx->dropin_ns[2] += now_ns() - ch->post_t0;
    if (rc == kExitedEarly) {
        // the kernel undid its pending proposal and never read this command: a fresh launch gets it
        // again, preceded by that proposal as a committed step if the caller accepted it
        ScriptStep st[kMaxScript];
        int nsteps = ch->post_nsteps;
        for (int k = 0; k < nsteps; ++k) st[k] = ch->post_steps[k];
        if (ch->post_decision == 1 && ch->post_had) {
            if (nsteps + 1 > kMaxScript) return set_err(ch->ctx, TD_ERR_HIP, "chain server: lost a pending commit");
            for (int k = nsteps; k > 0; --k) st[k] = st[k - 1];
            st[0] = ch->post_held;
            st[0].decision = 1;
            ++nsteps;
        }
        rc = server_post_eval(ch, 0, st, nsteps, true);  // (nothing pending on the new launch)
        if (rc) return rc;
        ch->post_open = false;
        rc = server_wait(ch, ch->post_seq);
        ch->ctx->dropin_ns[2] += now_ns() - ch->post_t0;
        if (rc == kExitedEarly) return set_err(ch->ctx, TD_ERR_HIP, "chain server returned before answering twice");
    }
    if (rc) return rc;
    ch->ctx->dropin_ns[16] += 10 * *vol(&ch->mb_host->diag[1]);  // (100 MHz ticks)
    ch->srv_pending = ch->post_steps[ch->post_nsteps - 1];
    ch->srv_has_pending = ch->srv_pending.decision == kDecideLater;
    ch->pq_expect = ch->srv_has_pending && ch->srv_pending.action == 2 ? ch->post_seq : -1;
    *k0_out = unpack_report(ch->script_host, ch->ctx->g.n, base_ptS, ptS_out);
    return TD_OK;
}

// The pending death's Interpolation at its killed site (x, y, z), answered by the kernel right after the
// evaluate (no command, no round trip): 1 and *val, or 0 (another point, nothing pending, no server).
int shadow_server_death_query(td_chain *ch, double x, double y, double z, double *val) {
    if (!ch->srv_running || ch->post_open || ch->pq_expect < 0 || !ch->srv_has_pending) return 0;
    const ScriptStep &st = ch->srv_pending;
    auto same = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; };
    if (st.action != 2 || !same(st.old[0], x) || !same(st.old[1], y) || !same(st.old[2], z)) return 0;
    Mailbox *m = ch->mb_host;
    const int64_t t0 = now_ns();
    for (long long spin = 0; *vol(&m->pq_seq) != ch->pq_expect; ++spin)
        if (*vol(&m->exited) || ((spin & 1023) == 1023 && now_ns() - t0 > 100000000)) return 0;  // (100 ms)
    std::atomic_thread_fence(std::memory_order_acquire);
    *val = *static_cast<volatile double *>(&m->pq_val);
    ch->ctx->dropin_ns[5] += now_ns() - t0;
    return 1;
}

int shadow_server_eval(td_chain *ch, int decision, const ScriptStep *steps, int nsteps, const double *base_ptS,
                       int64_t *k0_out, double *ptS_out) {
    const int rc = shadow_server_post(ch, decision, steps, nsteps);
    if (rc) return rc;
    return shadow_server_answer(ch, base_ptS, k0_out, ptS_out);
}

// One-point query, split like the evaluate: post, then the answer (the caller classifies meanwhile).
int shadow_server_query_post(td_chain *ch, double x, double y, double z, const ScriptStep *edit) {
    if (ch->post_open) return set_err(ch->ctx, TD_ERR_ARG, "server: a command is open");
    int rc = server_start(ch);
    if (rc) return rc;
    if (g_post_delay_ms.load() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(g_post_delay_ms.load()));
    Mailbox *m = ch->mb_host;
    m->type = kCmdQuery;
    m->q[0] = x;
    m->q[1] = y;
    m->q[2] = z;
    m->has_edit = edit ? 1 : 0;
    if (edit) m->qedit = *edit;
    ch->post_held = edit ? *edit : ScriptStep{};
    ch->post_had = edit != nullptr;
    ch->post_t0 = now_ns();
    ch->post_seq = m->seq + 1;
    post_seq(m, ch->post_seq);
    ch->post_open = true;
    return TD_OK;
}

int shadow_server_query_answer(td_chain *ch, double *val) {
    if (!ch->post_open) return set_err(ch->ctx, TD_ERR_ARG, "server: no query posted");
    ch->post_open = false;
    int rc = server_wait(ch, ch->post_seq);
    ch->ctx->dropin_ns[5] += now_ns() - ch->post_t0;
    if (rc == TD_OK) ch->ctx->dropin_ns[17] += 10 * *vol(&ch->mb_host->diag[1]);
    // the kernel had returned (its pending proposal undone: the caller sees the server
    // stopped and re-issues that proposal's commit): answer with a one-off launch
    const Mailbox *m = ch->mb_host;
    if (rc == kExitedEarly) return shadow_chain_query(ch, m->q[0], m->q[1], m->q[2], ch->post_had ? &ch->post_held : nullptr, val);
    if (rc) return rc;
    *val = m->qval;
    return TD_OK;
}

int shadow_server_query(td_chain *ch, double x, double y, double z, const ScriptStep *edit, double *val) {
    const int rc = shadow_server_query_post(ch, x, y, z, edit);
    if (rc) return rc;
    return shadow_server_query_answer(ch, val);
}

int shadow_server_stop(td_chain *ch) { return server_stop(ch); }

int shadow_profile(td_chain *ch, int64_t out[80]) {
    int rc = server_stop(ch);
    if (rc) return rc;
    return tdt_chain_profile(ch, 1, out);
}

void shadow_server_diag(const td_chain *ch, int64_t out[4]) {
    for (int k = 0; k < 4; ++k) out[k] = ch->mb_host ? ch->mb_host->diag[k] : 0;
}

}  // namespace tdstar

extern "C" {

// --------------------------------------------------------- testing hooks ----
void tdt_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    const tdchain::U4 r = tdchain::philox(tdchain::U4{ctr[0], ctr[1], ctr[2], ctr[3]}, key[0], key[1]);
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}
double tdt_det_log(double x) { return tdchain::det_log(x); }
double tdt_det_exp(double x) { return tdchain::det_exp(x); }
double tdt_normal_quantile(double p) { return tdchain::normal_quantile(p); }
void tdt_draws(uint64_t seed, uint32_t chain, uint64_t iter, double out[7]) {
    const tdchain::Draws d = tdchain::draw_iteration(seed, chain, iter);
    const double v[7] = {d.u_action, d.u_accept, d.u_a, d.u_b, d.u_c, d.u_zeta, d.u_index};
    std::memcpy(out, v, sizeof v);
}
int tdt_propose(const td_chain_params *prm, uint64_t iter, int64_t ncells, const double *cx, const double *cy,
                const double *cz, const double *czeta, double czeta_birth, double out[8]) {
    const tdchain::Params P = make_params(*prm);
    const tdchain::Draws d = tdchain::draw_iteration(prm->seed, (uint32_t)prm->chain, iter);
    tdchain::Proposal p = tdchain::propose(P, d, ncells);
    if (p.active && p.action != tdchain::kBirth) {
        const size_t k = (size_t)p.index;
        tdchain::complete_proposal(P, d, p, cx[k], cy[k], cz[k], czeta[k]);
    } else if (p.active) {
        tdchain::birth_zeta(P, p, czeta_birth);
    }
    const double v[8] = {(double)p.action, (double)p.active, (double)p.valid, (double)p.index, p.x, p.y, p.z, p.zeta};
    std::memcpy(out, v, sizeof v);
    return 0;
}
int tdt_dropin_timing(td_ctx *ctx, int reset, int64_t out[18]) {
    if (!ctx) return TD_ERR_ARG;
    if (out)
        for (int k = 0; k < 18; ++k) out[k] = ctx->dropin_ns[k];
    if (reset)
        for (int64_t &v : ctx->dropin_ns) v = 0;
    return TD_OK;
}
int tdt_rounds_force_exit(td_rounds *r, const int32_t *slots, int64_t nslots) {
    if (!r || nslots < 0 || (nslots > 0 && !slots)) return TD_ERR_ARG;
    const int nc = (int)r->chains.size();
    std::vector<char> f((size_t)nc, 0);
    for (int64_t i = 0; i < nslots; ++i) {
        if (slots[i] < 0 || slots[i] >= nc) return TD_ERR_ARG;
        f[(size_t)slots[i]] = 1;
    }
    // takes effect at the next launch: end the running one (states are consistent between rounds)
    const int rc = rounds_stop(r);
    if (rc) return rc;
    r->force_exit = nslots > 0 ? f : std::vector<char>();
    return TD_OK;
}
int tdt_set_server_post_delay(int ms) {
    if (ms < 0) return TD_ERR_ARG;
    g_post_delay_ms.store(ms);
    return TD_OK;
}
int tdt_chain_set_lds_mode(td_chain *ch, int mode) {
    if (!ch || ch->engine != TD_ENGINE_DEVICE || mode < 0 || mode > 3) return TD_ERR_ARG;
    ch->dev.lds_mode = mode;
    ch->desc_dirty = true;
    return TD_OK;
}

int tdt_chain_set_exact_every(td_chain *ch, int k) {
    if (!ch || ch->engine != TD_ENGINE_DEVICE || k < 0) return TD_ERR_ARG;
    ch->dev.exact_every = k;
    ch->desc_dirty = true;
    return TD_OK;
}

int tdt_chain_lds(td_chain *ch, int64_t out[4]) {
    if (!ch || ch->engine != TD_ENGINE_DEVICE || !out) return TD_ERR_ARG;
    chain_lds_sizes(ch->dev, out);
    return TD_OK;
}

int tdt_chain_query_lat(td_chain *ch, const double *pts, int nq, int mode, int64_t out[4]) {
    if (!ch || ch->engine != TD_ENGINE_DEVICE || !pts || nq < 1 || !out) return TD_ERR_ARG;
    td_ctx *c = ch->ctx;
    double *dp = nullptr;
    long long *dout = nullptr;
    hipError_t e = hipMalloc((void **)&dp, sizeof(double) * 3 * (size_t)nq);
    if (e == hipSuccess) e = hipMalloc((void **)&dout, sizeof(long long) * 4);
    if (e == hipSuccess) e = hipMemcpy(dp, pts, sizeof(double) * 3 * (size_t)nq, hipMemcpyHostToDevice);
    if (e == hipSuccess && ch->desc_dirty) {
        e = hipMemcpy(ch->dev_ptr, &ch->dev, sizeof(DevChain), hipMemcpyHostToDevice);
        ch->desc_dirty = false;
    }
    if (e == hipSuccess) e = test_query_lat(ch->dev_ptr, dp, nq, mode, dout, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    long long h[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
    if (dp) (void)hipFree(dp);
    if (dout) (void)hipFree(dout);
    if (e != hipSuccess) return hip_err(c, e, "tdt_chain_query_lat");
    for (int k = 0; k < 4; ++k) out[k] = h[k];
    return TD_OK;
}

int tdt_tile_filter(const float *lo, const float *hi, const double *maxd, int nt, const double *queries, int nq,
                    int mode, uint8_t *hit) {
    if (!lo || !hi || !maxd || !queries || !hit || nt < 1 || nq < 1 || (mode != 0 && mode != 1)) return TD_ERR_ARG;
    float *dlo = nullptr, *dhi = nullptr;
    double *dm = nullptr, *dq = nullptr;
    unsigned char *dh = nullptr;
    const size_t T = (size_t)nt, Q = (size_t)nq;
    hipError_t e = hipMalloc((void **)&dlo, sizeof(float) * 3 * T);
    if (e == hipSuccess) e = hipMalloc((void **)&dhi, sizeof(float) * 3 * T);
    if (e == hipSuccess) e = hipMalloc((void **)&dm, sizeof(double) * T);
    if (e == hipSuccess) e = hipMalloc((void **)&dq, sizeof(double) * 3 * Q);
    if (e == hipSuccess) e = hipMalloc((void **)&dh, T * Q);
    if (e == hipSuccess) e = hipMemcpy(dlo, lo, sizeof(float) * 3 * T, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dhi, hi, sizeof(float) * 3 * T, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dm, maxd, sizeof(double) * T, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dq, queries, sizeof(double) * 3 * Q, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = test_tile_filter(dlo, dhi, dm, nt, dq, nq, mode, dh, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(hit, dh, T * Q, hipMemcpyDeviceToHost);
    for (void *p : {(void *)dlo, (void *)dhi, (void *)dm, (void *)dq, (void *)dh})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return set_err(nullptr, TD_ERR_HIP, std::string("tdt_tile_filter: ") + hipGetErrorString(e));
    return TD_OK;
}

int tdt_chain_query_answers(td_chain *ch, const double *pts, int nq, int mode, double *dist, double *value,
                            int32_t *proven) {
    if (!ch || ch->engine != TD_ENGINE_DEVICE || !pts || nq < 1 || !dist || !value || !proven ||
        (mode != 0 && mode != 6))
        return TD_ERR_ARG;
    td_ctx *c = ch->ctx;
    double *dp = nullptr, *dd = nullptr, *dz = nullptr;
    int *dpr = nullptr;
    const size_t n = (size_t)nq;
    hipError_t e = hipMalloc((void **)&dp, sizeof(double) * 3 * n);
    if (e == hipSuccess) e = hipMalloc((void **)&dd, sizeof(double) * n);
    if (e == hipSuccess) e = hipMalloc((void **)&dz, sizeof(double) * n);
    if (e == hipSuccess) e = hipMalloc((void **)&dpr, sizeof(int) * n);
    if (e == hipSuccess) e = hipMemcpy(dp, pts, sizeof(double) * 3 * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && ch->desc_dirty) {
        e = hipMemcpy(ch->dev_ptr, &ch->dev, sizeof(DevChain), hipMemcpyHostToDevice);
        ch->desc_dirty = false;
    }
    if (e == hipSuccess) e = test_query_answers(ch->dev_ptr, dp, nq, mode, dd, dz, dpr, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(dist, dd, sizeof(double) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(value, dz, sizeof(double) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(proven, dpr, sizeof(int) * n, hipMemcpyDeviceToHost);
    for (void *q : {(void *)dp, (void *)dd, (void *)dz, (void *)dpr})
        if (q) (void)hipFree(q);
    if (e != hipSuccess) return hip_err(c, e, "tdt_chain_query_answers");
    return TD_OK;
}

int tdt_chain_profile(td_chain *ch, int enable, int64_t out[80]) {
    if (!ch || ch->engine != TD_ENGINE_DEVICE) return TD_ERR_ARG;
    ch->dev.profile = enable;
    ch->desc_dirty = true;
    if (out) {
        ChainScalars s{};
        hipError_t e = hipMemcpy(&s, ch->st_dev, sizeof s, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_err(ch->ctx, e, "tdt_chain_profile");
        std::memcpy(out, s.prof, sizeof s.prof);
    }
    return TD_OK;
}
int tdt_accept(const td_chain_params *prm, int action, double u_accept, double zeta_new, int64_t ncells, double phi,
               double phi_n, double czeta, double zeta_killed, double zetanew_death) {
    const tdchain::Params P = make_params(*prm);
    tdchain::Proposal p{};
    p.action = action;
    p.active = 1;
    p.valid = 1;
    p.u_accept = u_accept;
    p.zeta = zeta_new;
    if (action == tdchain::kBirth || action == tdchain::kChange) p.valid = tdchain::prior_valid(P, zeta_new);
    p.log_u = u_accept > 0.0 ? tdchain::det_log(u_accept) : -HUGE_VAL;
    double lnN[3];
    tdchain::log_window(lnN, ncells);
    return tdchain::accept(P, p, phi, phi_n, czeta, zeta_killed, zetanew_death, lnN) ? 1 : 0;
}

// The device's decision pre-filter (chain_logic.h decide_sure) on the bracket [phi_lo, phi_hi] x
// [phin_lo, phin_hi]: 1 (accept everywhere), -1 (reject everywhere) or 0 (undecided).
int tdt_decide_sure(const td_chain_params *prm, int action, double u_accept, double zeta_new, int64_t ncells,
                    double phi_lo, double phi_hi, double phin_lo, double phin_hi, double czeta, double zeta_killed,
                    double zetanew_death) {
    const tdchain::Params P = make_params(*prm);
    tdchain::Proposal p{};
    p.action = action;
    p.active = 1;
    p.valid = 1;
    p.u_accept = u_accept;
    p.zeta = zeta_new;
    if (action == tdchain::kBirth || action == tdchain::kChange) p.valid = tdchain::prior_valid(P, zeta_new);
    p.log_u = u_accept > 0.0 ? tdchain::det_log(u_accept) : -HUGE_VAL;
    double lnN[3];
    tdchain::log_window(lnN, ncells);
    const tdchain::AlphaParts a = tdchain::alpha_parts(P, p, czeta, zeta_killed, zetanew_death, lnN);
    return tdchain::decide_sure(a, p.log_u, (phi_lo - phin_hi) * P.inv_2t, (phi_hi - phin_lo) * P.inv_2t);
}


}  // extern "C"
