// eval_server.cpp -- host side of td_evaluate's resident full evaluate
// (eval_server.h; the kernel is k_eval_server in nn_grid.hip).
//
// evaluate_full (api.cpp) hands a grid-path evaluate here when no other
// resident launch of this thread is alive; this file posts it to the resident
// launch (starting one when none runs), waits for every workgroup's reply and
// leaves ptS in ctx->h_out + 1, where the launches would have put it.  A launch
// that quit on its own before taking the command is relaunched and takes it; a
// launch whose grid barrier failed turns the server off for the context (the
// launches answer from then on: *served = false).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "ctx.h"
#include "eval_server.h"

namespace tdstar {

struct EvalServer {
    bool running = false;
    bool disabled = false;  // a launch failed (or the geometry does not fit): the launches answer
    hipStream_t stream = nullptr;
    EvalCmd *mb = nullptr, *mb_dev = nullptr;      // pinned mailbox
    EvalCtl *ctl = nullptr, *ctl_dev = nullptr;    // pinned: what the host polls
    EvalStamps *stamps = nullptr, *stamps_dev = nullptr;  // pinned [nwg]: phase stamps (diag)
    void *dev = nullptr;                            // bcast | arrive | wg_ray | count[2][kGridMaxBuckets] | ent
    unsigned long long *bcast = nullptr;
    unsigned *arrive = nullptr;
    int *wg_ray = nullptr;
    int *count = nullptr;
    BucketEntry *ent = nullptr;
    int nwg = 0, lds_pts = 0;
    int par = 0;                  // the count set the next evaluate fills
    int64_t used[2] = {0, 0};     // buckets each set holds counts in (zeroed by the other's evaluate)
    long long seq = 0;            // the last seq posted
    long long idle_ticks = 2000000;   // 20 ms of the 100 MHz clock (tdt_eval_server_config)
    long long guard_ticks = 10000000; // 100 ms: a grid barrier that waits longer fails
    bool diag = false;            // phase stamps (tdt_eval_server_config mode 2)
    int64_t served = 0, launches = 0, failures = 0, busy_ns = 0, stamped = 0;
    int64_t search_ns[6] = {};  // diag: wave 0's first search round (see eval_server_run)
    int64_t phase_ns[10] = {};  // diag: summed over stamped evaluates, from workgroup 0's take to the
                                // LAST workgroup's EvalStamps::t[j]
};

namespace {

volatile long long *vol(long long *p) { return p; }

constexpr size_t kBcastBytes = sizeof(unsigned long long) * 64;
constexpr size_t kArriveBytes = sizeof(unsigned) * 16 * 32;  // 8 arrival shards, 8 finish shards

// Rays to workgroups: contiguous ranges with about P / nwg points each (the boundary nearer to each
// quantile), so that a workgroup sums the rays it searched.
std::vector<int> partition_rays(const std::vector<int> &off, int nwg, int *max_pts) {
    const int n = (int)off.size() - 1;
    const long long P = off.back();
    std::vector<int> r((size_t)nwg + 1, 0);
    r[(size_t)nwg] = n;
    for (int w = 1; w < nwg; ++w) {
        const long long q = P * w / nwg;
        int b = (int)(std::lower_bound(off.begin(), off.end(), (int)q) - off.begin());  // off[b] >= q
        if (b > 0 && q - off[(size_t)b - 1] < off[(size_t)b] - q) --b;
        r[(size_t)w] = std::min(std::max(b, r[(size_t)w - 1]), n);
    }
    int m = 1;
    for (int w = 0; w < nwg; ++w) m = std::max(m, off[(size_t)r[(size_t)w + 1]] - off[(size_t)r[(size_t)w]]);
    *max_pts = m;
    return r;
}

int setup(td_ctx *ctx, EvalServer *ev) {
    ev->nwg = std::max(1, ctx->num_cus);
    int mp = 1;
    const std::vector<int> wr = partition_rays(ctx->ray_off_host, ev->nwg, &mp);
    ev->lds_pts = mp;
    if (mp > kEvalMaxLdsPts) {  // a workgroup's share does not fit its LDS: the launches
        ev->disabled = true;
        return TD_OK;
    }
    TD_HIP(ctx, hipStreamCreateWithFlags(&ev->stream, hipStreamNonBlocking));
    TD_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&ev->mb), sizeof(EvalCmd),
                              hipHostMallocMapped | hipHostMallocCoherent));
    TD_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void **>(&ev->mb_dev), ev->mb, 0));
    TD_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&ev->ctl), sizeof(EvalCtl),
                              hipHostMallocMapped | hipHostMallocCoherent));
    TD_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void **>(&ev->ctl_dev), ev->ctl, 0));
    TD_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&ev->stamps), sizeof(EvalStamps) * (size_t)ev->nwg,
                              hipHostMallocMapped | hipHostMallocCoherent));
    TD_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void **>(&ev->stamps_dev), ev->stamps, 0));
    std::memset(ev->mb, 0, sizeof(EvalCmd));
    std::memset(ev->ctl, 0, sizeof(EvalCtl));
    std::memset(ev->stamps, 0, sizeof(EvalStamps) * (size_t)ev->nwg);
    const size_t wr_bytes = (sizeof(int) * ((size_t)ev->nwg + 1) + 255) & ~(size_t)255;
    const size_t cnt_bytes = sizeof(int) * 2 * (size_t)kGridMaxBuckets;
    const size_t ent_bytes = sizeof(BucketEntry) * (size_t)kGridMaxBuckets * kGridCap;
    TD_HIP(ctx, hipMalloc(&ev->dev, kBcastBytes + kArriveBytes + wr_bytes + cnt_bytes + ent_bytes));
    char *d = static_cast<char *>(ev->dev);
    ev->bcast = reinterpret_cast<unsigned long long *>(d);
    ev->arrive = reinterpret_cast<unsigned *>(d + kBcastBytes);
    ev->wg_ray = reinterpret_cast<int *>(d + kBcastBytes + kArriveBytes);
    ev->count = reinterpret_cast<int *>(d + kBcastBytes + kArriveBytes + wr_bytes);
    ev->ent = reinterpret_cast<BucketEntry *>(d + kBcastBytes + kArriveBytes + wr_bytes + cnt_bytes);
    TD_HIP(ctx, hipMemcpy(ev->wg_ray, wr.data(), sizeof(int) * wr.size(), hipMemcpyHostToDevice));
    TD_HIP(ctx, hipMemset(ev->count, 0, cnt_bytes));  // later evaluates zero the set they do not fill
    return TD_OK;
}

// start a launch; seq0 = the last seq it is not to run (a pending command is seq0 + 1)
int start(td_ctx *ctx, EvalServer *ev, long long seq0) {
    for (int j = 0; j < 8; ++j) ev->ctl->done[j] = seq0;
    ev->ctl->exited = 0;
    ev->ctl->failed = 0;
    std::atomic_thread_fence(std::memory_order_release);
    // a cleared broadcast (no stale tag) and arrival counters from zero: ordered before the launch
    TD_HIP(ctx, hipMemsetAsync(ev->bcast, 0, kBcastBytes + kArriveBytes, ev->stream));
    EvalArgs a{};
    a.mb = ev->mb_dev;
    a.ctl = ev->ctl_dev;
    a.stamps = ev->stamps_dev;
    a.bcast = ev->bcast;
    a.arrive = ev->arrive;
    a.count = ev->count;
    a.ent = ev->ent;
    a.wg_ray = ev->wg_ray;
    const Geometry &g = ctx->g;
    a.ray_off = g.ray_off;
    a.px = g.px;
    a.py = g.py;
    a.pz = g.pz;
    a.w = g.w;
    a.ptS = ctx->ptS;
    a.ptS_host = ctx->h_out_dev + 1;
    a.n = (int)g.n;
    a.nwg = ev->nwg;
    a.lds_pts = ev->lds_pts;
    a.seq0 = seq0;
    a.idle_ticks = ev->idle_ticks;
    a.guard_ticks = ev->guard_ticks;
    const hipError_t e = launch_eval_server(a, ev->stream);
    if (e != hipSuccess) return hip_err(ctx, e, "k_eval_server launch");
    ev->running = true;
    ev->launches += 1;
    resident_register_eval(ctx);
    return TD_OK;
}

// the launch has returned or is returning: wait for it
int join(td_ctx *ctx, EvalServer *ev) {
    const hipError_t e = hipStreamSynchronize(ev->stream);
    ev->running = false;
    resident_unregister_eval(ctx);
    if (e != hipSuccess) return hip_err(ctx, e, "k_eval_server exit");
    return TD_OK;
}

void post(EvalServer *ev, long long sq) {
    ev->mb->check = eval_check(ev->mb, sq);
    std::atomic_thread_fence(std::memory_order_release);
    *vol(&ev->mb->seq) = sq;
}

}  // namespace

int eval_server_run(td_ctx *ctx, int64_t ncells, const CellGrid &G, bool *served, int64_t *issue_ns) {
    *served = false;
    static const bool env_off = [] {  // TD_EVAL_SERVER=0: the launches (A/B)
        const char *v = std::getenv("TD_EVAL_SERVER");
        return v && std::atoi(v) == 0;
    }();
    if (!ctx->eval_server_mode || env_off) return TD_OK;
    EvalServer *ev = ctx->evs;
    if (!ev) {
        ev = ctx->evs = new EvalServer();
        if (ctx->eval_idle_us > 0) ev->idle_ticks = ctx->eval_idle_us * 100;
        if (ctx->eval_guard_us > 0) ev->guard_ticks = ctx->eval_guard_us * 100;
        ev->diag = ctx->eval_server_mode == 2;
        const int rc = setup(ctx, ev);
        if (rc) {
            ev->disabled = true;
            return rc;
        }
    }
    if (ev->disabled) return TD_OK;
    const int64_t t0 = now_ns();
    if (!ev->running) {
        const int rc = start(ctx, ev, ev->seq);
        if (rc) return rc;
    }
    const int par = ev->par;
    const int64_t nb = (int64_t)G.gx * G.gy * G.gz;
    EvalCmd *m = ev->mb;
    m->type = kEvalRun;
    m->ncells = (int)ncells;
    m->stride = (int)ctx->cell_stride;
    m->par = par;
    m->other_nb = (int)ev->used[par ^ 1];
    m->diag = ev->diag ? 1 : 0;
    m->cells = ctx->cells;
    m->stage = ctx->h_cells_dev;
    m->G = G;
    const long long sq = ++ev->seq;
    post(ev, sq);
    *issue_ns = now_ns() - t0;
    const auto tw = std::chrono::steady_clock::now();
    const int nsh = std::min(ev->nwg, 8);  // shards with workgroups
    EvalCtl *ct = ev->ctl;
    bool failed = false;
    for (long long spin = 0;; ++spin) {
        int j = 0;
        while (j < nsh && *vol(&ct->done[j]) == sq) ++j;
        if (j == nsh) break;
        if (*vol(&ct->failed) == sq) {
            failed = true;
            break;
        }
        if (*vol(&ct->exited)) {
            if (*vol(&ct->failed) == sq) {
                failed = true;
                break;
            }
            // quit on its own before taking sq (its watchdog): a new launch takes the pending command
            int rc = join(ctx, ev);
            if (rc) return rc;
            rc = start(ctx, ev, sq - 1);
            if (rc) return rc;
            continue;
        }
        if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - tw > std::chrono::seconds(5)) {
            ev->disabled = true;  // (the launch is left to its own watchdogs)
            return set_err(ctx, TD_ERR_HIP, "k_eval_server: no answer in 5 s");
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (failed) {  // a grid barrier timed out (a workgroup not resident): the launches from now on
        ev->failures += 1;
        ev->disabled = true;
        (void)join(ctx, ev);
        return TD_OK;
    }
    const long long t0d = ct->t_take;
    long long t_end = 0;
    for (int j = 0; j < nsh; ++j) t_end = std::max(t_end, ct->t_end[j]);
    ev->busy_ns += 10 * (t_end - t0d);  // (100 MHz ticks)
    if (ev->diag) {
        long long ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < ev->nwg; ++k)
            for (int j = 0; j < 10; ++j) ph[j] = std::max(ph[j], ev->stamps[k].t[j] - t0d);
        for (int j = 0; j < 10; ++j) ev->phase_ns[j] += 10 * ph[j];
        // wave 0's first search round, per workgroup: loads back, quads reduced, unproven points, most
        // entries in a bucket, unproven done -- summed over workgroups (the first three as durations)
        for (int k = 0; k < ev->nwg; ++k) {
            const long long *t = ev->stamps[k].t;
            ev->search_ns[0] += 10 * (t[10] - t[5]);
            ev->search_ns[1] += 10 * (t[11] - t[10]);
            ev->search_ns[2] += t[12];
            ev->search_ns[3] += t[13];
            ev->search_ns[4] += 10 * (t[14] - t[11]);
            ev->search_ns[5] += 10 * (t[6] - t[14]);
        }
        ev->stamped += 1;
    }
    ev->served += 1;
    ev->used[par ^ 1] = 0;
    ev->used[par] = nb;
    ev->par = par ^ 1;
    *served = true;
    return TD_OK;
}

int eval_server_stop(td_ctx *ctx) {
    EvalServer *ev = ctx ? ctx->evs : nullptr;
    if (!ev || !ev->running) return TD_OK;
    if (!*vol(&ev->ctl->exited)) {
        ev->mb->type = kEvalQuit;
        post(ev, ++ev->seq);
    }
    return join(ctx, ev);  // (QUIT, or its watchdog)
}

void eval_server_free(td_ctx *ctx) {
    EvalServer *ev = ctx ? ctx->evs : nullptr;
    if (!ev) return;
    (void)eval_server_stop(ctx);
    if (ev->dev) (void)hipFree(ev->dev);
    if (ev->mb) (void)hipHostFree(ev->mb);
    if (ev->ctl) (void)hipHostFree(ev->ctl);
    if (ev->stamps) (void)hipHostFree(ev->stamps);
    if (ev->stream) (void)hipStreamDestroy(ev->stream);
    delete ev;
    ctx->evs = nullptr;
}

}  // namespace tdstar

using namespace tdstar;

extern "C" {

int tdt_eval_server_config(td_ctx *ctx, int mode, int64_t idle_us, int64_t guard_us) {
    if (!ctx || mode < 0 || mode > 2) return TD_ERR_ARG;
    (void)eval_server_stop(ctx);
    ctx->eval_server_mode = mode;
    ctx->eval_idle_us = idle_us;
    ctx->eval_guard_us = guard_us;
    if (EvalServer *ev = ctx->evs) {
        if (idle_us > 0) ev->idle_ticks = idle_us * 100;
        if (guard_us > 0) ev->guard_ticks = guard_us * 100;
        ev->diag = mode == 2;
        if (mode) ev->disabled = ev->lds_pts > kEvalMaxLdsPts;
    }
    return TD_OK;
}

int tdt_eval_server_stats(td_ctx *ctx, int64_t out[20]) {
    if (!ctx || !out) return TD_ERR_ARG;
    const EvalServer *ev = ctx->evs;
    const int64_t v[8] = {ev ? ev->served : 0, ev ? ev->launches : 0, ev ? ev->failures : 0, ev ? ev->busy_ns : 0,
                          ev && ev->running ? 1 : 0, ev && ev->disabled ? 1 : 0, ev ? ev->nwg : 0,
                          ev ? ev->lds_pts : 0};
    std::memcpy(out, v, sizeof v);
    for (int j = 0; j < 10; ++j) out[8 + j] = ev ? ev->phase_ns[j] : 0;
    out[18] = ev ? ev->stamped : 0;
    out[19] = 0;
    return TD_OK;
}

// diagnostics: wave 0's first search round, summed over workgroups and stamped evaluates
int tdt_eval_server_search_diag(td_ctx *ctx, int64_t out[6]) {
    if (!ctx || !out) return TD_ERR_ARG;
    for (int j = 0; j < 6; ++j) out[j] = ctx->evs ? ctx->evs->search_ns[j] : 0;
    return TD_OK;
}

}  // extern "C"
