// incremental.cpp -- td_evaluate's incremental path: the drop-in boundary
// running the device chain's algorithm for an UNCHANGED Julia host.
//
// The reference's chain (TD_inversion_function.jl:70-274) calls evaluate on
// modeln = deepcopy(model) plus ONE edit: append! (birth, :85-88),
// deleteat! (death, :132-135), a new zeta (change, :189) or a new site (move,
// :234-236); if it accepts, the next modeln is an edit of this one, else of
// the previous model.  So every call's cells are one edit away from either the
// last committed model B or the last evaluated proposal Q = B + e.  The
// context keeps a "shadow" device chain holding B (per-point nearest cell,
// tiles, ray sums, chi^2 prefix sums -- chain_dev.h) and evaluates each
// recognised edit incrementally in one k_chain_run launch (scripted steps,
// no draws): when the new cells are an edit of Q, e is committed first (Julia
// accepted it), then the new edit is evaluated and undone.  The result is
// bit-identical to the full evaluate (the same invariant as the device chain,
// tests/test_gpu_incremental.py).  Anything else -- the first call, unrelated
// models, several edits at once, cells outside a sane range, nearest indices
// requested -- takes the full evaluate, and a shadow is built from a model
// only once the next call turns out to be an edit of it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "chain_dev.h"
#include "ctx.h"
#include "host_nn.h"

namespace tdstar {

struct Cells {
    std::vector<double> x, y, z, zeta;
    int64_t size() const { return (int64_t)x.size(); }
    void assign(const double *a, const double *b, const double *c, const double *d, int64_t n) {
        x.assign(a, a + n);
        y.assign(b, b + n);
        z.assign(c, c + n);
        zeta.assign(d, d + n);
    }
    void apply(const ScriptStep &e) {
        const size_t k = (size_t)e.index;
        switch (e.action) {
            case 1: x.push_back(e.x); y.push_back(e.y); z.push_back(e.z); zeta.push_back(e.zeta); break;
            case 2:
                x.erase(x.begin() + (long)k); y.erase(y.begin() + (long)k);
                z.erase(z.begin() + (long)k); zeta.erase(zeta.begin() + (long)k);
                break;
            case 3: zeta[k] = e.zeta; break;
            default: x[k] = e.x; y[k] = e.y; z[k] = e.z; break;
        }
    }
};

struct td_shadow {
    td_chain *ch = nullptr;
    Cells B;                 // committed model (Julia order), what the shadow chain holds
    HostNN nn;               // B's cells in a host bucket grid: one-point Interpolation queries (host_nn.h)
    double phiB = 0.0;
    std::vector<double> ptSB;
    std::vector<double> preB;  // B's chi^2 partial sums (MCsub.jl:169-172): phi_n is formed here, from them
    bool pending = false;    // Q = B + e evaluated (undone on the device, or held there undecided: dev_pending)
    bool dev_pending = false;  // server mode: the resident kernel holds e's overlay, awaiting its fate
    ScriptStep e{};
    double phiQ = 0.0;
    std::vector<double> ptSQ;
    std::vector<double> preQ;
    int64_t built_n = 0;     // cells when the shadow's bucket grid was sized
    // the last fully evaluated model, a shadow candidate
    bool have_last = false;
    Cells last;
    double last_phi = 0.0;
    std::vector<double> last_ptS;
};

namespace {

constexpr double kSane = 1e6;  // |coordinate| bound for the shadow (distances stay far below the 1e9 sentinel)

bool sane(double v) { return std::isfinite(v) && std::fabs(v) <= kSane; }

bool bits_eq(const double *a, const double *b, int64_t n) {
    return n <= 0 || std::memcmp(a, b, sizeof(double) * (size_t)n) == 0;
}

// phi of ptS (MCsub.jl:169-172: C = 0, then C += ((ptS - tS)^2 * 1.0) / sig^2 in ray order), the
// sequential sum resumed at ray k0 from the partial sums `pre` of a model whose t* agree with ptS below
// k0 -- bit for bit the full sum (host_chi2), in O(n - k0).  `out` receives ptS's own partial sums.
double chi2_resume(const td_ctx *ctx, const double *ptS, int64_t k0, const std::vector<double> &pre,
                   std::vector<double> &out) {
    const int64_t n = ctx->g.n;
    const double *tS = ctx->tS_host.data(), *sig = ctx->sig_host.data();
    out.resize((size_t)n);
    k0 = std::max<int64_t>(0, std::min(k0, n));
    if ((int64_t)pre.size() != n) k0 = 0;
    double C = k0 > 0 ? pre[(size_t)k0 - 1] : 0.0;
    if (k0 > 0 && &out != &pre) std::memcpy(out.data(), pre.data(), sizeof(double) * (size_t)k0);
    for (int64_t k = k0; k < n; ++k) {
        const double d = ptS[k] - tS[k];
        C = C + ((d * d) * 1.0) / (sig[k] * sig[k]);
        out[(size_t)k] = C;
    }
    return C;
}

// A model as the committed cells B plus at most one edit e (e.action 0: B
// itself), read without materialising it: the proposal Q = B + e costs no copy.
struct View {
    const Cells &B;
    ScriptStep e;
    double edited[4];  // the edited cell (change / move / birth), field by field
    View(const Cells &b, const ScriptStep *ed) : B(b), e{} {
        if (ed) e = *ed;
        if (e.action == 3 || e.action == 4) {
            const size_t k = (size_t)e.index;
            edited[0] = e.action == 4 ? e.x : B.x[k];
            edited[1] = e.action == 4 ? e.y : B.y[k];
            edited[2] = e.action == 4 ? e.z : B.z[k];
            edited[3] = e.action == 3 ? e.zeta : B.zeta[k];
        } else if (e.action == 1) {
            edited[0] = e.x, edited[1] = e.y, edited[2] = e.z, edited[3] = e.zeta;
        }
    }
    const double *arr(int a) const { return a == 0 ? B.x.data() : a == 1 ? B.y.data() : a == 2 ? B.z.data() : B.zeta.data(); }
    int64_t size() const { return B.size() + (e.action == 1 ? 1 : e.action == 2 ? -1 : 0); }
    // the contiguous run of field a from position j: pointer and length
    const double *run(int a, int64_t j, int64_t *len) const {
        const int64_t N = B.size(), k = e.index;
        switch (e.action) {
            case 1:
                if (j < N) { *len = N - j; return arr(a) + j; }
                *len = 1; return &edited[a];
            case 2:
                if (j < k) { *len = k - j; return arr(a) + j; }
                *len = N - 1 - j; return arr(a) + j + 1;
            case 3:
            case 4:
                if (j < k) { *len = k - j; return arr(a) + j; }
                if (j == k) { *len = 1; return &edited[a]; }
                *len = N - j; return arr(a) + j;
            default:
                *len = N - j; return arr(a) + j;
        }
    }
};

// in[0..len) == field a of v at [off, off + len)?
bool range_eq(const double *in, int a, int64_t off, int64_t len, const View &v) {
    while (len > 0) {
        int64_t r;
        const double *p = v.run(a, off, &r);
        r = std::min(r, len);
        if (!bits_eq(in, p, r)) return false;
        in += r, off += r, len -= r;
    }
    return true;
}

// first position where (x, y, z, zeta) differ bit-wise, up to lim
int64_t common_prefix(const double *const in[4], const View &v, int64_t lim) {
    for (int a = 0; a < 4; ++a) {
        int64_t k = 0;
        while (k < lim) {
            int64_t r;
            const double *p = v.run(a, k, &r);
            r = std::min(r, lim - k);
            int64_t j = 0;
            constexpr int64_t kBlk = 64;
            while (j + kBlk <= r && bits_eq(in[a] + k + j, p + j, kBlk)) j += kBlk;
            while (j < r && std::memcmp(in[a] + k + j, p + j, sizeof(double)) == 0) ++j;
            k += j;
            if (j < r) break;
        }
        lim = k;
    }
    return lim;
}

// O(1) guess whether `in` (M cells) descends from Q = B + e rather than from B:
// it holds e's mark where e left it (the appended cell at N, the cell after the
// killed one at k, the new value or site at k).  Only an order for the two
// classify scans (each reads the whole model): whichever base matches, the
// model evaluated is `in`, exactly.
bool looks_like_q(const double *const in[4], int64_t M, const Cells &B, const ScriptStep &e) {
    const int64_t N = B.size(), k = e.index;
    auto eq = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; };
    switch (e.action) {
        case 1:  // birth: Q has N + 1 cells, the new one last
            return M >= N + 1 && eq(in[0][N], e.x) && eq(in[1][N], e.y) && eq(in[2][N], e.z);
        case 2:  // death of k: Q[k] = B[k + 1]
            return k + 1 < N && k < M && !(eq(in[0][k], B.x[(size_t)k]) && eq(in[1][k], B.y[(size_t)k])) &&
                   eq(in[0][k], B.x[(size_t)k + 1]) && eq(in[1][k], B.y[(size_t)k + 1]);
        case 3:  // change of k
            return k < M && eq(in[3][k], e.zeta);
        case 4:  // move of k
            return k < M && eq(in[0][k], e.x) && eq(in[1][k], e.y) && eq(in[2][k], e.z);
        default:
            return false;
    }
}

// Whether `in` (M cells) is an edit of Q = B + e rather than of B, from e's mark where any one further
// edit leaves it (at its position, one lower after a death before it, or the whole count for a size
// change) -- every one-edit sequence of TD_inversion_function.jl, O(1).  Where both readings give the
// same model (a death of e's own cell, e's cell edited again) either base is right.
bool descends_from_q(const double *const in[4], int64_t M, const Cells &B, const ScriptStep &e) {
    const int64_t N = B.size(), k = e.index;
    auto eq = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; };
    auto cell_is = [&](int64_t i, double x, double y, double zeta) {  // in[i] has this site and value
        return i >= 0 && i < M && eq(in[0][i], x) && eq(in[1][i], y) && eq(in[3][i], zeta);
    };
    switch (e.action) {
        case 1:  // birth: Q has N + 1 cells, e's at N
            if (M == N + 2) return true;
            if (M == N - 1) return false;
            if (M == N + 1)  // Q changed / moved (its new cell keeps its site or its value), or B + a birth
                return (eq(in[0][N], e.x) && eq(in[1][N], e.y)) || eq(in[3][N], e.zeta);
            return M == N && cell_is(N - 1, e.x, e.y, e.zeta);  // Q less a cell before e's
        case 2: {  // death of k: Q[i] = B[i + 1] from k on, N - 1 cells
            if (M == N + 1) return false;
            if (M == N - 2) return true;
            const bool next_at_k = k + 1 < N && k < M && eq(in[0][k], B.x[(size_t)k + 1]) && eq(in[1][k], B.y[(size_t)k + 1]);
            if (M == N) return next_at_k;  // Q + a birth (B + a change / move keeps B[k] at k)
            // M == N - 1: Q changed / moved, or B less a cell (j < k puts B[k] at k - 1)
            const bool below = k == 0 || (eq(in[0][k - 1], B.x[(size_t)k - 1]) && eq(in[3][k - 1], B.zeta[(size_t)k - 1]));
            const bool at_k = k + 1 < N && k < M && (next_at_k || eq(in[3][k], B.zeta[(size_t)k + 1]));
            return below && at_k;
        }
        case 3:  // change of k: e.zeta at k, or at k - 1 after a death before it
            return (k < M && eq(in[3][k], e.zeta)) || (M == N - 1 && k >= 1 && eq(in[3][k - 1], e.zeta));
        case 4:  // move of k: e's site at k, or at k - 1 after a death before it
            return (k < M && eq(in[0][k], e.x) && eq(in[1][k], e.y)) ||
                   (M == N - 1 && k >= 1 && eq(in[0][k - 1], e.x) && eq(in[1][k - 1], e.y));
        default:
            return false;
    }
}

// The edit `in` (M cells) most likely makes to `v`, from its length and ONE field's first
// difference (x, else zeta): what classify finds when `in` is v plus one reference-shaped edit.
// Cheap (one array up to the edit), so the server can start on it while classify verifies.
// false: no guess (v itself, or a shape the probe does not cover).
bool probe_edit(const double *const in[4], int64_t M, const View &v, ScriptStep *e) {
    const int64_t N = v.size();
    std::memset(e, 0, sizeof *e);
    auto first_diff = [&](int a, int64_t lim) -> int64_t {
        int64_t k = 0;
        while (k < lim) {
            int64_t r;
            const double *p = v.run(a, k, &r);
            r = std::min(r, lim - k);
            int64_t j = 0;
            constexpr int64_t kBlk = 64;
            while (j + kBlk <= r && bits_eq(in[a] + k + j, p + j, kBlk)) j += kBlk;
            while (j < r && std::memcmp(in[a] + k + j, p + j, sizeof(double)) == 0) ++j;
            k += j;
            if (j < r) break;
        }
        return k;
    };
    auto at = [&](int a, int64_t j) {  // field a of v at position j
        int64_t r;
        return *v.run(a, j, &r);
    };
    auto same = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; };
    // O(1) spot checks of the guess (the last cell, the cells around the edit): they tell which of
    // two bases a model descends from; classify proves it
    if (M == N + 1) {  // birth: append! (:85-88)
        if (!sane(in[0][N]) || !sane(in[1][N]) || !sane(in[2][N]) || !std::isfinite(in[3][N])) return false;
        if (N > 0 && !(same(in[0][N - 1], at(0, N - 1)) && same(in[3][N - 1], at(3, N - 1)))) return false;
        e->action = 1;
        e->index = (int)N;
        e->x = in[0][N];
        e->y = in[1][N];
        e->z = in[2][N];
        e->zeta = in[3][N];
        return true;
    }
    if (M == N - 1 && M >= 1) {  // death: deleteat! (:132-135) where x first differs
        const int64_t p = first_diff(0, M);
        if (!same(in[0][M - 1], at(0, N - 1)) || !same(in[3][M - 1], at(3, N - 1))) return false;
        if (p < M && !(same(in[1][p], at(1, p + 1)) && same(in[3][p], at(3, p + 1)))) return false;
        e->action = 2;
        e->index = (int)p;
        return true;
    }
    if (M == N && N >= 1) {
        int64_t p = first_diff(0, N);
        if (p < N) {  // move (:234-236)
            if (!sane(in[0][p]) || !sane(in[1][p]) || !sane(in[2][p])) return false;
            if (!same(in[3][p], at(3, p))) return false;  // (a move keeps the value)
            if (p + 1 < N && !(same(in[0][N - 1], at(0, N - 1)) && same(in[3][N - 1], at(3, N - 1)))) return false;
            e->action = 4;
            e->index = (int)p;
            e->x = in[0][p];
            e->y = in[1][p];
            e->z = in[2][p];
            return true;
        }
        p = first_diff(3, N);
        if (p < N && std::isfinite(in[3][p])) {  // change (:189)
            if (p + 1 < N && !same(in[3][N - 1], at(3, N - 1))) return false;
            e->action = 3;
            e->index = (int)p;
            e->zeta = in[3][p];
            return true;
        }
    }
    return false;
}

// Is `in` (M cells) the model `base` plus one reference-shaped edit?  0:
// identical, 1: one edit (in *e, decision unset), -1: neither.
int classify(const double *const in[4], int64_t M, const View &base, ScriptStep *e) {
    const int64_t N = base.size();
    const int64_t p = common_prefix(in, base, std::min(M, N));
    std::memset(e, 0, sizeof *e);
    auto tail_eq = [&](int64_t from_in, int64_t from_base, int64_t t) {
        for (int a = 0; a < 4; ++a)
            if (!range_eq(in[a] + from_in, a, from_base, t, base)) return false;
        return true;
    };
    auto cell_eq = [&](int a, int64_t j) { return range_eq(in[a] + j, a, j, 1, base); };
    if (M == N) {
        if (p == N) return 0;
        if (!tail_eq(p + 1, p + 1, N - p - 1)) return -1;  // the rest must be unchanged
        const bool site = cell_eq(0, p) && cell_eq(1, p) && cell_eq(2, p);
        const bool val = cell_eq(3, p);
        e->index = (int)p;
        if (site && !val) {  // change (:189)
            if (!std::isfinite(in[3][p])) return -1;
            e->action = 3;
            e->zeta = in[3][p];
            return 1;
        }
        if (!site && val) {  // move (:234-236)
            if (!sane(in[0][p]) || !sane(in[1][p]) || !sane(in[2][p])) return -1;
            e->action = 4;
            e->x = in[0][p];
            e->y = in[1][p];
            e->z = in[2][p];
            return 1;
        }
        return -1;
    }
    if (M == N + 1 && p == N) {  // birth: append! (:85-88)
        if (!sane(in[0][N]) || !sane(in[1][N]) || !sane(in[2][N]) || !std::isfinite(in[3][N])) return -1;
        e->action = 1;
        e->index = (int)N;
        e->x = in[0][N];
        e->y = in[1][N];
        e->z = in[2][N];
        e->zeta = in[3][N];
        return 1;
    }
    if (M == N - 1 && M >= 1) {  // death: deleteat!(kill) (:132-135)
        if (!tail_eq(p, p + 1, M - p)) return -1;
        e->action = 2;
        e->index = (int)p;
        return 1;
    }
    return -1;
}

// The step as the device takes it: with the edited cell's values before it, read from `base`
// (the model the step applies to, the chain's model bit for bit).  The host's own copies of
// steps (td_shadow::e) keep them zero, as classify leaves them, so they compare as edits.
ScriptStep posted(ScriptStep e, const Cells &base) {
    if (e.action != 1) {
        const size_t k = (size_t)e.index;
        e.old[0] = base.x[k];
        e.old[1] = base.y[k];
        e.old[2] = base.z[k];
        e.old[3] = base.zeta[k];
    }
    return e;
}

bool all_sane(const double *const in[4], int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (!sane(in[0][i]) || !sane(in[1][i]) || !sane(in[2][i]) || !std::isfinite(in[3][i])) return false;
    return true;
}

// Julia went on from Q: the committed model takes the pending edit (host copy and host grid)
void commit_q(td_shadow *s) {
    s->B.apply(s->e);
    s->nn.apply(s->e);
}

// TD_HOST_QUERY=0: one-point queries go to the device server as before (A/B measurements)
bool host_query_on() {
    static const bool on = [] {
        const char *v = std::getenv("TD_HOST_QUERY");
        return !(v && v[0] == '0');
    }();
    return on;
}

void drop_chain(td_shadow *s) {
    if (s->ch) shadow_chain_destroy(s->ch);
    s->ch = nullptr;
    s->pending = false;
    s->dev_pending = false;
}

// Build the shadow chain from the last fully evaluated model.
int build_shadow(td_ctx *ctx, td_shadow *s) {
    drop_chain(s);
    const Cells &c = s->last;
    const int64_t n = c.size();
    double box[6] = {HUGE_VAL, -HUGE_VAL, HUGE_VAL, -HUGE_VAL, HUGE_VAL, -HUGE_VAL};
    const std::vector<double> *pts[3] = {&ctx->hx, &ctx->hy, &ctx->hz};
    const std::vector<double> *cel[3] = {&c.x, &c.y, &c.z};
    for (int a = 0; a < 3; ++a) {  // the cells' and the ray points' box: the bucket grid's extent
        for (double v : *pts[a]) box[2 * a] = std::min(box[2 * a], v), box[2 * a + 1] = std::max(box[2 * a + 1], v);
        for (double v : *cel[a]) box[2 * a] = std::min(box[2 * a], v), box[2 * a + 1] = std::max(box[2 * a + 1], v);
        if (!(box[2 * a] <= box[2 * a + 1])) box[2 * a] = box[2 * a + 1] = 0.0;
    }
    const int64_t cap = std::max<int64_t>(2 * n, n + 256);
    int rc = shadow_chain_create(ctx, c.x.data(), c.y.data(), c.z.data(), c.zeta.data(), n, cap, box, &s->ch);
    if (rc) return rc;
    s->B = c;
    s->nn.build(c.x.data(), c.y.data(), c.z.data(), c.zeta.data(), n);
    s->phiB = s->last_phi;
    s->ptSB = s->last_ptS;
    chi2_resume(ctx, s->ptSB.data(), 0, s->preB, s->preB);  // (== phiB: the same sequential sum)
    s->pending = false;
    s->built_n = n;
    return TD_OK;
}

}  // namespace

td_chain *shadow_chain_of(td_ctx *ctx) { return ctx->shadow ? ctx->shadow->ch : nullptr; }

void shadow_free(td_ctx *ctx) {
    if (!ctx->shadow) return;
    drop_chain(ctx->shadow);
    delete ctx->shadow;
    ctx->shadow = nullptr;
}

// td_evaluate without nearest indices (api.cpp); full = the plain evaluate.
int evaluate_incremental(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                         int64_t M, double *ptS_out, double *phi_out) {
    if (!ctx->shadow) ctx->shadow = new td_shadow();
    td_shadow *s = ctx->shadow;
    const int64_t n = ctx->g.n;
    const double *in[4] = {x, y, z, zeta};
    auto out = [&](double phi, const std::vector<double> &ptS) -> int {
        if (phi_out) *phi_out = phi;
        if (ptS_out && n) std::memcpy(ptS_out, ptS.data(), sizeof(double) * (size_t)n);
        return TD_OK;
    };
    auto full = [&]() -> int {  // the plain evaluate; its model becomes the shadow candidate
        ctx->dropin_ns[8] += 1;
        drop_chain(s);
        s->have_last = false;
        s->last_ptS.assign((size_t)n, 0.0);
        int rc = evaluate_full(ctx, x, y, z, zeta, M, s->last_ptS.data(), &s->last_phi);
        if (rc) return rc;
        if (M >= 1 && n > 0 && all_sane(in, M)) {
            s->last.assign(x, y, z, zeta, M);
            s->have_last = true;
        }
        return out(s->last_phi, s->last_ptS);
    };
    if (!s->ch) {
        ScriptStep e;
        if (!s->have_last || classify(in, M, View(s->last, nullptr), &e) < 0) return full();
        int rc = build_shadow(ctx, s);  // the caller is walking a chain: follow it on the device
        if (rc) return rc;
    }
    // server mode (incremental == 2): one resident launch answers every call
    const bool srv = ctx->incremental == 2;
    if (s->dev_pending && !(srv && shadow_server_alive(s->ch))) s->dev_pending = false;  // stopped: undone
    if (srv) {
        // Optimistic: guess the base (Q where it holds Q's mark, else B) and the edit (probe_edit: one
        // array scan), post that step to the server at once, and verify it with the full classify while
        // the device evaluates.  The host state then is exactly what the checked path below would leave.
        // A wrong guess (never, for a reference-shaped host) drops the shadow: the full evaluate answers.
        const int64_t tp = now_ns();
        const bool on_q = s->pending && descends_from_q(in, M, s->B, s->e);
        ScriptStep g;
        const bool guessed = probe_edit(in, M, on_q ? View(s->B, &s->e) : View(s->B, nullptr), &g);
        if (guessed && (on_q || !s->pending || std::memcmp(&g, &s->e, sizeof g) != 0)) {
            ScriptStep steps[kMaxScript];
            int nsteps = 0, decision = 0;
            if (on_q) {  // Julia went on from Q: the device commits it first
                if (s->dev_pending) {
                    decision = 1;
                } else {
                    ScriptStep c = posted(s->e, s->B);
                    c.decision = 1;
                    steps[nsteps++] = c;
                }
                commit_q(s);
                s->phiB = s->phiQ;
                s->ptSB.swap(s->ptSQ);
                s->preB.swap(s->preQ);
            }
            s->pending = false;  // (not on Q: Q, if any, was rejected -- undone, decision 0)
            const int64_t after = s->B.size() + (g.action == 1 ? 1 : g.action == 2 ? -1 : 0);
            if (after + 1 > shadow_chain_slots(s->ch) || after > 4 * std::max<int64_t>(s->built_n, 64)) {
                s->last = s->B;  // rebuilt from B (a pending commit step is then moot)
                s->last_phi = s->phiB;
                s->last_ptS = s->ptSB;
                s->have_last = true;
                int rc = build_shadow(ctx, s);
                if (rc) return rc;
                nsteps = 0;
            }
            ctx->dropin_ns[1] += now_ns() - tp;
            g.decision = kDecideLater;
            steps[nsteps++] = posted(g, s->B);
            g.decision = 0;
            int rc = shadow_server_post(s->ch, decision, steps, nsteps);
            ScriptStep v2;
            const int rv = rc ? -1 : classify(in, M, View(s->B, nullptr), &v2);  // (the device works meanwhile)
            s->ptSQ.resize((size_t)n);
            int64_t k0 = 0;
            if (!rc) rc = shadow_server_answer(s->ch, s->ptSB.data(), &k0, s->ptSQ.data());
            if (!rc) s->phiQ = chi2_resume(ctx, s->ptSQ.data(), k0, s->preB, s->preQ);
            if (rc || rv != 1 || std::memcmp(&v2, &g, sizeof g) != 0) {
                drop_chain(s);
                s->have_last = false;
                return rc ? rc : full();
            }
            s->e = g;
            s->pending = true;
            s->dev_pending = true;
            return out(s->phiQ, s->ptSQ);
        }
    }
    // which state is the new model an edit of?
    const int64_t tc = now_ns();
    struct Lap {  // (the classification's time, however this call leaves)
        td_ctx *c;
        int64_t t;
        bool on = true;
        void stop() {
            if (on) c->dropin_ns[1] += now_ns() - t;
            on = false;
        }
        ~Lap() { stop(); }
    } lap{ctx, tc};
    ScriptStep e2;
    ScriptStep steps[kMaxScript];
    int nsteps = 0, decision = 0;  // decision: the fate of the device's pending proposal
    // an edit of Q when the O(1) probe says so (Julia accepted Q: ~57 % of calls), else of B;
    // the other base only when the first scan fails (one model scan per call, mostly)
    int rq = -2;  // -2: Q not tried yet
    if (s->pending && looks_like_q(in, M, s->B, s->e)) {
        rq = classify(in, M, View(s->B, &s->e), &e2);
        if (rq == 0) return out(s->phiQ, s->ptSQ);
    }
    const int rb = rq == 1 ? -1 : classify(in, M, View(s->B, nullptr), &e2);
    if (rb == 0) return out(s->phiB, s->ptSB);
    if (rb == 1 && s->pending && std::memcmp(&e2, &s->e, sizeof e2) == 0) return out(s->phiQ, s->ptSQ);  // == Q again
    if (rb == 1) {
        s->pending = false;  // Q (if any) was rejected: undone (decision 0)
    } else if (s->pending) {
        if (rq == -2 || rq == -1) {
            if (rq == -1) return full();  // neither base
            rq = classify(in, M, View(s->B, &s->e), &e2);
        }
        if (rq < 0) return full();
        if (rq == 0) return out(s->phiQ, s->ptSQ);
        if (s->dev_pending) {
            decision = 1;  // Julia went on from Q: the device commits its pending overlay
        } else {
            ScriptStep c = posted(s->e, s->B);
            c.decision = 1;  // re-evaluate and commit Q first
            steps[nsteps++] = c;
        }
        commit_q(s);  // B := Q (in place: O(1) but for a death's shift)
        s->phiB = s->phiQ;
        s->ptSB.swap(s->ptSQ);
        s->preB.swap(s->preQ);
        s->pending = false;
    } else {
        return full();
    }
    // slots: a birth needs a free one; regrow (rebuild) when the chain is full or the
    // grid was sized for far fewer cells
    const int64_t after = s->B.size() + (e2.action == 1 ? 1 : e2.action == 2 ? -1 : 0);
    if (after + 1 > shadow_chain_slots(s->ch) || after > 4 * std::max<int64_t>(s->built_n, 64)) {
        s->last = s->B;  // rebuilt from B (a pending commit step is then moot)
        s->last_phi = s->phiB;
        s->last_ptS = s->ptSB;
        s->have_last = true;
        int rc = build_shadow(ctx, s);
        if (rc) return rc;
        nsteps = 0;
    }
    lap.stop();
    e2.decision = srv ? kDecideLater : 0;
    steps[nsteps++] = posted(e2, s->B);
    s->ptSQ.resize((size_t)n);
    int64_t k0 = 0;
    int rc = srv ? shadow_server_eval(s->ch, decision, steps, nsteps, s->ptSB.data(), &k0, s->ptSQ.data())
                 : shadow_chain_script(s->ch, steps, nsteps, s->ptSB.data(), &k0, s->ptSQ.data());
    if (!rc) s->phiQ = chi2_resume(ctx, s->ptSQ.data(), k0, s->preB, s->preQ);
    if (rc) {
        drop_chain(s);
        s->have_last = false;
        return rc;
    }
    e2.decision = 0;
    s->e = e2;
    s->pending = true;
    s->dev_pending = srv;
    return out(s->phiQ, s->ptSQ);
}

// td_interpolate of ONE point (the reference's birth / death queries,
// TD_inversion_function.jl:81,146) when the cells are the shadow's committed
// model or its pending proposal: answered on the device chain's bucket grid.
// Returns 1 (handled, *val set), 0 (not this context's model: caller takes the
// plain path) or an error status < 0 never (errors are returned as > 1 codes).
int interpolate_incremental(td_ctx *ctx, const double *x, const double *y, const double *z, const double *zeta,
                            int64_t M, double qx, double qy, double qz, double *val, int *handled) {
    *handled = 0;
    td_shadow *s = ctx->shadow;
    if (!s || !s->ch || !std::isfinite(qx) || !std::isfinite(qy) || !std::isfinite(qz)) return TD_OK;
    const double *in[4] = {x, y, z, zeta};
    ScriptStep e2;
    if (host_query_on()) {
        // the cells must be B or Q bit for bit (one scan); then the host grid answers (host_nn.h) and the
        // device -- its pending proposal untouched -- never sees the call
        const int64_t tc = now_ns();
        const int rb = classify(in, M, View(s->B, nullptr), &e2);
        const bool on_b = rb == 0, on_q = rb == 1 && s->pending && std::memcmp(&e2, &s->e, sizeof e2) == 0;
        ctx->dropin_ns[4] += now_ns() - tc;
        if (!on_b && !on_q) return TD_OK;  // another model: the plain path answers
        *val = s->nn.query(qx, qy, qz, on_q ? &s->e : nullptr);
        *handled = 1;
        return TD_OK;
    }
    if (s->dev_pending && !shadow_server_alive(s->ch)) s->dev_pending = false;
    if (shadow_server_alive(s->ch)) {
        // a running server: post the query on the model the cells most likely are (the pending proposal
        // where they hold its mark, else the committed one) and verify that while it is answered
        const bool on_q = s->pending && descends_from_q(in, M, s->B, s->e);
        if (on_q && s->dev_pending && s->e.action == 2) {
            // the death's query at its killed site (TD_inversion_function.jl:146): the kernel answered it
            // right after the evaluate; the cells are checked meanwhile
            const int rb = classify(in, M, View(s->B, nullptr), &e2);
            if (rb == 1 && std::memcmp(&e2, &s->e, sizeof e2) == 0 &&
                shadow_server_death_query(s->ch, qx, qy, qz, val)) {
                *handled = 1;
                return TD_OK;
            }
        }
        int rc = shadow_server_query_post(s->ch, qx, qy, qz, on_q ? &s->e : nullptr);
        if (rc) return rc;
        const int rb = classify(in, M, View(s->B, nullptr), &e2);  // (inside the round trip: not counted apart)
        rc = shadow_server_query_answer(s->ch, val);
        if (rc) return rc;
        const bool ok = on_q ? (rb == 1 && s->pending && std::memcmp(&e2, &s->e, sizeof e2) == 0) : rb == 0;
        *handled = ok ? 1 : 0;  // (a wrong guess: the plain path answers; nothing changed)
        return TD_OK;
    }
    const int64_t tc = now_ns();
    const int rb = classify(in, M, View(s->B, nullptr), &e2);
    ctx->dropin_ns[4] += now_ns() - tc;
    const ScriptStep *edit = nullptr;
    if (rb == 0) {
        edit = nullptr;  // the committed model
    } else if (rb == 1 && s->pending && std::memcmp(&e2, &s->e, sizeof e2) == 0) {
        edit = &s->e;  // the pending proposal (e.g. death's query on modeln, :146)
    } else {
        return TD_OK;
    }
    if (s->dev_pending && !shadow_server_alive(s->ch)) s->dev_pending = false;
    // a running server holds the state (its LDS mirrors are not written back): ask it
    int rc = shadow_server_alive(s->ch) ? shadow_server_query(s->ch, qx, qy, qz, edit, val)
                                        : shadow_chain_query(s->ch, qx, qy, qz, edit, val);
    if (rc) return rc;
    *handled = 1;
    return TD_OK;
}

}  // namespace tdstar

extern "C" int tdt_shadow_profile(td_ctx *ctx, int64_t out[80]) {
    if (!ctx || !out || !ctx->shadow || !ctx->shadow->ch) return TD_ERR_ARG;
    ctx->shadow->dev_pending = false;  // the server stops: its pending proposal is undone
    return tdstar::shadow_profile(ctx->shadow->ch, out);
}

extern "C" int tdt_shadow_diag(td_ctx *ctx, int64_t out[4]) {
    if (!ctx || !out) return TD_ERR_ARG;
    for (int k = 0; k < 4; ++k) out[k] = 0;
    if (ctx->shadow && ctx->shadow->ch) tdstar::shadow_server_diag(ctx->shadow->ch, out);
    return TD_OK;
}

extern "C" int tdt_host_nn_query(const double *x, const double *y, const double *z, const double *zeta, int64_t n,
                                 const double *edits, int64_t nedits, const double *pending, const double *qx,
                                 const double *qy, const double *qz, int64_t nq, double *val_out, int64_t *pos_out) {
    if (n < 0 || nedits < 0 || nq < 0 || (n > 0 && (!x || !y || !z || !zeta)) || (nedits > 0 && !edits) ||
        (nq > 0 && (!qx || !qy || !qz || !val_out)))
        return TD_ERR_ARG;
    auto step = [](const double *r) {
        tdstar::ScriptStep e{};
        e.action = (int)r[0];
        e.index = (int)r[1];
        e.x = r[2], e.y = r[3], e.z = r[4], e.zeta = r[5];
        return e;
    };
    tdstar::HostNN nn;
    nn.build(x, y, z, zeta, n);
    int64_t size = n;
    auto valid = [&](const tdstar::ScriptStep &e) {
        if (e.action < 1 || e.action > 4) return false;
        if (e.action != 1 && (e.index < 0 || e.index >= size)) return false;
        return !(e.action == 2 && size < 1);
    };
    for (int64_t k = 0; k < nedits; ++k) {
        const tdstar::ScriptStep e = step(edits + 6 * k);
        if (!valid(e)) return TD_ERR_ARG;
        nn.apply(e);
        size += e.action == 1 ? 1 : e.action == 2 ? -1 : 0;
    }
    tdstar::ScriptStep pe{};
    if (pending) {
        pe = step(pending);
        if (!valid(pe)) return TD_ERR_ARG;
    }
    for (int64_t k = 0; k < nq; ++k) {
        int64_t pos = -1;
        val_out[k] = nn.query(qx[k], qy[k], qz[k], pending ? &pe : nullptr, &pos);
        if (pos_out) pos_out[k] = pos;
    }
    return TD_OK;
}
