// host_nn.h -- v_nearest (MCsub.jl:247-263) of ONE point on the drop-in path's committed model,
// answered on the host.
//
// An unchanged Julia host calls Interpolation(model, site) once per birth (TD_inversion_function.jl:81)
// and once per death (:146) between its evaluates.  The model is the shadow's committed cells B, or B
// plus the pending edit e (Q); the host keeps B bit for bit anyway (incremental.cpp), so the one-point
// answer is a bucket-grid query over it here -- ~0.2 us -- where the device server needs a pinned-memory
// round trip (>= 2.8 us handshake, plus waiting out the previous step's phase F).  The device keeps every
// ray point x cell search (the evaluate, the chain); this is the proposal side's one point.
//
// The answer is v_nearest's exactly: the first cell in Julia order whose squared distance (left to right,
// (mx - x)^2 + (my - y)^2 + (mz - z)^2, no FMA: -ffp-contract=off) is the least below the 1e9 sentinel,
// i.e. the lexicographic minimum of (distance, position) over the cells with distance < 1e9; 0.0 if none.
// Julia position order is kept as a stamp per cell (append! takes a new largest stamp; deleteat! keeps
// the others' relative order), so a death shifts no index here.  The grid search stops only when every
// cell outside the scanned block of buckets is provably farther (strictly) than the best found.
// Tested against the C oracle on ties, duplicates, points far outside the cells' box and the sentinel
// (tests/test_host_nn.py, tdt_host_nn_query).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "chain_dev.h"

namespace tdstar {

class HostNN {
  public:
    static constexpr double kSentinel = 1e9;  // MCsub.jl:250

    void build(const double *x, const double *y, const double *z, const double *zeta, int64_t n) {
        cell_.clear();
        slot_of_.clear();
        free_.clear();
        next_stamp_ = 0;
        double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
        const double *c[3] = {x, y, z};
        for (int a = 0; a < 3; ++a) {
            if (n > 0) {
                lo[a] = hi[a] = c[a][0];
                for (int64_t i = 1; i < n; ++i) lo[a] = std::min(lo[a], c[a][i]), hi[a] = std::max(hi[a], c[a][i]);
            }
        }
        // ~2 cells per bucket, buckets about cubic; a flat axis gets one bucket
        const double target = std::max<double>(1.0, (double)n / 2.0);
        double vol = 1.0;
        int live = 0;
        for (int a = 0; a < 3; ++a)
            if (hi[a] - lo[a] > 0) vol *= hi[a] - lo[a], ++live;
        const double side = live ? std::pow(vol / target, 1.0 / live) : 1.0;
        for (int a = 0; a < 3; ++a) {
            const double s = hi[a] - lo[a];
            lo_[a] = lo[a];
            if (!(s > 0) || !(side > 0)) {
                nb_[a] = 1;
                inv_[a] = 0.0;
                h_[a] = 0.0;
                span_[a] = 0.0;
                continue;
            }
            nb_[a] = (int)std::min(128.0, std::max(1.0, std::round(s / side)));
            span_[a] = s;
            h_[a] = s / nb_[a];
            inv_[a] = nb_[a] / s;
        }
        bucket_.assign((size_t)nb_[0] * nb_[1] * nb_[2], {});
        cell_.reserve((size_t)(2 * n + 256));
        slot_of_.reserve((size_t)(2 * n + 256));
        for (int64_t i = 0; i < n; ++i) {
            slot_of_.push_back(add(x[i], y[i], z[i], zeta[i], next_stamp_++));
        }
    }

    // the committed model takes the edit (incremental.cpp Cells::apply, the same positions)
    void apply(const ScriptStep &e) {
        const size_t k = (size_t)e.index;
        switch (e.action) {
            case 1:  // append!
                slot_of_.push_back(add(e.x, e.y, e.z, e.zeta, next_stamp_++));
                break;
            case 2: {  // deleteat!
                const int s = slot_of_[k];
                unlink(s);
                free_.push_back(s);
                slot_of_.erase(slot_of_.begin() + (long)k);
                break;
            }
            case 3:
                cell_[(size_t)slot_of_[k]].v = e.zeta;
                break;
            default: {  // a new site, same position and value
                const int s = slot_of_[k];
                unlink(s);
                Cell &c = cell_[(size_t)s];
                c.x = e.x, c.y = e.y, c.z = e.z;
                link(s);
                break;
            }
        }
    }

    int64_t size() const { return (int64_t)slot_of_.size(); }

    // v_nearest at (qx, qy, qz) on the committed model (edit null) or on it plus *edit; *pos_out (if
    // given): the winner's 0-based Julia position in that model, -1 when no cell is below the sentinel.
    double query(double qx, double qy, double qz, const ScriptStep *edit, int64_t *pos_out = nullptr) const {
        Best b;
        int skip = -1, slot_k = -1;
        const int64_t birth_stamp = next_stamp_;
        if (edit && edit->action != 1) slot_k = slot_of_[(size_t)edit->index];
        if (edit && (edit->action == 2 || edit->action == 4)) skip = slot_k;  // the killed / moved cell's old site
        if (edit && edit->action == 4) {  // the moved cell at its new site, in its own position
            const Cell &c = cell_[(size_t)slot_k];
            b.consider(dist2(edit->x, edit->y, edit->z, qx, qy, qz), c.stamp, slot_k, c.v);
        }
        if (edit && edit->action == 1)  // the appended cell: last in Julia order
            b.consider(dist2(edit->x, edit->y, edit->z, qx, qy, qz), birth_stamp, -2, edit->zeta);
        if (!slot_of_.empty()) search(qx, qy, qz, skip, b);
        double val = b.found ? b.v : 0.0;  // :249 v = zero(Float64) when nothing is below the sentinel
        if (b.found && edit && edit->action == 3 && b.slot == slot_k) val = edit->zeta;  // the new value
        if (pos_out) {
            int64_t pos = -1;
            if (b.found) {
                pos = 0;  // the cells before the winner in Julia order (a killed cell is not one)
                const int gone = edit && edit->action == 2 ? slot_k : -1;
                for (int s : slot_of_)
                    if (s != gone && cell_[(size_t)s].stamp < b.stamp) ++pos;
            }
            *pos_out = pos;
        }
        return val;
    }

  private:
    struct Cell {
        double x, y, z, v;
        int64_t stamp;   // Julia position order
        int32_t bucket;  // its bucket, and its index in that bucket's list
        int32_t at;
    };
    struct Best {
        bool found = false;
        double d = kSentinel, v = 0.0;
        int64_t stamp = std::numeric_limits<int64_t>::max();
        int slot = -1;
        void consider(double dd, int64_t st, int s, double val) {
            // MCsub.jl:255 strict `<` in Julia order == the least (distance, position) below the sentinel
            if (dd < kSentinel && (!found || dd < d || (dd == d && st < stamp))) {
                found = true;
                d = dd;
                stamp = st;
                slot = s;
                v = val;
            }
        }
    };

    static double dist2(double mx, double my, double mz, double x, double y, double z) {
        const double dx = mx - x, dy = my - y, dz = mz - z;  // :254, left to right
        double d = dx * dx;
        d = d + dy * dy;
        d = d + dz * dz;
        return d;
    }

    // bucket index along axis a: monotone in v (a subtraction, a product by a positive constant, floor and a
    // clamp), so every cell in a bucket below b0 lies below the edge between buckets b0 - 1 and b0
    int coord(int a, double v) const {
        if (nb_[a] == 1) return 0;
        double t = std::floor((v - lo_[a]) * inv_[a]);
        t = t >= 0.0 ? std::min(t, (double)(nb_[a] - 1)) : 0.0;  // (NaN: bucket 0; its distances never count)
        return (int)t;
    }
    int bucket_of(double x, double y, double z) const { return (coord(2, z) * nb_[1] + coord(1, y)) * nb_[0] + coord(0, x); }

    int add(double x, double y, double z, double v, int64_t stamp) {
        int s;
        if (!free_.empty()) {
            s = free_.back();
            free_.pop_back();
        } else {
            s = (int)cell_.size();
            cell_.push_back({});
        }
        cell_[(size_t)s] = Cell{x, y, z, v, stamp, 0, 0};
        link(s);
        return s;
    }
    void link(int s) {
        Cell &c = cell_[(size_t)s];
        c.bucket = bucket_of(c.x, c.y, c.z);
        std::vector<int32_t> &l = bucket_[(size_t)c.bucket];
        c.at = (int32_t)l.size();
        l.push_back(s);
    }
    void unlink(int s) {
        const Cell &c = cell_[(size_t)s];
        std::vector<int32_t> &l = bucket_[(size_t)c.bucket];
        const int32_t last = l.back();
        l[(size_t)c.at] = last;
        cell_[(size_t)last].at = c.at;
        l.pop_back();
    }

    // rings of buckets around the query's bucket until every unscanned cell is provably farther
    void search(double qx, double qy, double qz, int skip, Best &b) const {
        const double q[3] = {qx, qy, qz};
        int c[3];
        for (int a = 0; a < 3; ++a) c[a] = coord(a, q[a]);
        const int rmax = std::max(std::max(nb_[0], nb_[1]), nb_[2]);
        for (int r = 0; r <= rmax; ++r) {
            int lo[3], hi[3];
            for (int a = 0; a < 3; ++a) lo[a] = std::max(c[a] - r, 0), hi[a] = std::min(c[a] + r, nb_[a] - 1);
            for (int k = lo[2]; k <= hi[2]; ++k) {
                const bool kr = k == c[2] - r || k == c[2] + r;
                for (int j = lo[1]; j <= hi[1]; ++j) {
                    const bool jr = kr || j == c[1] - r || j == c[1] + r;
                    auto scan = [&](int i) {
                        for (int32_t s : bucket_[(size_t)((k * nb_[1] + j) * nb_[0] + i)]) {
                            if (s == skip) continue;
                            const Cell &cl = cell_[(size_t)s];
                            b.consider(dist2(cl.x, cl.y, cl.z, qx, qy, qz), cl.stamp, s, cl.v);
                        }
                    };
                    if (jr) {  // a face row of the shell: all of it
                        for (int i = lo[0]; i <= hi[0]; ++i) scan(i);
                    } else {  // an inner row: its two ends (the rest was scanned in earlier rings)
                        if (c[0] - r >= 0) scan(c[0] - r);
                        if (r > 0 && c[0] + r < nb_[0]) scan(c[0] + r);
                    }
                }
            }
            // every cell outside the block lies beyond one of its faces: at least the least face gap away
            // (a face on the grid's edge has no cells beyond it); the gaps are shrunk by far more than the
            // roundings of the bucket index and the edge, and the squared gap is shrunk past the distance's
            // own roundings, so a cell outside is never at or below `bound`
            double g = std::numeric_limits<double>::infinity();
            for (int a = 0; a < 3; ++a) {
                const double tol = 1e-12 * (std::fabs(lo_[a]) + span_[a] + std::fabs(q[a]));
                if (lo[a] > 0) g = std::min(g, q[a] - (lo_[a] + lo[a] * h_[a]) - tol);
                if (hi[a] < nb_[a] - 1) g = std::min(g, (lo_[a] + (hi[a] + 1) * h_[a]) - q[a] - tol);
            }
            if (g == std::numeric_limits<double>::infinity()) return;  // the block is the whole grid
            if (!(g > 0)) continue;
            const double bound = (g * g) * (1.0 - 1e-12);
            if (b.found ? b.d < bound : bound >= kSentinel) return;
        }
    }

    std::vector<Cell> cell_;          // by slot
    std::vector<int32_t> slot_of_;    // Julia position -> slot
    std::vector<int32_t> free_;
    std::vector<std::vector<int32_t>> bucket_;
    double lo_[3] = {0, 0, 0}, h_[3] = {0, 0, 0}, inv_[3] = {0, 0, 0}, span_[3] = {0, 0, 0};
    int nb_[3] = {1, 1, 1};
    int64_t next_stamp_ = 0;
};

}  // namespace tdstar
