// eval_server.h -- td_evaluate's full path as ONE resident launch (k_eval_server,
// nn_grid.hip; host side eval_server.cpp).
//
// The three launches of a full evaluate (bucket fill, grid search, ray sums)
// cost 18 us issue-to-done before any work.  The server is one
// launch of one 512-thread workgroup per CU that stays resident between calls:
// the host writes a command into pinned memory (EvalCmd: the cells' grid and
// where the staged cells are), workgroup 0 polls it over PCIe and forwards it
// to the others through device memory, and every workgroup then
//   fills its share of the bucket grid from the staged cells (pinned memory),
//   meets the others at one grid barrier (8 sharded arrival counters),
//   searches the points of ITS rays (a contiguous range of rays, balanced by
//     point count: no hand-off between the search and the sums),
//   sums its rays (ray_sum.h, Julia's association) into pinned memory,
//   and reports done = seq in its own reply line.
// The host adds chi^2 in k order from the pinned ptS, as for the launches.
// Workgroup 0 alone takes commands and alone decides to quit (QUIT, or its idle
// watchdog): the others follow its forwarded command, so a command is either
// run by every workgroup or by none (then EvalReply::exited is set and the
// host relaunches).  Every spin is bounded; a grid barrier that never completes
// (a workgroup not resident) ends the launch with done = -seq, and the host
// takes the launches from then on.
#pragma once
#include <cstddef>

#include "internal.h"

namespace tdstar {

enum EvalCmdType : int { kEvalRun = 1, kEvalQuit = 3 };

struct EvalCmd {  // pinned host memory, host -> device: check, then seq, written last
    long long seq;
    int type, ncells;
    int stride, par;       // par: the bucket-count set this evaluate fills
    int other_nb, diag;    // buckets of the other set (the previous evaluate's) to zero; diag: stamp phases
    double *cells;         // device cell copy (SoA x|y|z|zeta, `stride`), written by the fill
    const double *stage;   // the staged cells: pinned host memory, as the device addresses it
    CellGrid G;
    unsigned long long check;  // mailbox mix of words 1 .. check - 1 with seq (chain_dev.h mailbox_word_mix)
};
constexpr int kEvalCmdWords = (int)(offsetof(EvalCmd, check) / sizeof(long long)) + 1;  // seq .. check
static_assert(sizeof(EvalCmd) == sizeof(long long) * kEvalCmdWords, "EvalCmd: no tail padding");
static_assert(2 * kEvalCmdWords <= 64, "EvalCmd: one 32-bit granule per lane");

// What the host polls: pinned host memory, device -> host, two 64-B lines.  The workgroups of each
// of 8 shards (wg % 8) count their finished evaluates on a device counter; the shard's last one
// writes done[shard] = seq (after every workgroup's replies were acknowledged), so the host reads
// one line, not one per workgroup.
struct EvalCtl {
    long long done[8];   // per shard: seq of the last command all its workgroups finished
    long long t_end[8];  // 100 MHz wall clock: when that shard finished (written before done)
    long long t_take;    // workgroup 0: the command seen
    long long exited;    // workgroup 0: the launch is ending (set before it forwards its QUIT)
    long long failed;    // seq of a command some workgroup abandoned (its grid barrier timed out)
    long long pad[13];
};
static_assert(sizeof(EvalCtl) == 256, "EvalCtl: four lines");

// Per-workgroup phase stamps (diagnostics: EvalCmd::diag != 0), pinned, one 128-B record each; the
// 100 MHz clock: [0] command seen, [1] its cells loaded, [2] bucket slots returned, [3] fill drained,
// [4] released, [5] grid barrier passed, [6] first search round done (wave 0), [7] search done,
// [8] ray sums done, [9] replies acknowledged
struct EvalStamps {
    long long t[16];
};

struct EvalArgs {  // k_eval_server's argument block
    EvalCmd *mb;                 // pinned mailbox (device address)
    EvalCtl *ctl;                // pinned (device address)
    EvalStamps *stamps;          // pinned [nwg] (device address): diagnostics
    unsigned long long *bcast;   // device: the forwarded command, 2 * kEvalCmdWords granules {32-bit word, tag}
    unsigned *arrive;            // device: 8 arrival shards, 32 words (128 B) apart; then 8 finish shards
    int *count;                  // device: [2][kGridMaxBuckets] bucket counts
    BucketEntry *ent;            // device: [kGridMaxBuckets * kGridCap]
    const int *wg_ray;           // device: [nwg + 1] first ray of each workgroup
    const int *ray_off;          // the geometry (Geometry)
    const double *px, *py, *pz, *w;
    double *ptS;                 // device copy of ptS [n]
    double *ptS_host;            // pinned ptS [n] (device address)
    int n, nwg;
    int lds_pts;                 // points of the largest workgroup share (dynamic LDS: lds_pts doubles)
    int pad0;
    long long seq0;              // the mailbox's seq when launched: the first command is seq0 + 1
    long long idle_ticks;        // workgroup 0 quits after this much silence (100 MHz ticks)
    long long guard_ticks;       // a grid barrier waited this long: the command fails
};

// The command check: each word mixed with its position and the seq (splitmix64's finaliser), xor-combined;
// the kernel forms it with one DPP xor over the lanes holding words 1 .. check - 1.
__host__ __device__ inline unsigned long long eval_mix(unsigned long long w, int i, long long seq) {
    unsigned long long z = w ^ ((unsigned long long)i * 0x9E3779B97F4A7C15ull) ^
                           ((unsigned long long)seq * 0xD1B54A32D192ED03ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline unsigned long long eval_check(const EvalCmd *c, long long seq) {
    const unsigned long long *w = reinterpret_cast<const unsigned long long *>(c);
    unsigned long long h = 0;
    for (int i = 1; i < kEvalCmdWords - 1; ++i) h ^= eval_mix(w[i], i, seq);
    return h;
}

constexpr int kEvalThreads = 512;
constexpr int kEvalMaxLdsPts = 6144;  // a larger workgroup share (very long rays): the launches
// the forwarded command's tag: never 0 (a cleared broadcast), unique among consecutive seqs
__host__ __device__ inline unsigned eval_tag(long long seq) { return 0x80000000u | (unsigned)(seq & 0x7fffffff); }

// k_eval_server, launched on `s` with nwg workgroups
hipError_t launch_eval_server(const EvalArgs &a, hipStream_t s);

}  // namespace tdstar
