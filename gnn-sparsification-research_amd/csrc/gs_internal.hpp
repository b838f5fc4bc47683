// gs_internal.hpp -- context, device buffers, error plumbing for libgsparse.
// gfx950 only; compiled with -ffp-contract=off so every product is rounded
// before it is summed unless a kernel asks for fma() explicitly.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/gsparse.h"

namespace gs {

void set_error(const char *fmt, ...);

struct GsError {
    int code;
};

#define GS_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            ::gs::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
            throw ::gs::GsError{_e == hipErrorOutOfMemory ? GS_ENOMEM : GS_EHIP};           \
        }                                                                                   \
    } while (0)

#define GS_CHECK(cond, code, ...)        \
    do {                                 \
        if (!(cond)) {                   \
            ::gs::set_error(__VA_ARGS__); \
            throw ::gs::GsError{code};   \
        }                                \
    } while (0)

// Grow-only device buffer.
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    void *ensure(size_t n) {
        if (n <= bytes) return ptr;
        if (ptr) GS_HIP(hipFree(ptr));
        ptr = nullptr;
        bytes = 0;
        if (n == 0) return nullptr;
        GS_HIP(hipMalloc(&ptr, n));
        bytes = n;
        return ptr;
    }
    template <class T>
    T *as() const { return static_cast<T *>(ptr); }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

struct ProfEntry {
    int64_t launches = 0;
    double ms = 0.0;
    double bytes = 0.0;
};

struct ProfPending {
    std::string name;
    hipEvent_t start, stop;
    double bytes;
    // optional: + its_bytes x (an int64 the device wrote to slot its_slot of the
    // context's "prof_its" buffer), read when the entries are flushed -- e.g. the CG's
    // bytes per executed iteration, without a host round trip per solve
    int64_t its_slot = -1;
    double its_bytes = 0.0;
};
static constexpr int kProfPendingMax = 4096;
// int32 entries allocated past the last column index: the Jaccard probe loop reads
// lists in unconditional 64-lane steps (up to 511 entries past a list's end, masked)
static constexpr int64_t kIxPad = 1024;

struct Graph {
    int64_t n = 0, nnz = 0;
    int symmetric = 0;
    DevBuf indptr;    // int64 [n+1]
    DevBuf indices;   // int32 [nnz]
    DevBuf data;      // f64 [nnz] multiplicity / weight
    DevBuf rows;      // int32 [nnz] row of each entry
    DevBuf tptr;      // int64 [n+1] transpose (in-lists), only if !symmetric
    DevBuf tidx;      // int32 [nnz]
    DevBuf tpos;      // int64 [nnz] CSR position of each transposed entry
    bool has_transpose = false;
    int64_t epoch = 0;  // bumped whenever a new graph is set (keys the per-graph caches)
};

// Row ranges of the sharded Jaccard (gs_jaccard_shares): cuts = [R | E | O], P + 1
// values each -- cut rows, their first CSR entries, owner entries before them
struct JacShares {
    std::vector<int64_t> cuts;
    int P() const { return (int)(cuts.size() / 3) - 1; }
    int64_t R(int r) const { return cuts[r]; }
    int64_t E(int r) const { return cuts[P() + 1 + r]; }
    int64_t O(int r) const { return cuts[2 * (P() + 1) + r]; }
};

struct ErState {
    int64_t k = 0, m = 0, n = 0;
    int64_t ld = 0;         // row stride of the n x k arrays (k rounded up to 8)
    int64_t lnnz = 0;       // entries of L_reg
    int64_t proj_next = 0;  // next R row expected by project_rows
    double reg = 0.0;       // L_reg = L + reg I of the last gs_er_prepare
    DevBuf edge_id;   // int64 [nnz] undirected edge id of CSR entry (u<v), -1 otherwise
    DevBuf bptr;      // int64 [n+1] incidence rows (B, metrics.py:260-269)
    DevBuf bcol;      // int64 [2m] edge id (ascending within row)
    DevBuf bsgn;      // int8  [2m] +1 / -1
    DevBuf bcur;      // int64 [n] streaming cursor into B rows
    DevBuf lp, li, lv;  // L_reg CSR (int64, int32, f64)
    DevBuf X, Rr, P0, P1, Q;  // n x k row-major f64 (Rr starts as Y)
    DevBuf colstate;  // per-column scalars
    DevBuf acc;       // dot partial accumulators
    DevBuf iters;     // int32 [k]
    DevBuf rawbuf;    // staging for host-streamed raw normals
    int pcur = 0;     // which of P0/P1 holds the current p
    bool solved = false;
    int64_t proj_c0 = 0, proj_c1 = 0;  // JL columns of Y the projection fills (a rank's slice)
    std::vector<int64_t> prep_key;      // (graph epoch, k, reg) the state above was built for
    void *rr_zeroed = nullptr;          // Rr allocation whose row padding has been zeroed
    int64_t rr_k = 0;                   // ... for this k (the padding is [k, ld) of each row)
    std::vector<uint8_t> col_solved;    // [k] solved since the last gs_er_prepare
    // mode 4 / 5 setup read back once per (graph epoch, reg): unit-weight flags, SELL
    // entry count and slice widths (no host round trip on later solves)
    std::vector<int64_t> unit_key;
    int32_t unit_flags = 0;
    int64_t sell_sent = 0;
    std::vector<int32_t> sell_wid;
};

}  // namespace gs

struct gs_ctx;
namespace gs {
struct BbRun;  // the staged metric backbone's state (gs_backbone.hip)
void project_rows(gs_ctx *c, int64_t e0, int64_t e1, const double *draw, int64_t kraw, int64_t col0,
                  int64_t col1, double sqrt_k);
}  // namespace gs

struct gs_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t aux[4] = {nullptr, nullptr, nullptr, nullptr};  // side streams (Jaccard classes)
    hipEvent_t aux_ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    hipEvent_t order_ev = nullptr;  // gs_stream_wait / gs_stream_signal (timing off)
    bool async_ = false;
    bool profiling = false;
    std::map<std::string, gs::ProfEntry> prof;
    std::vector<std::string> prof_order;
    std::vector<gs::ProfPending> pending;
    gs::Graph g;
    gs::ErState er;
    // symmetric Jaccard: the plan of the last call (graph epoch, part rows) kept with
    // its task lists, so a repeated call plans nothing and does not wait for the host
    std::vector<int64_t> jac_plan_key;
    unsigned long long jac_plan_tot[8] = {};
    std::vector<std::array<int64_t, 4>> jac_plan_bm;  // bitmap batches: g0, g1, task range
    int64_t jac_bytes_epoch = -1;
    double jac_bytes_sum = 0.0;
    std::vector<uint64_t> zig_key;  // (PCG64 state, stream length, block) of a parsed stream
    int64_t zig_draws = 0;          // draws known to cover it
    gs::DevBuf scratch[6];
    gs::DevBuf outbuf, inbuf, inbuf2;
    std::map<std::string, gs::DevBuf> named;  // per-subsystem buffers (backbone, ...)
    std::map<int, gs::JacShares> jac_shares;  // sharded Jaccard row ranges, by part count
    int64_t jac_epoch = -1;                   // graph epoch jac_shares belong to
    // register-resident CG (gs_cg_reg.hip): the ELL-8 copies are kept while their key
    // (graph epoch, L_reg shift, chunk / LDS layout) is unchanged; the split form is
    // switched off for the context after a hand-off gave up (its parts could not all
    // be resident: another process or stream held CUs)
    std::vector<int64_t> reg_ell_key, reg_split_key;
    int64_t reg_nov = 0;
    std::vector<int64_t> reg_hch;  // host copy of the chunk table (outlives its async copy)
    bool reg_split_off = false;
    int64_t reg_split_off_epoch = -1;      // graph epoch the split form was turned off for
    std::vector<int32_t> reg_split_hpt;    // host copies of the split tables (outlive their
    std::vector<int64_t> reg_split_htab;   // stream-ordered uploads)
    int32_t *split_abort_host = nullptr;   // pinned: the last split launch's abort word
    hipEvent_t split_abort_ev = nullptr;   // its copy has landed
    bool split_abort_pending = false;
    int split_abort_parts = 0;
    int64_t split_aborts = 0;              // aborts seen by this context
    std::shared_ptr<gs::BbRun> bb;         // staged metric backbone (gs_bb_*)
    gs::DevBuf &buf(const char *name) { return named[name]; }
};

namespace gs {

// Record a profiled launch: call prof_begin before the launch and prof_end after.
hipEvent_t prof_begin(gs_ctx *c);
void prof_end(gs_ctx *c, hipEvent_t start, const char *name, double bytes);
// count an event under `name` in the profile (launches += 1, no time)
void prof_note(gs_ctx *c, const char *name);
void prof_flush(gs_ctx *c);
void sync_if_needed(gs_ctx *c);

template <class F>
int guard(F &&f) {
    try {
        f();
        return GS_OK;
    } catch (const GsError &e) {
        return e.code;
    } catch (const std::exception &e) {
        set_error("std::exception: %s", e.what());
        return GS_EHIP;
    } catch (...) {
        set_error("unknown exception");
        return GS_EHIP;
    }
}

inline unsigned grid_for(int64_t work, int block, int64_t cap = 1 << 20) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// Host pointer in -> device copy (staging into buf); device pointer passes through.
const void *to_device(gs_ctx *c, DevBuf &buf, const void *p, size_t bytes, int loc);
// Output helper: returns a device pointer to write into; finish_out copies to host if needed.
void *out_device(gs_ctx *c, DevBuf &buf, void *p, size_t bytes, int loc);
void finish_out(gs_ctx *c, void *host, const void *dev, size_t bytes, int loc);

// Device-wide helpers (gs_prims.hip)
void exclusive_scan_i64(gs_ctx *c, const int64_t *in, int64_t *out, int64_t n);
void sort_keys_u64(gs_ctx *c, uint64_t *keys, int64_t n, int end_bit);
void sort_pairs_u64_i64(gs_ctx *c, uint64_t *keys, int64_t *vals, int64_t n, int end_bit);

// Graph helpers used by the ER path (gs_graph.hip)
void ensure_transpose(gs_ctx *c);

// Register-resident CG (ApproxER mode 5, gs_cg_reg.hip): applies when the T BLAS
// chunks (lengths len[t]) fit its thread geometry; solves columns [col0, col0+ncols)
// of L_reg (CSR lp/li/lv) into Xc (column-major, ldn per column)
bool cg_regres_applies(int64_t n, int T, const int64_t *len);
bool cg_regres_wide(int64_t n, int T, const int64_t *len);  // its 512-thread form applies
void split_abort_poll(gs_ctx *c, bool wait);
void cg_regres_solve(gs_ctx *c, int64_t n, const int64_t *lp, const int32_t *li, const double *lv,
                     int unit, int dcount, const double *diag, const double *Rr, int64_t ld,
                     int64_t col0, int64_t ncols, int32_t maxiter, double rtol, int T,
                     const int64_t *ha, const int64_t *hlen, double *Xc, int64_t ldn,
                     int32_t *iters, int64_t slots, long long *prof);

// Whole-graph Jaccard of a symmetric graph (gs_jaccard.hip)
// counts != 0: |N(u) ∩ N(v)| per entry instead of the Jaccard ratio
// cc != nullptr: the part's raw counts into its compact owner-entry array
void jaccard_symmetric(gs_ctx *c, double *out, int part, int nparts, int counts = 0,
                       uint32_t *cc = nullptr);
const JacShares &jaccard_shares(gs_ctx *c, int P);
void jaccard_from_counts(gs_ctx *c, int P, const uint32_t *cc, int64_t stride, double *out);

// Dense grounded-Laplacian machinery (gs_exact_er.hip): component labels of the
// resident graph (smallest node id per component, device), and W = L^{-1} of
// M = L L^T for the grounded M (identity rows where flag[u], N x N scratch A, W)
int32_t *components(gs_ctx *c);
void grounded_inverse(gs_ctx *c, int64_t N, const uint8_t *flag, double *A, double *W);
void transpose_square(gs_ctx *c, int64_t N, const double *W, double *U);

}  // namespace gs
