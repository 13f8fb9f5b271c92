// plba.hip — host side of the MI355X LBA backend: context, structure preparation, the
// Levenberg–Marquardt driver and the C ABI of include/plba.h.
//
// Control flow mirrors g2o exactly:
//   SparseOptimizer::initializeOptimization(level)   -> plba_initialize_optimization
//   SparseOptimizer::optimize(n)                     -> plba_optimize
//     OptimizationAlgorithmLevenberg::solve(it)      -> one iteration launch + trial launches
// The numerical work is all on the device (plba_kernels.hpp); the host only reads back the
// 80-byte control block after each trial to decide whether another trial runs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/plba.h"
#include "plba_build.hpp"
#include "plba_kernels.hpp"

namespace plba {

#define PLBA_CHECK(expr)                                                                       \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) {                                                                \
            (void)hipGetLastError(); /* do not leak into the next launch check */              \
            ctx->set_error("HIP error %s at %s:%d: %s", hipGetErrorString(_e), __FILE__,       \
                           __LINE__, #expr);                                                   \
            return PLBA_E_DEVICE;                                                              \
        }                                                                                      \
    } while (0)

enum KernelId {
    K_LINEARIZE, K_REDUCE, K_ITER_INIT, K_ESCHUR, K_MEMSET, K_ASSEMBLE, K_FINALIZE, K_FACTOR,
    K_POSE_UPDATE, K_LM_UPDATE, K_EVAL, K_DECIDE, K_DENSE_PANEL, K_DENSE_UPDATE,
    K_PACK,  // sharded: this rank's partials packed for an exchange (per-rank work)
    K_COMM,  // sharded: the collectives themselves (RCCL, or the host transport's round trip)
    K_COUNT
};
static const char *kKernelNames[K_COUNT] = {
    "k_linearize", "k_iter_reduce", "k_iter_init", "k_edge_schur", "memset_rcs",
    "k_rcs_chunk", "k_rcs_finalize", "k_rcs_factor", "k_pose_update", "k_lm_solve", "k_edge_eval", "k_decide",
    "k_dense_panel", "k_dense_update", "k_shard_pack", "collectives"};

}  // namespace plba

using namespace plba;

struct plba_ctx {
    plba_opts opts;
    std::string err;
    hipStream_t stream = nullptr;
    bool uploaded = false, initialized = false;
    int level = 0;
    int robust = 1;
    Dev d{};
    // sharded windows: transport of the three per-step all-reduces
    struct Comm {
        enum Kind { NONE, RCCL, HOST } kind = NONE;
        int nranks = 1, rank = 0;
        ncclComm_t nccl = nullptr;
        plba_host_allreduce_fn fn = nullptr;
        void *user = nullptr;
        double *hbuf = nullptr;  // pinned staging (HOST)
        size_t hcap = 0;
    } comm;
    // device arena: ONE grow-only allocation carved per window (no hipMalloc / hipFree per
    // upload), filled by one memset and one host->device copy from pinned staging
    struct Item {
        void **field;
        size_t bytes, src_bytes;
        const void *src;
        bool zero;
        size_t off;
        const void *dsrc = nullptr;  // device source (copied D2D after the arena is carved)
    };
    std::vector<Item> plan;
    BuildMem bmemA, bmemB;   // device window build scratch (plba_build.hip), grow-only
    char *arena = nullptr, *staging = nullptr;
    size_t arena_cap = 0, staging_cap = 0;
    Ctrl *h_ctrl = nullptr;  // pinned
    uint8_t *d_depth = nullptr;  // [Ep] isDepthPositive flags
    double *d_outd = nullptr;    // download staging, caller order: Tcw | pt_xyz | ln_orth | χ² (points,
                                 // lines) | bytes: depth flags [Ep] | levels (points, lines)
    char *h_out = nullptr;       // pinned host copy of it (grow-only)
    size_t h_out_cap = 0;
    // host-side bookkeeping
    int32_t n_kf = 0, n_pt = 0, n_ln = 0, Ep = 0, El = 0;
    std::vector<int32_t> e_orig;        // CSR edge -> original index within its type
    std::vector<int32_t> h_tile_last;   // dense path: last row tile of each column tile's envelope
    std::vector<int32_t> lm_gpos;       // local landmark -> whole-window landmark (points, then lines)
    std::vector<uint8_t> h_level;       // [E] CSR order
    std::vector<plba_iter_trace> trace;
    int stage = 0;
    size_t n_triples = 0;
    int64_t n_free_edges = 0;  // edges whose pose vertex is free
    // captured step graph (one LM trial + guarded iteration / stage-switch work)
    hipGraph_t step_graph = nullptr;
    hipGraphExec_t step_exec = nullptr;
    bool graphs_stale = false;  // captured for a previous window (update before use)
    std::vector<int64_t> graph_sig;  // launch signature the executable graphs were built for
    // the same step captured 2, 4, 8, 16 times back to back: a batch of N steps is launched as
    // its binary decomposition (a graph-to-graph transition costs ~8 us on the device)
    static constexpr int kMultiLevels = 4;
    hipGraph_t multi_graph[kMultiLevels] = {};
    hipGraphExec_t multi_exec[kMultiLevels] = {};
    int last_steps = 16;     // steps the previous schedule needed (first batch size)
    int cur = 0;             // which state buffer holds the current estimate (mirror of Ctrl::cur)
    int last_ok = 0, chi_src = 0;  // x_p / x_l and χ² buffer indices (mirrors of Ctrl::last_ok / chi_src)
    bool no_graph = false;   // set when the step cannot be captured (RCCL without capture support)
    // block cyclic reduction safety net: a BCR hand-off wait that timed out (Ctrl::dev_error)
    // makes run_schedule restore the schedule's starting state from these copies, switch this
    // context to the column-lane factorisation for good (no_bcr) and solve the window again
    bool no_bcr = false;
    int bcr_fallbacks = 0;
    bool pool_hold = false;  // this context keeps the device pool's release threshold raised (prewarm)
    int dev_build = 0;  // the last upload's window structure was built on the device
    int fb_cl = 0, fb_twisted = 0, fb_tw_m = 0;  // the factorisation the window falls back to
    double *bk_T = nullptr, *bk_X = nullptr, *bk_xp = nullptr, *bk_xk = nullptr, *bk_Lpb = nullptr, *bk_XL = nullptr,
           *bk_xl = nullptr;
    uint8_t *bk_level = nullptr;
    int steps_launched = 0;
    // kernel timing (optional)
    bool timing = false;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_used;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_next = 0;
    double k_ms[K_COUNT] = {0};
    int32_t k_n[K_COUNT] = {0};
    // loop-closure pose graph (plba_pgo_optimize): its own grow-only device block, independent
    // of the window arena (a PGO call leaves an uploaded window intact)
    char *pgo_mem = nullptr;
    size_t pgo_cap = 0;
    double *pgo_hout = nullptr;  // pinned [4]

    void set_error(const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        if (opts.verbose) fprintf(stderr, "[plba] %s\n", buf);
    }
    // A new window keeps the instantiated step graphs: the next capture updates them in place
    // (hipGraphExecUpdate, same topology, new kernel arguments and grids) instead of destroying
    // and re-instantiating five executable graphs (capture_step).
    void free_all() {
        graphs_stale = true;
        plan.clear();
        d = Dev{};
        bk_T = bk_X = bk_xp = bk_xk = bk_Lpb = bk_XL = bk_xl = nullptr;
        bk_level = nullptr;
        uploaded = initialized = false;
    }
    // Records a device array of `count` T (at least 128 bytes: kernels issue unconditional
    // loads of one record for dead lanes, which must stay inside the array). `src` (host, kept
    // alive until commit_plan) is uploaded; everything else starts zeroed (`zero`: must stay
    // zero even under PLBA_POISON).
    template <typename T>
    void alloc(T *&p, size_t count, const void *src = nullptr, bool zero = false) {
        p = nullptr;
        const size_t sb = count * sizeof(T);
        plan.push_back(Item{(void **)&p, std::max(sb, (size_t)128), src ? sb : 0, src, zero, 0});
    }
    // a device array filled from device memory (the device window build's outputs)
    template <typename T>
    void alloc_dev(T *&p, size_t count, const void *dsrc) {
        p = nullptr;
        const size_t sb = count * sizeof(T);
        plan.push_back(Item{(void **)&p, std::max(sb, (size_t)128), sb, nullptr, false, 0, dsrc});
    }
    int commit_plan() {
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        size_t up = 0, tot = 0;
        for (auto &it : plan)
            if (it.src) { it.off = up; up = al(up + it.bytes); }
        size_t dv = up;  // device-sourced arrays after the host-sourced ones, outside the memset
        for (auto &it : plan)
            if (it.dsrc) { it.off = dv; dv = al(dv + it.bytes); }
        tot = dv;
        for (auto &it : plan)
            if (!it.src && !it.dsrc) { it.off = tot; tot = al(tot + it.bytes); }
        if (tot > arena_cap) {
            // stream-ordered: hipFree / hipMalloc would synchronise the whole device, which fails
            // (and invalidates the capture) while another context of the process captures its
            // step graphs
            if (arena) (void)hipFreeAsync(arena, stream);
            arena = nullptr;
            arena_cap = 0;
            const size_t cap = tot + tot / 4;
            if (hipMallocAsync((void **)&arena, cap, stream) != hipSuccess) {
                (void)hipGetLastError();
                set_error("hipMalloc(%zu bytes) of the window arena failed", cap);
                return PLBA_E_NOMEM;
            }
            arena_cap = cap;
        }
        if (up > staging_cap) {
            (void)hipStreamSynchronize(stream);
            retire_pinned(staging);
            staging = nullptr;
            staging_cap = 0;
            const size_t cap = up + up / 4;
            if (hipHostMalloc((void **)&staging, cap, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                set_error("hipHostMalloc(%zu bytes) of the upload staging failed", cap);
                return PLBA_E_NOMEM;
            }
            staging_cap = cap;
        }
        for (auto &it : plan) {
            *it.field = arena + it.off;
            if (it.src) {
                if (it.src_bytes) std::memcpy(staging + it.off, it.src, it.src_bytes);
                if (it.bytes > it.src_bytes) std::memset(staging + it.off + it.src_bytes, 0, it.bytes - it.src_bytes);
            }
        }
        // PLBA_POISON=1 (diagnostics only): non-uploaded arrays start as NaN (0xFF bytes) to expose
        // reads of memory no kernel wrote; arrays whose zero start is part of the contract stay 0
        const char *poison = getenv("PLBA_POISON");
        const bool pz = poison && poison[0] == '1';
        // device-sourced arrays [up, dv) are zeroed too before their payload is copied in, so the
        // padding past their payload reads as zero like a host array's (the 128-byte over-read
        // contract of alloc) — one memset of [up, tot) unless the rest is poisoned
        hipError_t e = pz ? hipMemsetAsync(arena + up, 0, dv - up, stream) : hipSuccess;
        if (e == hipSuccess) e = pz ? hipMemsetAsync(arena + dv, 0xFF, tot - dv, stream) : hipMemsetAsync(arena + up, 0, tot - up, stream);
        for (auto &it : plan)
            if (it.dsrc && it.src_bytes && e == hipSuccess)
                e = hipMemcpyAsync(arena + it.off, it.dsrc, it.src_bytes, hipMemcpyDeviceToDevice, stream);
        if (e == hipSuccess && pz)
            for (auto &it : plan)
                if (it.zero && e == hipSuccess) e = hipMemsetAsync(arena + it.off, 0, it.bytes, stream);
        if (e == hipSuccess && up) e = hipMemcpyAsync(arena, staging, up, hipMemcpyHostToDevice, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            set_error("window arena fill failed: %s", hipGetErrorString(e));
            return PLBA_E_DEVICE;
        }
        return PLBA_OK;
    }
    // Pinned host blocks outgrown by a bigger window are freed only when the context is destroyed:
    // hipHostFree synchronises the device (see commit_plan). Growth is geometric, so few retire.
    std::vector<void *> retired;
    void retire_pinned(void *p) {
        if (p) retired.push_back(p);
    }
    hipEvent_t next_event() {
        if (ev_next == ev_pool.size()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            ev_pool.push_back(e);
        }
        return ev_pool[ev_next++];
    }
};

namespace {

inline int blocks_for(int n, int b = kBlock) { return (n + b - 1) / b; }

// Landmark -> rank: landmarks ordered by the id rank of the keyframe of their
// first observation (kf_obs_list[0]), cut into nranks contiguous runs of ~equal edge count.
void shard_plan(const plba_graph *g, int R, int32_t *pt_owner, int32_t *ln_owner) {
    std::vector<int32_t> korder(g->n_kf), kpos(g->n_kf);
    std::iota(korder.begin(), korder.end(), 0);
    std::stable_sort(korder.begin(), korder.end(), [&](int a, int b) { return g->kf_id[a] < g->kf_id[b]; });
    for (int i = 0; i < g->n_kf; ++i) kpos[korder[i]] = i;
    const int np = g->n_pt, nl = g->n_ln;
    std::vector<int32_t> key(np + nl, INT32_MAX), cnt(np + nl, 0);
    for (int e = 0; e < g->n_ept; ++e) {
        const int l = g->ept_lm[e];
        if (cnt[l]++ == 0) key[l] = kpos[g->ept_kf[e]];
    }
    for (int e = 0; e < g->n_eln; ++e) {
        const int l = np + g->eln_lm[e];
        if (cnt[l]++ == 0) key[l] = kpos[g->eln_kf[e]];
    }
    std::vector<int32_t> ord(np + nl);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return key[a] < key[b]; });
    int64_t total = 0, acc = 0;
    for (int c : cnt) total += c;
    for (int l : ord) {
        // rank of this landmark's edge-count midpoint
        const int64_t mid2 = 2 * acc + cnt[l];
        int r = total > 0 ? (int)((mid2 * R) / (2 * total)) : 0;
        r = std::min(std::max(r, 0), R - 1);
        acc += cnt[l];
        if (l < np) pt_owner[l] = r;
        else ln_owner[l - np] = r;
    }
}

inline bool env_flag(const char *name) {
    const char *v = getenv(name);
    return v && v[0] == '1';
}
inline size_t band_lds_bytes(int bw) { return sizeof(double) * band_lds_doubles(bw, 0); }
template <int... B>
const void *band_kernel_impl(int bw, std::integer_sequence<int, B...>) {
    const void *k = nullptr;
    ((bw == B ? (k = (const void *)k_rcs_factor_band<B>, 0) : 0), ...);
    return k;
}
inline const void *band_kernel(int bw) {
    return band_kernel_impl(bw, std::make_integer_sequence<int, kBandMax + 1>{});
}
template <int... B>
const void *twisted_kernel_impl(int bw, std::integer_sequence<int, B...>) {
    const void *k = nullptr;
    ((bw == B ? (k = (const void *)k_rcs_factor_twisted<B>, 0) : 0), ...);
    return k;
}
inline const void *twisted_kernel(int bw) {
    return twisted_kernel_impl(bw, std::make_integer_sequence<int, kBandMax + 1>{});
}
static_assert(band_lds_doubles(kBandMax, 1) * sizeof(double) + band_static_bytes(kBandMax) <= 158 * 1024,
              "kBandMax window must fit LDS");
inline int band_ring(int bw, int nf) {
    const size_t budget = 158 * 1024 - band_static_bytes(bw), base = band_lds_bytes(bw);
    const size_t per = sizeof(double) * ((size_t)bw * 36 + 36 + 6);
    int R = base + per < budget ? (int)((budget - base - per) / per) : 1;
    return std::max(1, std::min(R, 16));
}
inline size_t band_lds_bytes(int bw, int nf) { return sizeof(double) * band_lds_doubles(bw, band_ring(bw, nf)); }
inline size_t twisted_lds_bytes(int bw, int nf) {
    // x_p staging [nf][6], then the separator merge or (bw >= 11) the streamed back substitution
    const size_t tail = std::max(twisted_merge_doubles(bw), bw * 6 > 64 ? bstream_doubles(bw) : (size_t)0);
    return std::max(band_lds_bytes(bw, nf), sizeof(double) * ((size_t)nf * 6 + tail));
}
template <int... B>
const void *cl_kernel_impl(int bw, bool twisted, std::integer_sequence<int, B...>) {
    const void *k = nullptr;
    ((bw == B ? (k = twisted ? (const void *)k_rcs_factor_twisted_cl<B> : (const void *)k_rcs_factor_band_cl<B>, 0) : 0),
     ...);
    return k;
}
// column-lane factorisation (plba_band_cl.hpp) for bandwidths up to kClMaxBW
inline bool use_cl(int bw) {
    const char *f = getenv("PLBA_FACTOR");
    if (f && std::string(f) == "band") return false;
    return bw >= 1 && bw <= kClMaxBW && !env_flag("PLBA_NO_CL");
}
// Two-sided split: rows 0..m-1 top-down, nf-1..m+bw bottom-up. An odd remainder goes to the top
// segment, so workgroup 0 usually arrives last and merges with the separator window already in
// its LDS (workgroup 1 as the last arriver must first reload segment 0's window from global
// memory): C3 hand-off + merge 10.9 k -> 8.1 k cycles, factorisation 74.8 -> 73.3 µs.
inline int tw_split(int nf, int bw) { return (nf - bw + 1) / 2; }
inline size_t cl_lds_bytes(int bw, int nf, bool twisted) {
    return sizeof(double) * (cl_lds_doubles(bw) + (twisted ? (size_t)nf * 6 : 0));
}
template <int... B>
const void *bcr_kernel_impl(int bw, std::integer_sequence<int, B...>) {
    const void *k = nullptr;
    ((bw == B ? (k = (const void *)k_rcs_factor_bcr<B>, 0) : 0), ...);
    return k;
}
inline const void *bcr_kernel(int bw) { return bcr_kernel_impl(bw, std::make_integer_sequence<int, kBcrMaxBW + 1>{}); }
inline size_t bcr_lds_bytes(int bw) { return sizeof(double) * bcr_lds_doubles(bw); }
// n up to which the dense solve keeps y in LDS; PLBA_SOLVE_LDS_N lowers it (tests: the global-y path
// at sizes the oracle finishes)
inline int solve_lds_limit() {
    const char *e = getenv("PLBA_SOLVE_LDS_N");
    return e && e[0] ? std::min(atoi(e), kSolveLdsN) : kSolveLdsN;
}
// Factorisation mode of a banded window: PLBA_FACTOR=bcr|cl|band forces one (diagnostics / A-B
// runs); by default block cyclic reduction once the window has enough super-rows for its
// log-depth chain to beat the two-sided column-lane chain of (nf+bw)/2 pivot steps.
inline size_t bcr_back_lds_bytes(int bw) { return sizeof(double) * bcr_back_lds_doubles(bw); }
template <int... B>
const void *bcr_back_kernel_impl(int bw, std::integer_sequence<int, B...>) {
    const void *k = nullptr;
    ((bw == B ? (k = (const void *)k_rcs_bcr_back<B>, 0) : 0), ...);
    return k;
}
inline const void *bcr_back_kernel(int bw) {
    return bcr_back_kernel_impl(bw, std::make_integer_sequence<int, kBcrMaxBW + 1>{});
}
// Workgroups of the BCR forward kernel the device holds at once: CUs x occupancy (LDS-bound, one
// per CU above 80 KB). PLBA_BCR_RESIDENT overrides it (tests: force the column-lane choice).
inline int bcr_resident(int device, int bw) {
    const char *e = getenv("PLBA_BCR_RESIDENT");
    if (e && e[0]) return atoi(e);
    if (bw < 1 || bw > kBcrMaxBW || bcr_lds_bytes(bw) > 159 * 1024) return 0;
    int cus = 0, occ = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        hipFuncSetAttribute(bcr_kernel(bw), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bcr_lds_bytes(bw)) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bcr_kernel(bw), kBcrNT, bcr_lds_bytes(bw)) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return cus * occ;
}
// Factorisation mode of a banded window: PLBA_FACTOR=bcr|cl|band forces one (diagnostics / A-B
// runs); by default block cyclic reduction once the window has enough super-rows for its
// log-depth chain to beat the two-sided column-lane chain of (nf+bw)/2 pivot steps. BCR only when
// its N workgroups fit the device at once (`resident`): a launch that cannot hold them all still
// completes (ticket order, plba_bcr.hpp) but serialises the levels it exists to overlap.
inline bool want_bcr(int bw, int nf, int resident) {
    if (bw < 1 || bw > kBcrMaxBW) return false;
    const int N = (nf + bw - 1) / bw;
    if (N < 2 || N > resident || bcr_lds_bytes(bw) > 159 * 1024) return false;
    const char *f = getenv("PLBA_FACTOR");
    if (f && f[0]) return std::string(f) == "bcr";
    // latency model calibrated on C3/C4/C5 (profiles/r02): the two-sided column-lane
    // chain costs ~1.3 µs per pivot block, (nf + bw)/2 of them; BCR ~(2.6·bw + 4.8) µs per level,
    // ceil(log2 N) + 1 levels. C3 (N = 13): 76 vs 116 µs -> column lane; C4 (N = 52): 230 vs
    // 157 µs and C5 (N = 129): 539 vs 198 µs -> BCR.
    int levels = 1;
    while ((1 << (levels - 1)) < N) ++levels;
    const double t_cl = 1.3 * (nf + bw) / 2.0, t_bcr = levels * (2.6 * bw + 4.8);
    return t_bcr < t_cl;
}
// Trial slots per step and when to use them (DESIGN §2 "Speculative trials"). PLBA_SPEC=<slots>
// and PLBA_SPEC_POLICY=<0 off | 1 always | 2 after a rejection in the iteration | 3 after the first
// rejection of the optimize() call> override (A/B runs; results are identical in every setting).
struct SpecChoice {
    int slots, policy;
};
// bcr_fit: how many BCR factorisations the device holds at once (resident workgroups / super-rows);
// trial slots of a BCR window run side by side only if they all fit (else the second slot's
// super-rows would wait for the first's to retire and the levels would serialise). A/B at C4
// (DESIGN §2): 1,551 -> 1,817 LM it/s (31 -> 22 steps per LBA); PLBA_SPEC_BCR=0 disables.
inline SpecChoice spec_choice(bool band1, bool wide, bool bcr, int bcr_fit, bool sharded, bool has_trials) {
    SpecChoice r{1, kSpecOff};
    if (sharded || !has_trials || !(band1 || bcr)) return r;
    int cap = kMaxSpec;
    if (bcr) {
        const char *b = getenv("PLBA_SPEC_BCR");
        if ((b && b[0] == '0') || bcr_fit < 2) return r;
        cap = std::min(cap, bcr_fit);
    }
    // wide bands (bw > 9: the register-window kernel, ≈0.5 ms a factorisation at C3R) take every
    // slot: C3R 21 -> 17 steps per LBA, 1,000 -> 1,194 LM it/s (2 / 3 / 4 slots); so do
    // BCR windows, as far as the device holds the slots' super-rows (C4: 4 fit, 22 -> 17 steps,
    // 1,822 -> 1,851 LM it/s); the column-lane windows keep two (C3: 3 slots 5,248 vs 5,304)
    r.slots = (wide || bcr) ? kMaxSpec : 2;
    r.policy = kSpecSticky;
    const char *e = getenv("PLBA_SPEC");
    if (e && e[0]) r.slots = std::max(1, std::min(atoi(e), kMaxSpec));
    r.slots = std::min(r.slots, cap);
    const char *p = getenv("PLBA_SPEC_POLICY");
    if (p && p[0]) r.policy = std::max(0, std::min(atoi(p), 3));
    if (r.policy == kSpecOff) r.slots = 1;
    if (r.slots == 1) r.policy = kSpecOff;
    return r;
}
// the banded factorisation's launch(es); the first failing launch's status is returned
inline hipError_t launch_band(Dev &d, hipStream_t s) {
    void *args[] = {&d};
    if (d.bcr) {  // forward elimination, then back substitution + pose update (plba_bcr.hpp)
        hipError_t e = hipLaunchKernel(bcr_kernel(d.bw), dim3(d.bcr_N, d.spec_max), dim3(kBcrNT), args, bcr_lds_bytes(d.bw), s);
        if (e != hipSuccess || d.bcr_fused) return e;
        return hipLaunchKernel(bcr_back_kernel(d.bw), dim3(d.bcr_N, d.spec_max), dim3(kBcrBackNT), args,
                               bcr_back_lds_bytes(d.bw), s);
    }
    if (d.cl) {
        const void *k = cl_kernel_impl(d.bw, d.twisted != 0, std::make_integer_sequence<int, kClMaxBW + 1>{});
        return hipLaunchKernel(k, dim3(d.twisted ? 2 : 1, d.spec_max), dim3(kClNT), args, cl_lds_bytes(d.bw, d.nf, d.twisted != 0), s);
    }
    if (d.twisted)
        return hipLaunchKernel(twisted_kernel(d.bw), dim3(2, d.spec_max), dim3(band_nt(d.bw)), args, twisted_lds_bytes(d.bw, d.nf), s);
    return hipLaunchKernel(band_kernel(d.bw), dim3(1, d.spec_max), dim3(band_nt(d.bw)), args, band_lds_bytes(d.bw, d.nf), s);
}

// time a launch when kernel timing is enabled
template <typename F>
int timed(plba_ctx *ctx, int kid, F &&launch) {
    hipEvent_t a = nullptr, b = nullptr;
    if (ctx->timing) {
        a = ctx->next_event();
        b = ctx->next_event();
        (void)hipEventRecord(a, ctx->stream);
    }
    (void)hipGetLastError();  // launch errors below belong to this launch only
    launch();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        ctx->set_error("kernel %s launch failed: %s", kKernelNames[kid], hipGetErrorString(e));
        return PLBA_E_DEVICE;
    }
    if (ctx->timing) {
        (void)hipEventRecord(b, ctx->stream);
        ctx->ev_used.push_back({kid, {a, b}});
    }
    return PLBA_OK;
}

#define LAUNCH(kid, ...)                                   \
    do {                                                   \
        int _rc = timed(ctx, kid, [&] { __VA_ARGS__; });   \
        if (_rc) return _rc;                               \
    } while (0)

int collect_timing(plba_ctx *ctx) {
    if (!ctx->timing) return PLBA_OK;
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    for (auto &u : ctx->ev_used) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, u.second.first, u.second.second);
        ctx->k_ms[u.first] += ms;
        ctx->k_n[u.first] += 1;
    }
    ctx->ev_used.clear();
    ctx->ev_next = 0;
    return PLBA_OK;
}


// ------------------------------------------------------------------ upload / structure prep
// Reverse Cuthill–McKee order of the free poses (hidx 0..nf-1) on the graph "two free poses
// observe a common landmark": BFS from a pseudo-peripheral vertex of each component, neighbours
// by increasing degree, then reversed. Returns rcm[i] = the hidx placed at position i.
std::vector<int32_t> rcm_from_adj(std::vector<std::vector<int32_t>> &adj);
// doubles of the download staging block before its byte outputs
inline size_t out_doubles(size_t n_kf, size_t n_pt, size_t n_ln, size_t E) { return n_kf * 12 + n_pt * 3 + n_ln * 4 + E; }
std::vector<int32_t> rcm_order(const plba_graph *g, const std::vector<int32_t> &kf_hidx, int nf) {
    // landmark -> free poses as a CSR (counting sort of the edges by landmark), then the coupling
    // graph as an nf x nf bit matrix: its rows are the sorted, duplicate-free adjacency lists
    const int np_ = g->n_pt, nl = np_ + g->n_ln;
    std::vector<int32_t> off(nl + 1, 0);
    for (int e = 0; e < g->n_ept; ++e) off[g->ept_lm[e] + 1] += kf_hidx[g->ept_kf[e]] >= 0;
    for (int e = 0; e < g->n_eln; ++e) off[np_ + g->eln_lm[e] + 1] += kf_hidx[g->eln_kf[e]] >= 0;
    for (int l = 0; l < nl; ++l) off[l + 1] += off[l];
    std::vector<int32_t> fill(off.begin(), off.end() - 1), hs(off[nl]);
    for (int e = 0; e < g->n_ept; ++e) {
        const int h = kf_hidx[g->ept_kf[e]];
        if (h >= 0) hs[fill[g->ept_lm[e]]++] = h;
    }
    for (int e = 0; e < g->n_eln; ++e) {
        const int h = kf_hidx[g->eln_kf[e]];
        if (h >= 0) hs[fill[np_ + g->eln_lm[e]]++] = h;
    }
    const size_t W = ((size_t)nf + 63) / 64;
    std::vector<uint64_t> bits((size_t)nf * W, 0);
    for (int l = 0; l < nl; ++l)
        for (int i = off[l]; i < off[l + 1]; ++i)
            for (int j = i + 1; j < off[l + 1]; ++j) {
                const int a = hs[i], b = hs[j];
                if (a == b) continue;
                bits[(size_t)a * W + b / 64] |= 1ull << (b % 64);
                bits[(size_t)b * W + a / 64] |= 1ull << (a % 64);
            }
    std::vector<std::vector<int32_t>> adj(nf);
    for (int h = 0; h < nf; ++h) {
        const uint64_t *row = bits.data() + (size_t)h * W;
        int cnt = 0;
        for (size_t w = 0; w < W; ++w) cnt += __builtin_popcountll(row[w]);
        adj[h].reserve(cnt);
        for (size_t w = 0; w < W; ++w)
            for (uint64_t m = row[w]; m; m &= m - 1) adj[h].push_back((int32_t)(w * 64 + __builtin_ctzll(m)));
    }
    return rcm_from_adj(adj);
}
// RCM of an undirected graph given as adjacency lists (duplicates allowed; sorted in place)
std::vector<int32_t> rcm_from_adj(std::vector<std::vector<int32_t>> &adj) {
    const int nf = (int)adj.size();
    std::vector<int32_t> deg(nf);
    for (int h = 0; h < nf; ++h) {
        auto &a = adj[h];
        std::sort(a.begin(), a.end());
        a.erase(std::unique(a.begin(), a.end()), a.end());
        deg[h] = (int32_t)a.size();
    }
    for (int h = 0; h < nf; ++h)
        std::stable_sort(adj[h].begin(), adj[h].end(), [&](int x, int y) { return deg[x] < deg[y]; });
    std::vector<int32_t> order;
    order.reserve(nf);
    std::vector<char> seen(nf, 0);
    auto bfs = [&](int root, std::vector<int32_t> &out) {  // returns the last level's min-degree vertex
        std::vector<int32_t> lev(nf, -1);
        out.clear();
        out.push_back(root);
        lev[root] = 0;
        for (size_t q = 0; q < out.size(); ++q)
            for (int v : adj[out[q]])
                if (lev[v] < 0) {
                    lev[v] = lev[out[q]] + 1;
                    out.push_back(v);
                }
        const int last = lev[out.back()];
        int best = out.back();
        for (int v : out)
            if (lev[v] == last && deg[v] < deg[best]) best = v;
        return std::make_pair(best, last);
    };
    std::vector<int32_t> comp;
    for (int s0 = 0; s0 < nf; ++s0) {
        if (seen[s0]) continue;
        // pseudo-peripheral start: repeat BFS from the far end while the depth grows
        int root = s0;
        auto r = bfs(root, comp);
        for (int it = 0; it < 8; ++it) {
            auto r2 = bfs(r.first, comp);
            if (r2.second <= r.second) break;
            root = r.first;
            r = r2;
        }
        bfs(root, comp);  // Cuthill–McKee order of this component (neighbours by degree)
        for (int v : comp) {
            seen[v] = 1;
            order.push_back(v);
        }
    }
    std::reverse(order.begin(), order.end());
    // refinement: a few passes of "sort by the mean position of self and neighbours" (a discrete
    // smoothing that straightens thick paths, where level-by-level orders give ~2x the band);
    // the narrowest order seen wins
    auto bandwidth = [&](const std::vector<int32_t> &ord) {
        std::vector<int32_t> p(nf);
        for (int i = 0; i < nf; ++i) p[ord[i]] = i;
        int w = 0;
        for (int h = 0; h < nf; ++h)
            for (int v : adj[h]) w = std::max(w, std::abs(p[h] - p[v]));
        return w;
    };
    std::vector<int32_t> best = order, cur = order, p(nf);
    int bw_best = bandwidth(best);
    for (int it = 0; it < 24 && bw_best > 0; ++it) {
        for (int i = 0; i < nf; ++i) p[cur[i]] = i;
        std::vector<double> key(nf);
        for (int h = 0; h < nf; ++h) {
            double s = p[h];
            for (int v : adj[h]) s += p[v];
            key[h] = s / (double)(adj[h].size() + 1);
        }
        std::stable_sort(cur.begin(), cur.end(), [&](int a, int b) { return key[a] < key[b]; });
        const int w = bandwidth(cur);
        if (w < bw_best) {
            bw_best = w;
            best = cur;
        }
    }
    return best;
}

int allreduce(plba_ctx *ctx, const double *send, double *recv, size_t n);
// Sharded windows: the RCS exchange. PLBA_SHARD_XCHG=allreduce restores the all-reduce of the
// whole partial system (A/B runs); the default all-gathers each rank's nonzero runs.
inline bool xchg_gather() {
    const char *e = getenv("PLBA_SHARD_XCHG");
    return !(e && std::string(e) == "allreduce");
}
int do_upload(plba_ctx *ctx, const plba_graph *g) {
    if (!g || g->n_kf < 0 || g->n_pt < 0 || g->n_ln < 0 || g->n_ept < 0 || g->n_eln < 0) {
        ctx->set_error("invalid graph sizes");
        return PLBA_E_INVALID;
    }
    if ((g->n_kf && (!g->kf_Tcw || !g->kf_fixed || !g->kf_id)) || (g->n_pt && (!g->pt_xyz || !g->pt_id)) ||
        (g->n_ln && (!g->ln_orth || !g->ln_id)) ||
        (g->n_ept && (!g->ept_lm || !g->ept_kf || !g->ept_obs || !g->ept_info)) ||
        (g->n_eln && (!g->eln_lm || !g->eln_kf || !g->eln_obs || !g->eln_info))) {
        ctx->set_error("null array in graph");
        return PLBA_E_INVALID;
    }
    // Window structure on the device (plba_build.hip: sorts / scans / scatters on the solver
    // stream) unless PLBA_HOST_BUILD=1 (the host build below, kept as the reference the device
    // build is tested against bit for bit, and for windows whose envelope needs the RCM order).
    const bool devb_wanted = g->n_kf > 0 && !env_flag("PLBA_HOST_BUILD");
    if (!devb_wanted) {  // (the device build validates the edges itself)
        for (int e = 0; e < g->n_ept; ++e)
            if (g->ept_lm[e] < 0 || g->ept_lm[e] >= g->n_pt || g->ept_kf[e] < 0 || g->ept_kf[e] >= g->n_kf) {
                ctx->set_error("point edge %d references a missing vertex", e);
                return PLBA_E_INVALID;
            }
        for (int e = 0; e < g->n_eln; ++e)
            if (g->eln_lm[e] < 0 || g->eln_lm[e] >= g->n_ln || g->eln_kf[e] < 0 || g->eln_kf[e] >= g->n_kf) {
                ctx->set_error("line edge %d references a missing vertex", e);
                return PLBA_E_INVALID;
            }
    }
    auto tmark = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        const auto t = std::chrono::steady_clock::now();
        if (env_flag("PLBA_TIMING"))
            fprintf(stderr, "[plba upload] %-24s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - tmark).count());
        tmark = t;
    };
    ctx->free_all();
    mark("free");
    const int n_kf = g->n_kf, n_pt_g = g->n_pt, n_ln_g = g->n_ln, Ep_g = g->n_ept, El_g = g->n_eln;
    const int R = ctx->comm.nranks, rank = ctx->comm.rank;
    ctx->n_kf = n_kf; ctx->n_pt = n_pt_g; ctx->n_ln = n_ln_g; ctx->Ep = Ep_g; ctx->El = El_g;

    std::vector<int32_t> lm_gpos, kf_hidx, first_blk, e_lm, e_kf, e_hidx, e_orig, e_gpos, lm_off, pe_off, pe_list;
    std::vector<double> e_obs, e_info;
    int n_pt = 0, n_ln = 0, Ep = 0, El = 0, nf = 0, bw = 0;
    WindowBuild wb;
    bool devb = false;
    if (devb_wanted) {
        // free poses by vertex id (buildIndexMapping) and the id rank of every keyframe
        std::vector<int32_t> korder(n_kf), kpos(n_kf);
        std::iota(korder.begin(), korder.end(), 0);
        std::stable_sort(korder.begin(), korder.end(), [&](int a, int b) { return g->kf_id[a] < g->kf_id[b]; });
        kf_hidx.assign(n_kf, -1);
        for (int i = 0; i < n_kf; ++i) {
            kpos[korder[i]] = i;
            if (!g->kf_fixed[korder[i]]) kf_hidx[korder[i]] = nf++;
        }
        wb.g = g;
        wb.nranks = R;
        wb.rank = rank;
        wb.nf = nf;
        wb.kf_hidx = kf_hidx.data();
        wb.kpos = kpos.data();
        wb.stream = ctx->stream;
        char msg[256] = {0};
        const int brc = build_stage1(ctx->bmemA, wb, msg, sizeof msg);
        if (brc) {
            ctx->set_error("%s", msg);
            return brc;
        }
        first_blk = wb.first_blk;
        for (int h = 0; h < nf; ++h) bw = std::max(bw, h - first_blk[h]);
        // an envelope the banded kernels cannot take may narrow under the RCM order (the host
        // build's rule, same permutation: rcm_order over the whole graph): build again with the
        // reordered free poses, kept when the envelope narrows, else built once more in id order
        if (bw > kClMaxBW && nf > 2 && !env_flag("PLBA_NO_RCM")) {
            const std::vector<int32_t> rcm = rcm_order(g, kf_hidx, nf);
            std::vector<int32_t> pos(nf), h2(n_kf, -1);
            for (int i = 0; i < nf; ++i) pos[rcm[i]] = i;
            for (int k = 0; k < n_kf; ++k) h2[k] = kf_hidx[k] >= 0 ? pos[kf_hidx[k]] : -1;
            wb.kf_hidx = h2.data();
            int brc2 = build_stage1(ctx->bmemA, wb, msg, sizeof msg);
            int bw2 = 0;
            for (int h = 0; h < nf && !brc2; ++h) bw2 = std::max(bw2, h - wb.first_blk[h]);
            if (!brc2 && bw2 < bw) {
                kf_hidx = h2;
                wb.kf_hidx = kf_hidx.data();  // (h2 dies with this block)
                first_blk = wb.first_blk;
                bw = bw2;
            } else {
                wb.kf_hidx = kf_hidx.data();
                if (!brc2) brc2 = build_stage1(ctx->bmemA, wb, msg, sizeof msg);
            }
            if (brc2) {
                ctx->set_error("%s", msg);
                return brc2;
            }
            mark("device build (RCM order)");
        }
        devb = true;
        mark("device build (stage 1 proper)");
        if (devb) {
            n_pt = wb.n_pt; n_ln = wb.n_ln; Ep = wb.Ep; El = wb.El;
            ctx->n_free_edges = wb.n_free_edges;
            // host mirrors of the output maps (plba_download / plba_get_edge_chi2)
            lm_gpos.resize(wb.n_lm);
            e_orig.resize(wb.E);
            if (wb.n_lm)
                PLBA_CHECK(hipMemcpyAsync(lm_gpos.data(), wb.lm_gpos, sizeof(int32_t) * wb.n_lm, hipMemcpyDeviceToHost, ctx->stream));
            if (wb.E)
                PLBA_CHECK(hipMemcpyAsync(e_orig.data(), wb.e_orig, sizeof(int32_t) * wb.E, hipMemcpyDeviceToHost, ctx->stream));
            PLBA_CHECK(hipStreamSynchronize(ctx->stream));
            ctx->lm_gpos = lm_gpos;
            ctx->e_orig = e_orig;
            ctx->h_level.assign(wb.E, 0);
        } else {
            bw = 0;
            nf = 0;
        }
        mark("device build (stage 1)");
    }
    ctx->dev_build = devb ? 1 : 0;
    if (!devb) {
    // landmarks owned by this rank (all of them unless the window is sharded)
    std::vector<int32_t> pt_owner(n_pt_g, 0), ln_owner(n_ln_g, 0);
    if (R > 1) shard_plan(g, R, pt_owner.data(), ln_owner.data());
    // Local landmark order: points then lines, each sorted (stably) by the id rank of the
    // keyframe of their first observation, so the edges of one pose — and the landmarks one RCS
    // block couples — sit in a narrow range of the landmark-major edge array (cache locality of
    // the pose reduction and the Schur assembly; any order gives the same solution).
    std::vector<int32_t> pt_loc(n_pt_g, -1), ln_loc(n_ln_g, -1);
    lm_gpos.clear();
    {
        std::vector<int32_t> korder_(n_kf), kpos(n_kf);
        std::iota(korder_.begin(), korder_.end(), 0);
        std::stable_sort(korder_.begin(), korder_.end(), [&](int a, int b) { return g->kf_id[a] < g->kf_id[b]; });
        for (int i = 0; i < n_kf; ++i) kpos[korder_[i]] = i;
        std::vector<int32_t> key_pt(n_pt_g, INT32_MAX), key_ln(n_ln_g, INT32_MAX);
        for (int e = Ep_g - 1; e >= 0; --e) key_pt[g->ept_lm[e]] = kpos[g->ept_kf[e]];
        for (int e = El_g - 1; e >= 0; --e) key_ln[g->eln_lm[e]] = kpos[g->eln_kf[e]];
        // stable counting sort by key (key in [0, n_kf], n_kf = never observed)
        auto order = [&](int n, const std::vector<int32_t> &own, const std::vector<int32_t> &key,
                         std::vector<int32_t> &loc, int &cnt, int gbase) {
            std::vector<int32_t> c(n_kf + 2, 0);
            for (int i = 0; i < n; ++i)
                if (own[i] == rank) c[std::min(key[i], n_kf) + 1]++;
            for (int k = 0; k <= n_kf; ++k) c[k + 1] += c[k];
            const int base = (int)lm_gpos.size();
            lm_gpos.resize(base + c[n_kf + 1]);
            for (int i = 0; i < n; ++i)
                if (own[i] == rank) {
                    const int pos = c[std::min(key[i], n_kf)]++;
                    loc[i] = pos;
                    lm_gpos[base + pos] = gbase + i;
                }
            cnt = (int)lm_gpos.size() - base;
        };
        order(n_pt_g, pt_owner, key_pt, pt_loc, n_pt, 0);
        order(n_ln_g, ln_owner, key_ln, ln_loc, n_ln, n_pt_g);
    }
    ctx->lm_gpos = lm_gpos;
    for (int e = 0; e < Ep_g; ++e) Ep += pt_loc[g->ept_lm[e]] >= 0;
    for (int e = 0; e < El_g; ++e) El += ln_loc[g->eln_lm[e]] >= 0;
    const int n_lm = n_pt + n_ln, E = Ep + El;

    // free poses ordered by vertex id (buildIndexMapping)
    std::vector<int32_t> korder(n_kf);
    std::iota(korder.begin(), korder.end(), 0);
    std::stable_sort(korder.begin(), korder.end(), [&](int a, int b) { return g->kf_id[a] < g->kf_id[b]; });
    kf_hidx.assign(n_kf, -1);
    for (int k : korder)
        if (!g->kf_fixed[k]) kf_hidx[k] = nf++;
    first_blk.assign(nf, 0);
    auto envelope = [&](const std::vector<int32_t> &hidx, std::vector<int32_t> &fb) {
        for (int h = 0; h < nf; ++h) fb[h] = h;
        std::vector<int32_t> lmin(n_pt_g + n_ln_g, INT32_MAX);
        for (int e = 0; e < Ep_g; ++e) {
            const int h = hidx[g->ept_kf[e]];
            if (h >= 0) lmin[g->ept_lm[e]] = std::min(lmin[g->ept_lm[e]], h);
        }
        for (int e = 0; e < El_g; ++e) {
            const int h = hidx[g->eln_kf[e]];
            if (h >= 0) lmin[n_pt_g + g->eln_lm[e]] = std::min(lmin[n_pt_g + g->eln_lm[e]], h);
        }
        for (int e = 0; e < Ep_g; ++e) {
            const int h = hidx[g->ept_kf[e]];
            if (h >= 0) fb[h] = std::min(fb[h], lmin[g->ept_lm[e]]);
        }
        for (int e = 0; e < El_g; ++e) {
            const int h = hidx[g->eln_kf[e]];
            if (h >= 0) fb[h] = std::min(fb[h], lmin[n_pt_g + g->eln_lm[e]]);
        }
        int w = 0;
        for (int h = 0; h < nf; ++h) w = std::max(w, h - fb[h]);
        return w;
    };
    bw = envelope(kf_hidx, first_blk);
    // Reverse Cuthill–McKee on the free-pose coupling graph when the natural (id) order leaves an
    // envelope wider than the column-lane / BCR kernels take: windows that revisit old keyframes
    // couple poses a loop apart. LinearSolverEigen orders the same matrix by AMD; any symmetric
    // permutation gives the same exact LDLᵀ solution (rounding aside). PLBA_NO_RCM=1 disables.
    if (bw > kClMaxBW && nf > 2 && !env_flag("PLBA_NO_RCM")) {
        std::vector<int32_t> rcm = rcm_order(g, kf_hidx, nf);
        std::vector<int32_t> pos(nf), h2(n_kf, -1), fb2(nf);
        for (int i = 0; i < nf; ++i) pos[rcm[i]] = i;
        for (int k = 0; k < n_kf; ++k) h2[k] = kf_hidx[k] >= 0 ? pos[kf_hidx[k]] : -1;
        const int bw2 = envelope(h2, fb2);
        if (bw2 < bw) {
            kf_hidx = h2;
            first_blk = fb2;
            bw = bw2;
        }
    }
    mark("envelope (+ RCM)");

    // landmark-major CSR of the local landmarks (stable within a landmark = g2o insertion order)
    std::vector<int32_t> lm_cnt(n_lm + 1, 0);
    for (int e = 0; e < Ep_g; ++e)
        if (pt_loc[g->ept_lm[e]] >= 0) lm_cnt[pt_loc[g->ept_lm[e]] + 1]++;
    for (int e = 0; e < El_g; ++e)
        if (ln_loc[g->eln_lm[e]] >= 0) lm_cnt[n_pt + ln_loc[g->eln_lm[e]] + 1]++;
    lm_off.assign(n_lm + 1, 0);
    for (int l = 0; l < n_lm; ++l) lm_off[l + 1] = lm_off[l] + lm_cnt[l + 1];
    std::vector<int32_t> fill(lm_off.begin(), lm_off.end() - 1);
    e_lm.assign(E, 0); e_kf.assign(E, 0); e_hidx.assign(E, 0); e_orig.assign(E, 0); e_gpos.assign(E, 0);
    e_obs.assign((size_t)E * 4, 0.0); e_info.assign(E, 0.0);
    for (int e = 0; e < Ep_g; ++e) {
        const int l = pt_loc[g->ept_lm[e]];
        if (l < 0) continue;
        const int pos = fill[l]++;
        e_lm[pos] = l;
        e_kf[pos] = g->ept_kf[e];
        e_orig[pos] = e;
        e_gpos[pos] = e;
        e_obs[(size_t)pos * 4] = g->ept_obs[2 * e];
        e_obs[(size_t)pos * 4 + 1] = g->ept_obs[2 * e + 1];
        e_info[pos] = g->ept_info[e];
    }
    for (int e = 0; e < El_g; ++e) {
        if (ln_loc[g->eln_lm[e]] < 0) continue;
        const int l = n_pt + ln_loc[g->eln_lm[e]], pos = fill[l]++;
        e_lm[pos] = l;
        e_kf[pos] = g->eln_kf[e];
        e_orig[pos] = e;
        e_gpos[pos] = Ep_g + e;
        for (int k = 0; k < 4; ++k) e_obs[(size_t)pos * 4 + k] = g->eln_obs[4 * e + k];
        e_info[pos] = g->eln_info[e];
    }
    for (int e = 0; e < E; ++e) e_hidx[e] = kf_hidx[e_kf[e]];
    ctx->n_free_edges = std::count_if(e_hidx.begin(), e_hidx.end(), [](int32_t h) { return h >= 0; });
    ctx->e_orig = e_orig;
    ctx->h_level.assign(E, 0);

    mark("landmark order + CSR");
    // free-pose-major edge lists (ascending CSR edge index)
    pe_off.assign(nf + 1, 0);
    for (int e = 0; e < E; ++e)
        if (e_hidx[e] >= 0) pe_off[e_hidx[e] + 1]++;
    for (int h = 0; h < nf; ++h) pe_off[h + 1] += pe_off[h];
    pe_list.assign(pe_off[nf], 0);
    {
        std::vector<int32_t> f(pe_off.begin(), pe_off.end() - 1);
        for (int e = 0; e < E; ++e)
            if (e_hidx[e] >= 0) pe_list[f[e_hidx[e]]++] = e;
    }
    }  // host build
    const int n_lm = n_pt + n_ln, E = Ep + El;

    // Reduced-camera block pattern: the envelope of the lower triangle. first_blk[i2] = the lowest
    // free pose sharing a landmark with free pose i2, over the WHOLE window on every rank (the
    // all-reduced value array must have one layout). Blocks are indexed densely within the
    // envelope in (i2, i1) order; Schur triples (e1 at pose i1 <= e2 at pose i2, same landmark,
    // local landmarks only) are counting-sorted by block, landmark order inside a block.
    // PLBA_FORCE_DENSE=1 (diagnostics only) routes a narrow envelope through the dense path.
    const char *force_dense = getenv("PLBA_FORCE_DENSE");
    const bool band_mode = bw <= kBandMax && !(force_dense && force_dense[0] == '1');
    std::vector<int64_t> blk_base(nf + 1, 0);
    for (int h = 0; h < nf; ++h) blk_base[h + 1] = blk_base[h] + (h - first_blk[h] + 1);
    if (blk_base[nf] > INT32_MAX / 64) {
        ctx->set_error("reduced camera envelope too large (%lld blocks)", (long long)blk_base[nf]);
        return PLBA_E_INVALID;
    }
    const int nblk = (int)blk_base[nf];
    std::vector<int32_t> blk_i1(nblk), blk_i2(nblk), blk_off(nblk + 1, 0), trip;
    for (int h = 0; h < nf; ++h)
        for (int i1 = first_blk[h]; i1 <= h; ++i1) {
            const int b = (int)(blk_base[h] + (i1 - first_blk[h]));
            blk_i1[b] = i1;
            blk_i2[b] = h;
        }
    if (devb) {  // device build, stage 2: Schur triples sorted by block on the device
        char msg[256] = {0};
        const int brc = build_stage2(ctx->bmemA, ctx->bmemB, wb, blk_base, nblk, msg, sizeof msg);
        if (brc) {
            ctx->set_error("%s", msg);
            return brc;
        }
        blk_off = wb.h_blk_off;
        ctx->n_triples = (size_t)wb.n_triples;
    } else {
        auto for_pairs = [&](auto &&f) {
            for (int l = 0; l < n_lm; ++l)
                for (int a = lm_off[l]; a < lm_off[l + 1]; ++a) {
                    const int i1 = e_hidx[a];
                    if (i1 < 0) continue;
                    for (int b = lm_off[l]; b < lm_off[l + 1]; ++b) {
                        const int i2 = e_hidx[b];
                        if (i2 < i1) continue;
                        f(a, b, (int)(blk_base[i2] + (i1 - first_blk[i2])));
                    }
                }
        };
        for_pairs([&](int, int, int blk) { blk_off[blk + 1]++; });
        for (int k = 0; k < nblk; ++k) blk_off[k + 1] += blk_off[k];
        trip.resize(2 * (size_t)blk_off[nblk]);
        std::vector<int32_t> pos(blk_off.begin(), blk_off.end() - 1);
        for_pairs([&](int a, int b, int blk) {
            const size_t t = (size_t)pos[blk]++;
            trip[2 * t] = a;
            trip[2 * t + 1] = b;
        });
        ctx->n_triples = (size_t)blk_off[nblk];
    }
    mark("blocks + triples");
    // chunks of <= chunk triples, never spanning two blocks
    // (at least one chunk per block, possibly empty: the last chunk of a block to finish
    // assembles it, so every envelope block — zero ones included — is written each trial).
    // Windows up to 600 k triples take half-size chunks: twice the waves, each half as long, the
    // assembly being one round of waves there (C3: 25.5 -> 23.9 µs; C5 keeps 256: 115.3 vs 117.9);
    // PLBA_CHUNK_TRIPLES overrides (<= kChunk)
    int chunk = ctx->n_triples <= 600000 ? kChunk / 2 : kChunk;
    if (const char *ce = getenv("PLBA_CHUNK_TRIPLES")) chunk = std::max(1, std::min(atoi(ce), kChunk));
    std::vector<int32_t> ch_blk, ch_off, blk_ch(nblk + 1, 0);
    for (int k = 0; k < nblk; ++k) {
        blk_ch[k] = (int32_t)ch_blk.size();
        int t = blk_off[k];
        do {
            ch_blk.push_back(k);
            ch_off.push_back(t);
            t += chunk;
        } while (t < blk_off[k + 1]);
    }
    blk_ch[nblk] = (int32_t)ch_blk.size();
    ch_off.push_back(blk_off[nblk]);
    const int nch = (int)ch_blk.size();
    // envelope of the lower triangle (per 6-row pose block: first pose block column)
    const int n = 6 * nf;
    const int ntiles = (n + kTile - 1) / kTile;
    std::vector<int32_t> tile_first(std::max(ntiles, 1), 0), tile_last(std::max(ntiles, 1), 0);
    for (int I = 0; I < ntiles; ++I) {
        int f = I;
        for (int r = I * kTile; r < std::min(n, (I + 1) * kTile); ++r) f = std::min(f, (6 * first_blk[r / 6]) / kTile);
        tile_first[I] = f;
    }
    for (int K = 0; K < ntiles; ++K) {
        int last = K;
        for (int I = K; I < ntiles; ++I)
            if (tile_first[I] <= K) last = I;
        tile_last[K] = last;
    }
    ctx->h_tile_last = tile_last;

    mark("chunks + envelope");
    // ---- device allocation
    Dev &d = ctx->d;
    d.n_kf = n_kf; d.n_pt = n_pt; d.n_ln = n_ln; d.n_lm = n_lm; d.Ep = Ep; d.El = El; d.E = E;
    d.nf = nf; d.n = n; d.nblk = nblk; d.ntiles = ntiles;
    // any transport selects the sharded code path (a 1-rank RCCL window exercises it on one GPU)
    const bool sharded = ctx->comm.kind != plba_ctx::Comm::NONE;
    d.sharded = sharded ? 1 : 0;
    d.nranks = R;
    d.rank = rank;
    d.n_lm_g = n_pt_g + n_ln_g;
    d.E_g = Ep_g + El_g;
    d.bw = bw;
    d.band_mode = band_mode ? 1 : 0;
    // dense RCS: multi-workgroup blocked LDLᵀ with MFMA trailing updates; PLBA_DENSE_SCALAR=1
    // selects the single-workgroup scalar k_rcs_factor (A/B runs)
    d.dense_mfma = !band_mode && !env_flag("PLBA_DENSE_SCALAR") ? 1 : 0;
    d.ring = band_ring(bw, nf);
    // two-sided factorisation when the chain is long enough to halve and the separator's dense
    // system fits next to the band window in LDS (PLBA_NO_TWIST=1 disables, diagnostics only)
    const char *no_twist = getenv("PLBA_NO_TWIST");
    const int bcr_res = band_mode && !ctx->no_bcr ? bcr_resident(ctx->opts.device, bw) : 0;
    const bool bcr = band_mode && !ctx->no_bcr && want_bcr(bw, nf, bcr_res);
    d.bcr = bcr ? 1 : 0;
    d.bcr_N = bcr ? (nf + bw - 1) / bw : 0;
    // BCR back substitution inside the forward launch (PLBA_BCR_SPLIT=1: the second launch)
    d.bcr_fused = bcr && !env_flag("PLBA_BCR_SPLIT") ? 1 : 0;
    const bool cl = band_mode && !bcr && use_cl(bw);
    const bool twisted = band_mode && !bcr && bw >= 1 && nf >= 2 * bw + 16 &&
                         (cl ? cl_lds_bytes(bw, nf, true) : twisted_lds_bytes(bw, nf) + band_static_bytes(bw)) <= 159 * 1024 &&
                         !(no_twist && no_twist[0] == '1');
    // the column-lane factorisation a BCR window falls back to (run_schedule) and its arrays
    // (the same checks as the normal column-lane choice; without it, the one-sweep band kernel)
    static_assert(kBcrMaxBW <= kClMaxBW, "a BCR window must be able to fall back to the column-lane kernel");
    const bool fb_cl = bcr && use_cl(bw) && cl_lds_bytes(bw, nf, false) <= 159 * 1024;
    const bool fb_tw = fb_cl && nf >= 2 * bw + 16 && cl_lds_bytes(bw, nf, true) <= 159 * 1024 &&
                       !(no_twist && no_twist[0] == '1');
    ctx->fb_cl = fb_cl ? 1 : 0;
    ctx->fb_twisted = fb_tw ? 1 : 0;
    ctx->fb_tw_m = fb_tw ? tw_split(nf, bw) : 0;
    d.cl = cl && cl_lds_bytes(bw, nf, twisted) <= 159 * 1024 ? 1 : 0;
    d.twisted = twisted ? 1 : 0;
    d.tw_m = twisted ? tw_split(nf, bw) : 0;
    d.corrected = ctx->opts.corrected_line_jacobian;
    // Speculative trials: worth it where the step is bound by the serial factorisation
    // chain and the rest of the chip idles during it — the banded one- or two-workgroup
    // factorisations (column-lane, LDS window) and BCR windows whose slots' super-rows all fit the device at once;
    // the extra slots' edge and landmark kernels are then the price. Not for the dense path or
    // sharded windows (collectives per slot).
    {
        const SpecChoice sp = spec_choice(band_mode && !bcr, band_mode && !bcr && !d.cl, bcr, bcr ? bcr_res / std::max(d.bcr_N, 1) : 0, sharded,
                                          n_lm > 0 && nch > 0);
        d.spec_max = sp.slots;
        d.spec_policy = sp.policy;
        d.nbs = d.spec_max + 1;
        d.nbx = d.spec_max > 1 ? d.spec_max + 1 : 1;
    }
    {  // timing experiments only (wrong results): PLBA_DIAG bit mask read by some kernels
        const char *dg = getenv("PLBA_DIAG");
        d.diag = dg ? atoi(dg) : 0;
    }
    d.solve_lds_n = solve_lds_limit();
    d.cam = Cam{g->fx, g->fy, g->cx, g->cy};
    d.huber_pt = g->huber_pt;
    d.huber_ln = g->huber_ln;
    d.tau = ctx->opts.tau;
    d.n_lin_blocks = blocks_for(E);
    d.n_lm_blocks = blocks_for(n_lm, kLmBlock);
    d.n_lms_blocks = blocks_for(n_lm * kLmLanes, kLmsNT);
    d.n_kf_blocks = blocks_for(n_kf);

    std::vector<double> T(g->kf_Tcw, g->kf_Tcw + (size_t)n_kf * 12), X;
    if (!devb) {
        X.assign((size_t)n_lm * 4, 0.0);
        for (int p = 0; p < n_pt; ++p)
            for (int k = 0; k < 3; ++k) X[(size_t)p * 4 + k] = g->pt_xyz[3 * (size_t)lm_gpos[p] + k];
        for (int l = 0; l < n_ln; ++l)
            for (int k = 0; k < 4; ++k)
                X[(size_t)(n_pt + l) * 4 + k] = g->ln_orth[4 * (size_t)(lm_gpos[n_pt + l] - n_pt_g) + k];
    }

    // sharded, all-gather exchange: this rank's block-row range [lo, hi] (rows of the blocks that
    // hold one of its Schur triples — every local edge of a free pose has its diagonal triple), as
    // two runs of red_rcs; every rank's runs are exchanged here, so all ranks size the same record
    std::vector<int64_t> xg_rng;
    int64_t xg_P = 0;
    if (sharded && nblk > 0 && xchg_gather()) {
        int lo = nf, hi = -1;
        for (int b = 0; b < nblk; ++b)
            if (blk_off[b + 1] > blk_off[b]) {
                lo = std::min(lo, blk_i2[b]);
                hi = std::max(hi, blk_i2[b]);
            }
        std::vector<double> mine(4 * (size_t)R, 0.0);
        if (hi >= lo) {
            mine[4 * rank + 0] = (double)(blk_base[lo] * 36);
            mine[4 * rank + 1] = (double)((blk_base[hi + 1] - blk_base[lo]) * 36);
            mine[4 * rank + 2] = (double)((int64_t)nblk * 36 + 6 * (int64_t)lo);
            mine[4 * rank + 3] = (double)(6 * (int64_t)(hi - lo + 1));
        }
        double *tmp = nullptr;
        PLBA_CHECK(hipMallocAsync((void **)&tmp, mine.size() * sizeof(double), ctx->stream));
        PLBA_CHECK(hipMemcpyAsync(tmp, mine.data(), mine.size() * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
        int xrc = allreduce(ctx, tmp, tmp, mine.size());
        if (!xrc) {
            xrc = hipMemcpyAsync(mine.data(), tmp, mine.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream) ==
                          hipSuccess && hipStreamSynchronize(ctx->stream) == hipSuccess
                      ? PLBA_OK : PLBA_E_DEVICE;
        }
        (void)hipFreeAsync(tmp, ctx->stream);
        if (xrc) {
            if (xrc == PLBA_E_DEVICE) ctx->set_error("shard range exchange: device copy failed");
            return xrc;
        }
        xg_rng.resize(4 * (size_t)R);
        for (int r = 0; r < R; ++r) {
            for (int k = 0; k < 4; ++k) xg_rng[4 * r + k] = (int64_t)mine[4 * r + k];
            xg_P = std::max(xg_P, xg_rng[4 * r + 1] + xg_rng[4 * r + 3]);
        }
        xg_P = std::max<int64_t>(xg_P, 2);
    }
    std::vector<int32_t> h_kf(bcr ? nf : 0, 0);
    for (int k = 0; k < n_kf && bcr; ++k)
        if (kf_hidx[k] >= 0) h_kf[kf_hidx[k]] = k;
    // every device array of the window, carved from the arena (commit_plan assigns the pointers)
#define ALLOC(p, n_) ctx->alloc(p, (size_t)(n_))
#define ZALLOC(p, n_) ctx->alloc(p, (size_t)(n_), nullptr, true)
#define UPLOAD(p, v) ctx->alloc(p, (v).size(), (v).data())
// host vector (host build) or the device build's array of n_ elements
#define UPLOAD_D(p, v, dptr, n_)                           \
    do {                                                  \
        if (devb) ctx->alloc_dev(p, (size_t)(n_), (dptr)); \
        else UPLOAD(p, v);                                \
    } while (0)
    const int nbs = d.nbs, nbx = d.nbx, W = d.spec_max;
    UPLOAD(d.T_init, T);
    UPLOAD(d.Tb[0], T);
    for (int b = 1; b < nbs; ++b) ALLOC(d.Tb[b], T.size());
    UPLOAD_D(d.X_init, X, wb.X, (size_t)n_lm * 4);
    UPLOAD_D(d.Xb[0], X, wb.X, (size_t)n_lm * 4);
    for (int b = 1; b < nbs; ++b) ALLOC(d.Xb[b], (size_t)n_lm * 4);
    for (int b = 0; b < nbs; ++b) ALLOC(d.xk[b], (size_t)n_kf * 6);
    // hand-rolled GBA: endpoint lines in the reference's (global) order, their 6x6 blocks
    for (int b = 0; b < nbs; ++b) ALLOC(d.XL[b], (size_t)std::max(n_ln_g, 1) * 6);
    ALLOC(d.Hl6, (size_t)std::max(n_ln, 1) * 21);
    ALLOC(d.bl6, (size_t)std::max(n_ln, 1) * 6);
    std::vector<int32_t> ln_gidx(std::max(n_ln, 1), 0);
    for (int i = 0; i < n_ln; ++i) ln_gidx[i] = lm_gpos[n_pt + i] - n_pt_g;
    UPLOAD(d.ln_gidx, ln_gidx);
    for (int b = 0; b < nbs; ++b) ALLOC(d.Lpb[b], (size_t)std::max(n_ln, 1) * 8);
    UPLOAD(d.kf_hidx, kf_hidx);
    UPLOAD_D(d.e_lm, e_lm, wb.e_lm, E);
    UPLOAD_D(d.e_kf, e_kf, wb.e_kf, E);
    UPLOAD_D(d.e_hidx, e_hidx, wb.e_hidx, E);
    UPLOAD_D(d.e_obs, e_obs, wb.e_obs, (size_t)E * 4);
    UPLOAD_D(d.e_info, e_info, wb.e_info, E);
    ZALLOC(d.e_level, E);
    ALLOC(d.e_active, E);
    UPLOAD_D(d.lm_off, lm_off, wb.lm_off, n_lm + 1);
    ALLOC(d.lm_active, n_lm);
    UPLOAD_D(d.pe_off, pe_off, wb.pe_off, nf + 1);
    UPLOAD_D(d.pe_list, pe_list, wb.pe_list, ctx->n_free_edges);
    ALLOC(d.A, (size_t)E * 12);
    ALLOC(d.cvec, (size_t)E * 2);
    ALLOC(d.B, (size_t)E * 8);
    for (int b = 0; b < nbx; ++b) ZALLOC(d.chi2b[b], E);
    // Hpp | b_p | #active edges | χ² | active | landmark max per rank: one array, all-reduced when sharded
    // unsharded: Hpp | b_p | active | χ² | any | max; sharded: diag(Hpp) | b_p | active | χ² | any |
    // per-rank maxima, all-reduced (the full partial Hpp stays local: Hpp_w)
    ALLOC(d.red_iter, (size_t)nf * (sharded ? 13 : 43) + 2 + R);
    if (sharded) {
        ALLOC(d.red_iter_loc, (size_t)nf * 13 + 2 + R);
        ALLOC(d.Hpp_w, (size_t)nf * 36);
    }
    ALLOC(d.Hll, (size_t)n_lm * 10);
    ALLOC(d.bl, (size_t)n_lm * 4);
    // λ-dependent arrays: one copy per trial slot, back to back (slot_view, sl_* in plba_kernels.hpp)
    ALLOC(d.Z, (size_t)W * E * 8);
    ALLOC(d.q, (size_t)W * E * 2);
    for (int b = 0; b < nbx; ++b) ZALLOC(d.xlb[b], (size_t)n_lm * 4);
    UPLOAD(d.blk_i1, blk_i1);
    UPLOAD(d.blk_i2, blk_i2);
    UPLOAD(d.blk_off, blk_off);
    UPLOAD_D(d.trip, trip, wb.trip, 2 * (size_t)ctx->n_triples);
    d.nch = nch;
    UPLOAD(d.ch_blk, ch_blk);
    UPLOAD(d.ch_off, ch_off);
    UPLOAD(d.blk_ch, blk_ch);
    d.nch = nch;  // (sl_chp)
    ALLOC(d.ch_part, (size_t)W * sl_chp(d));
    ALLOC(d.Ad, band_mode ? 1 : (size_t)n * n);
    UPLOAD(d.first_blk, first_blk);
    // band blocks outside the envelope (w > i - first_blk[i]) are never assembled and must
    // read as zero: the band kernels sweep all BW block columns of every row
    ZALLOC(d.Bd, (size_t)W * sl_band(d));
    ALLOC(d.Lband, (size_t)W * sl_band(d));
    ALLOC(d.Kinv, (size_t)W * nf * 36);
    ALLOC(d.zb, (size_t)W * nf * 6);
    if (twisted || fb_tw) {
        ZALLOC(d.Bd2, (size_t)W * sl_tw(d));
        ALLOC(d.bs2, (size_t)W * nf * 6);
        ALLOC(d.Lband2, (size_t)W * sl_tw(d));
        ALLOC(d.Kinv2, (size_t)W * nf * 36);
        ALLOC(d.zb2, (size_t)W * nf * 6);
        ALLOC(d.tw_sep, (size_t)W * sl_sep(d));
        ZALLOC(d.tw_fail, 2 * (size_t)W);
        ZALLOC(d.tw_count, (size_t)W);
    }
    if (bcr) {  // flags carry epochs from bcr_ctl[0]: start from a clean slate (one set per trial slot)
        const int64_t N = d.bcr_N;
        d.bcr_sl[0] = N * (int64_t)bcr_pub_doubles(bw);
        d.bcr_sl[1] = N * (int64_t)bcr_xrec(bw);
        d.bcr_sl[2] = N * (int64_t)bcr_X_doubles(bw);
        d.bcr_sl[3] = 2 * N;
        d.bcr_sl[4] = kBcrCtl;
        d.bcr_sl[5] = N * (int64_t)kBcrStamps;
        ALLOC(d.bcr_pub, (size_t)W * d.bcr_sl[0]);
        ALLOC(d.bcr_x, (size_t)W * d.bcr_sl[1]);
        ALLOC(d.bcr_X, (size_t)W * d.bcr_sl[2]);

        UPLOAD(d.h_kf, h_kf);
        ZALLOC(d.bcr_flag, (size_t)W * d.bcr_sl[3]);
        ZALLOC(d.bcr_ctl, (size_t)W * kBcrCtl);
        ZALLOC(d.bcr_stamps, (size_t)W * d.bcr_sl[5]);
        // the schedule's starting state, restored if a hand-off wait times out (run_schedule)
        ctx->alloc(ctx->bk_T, (size_t)n_kf * 12);
        ctx->alloc(ctx->bk_X, (size_t)std::max(n_lm, 1) * 4);
        ctx->alloc(ctx->bk_xp, (size_t)std::max(n, 6));
        ctx->alloc(ctx->bk_xk, (size_t)n_kf * 6);
        ctx->alloc(ctx->bk_Lpb, (size_t)std::max(n_ln, 1) * 8);
        ctx->alloc(ctx->bk_XL, (size_t)std::max(n_ln_g, 1) * 6);
        ctx->alloc(ctx->bk_level, (size_t)std::max(E, 1));
        ctx->alloc(ctx->bk_xl, (size_t)std::max(n_lm, 1) * 4);
    }
    if (!band_mode) ZALLOC(d.bcr_stamps, kBcrStamps);  // dense-path phase stamps (PLBA_DIAG bit 8)
    ALLOC(d.bs, (size_t)W * n);
    // k_lm_solve reads x_p[6·max(h, 0) ..] for fixed-pose slots too
    for (int b = 0; b < nbx; ++b) ZALLOC(d.xpb[b], std::max(n, 6));
    ALLOC(d.Wbuf, (size_t)std::max(n, 1) * (kTile + 1));  // W panel + y of the dense path
    UPLOAD(d.tile_first, tile_first);
    UPLOAD(d.tile_last, tile_last);
    ALLOC(d.part_chi2, d.n_lin_blocks);
    ALLOC(d.part_any, d.n_lm_blocks);
    ALLOC(d.part_max, nf + d.n_lm_blocks);
    ALLOC(d.pose_part, (size_t)std::max(nf, 1) * kPoseParts * kPP);
    ALLOC(d.part_lm, (size_t)W * sl_lms(d));
    ALLOC(d.part_lms, (size_t)W * sl_lms(d));
    d.fold = sharded ? 0 : 1;
    d.fold_init = d.fold && !getenv("PLBA_NO_FOLD_INIT");
    // arrival counters: lm_solve, iter_reduce (top), RCS blocks, poses, iter_reduce groups
    const int nred = kPoseParts * nf + (d.n_lm > 0 ? d.n_lm_blocks : 0), ngrp = (nred + kRedGrp - 1) / kRedGrp;
    ZALLOC(d.cnt, 2 + (size_t)nblk + nf + ngrp);
    ZALLOC(d.cnt_rcs, (size_t)W * nblk);  // per trial slot: arrivals per RCS block
    ALLOC(d.wg_red, 3 * (size_t)std::max(nred, 1));
    ALLOC(d.grp_red, 3 * (size_t)std::max(ngrp, 1));
    d.n_ps = std::max(d.n_kf_blocks, d.bcr_N);
    ZALLOC(d.part_ps, (size_t)W * d.n_ps);
    ZALLOC(d.ctrl, 1);
    ALLOC(d.trace, kTraceCap);
    ALLOC(ctx->d_depth, Ep);
    ALLOC(d.red_rcs, (size_t)nblk * 36 + (size_t)nf * 6);
    ALLOC(d.red_dec, 3);
    if (sharded) {
        ALLOC(d.red_rcs_loc, (size_t)nblk * 36 + (size_t)nf * 6);
        ALLOC(d.red_dec_loc, 4);  // + the hand-off error agreement slot (agree_dev_error)
    }
    d.xg_P = 0;
    d.xg_host = ctx->comm.kind == plba_ctx::Comm::HOST ? 1 : 0;
    if (sharded && xg_rng.size()) {
        d.xg_P = xg_P;
        UPLOAD(d.xg_rng, xg_rng);
        // zeroed once: blockpart rewrites the same in-run positions every step, the padding (and,
        // host transport, the other ranks' slots) stays zero
        ZALLOC(d.xg_send, (size_t)(d.xg_host ? R : 1) * xg_P);
        ALLOC(d.xg_recv, (size_t)R * xg_P);
    }
    // output maps (local landmark / edge -> whole-window position): the download scatter
    // (k_out_scatter) or, sharded, the final gather of the full window X | χ² | depth | level
    UPLOAD_D(d.lm_gpos, lm_gpos, wb.lm_gpos, n_lm);
    UPLOAD_D(d.e_gpos, e_gpos, wb.e_gpos, E);
    if (sharded) {
        ALLOC(d.gat, (size_t)(n_pt_g + n_ln_g) * 4 + 3 * (size_t)(Ep_g + El_g));
    } else {
        // one staging block: Tcw | pt_xyz | ln_orth | χ² (doubles), then the byte outputs
        ALLOC(ctx->d_outd, out_doubles(n_kf, n_pt, n_ln, E) + ((size_t)Ep + E + 7) / 8);
    }
#if defined(PLBA_STAMPS) || defined(PLBA_PHASE_STAMPS) || defined(PLBA_LMS_STAMPS)
    ZALLOC(d.stamps, 17 * 8);
#endif
#undef ALLOC
#undef ZALLOC
#undef UPLOAD
#undef UPLOAD_D
    mark("host arrays staged");
    int rc = ctx->commit_plan();
    if (rc) return rc;
    // slot 0's buffers for the kernels that never run speculatively (one χ² / solve buffer then)
    d.xp = d.xpb[0];
    d.xl = d.xlb[0];
    d.chi2_last = d.chi2b[0];
    if (sharded) {
        d.Hpp = nullptr;
        d.Hdg = d.red_iter;
        d.bp = d.red_iter + (size_t)nf * 6;
        d.pact = d.red_iter + (size_t)nf * 12;
        d.Hdg_w = d.red_iter_loc;
        d.bp_w = d.red_iter_loc + (size_t)nf * 6;
        d.pact_w = d.red_iter_loc + (size_t)nf * 12;
    } else {
        d.Hpp = d.red_iter;
        d.bp = d.red_iter + (size_t)nf * 36;
        d.pact = d.red_iter + (size_t)nf * 42;
        d.red_iter_loc = d.red_iter;
        d.Hpp_w = d.red_iter_loc;
        d.bp_w = d.red_iter_loc + (size_t)nf * 36;
        d.pact_w = d.red_iter_loc + (size_t)nf * 42;
        d.Hdg = d.Hdg_w = nullptr;
    }
    if (band_mode) PLBA_CHECK(hipFuncSetAttribute(band_kernel(bw), hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  (int)band_lds_bytes(bw, nf)));
    if (bcr) {
        PLBA_CHECK(hipFuncSetAttribute(bcr_kernel(bw), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bcr_lds_bytes(bw)));
        PLBA_CHECK(hipFuncSetAttribute(bcr_back_kernel(bw), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)bcr_back_lds_bytes(bw)));
        if (fb_tw) {
            const void *k = cl_kernel_impl(bw, true, std::make_integer_sequence<int, kClMaxBW + 1>{});
            PLBA_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cl_lds_bytes(bw, nf, true)));
        } else {
            const void *k = cl_kernel_impl(bw, false, std::make_integer_sequence<int, kClMaxBW + 1>{});
            PLBA_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cl_lds_bytes(bw, nf, false)));
        }
    }
    if (d.cl) {  // the column-lane kernel's LDS grows with nf (x_p staging of the two-sided variant)
        const void *k = cl_kernel_impl(bw, twisted, std::make_integer_sequence<int, kClMaxBW + 1>{});
        PLBA_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cl_lds_bytes(bw, nf, twisted)));
    }
    if (twisted)
        PLBA_CHECK(hipFuncSetAttribute(twisted_kernel(bw), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)twisted_lds_bytes(bw, nf)));
    mark("alloc + copy + memset");
    ctx->uploaded = true;
    ctx->initialized = false;
    ctx->cur = ctx->last_ok = ctx->chi_src = 0;
    return PLBA_OK;
}

// One "step": [stage switch] -> [iteration: linearise + reductions + λ init] -> one damped
// trial -> decide -> commit. Every kernel is guarded by the device control block, so a fixed
// sequence can be captured once and replayed; steps after the schedule finished are no-ops.
// Sum of n doubles over the ranks of a sharded window: send (this rank's partials) -> recv.
// Device -> host read on the context's own stream. Never the legacy stream (plain hipMemcpy):
// while another context of the process captures its step graphs (first batch of a new window),
// a legacy-stream copy is refused and invalidates that capture.
hipError_t d2h(plba_ctx *ctx, void *dst, const void *src, size_t bytes) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
    return e == hipSuccess ? hipStreamSynchronize(ctx->stream) : e;
}
int allreduce(plba_ctx *ctx, const double *send, double *recv, size_t n) {
    auto &c = ctx->comm;
    if (n == 0) return PLBA_OK;
    if (c.kind == plba_ctx::Comm::RCCL) {
        const ncclResult_t r = ncclAllReduce(send, recv, n, ncclDouble, ncclSum, c.nccl, ctx->stream);
        if (r != ncclSuccess) {
            ctx->set_error("ncclAllReduce(%zu doubles): %s", n, ncclGetErrorString(r));
            return PLBA_E_COMM;
        }
        return PLBA_OK;
    }
    if (c.kind == plba_ctx::Comm::HOST) {
        if (c.hcap < n) {
            PLBA_CHECK(hipStreamSynchronize(ctx->stream));
            ctx->retire_pinned(c.hbuf);
            c.hbuf = nullptr;
            PLBA_CHECK(hipHostMalloc((void **)&c.hbuf, n * sizeof(double), hipHostMallocDefault));
            c.hcap = n;
        }
        PLBA_CHECK(hipMemcpyAsync(c.hbuf, send, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        PLBA_CHECK(hipStreamSynchronize(ctx->stream));
        const int rc = c.fn(c.user, c.hbuf, (int64_t)n);
        if (rc) {
            ctx->set_error("host all-reduce callback returned %d", rc);
            return PLBA_E_COMM;
        }
        PLBA_CHECK(hipMemcpyAsync(recv, c.hbuf, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
        return PLBA_OK;
    }
    ctx->set_error("sharded window without a transport");
    return PLBA_E_COMM;
}
// All-gather of P doubles per rank: recv = [rank 0's P | rank 1's P | ...]. The host transport
// only sums, so there each rank's send is its own slot of an R x P array, zero elsewhere.
int allgather(plba_ctx *ctx, const double *send, double *recv, size_t P) {
    auto &c = ctx->comm;
    if (P == 0) return PLBA_OK;
    if (c.kind == plba_ctx::Comm::RCCL) {
        const ncclResult_t r = ncclAllGather(send, recv, P, ncclDouble, c.nccl, ctx->stream);
        if (r != ncclSuccess) {
            ctx->set_error("ncclAllGather(%zu doubles): %s", P, ncclGetErrorString(r));
            return PLBA_E_COMM;
        }
        return PLBA_OK;
    }
    return allreduce(ctx, send, recv, (size_t)c.nranks * P);
}
#define COMM(send, recv, n)                                                        \
    do {                                                                           \
        int _crc = 0;                                                              \
        LAUNCH(K_COMM, _crc = allreduce(ctx, (send), (recv), (size_t)(n)));        \
        if (_crc) return _crc;                                                     \
    } while (0)

// Schur assembly with two lanes per triple (k_rcs_chunk_h) once a slot's chunk waves exceed what
// k_rcs_chunk keeps resident (1.75 waves per SIMD x 1024 SIMDs) — per slot, so that the choice
// (and the rounding) does not depend on the trial-slot count; PLBA_CHUNK_HALF_MIN overrides the
// threshold (0: always, a huge value: never)
bool chunk_half(const Dev &d) {
    const char *e = getenv("PLBA_CHUNK_HALF_MIN");  // (read per capture: tests switch it)
    const long long thr = e ? atoll(e) : 1792LL;
    return (long long)d.nch > thr;
}
int launch_step(plba_ctx *ctx) {
    Dev &d = ctx->d;
    hipStream_t s = ctx->stream;
    // PLBA_CHUNK_DIRECT=1: per-lane A/Z row loads in the Schur assembly (A/B of the staged copy)
    const bool chunk_direct = getenv("PLBA_CHUNK_DIRECT") != nullptr;  // (read per capture: tests switch it)

    if (d.E > 0) LAUNCH(K_LINEARIZE, hipLaunchKernelGGL(k_linearize, dim3(d.n_lin_blocks), dim3(kBlock), 0, s, d));
    if (d.nf > 0 || d.n_lm > 0) {
        const int nred = kPoseParts * d.nf + (d.n_lm > 0 ? d.n_lm_blocks : 0);
        LAUNCH(K_REDUCE, hipLaunchKernelGGL(k_iter_reduce, dim3(nred), dim3(kLmBlock), 0, s, d));
    }
    if (d.sharded) {
        LAUNCH(K_PACK, hipLaunchKernelGGL(k_iter_pack, dim3(1), dim3(kInitNT), 0, s, d));
        COMM(d.red_iter_loc, d.red_iter, (size_t)d.nf * 13 + 2 + d.nranks);
    }
    const bool reduced = d.nf > 0 || d.n_lm > 0;
    if (!(d.fold_init && reduced))  // (folded into the last k_iter_reduce workgroup otherwise)
        LAUNCH(K_ITER_INIT, hipLaunchKernelGGL(k_iter_init, dim3(1), dim3(kInitNT), 0, s, d));
    if (d.n_lm > 0) {
        LAUNCH(K_ESCHUR, hipLaunchKernelGGL(k_edge_schur, dim3(d.n_lin_blocks, d.spec_max), dim3(kBlock), 0, s, d));
    }
    if (d.n > 0) {
        if (!d.band_mode) LAUNCH(K_MEMSET, (void)hipMemsetAsync(d.Ad, 0, sizeof(double) * (size_t)d.n * d.n, s));
        if (d.nch > 0) LAUNCH(K_ASSEMBLE, hipLaunchKernelGGL(chunk_direct ? k_rcs_chunk<false> : chunk_half(d) ? k_rcs_chunk_h : k_rcs_chunk<true>, dim3(8 * ((d.nch + 7) / 8), d.spec_max), dim3(64), 0, s, d));
        if (d.sharded) {
            LAUNCH(K_PACK, hipLaunchKernelGGL(k_rcs_blockpart, dim3(blocks_for(d.nblk * 42)), dim3(kBlock), 0, s, d));
            if (d.xg_P > 0) {  // all-gather of every rank's nonzero runs, summed in rank order
                int grc = 0;
                LAUNCH(K_COMM, grc = allgather(ctx, d.xg_send, d.xg_recv, (size_t)d.xg_P));
                if (grc) return grc;
                LAUNCH(K_FINALIZE, hipLaunchKernelGGL(k_rcs_xunpack, dim3(blocks_for(d.nblk * 36 + d.nf * 6)), dim3(kBlock), 0, s, d));
            } else {
                COMM(d.red_rcs_loc, d.red_rcs, (size_t)d.nblk * 36 + (size_t)d.nf * 6);
            }
        }
        if (!(d.fold && d.nch > 0))  // (folded into the last chunk of each block otherwise)
            LAUNCH(K_FINALIZE, hipLaunchKernelGGL(k_rcs_finalize, dim3(blocks_for(d.nblk * 42)), dim3(kBlock), 0, s, d));
        const size_t solve_lds = d.n <= d.solve_lds_n ? sizeof(double) * (size_t)d.n : 0;  // y of dense_solve_wg
        if (d.band_mode) {
            hipError_t fe = hipSuccess;
            LAUNCH(K_FACTOR, fe = launch_band(d, s));
            if (fe != hipSuccess) {
                (void)hipGetLastError();
                ctx->set_error("factorisation launch failed: %s", hipGetErrorString(fe));
                return PLBA_E_DEVICE;
            }
        } else if (d.dense_mfma) {  // blocked LDLᵀ, MFMA trailing updates (plba_dense.hpp)
            for (int K = 0; K < d.ntiles; ++K) {  // the envelope's row tiles K..tile_last[K] only
                const int m = ctx->h_tile_last[K] - K;
                LAUNCH(K_DENSE_PANEL, hipLaunchKernelGGL(k_dense_panel, dim3((m + 2) / 2), dim3(kDensePanelNT), 0, s, d, K));
                if (m > 0)
                    LAUNCH(K_DENSE_UPDATE, hipLaunchKernelGGL(k_dense_update, dim3(m * (m + 1) / 2), dim3(64), 0, s, d, K));
            }
            LAUNCH(K_FACTOR, hipLaunchKernelGGL(k_dense_solve, dim3(1), dim3(kFacThreads), solve_lds, s, d));
        } else {
            LAUNCH(K_FACTOR, hipLaunchKernelGGL(k_rcs_factor, dim3(1), dim3(kFacThreads), solve_lds, s, d));
        }
    }
    // the factorisation kernels end with the pose update; without free poses it runs alone
    if (d.n == 0 && d.n_kf > 0) LAUNCH(K_POSE_UPDATE, hipLaunchKernelGGL(k_pose_update, dim3(1), dim3(kBlock), 0, s, d));
    if (d.n_lm > 0) {
        LAUNCH(K_LM_UPDATE, hipLaunchKernelGGL(k_lm_solve, dim3(d.n_lms_blocks, d.spec_max), dim3(kLmsNT), 0, s, d));
    }
    if (d.sharded) {
        LAUNCH(K_PACK, hipLaunchKernelGGL(k_decide_pack, dim3(1), dim3(kBlock), 0, s, d));
        COMM(d.red_dec_loc, d.red_dec, 3);
    }
    if (!(d.fold && d.n_lm > 0))  // (folded into the last k_lm_solve workgroup otherwise)
        LAUNCH(K_DECIDE, hipLaunchKernelGGL(k_decide, dim3(1), dim3(kBlock), 0, s, d));
    return PLBA_OK;
}

void destroy_graphs(plba_ctx *ctx) {
    if (ctx->step_exec) (void)hipGraphExecDestroy(ctx->step_exec);
    if (ctx->step_graph) (void)hipGraphDestroy(ctx->step_graph);
    ctx->step_exec = nullptr;
    ctx->step_graph = nullptr;
    for (int i = 0; i < plba_ctx::kMultiLevels; ++i) {
        if (ctx->multi_exec[i]) (void)hipGraphExecDestroy(ctx->multi_exec[i]);
        if (ctx->multi_graph[i]) (void)hipGraphDestroy(ctx->multi_graph[i]);
        ctx->multi_exec[i] = nullptr;
        ctx->multi_graph[i] = nullptr;
    }
}

int capture_steps(plba_ctx *ctx, int nsteps, hipGraph_t &graph, hipGraphExec_t &exec) {
    const bool t = ctx->timing;
    ctx->timing = false;
    PLBA_CHECK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    int rc = 0;
    for (int i = 0; i < nsteps && !rc; ++i) rc = launch_step(ctx);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    ctx->timing = t;
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess) {
        ctx->set_error("graph capture failed: %s", hipGetErrorString(e));
        return PLBA_E_DEVICE;
    }
    if (exec) {  // a previous window's executable graph: update it in place when the topology matches
        hipGraphNode_t bad = nullptr;
        hipGraphExecUpdateResult res = hipGraphExecUpdateSuccess;
        if (hipGraphExecUpdate(exec, g, &bad, &res) == hipSuccess && res == hipGraphExecUpdateSuccess) {
            if (graph) (void)hipGraphDestroy(graph);
            graph = g;
            return PLBA_OK;
        }
        (void)hipGetLastError();
        (void)hipGraphExecDestroy(exec);
        exec = nullptr;
    }
    if (graph) (void)hipGraphDestroy(graph);
    graph = g;
    PLBA_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    return PLBA_OK;
}
// Which kernels (template instances) a step launches, in which order: an executable graph is
// updated in place only for a window with the same signature (hipGraphExecUpdate changes kernel
// arguments and grids, never the kernel a node runs).
// multi-step graphs captured: 2, 4, .. 2^L steps (PLBA_GRAPH_LEVELS overrides, for measurements)
int graph_levels() {  // (read per capture: tests switch it)
    const char *e = getenv("PLBA_GRAPH_LEVELS");
    return e ? std::max(0, std::min(atoi(e), (int)plba_ctx::kMultiLevels)) : (int)plba_ctx::kMultiLevels;
}
std::vector<int64_t> launch_signature(const plba_ctx *ctx) {
    const Dev &d = ctx->d;
    return {d.E > 0, d.nf > 0, d.n_lm > 0, d.n > 0, d.nch > 0, d.band_mode, d.dense_mfma, d.dense_mfma ? d.ntiles : 0,
            d.bw, d.bcr, d.bcr_fused, d.cl, d.twisted, d.sharded, d.xg_P, d.fold, d.fold_init, d.n_kf > 0, d.spec_max,
            (int64_t)(getenv("PLBA_CHUNK_DIRECT") != nullptr), (int64_t)chunk_half(d), (int64_t)ctx->comm.kind};
}
int capture_step(plba_ctx *ctx) {
    if (ctx->step_exec && !ctx->graphs_stale) return PLBA_OK;
    ctx->graphs_stale = false;
    const std::vector<int64_t> sig = launch_signature(ctx);
    if (ctx->step_exec && sig != ctx->graph_sig) destroy_graphs(ctx);  // different kernels: rebuild
    ctx->graph_sig = sig;
    const auto t0 = std::chrono::steady_clock::now();
    int rc = capture_steps(ctx, 1, ctx->step_graph, ctx->step_exec);
    for (int i = 0; i < graph_levels() && !rc; ++i)
        rc = capture_steps(ctx, 2 << i, ctx->multi_graph[i], ctx->multi_exec[i]);
    if (env_flag("PLBA_TIMING"))
        fprintf(stderr, "[plba upload] %-24s %8.3f ms\n", "graph capture",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return rc;
}
// launch n replays of the step as the binary decomposition of n over the captured graphs
int launch_steps_graph(plba_ctx *ctx, int n) {
    const int L = graph_levels();
    if (L == 0) {
        for (int i = 0; i < n; ++i) PLBA_CHECK(hipGraphLaunch(ctx->step_exec, ctx->stream));
        return PLBA_OK;
    }
    while (n >= (2 << (L - 1))) {
        PLBA_CHECK(hipGraphLaunch(ctx->multi_exec[L - 1], ctx->stream));
        n -= 2 << (L - 1);
    }
    for (int i = L - 1; i >= 0; --i)
        if (n & (2 << i)) PLBA_CHECK(hipGraphLaunch(ctx->multi_exec[i], ctx->stream));
    if (n & 1) PLBA_CHECK(hipGraphLaunch(ctx->step_exec, ctx->stream));
    return PLBA_OK;
}

int read_ctrl(plba_ctx *ctx) {
    PLBA_CHECK(hipMemcpyAsync(ctx->h_ctrl, ctx->d.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, ctx->stream));
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    return PLBA_OK;
}


// Copies of the state a schedule starts from (BCR windows only): save = true before the first
// batch, save = false to put it back after a hand-off timeout.
int bcr_state_copy(plba_ctx *ctx, bool save) {
    Dev &d = ctx->d;
    const int c = ctx->cur;
    hipStream_t s = ctx->stream;
    auto cp = [&](void *bk, void *live, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        return save ? hipMemcpyAsync(bk, live, bytes, hipMemcpyDeviceToDevice, s)
                    : hipMemcpyAsync(live, bk, bytes, hipMemcpyDeviceToDevice, s);
    };
    PLBA_CHECK(cp(ctx->bk_T, d.Tb[c], sizeof(double) * (size_t)d.n_kf * 12));
    PLBA_CHECK(cp(ctx->bk_X, d.Xb[c], sizeof(double) * (size_t)d.n_lm * 4));
    PLBA_CHECK(cp(ctx->bk_xp, d.xp, sizeof(double) * (size_t)d.n));
    PLBA_CHECK(cp(ctx->bk_xk, d.xk[c], sizeof(double) * (size_t)d.n_kf * 6));
    PLBA_CHECK(cp(ctx->bk_Lpb, d.Lpb[c], sizeof(double) * (size_t)d.n_ln * 8));
    PLBA_CHECK(cp(ctx->bk_XL, d.XL[c], sizeof(double) * (size_t)ctx->n_ln * 6));
    PLBA_CHECK(cp(ctx->bk_level, d.e_level, (size_t)d.E));
    PLBA_CHECK(cp(ctx->bk_xl, d.xl, sizeof(double) * (size_t)d.n_lm * 4));
    return PLBA_OK;
}

// Sharded windows: every rank learns whether any rank hit a hand-off timeout in this batch, so
// that all of them fall back together (a collective cannot be re-run by one rank alone).
int agree_dev_error(plba_ctx *ctx, int mine, int *any) {
    *any = mine;
    if (!ctx->d.sharded) return PLBA_OK;
    double *buf = ctx->d.red_dec_loc + 3;  // spare slot after the three decision terms
    const double v = mine ? 1.0 : 0.0;
    PLBA_CHECK(hipMemcpyAsync(buf, &v, sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    int rc = allreduce(ctx, buf, buf, 1);
    if (rc) return rc;
    double out = 0.0;
    PLBA_CHECK(hipMemcpyAsync(&out, buf, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    *any = out != 0.0 ? 1 : 0;
    return PLBA_OK;
}

// Run a schedule of 1 or 2 optimize() calls entirely on the device: replay the step graph in
// batches, polling the control block once per batch.
// every launch outside the step graphs is checked where it is issued (the graph launches are
// checked by LAUNCH / launch_band)
#define PLBA_LAUNCHED(ctx_, name_)                                                        \
    do {                                                                                  \
        const hipError_t le_ = hipGetLastError();                                         \
        if (le_ != hipSuccess) {                                                          \
            (ctx_)->set_error("kernel %s launch failed: %s", name_, hipGetErrorString(le_)); \
            return PLBA_E_DEVICE;                                                         \
        }                                                                                 \
    } while (0)
int run_schedule_once(plba_ctx *ctx, const Ctrl &init, bool &dev_error) {
    dev_error = false;
    Dev &d = ctx->d;
    *ctx->h_ctrl = init;
    PLBA_CHECK(hipMemcpyAsync(d.ctrl, ctx->h_ctrl, sizeof(Ctrl), hipMemcpyHostToDevice, ctx->stream));
    if (d.n_ln > 0 && !init.hlm) {  // Plücker vectors of the current line states (read by k_linearize;
                                     // the hand-rolled LM starts from the map's NDw, uploaded instead)
        hipLaunchKernelGGL(k_line_pluker, dim3(blocks_for(d.n_ln)), dim3(kBlock), 0, ctx->stream, d); PLBA_LAUNCHED(ctx, "k_line_pluker");
        PLBA_CHECK(hipGetLastError());
    }
    // the host transport synchronises inside the step: no graph then
    bool use_graph = !ctx->timing && ctx->comm.kind != plba_ctx::Comm::HOST && !ctx->no_graph;
    // A new window's step graphs are captured (or updated) on the host while the device runs the
    // first batch, launched directly: the capture leaves the end-to-end call's critical path.
    bool capture_pending = use_graph && (!ctx->step_exec || ctx->graphs_stale);
    auto capture_now = [&]() -> int {
        capture_pending = false;
        int rc = capture_step(ctx);
        if (rc) {
            // a step that cannot be captured (collectives that refuse stream capture, graph
            // instantiation failing for lack of memory): the first batch is already running as
            // direct launches, so keep launching that way for the rest of this context's life
            (void)hipGetLastError();
            destroy_graphs(ctx);
            ctx->no_graph = true;
            use_graph = false;
            if (ctx->opts.verbose) fprintf(stderr, "[plba] step capture failed (%s); direct launches\n", ctx->err.c_str());
            ctx->err.clear();
        }
        return PLBA_OK;
    };
    int launched = 0;
    int batch = std::max(4, ctx->last_steps);
    const bool tlog = env_flag("PLBA_TIMING");
    auto tb0 = std::chrono::steady_clock::now();
    const int max_steps = init.n_stages * 10 * (init.max_iters[0] + init.max_iters[1] + 2) + 8;
    for (;;) {
        if (use_graph && !capture_pending) {
            int rc = launch_steps_graph(ctx, batch);
            if (rc) return rc;
        } else {
            for (int b = 0; b < batch; ++b) {
                int rc = launch_step(ctx);
                if (rc) return rc;
            }
            if (capture_pending)
                if (int rc = capture_now()) return rc;
        }
        launched += batch;
        int rc = read_ctrl(ctx);
        if (rc) return rc;
        if (tlog) {
            const auto tb1 = std::chrono::steady_clock::now();
            fprintf(stderr, "[plba schedule] batch of %3d steps (%3d so far, device step %3d) %8.3f ms\n", batch, launched,
                    ctx->h_ctrl->steps, std::chrono::duration<double, std::milli>(tb1 - tb0).count());
            tb0 = tb1;
        }
        int any_error = ctx->h_ctrl->dev_error;
        if (d.sharded && d.bcr && (rc = agree_dev_error(ctx, any_error, &any_error))) return rc;
        if (any_error) {
            dev_error = true;
            ctx->set_error("a bounded in-kernel hand-off wait timed out");
            return PLBA_E_DEVICE;
        }
        if (ctx->h_ctrl->all_done) break;
        if (launched >= max_steps) {
            ctx->set_error("LM schedule did not terminate after %d steps", launched);
            return PLBA_E_STATE;
        }
        // steps still needed: at least one per remaining trial; keep batches small near the end
        batch = 4;
    }
    ctx->steps_launched = launched;
    ctx->last_steps = std::max(4, ctx->h_ctrl->steps + 1);
    ctx->cur = ctx->h_ctrl->cur;
    ctx->last_ok = ctx->h_ctrl->last_ok;
    ctx->chi_src = ctx->h_ctrl->chi_src;
    // per-iteration trace written by k_decide
    const int nt = std::min(ctx->h_ctrl->ntrace, kTraceCap);
    std::vector<plba_iter_trace> tr(nt);
    if (nt) PLBA_CHECK(d2h(ctx, tr.data(), d.trace, sizeof(plba_iter_trace) * nt));
    ctx->trace.insert(ctx->trace.end(), tr.begin(), tr.end());
    return PLBA_OK;
}

// run_schedule_once with the BCR safety net: the starting state is copied first; if a hand-off
// wait times out (Ctrl::dev_error — every later kernel of that batch is a no-op), the state is put
// back, the window is switched to the column-lane factorisation for the rest of this context's
// life (its arrays were allocated with the BCR ones) and the same schedule runs again, in this
// process. Sharded windows agree on the error first, so every rank falls back together.
int run_schedule(plba_ctx *ctx, const Ctrl &init) {
    Dev &d = ctx->d;
    int rc;
    if (d.bcr && (rc = bcr_state_copy(ctx, true))) return rc;
    bool dev_error = false;
    rc = run_schedule_once(ctx, init, dev_error);
    if (!rc || !dev_error || !d.bcr) return rc;
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    if ((rc = bcr_state_copy(ctx, false))) return rc;
    if (ctx->opts.verbose)
        fprintf(stderr, "[plba] BCR hand-off timed out; re-solving with the column-lane factorisation\n");
    destroy_graphs(ctx);
    d.bcr = 0;
    d.bcr_N = 0;
    d.cl = ctx->fb_cl;
    d.twisted = ctx->fb_twisted;
    d.tw_m = ctx->fb_tw_m;
    ctx->no_bcr = true;
    ++ctx->bcr_fallbacks;
    ctx->err.clear();
    rc = run_schedule_once(ctx, init, dev_error);
    return rc;
}

Ctrl schedule_init(plba_ctx *ctx, int n_stages) {
    Ctrl c{};
    c.stage = -1;
    c.n_stages = n_stages;
    c.switch_pending = 1;
    c.solve_ok[0] = 1;
    c.max_trials = ctx->opts.max_trials;
    c.cur = ctx->cur;
    c.last_ok = ctx->last_ok;
    c.chi_src = ctx->chi_src;
    c.spec_w = 1;
    return c;
}

int do_optimize(plba_ctx *ctx, int iterations, int32_t *iters_done, double *final_chi2) {
    Ctrl c = schedule_init(ctx, 1);
    c.max_iters[0] = iterations;
    c.stage_robust[0] = ctx->robust;
    c.stage_level[0] = ctx->level;
    c.stage_classify[0] = 0;
    if (iterations <= 0) {
        if (iters_done) *iters_done = 0;
        if (final_chi2) *final_chi2 = 0.0;
        return PLBA_OK;
    }
    int rc = run_schedule(ctx, c);
    if (rc) return rc;
    if (iters_done) *iters_done = ctx->h_ctrl->iters_done[0];
    if (final_chi2) *final_chi2 = ctx->h_ctrl->chi2_final[0];
    return PLBA_OK;
}

int launch_edges(plba_ctx *ctx, void (*k)(Dev, int), int arg) {
    if (ctx->d.E > 0) hipLaunchKernelGGL(k, dim3(blocks_for(ctx->d.E)), dim3(kBlock), 0, ctx->stream, ctx->d, arg); PLBA_LAUNCHED(ctx, "edge kernel");
    PLBA_CHECK(hipGetLastError());
    return PLBA_OK;
}

// Sharded windows: whole-window landmark states and per-edge outputs on every rank
// (one all-reduce of a zero-filled, scattered buffer). Collective: all ranks call it.
int gather_outputs(plba_ctx *ctx, std::vector<double> &out) {
    Dev &d = ctx->d;
    const size_t n = (size_t)d.n_lm_g * 4 + 3 * (size_t)d.E_g;
    PLBA_CHECK(hipMemsetAsync(d.gat, 0, n * sizeof(double), ctx->stream));
    if (d.Ep) hipLaunchKernelGGL(k_depth, dim3(blocks_for(d.Ep)), dim3(kBlock), 0, ctx->stream, d, ctx->d_depth); PLBA_LAUNCHED(ctx, "k_depth");
    const int m = std::max(d.n_lm, d.E);
    if (m) hipLaunchKernelGGL(k_gather, dim3(blocks_for(m)), dim3(kBlock), 0, ctx->stream, d, ctx->d_depth); PLBA_LAUNCHED(ctx, "k_gather");
    PLBA_CHECK(hipGetLastError());
    int rc = allreduce(ctx, d.gat, d.gat, n);
    if (rc) return rc;
    out.resize(n);
    PLBA_CHECK(hipMemcpyAsync(out.data(), d.gat, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    return PLBA_OK;
}

// Unsharded windows: every requested output in the caller's order, scattered on the device
// (k_out_scatter) into one staging block, one copy into pinned memory, one synchronisation, then
// host copies into the caller's arrays.
int download_outputs(plba_ctx *ctx, double *kf_Tcw, double *pt_xyz, double *ln_orth, double *ept_chi2,
                     uint8_t *ept_depth_ok, double *eln_chi2, uint8_t *ept_level, uint8_t *eln_level) {
    Dev &d = ctx->d;
    hipStream_t s = ctx->stream;
    const size_t nk = (size_t)d.n_kf, np = (size_t)d.n_pt, nl = (size_t)d.n_ln, Ep = (size_t)d.Ep, El = (size_t)d.El;
    const size_t nd = out_doubles(nk, np, nl, Ep + El), bytes = nd * sizeof(double) + Ep + (Ep + El);
    const int m = std::max({d.n_lm, d.E, d.n_kf});
    const bool any = kf_Tcw || pt_xyz || ln_orth || ept_chi2 || ept_depth_ok || eln_chi2 || ept_level || eln_level;
    if (!m || !any) return PLBA_OK;
    if (bytes > ctx->h_out_cap) {  // grow-only, with slack: the next windows of a session are similar
        PLBA_CHECK(hipStreamSynchronize(ctx->stream));
        ctx->retire_pinned(ctx->h_out);
        ctx->h_out = nullptr;
        ctx->h_out_cap = 0;
        const size_t cap = bytes + bytes / 2;
        PLBA_CHECK(hipHostMalloc((void **)&ctx->h_out, cap));
        ctx->h_out_cap = cap;
    }
    hipLaunchKernelGGL(k_out_scatter, dim3(blocks_for(m)), dim3(kBlock), 0, s, d, ctx->d_outd, ept_depth_ok ? 1 : 0,
                       ctx->cur, ctx->chi_src); PLBA_LAUNCHED(ctx, "k_out_scatter");
    PLBA_CHECK(hipGetLastError());
    PLBA_CHECK(hipMemcpyAsync(ctx->h_out, ctx->d_outd, bytes, hipMemcpyDeviceToHost, s));
    PLBA_CHECK(hipStreamSynchronize(s));
    const double *od = reinterpret_cast<const double *>(ctx->h_out);
    const uint8_t *ob = reinterpret_cast<const uint8_t *>(od + nd);
    auto put = [](void *dst, const void *src, size_t b) {
        if (dst && b) std::memcpy(dst, src, b);
    };
    put(kf_Tcw, od, sizeof(double) * nk * 12);
    put(pt_xyz, od + nk * 12, sizeof(double) * np * 3);
    put(ln_orth, od + nk * 12 + np * 3, sizeof(double) * nl * 4);
    put(ept_chi2, od + nk * 12 + np * 3 + nl * 4, sizeof(double) * Ep);
    put(eln_chi2, od + nk * 12 + np * 3 + nl * 4 + Ep, sizeof(double) * El);
    put(ept_depth_ok, ob, Ep);
    put(ept_level, ob + Ep, Ep);
    put(eln_level, ob + 2 * Ep, El);
    return PLBA_OK;
}

}  // namespace

// ==================================================================================== C ABI
extern "C" {

void plba_default_opts(plba_opts *o) {
    if (!o) return;
    o->device = 0;
    o->corrected_line_jacobian = 0;
    o->verbose = 0;
    o->max_trials = 10;
    o->tau = 1e-5;
}

// The device's default memory pool is process-wide: its release threshold is raised while at
// least one context of the device lives and the value found before the first one is put back when
// the last one is destroyed (other users of the pool in the process see their own setting again).
void pool_hold(plba_ctx *ctx, bool on) {
    static std::mutex mu;
    static std::map<int, std::pair<int, uint64_t>> held;  // device -> (contexts holding, previous threshold)
    if (ctx->pool_hold == on) return;
    std::lock_guard<std::mutex> lk(mu);
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetDefaultMemPool(&pool, ctx->opts.device) != hipSuccess || !pool) {
        (void)hipGetLastError();
        return;
    }
    auto &h = held[ctx->opts.device];
    if (on) {
        if (h.first++ == 0) {
            uint64_t prev = 0;
            if (hipMemPoolGetAttribute(pool, hipMemPoolAttrReleaseThreshold, &prev) != hipSuccess) prev = 0;
            h.second = prev;
            uint64_t thr = UINT64_MAX;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
        }
    } else if (--h.first == 0) {
        uint64_t prev = h.second;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &prev);
    }
    (void)hipGetLastError();
    ctx->pool_hold = on;
}

// A three-keyframe window with points and a line solved once through the whole path (device
// build, step graphs, every kernel of a step, output scatter); the context is left without a
// window, as plba_create returns it.
int prewarm(plba_ctx *ctx) {
    // Device memory: windows are carved from stream-ordered allocations (hipMallocAsync); keep what
    // they free in the device's default pool (release threshold: never) and grow the pool once
    // here (PLBA_PREWARM_MB, default 256 MB of the 288 GB), so that a first window does not pay
    // the pool's growth; the first pinned upload staging likewise.
    {
        pool_hold(ctx, true);
        const char *mb = getenv("PLBA_PREWARM_MB");
        const size_t bytes = (size_t)(mb && mb[0] ? std::max(0, atoi(mb)) : 256) << 20;
        void *p = nullptr;
        if (bytes && hipMallocAsync(&p, bytes, ctx->stream) == hipSuccess) (void)hipFreeAsync(p, ctx->stream);
        (void)hipGetLastError();
        constexpr size_t kStage = 8u << 20;
        if (!ctx->staging && hipHostMalloc((void **)&ctx->staging, kStage, hipHostMallocDefault) == hipSuccess)
            ctx->staging_cap = kStage;
        (void)hipGetLastError();
        PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    }
    // a window of nk poses, np points and nl lines, each landmark seen by two consecutive poses:
    // large enough that the device build takes its full-size sort paths (first-call costs of a
    // small window differ from a real one's)
    const int nk = 8, np = 4096, nl = 256, nep = 2 * np, nel = 2 * nl;
    std::vector<double> T((size_t)nk * 12, 0.0), P((size_t)np * 3), L((size_t)nl * 4), eobs((size_t)nep * 2),
        einfo(nep, 1.0), lobs((size_t)nel * 4), linfo(nel, 1.0);
    std::vector<uint8_t> fixed(nk, 0);
    std::vector<int32_t> kf_id(nk), pt_id(np), ln_id(nl), elm(nep), ekf(nep), llm(nel), lkf(nel);
    fixed[0] = 1;
    for (int k = 0; k < nk; ++k) {
        T[(size_t)k * 12 + 0] = T[(size_t)k * 12 + 5] = T[(size_t)k * 12 + 10] = 1.0;
        T[(size_t)k * 12 + 3] = -0.1 * k;  // t_x
        kf_id[k] = k;
    }
    const double fx = 458.654, fy = 457.296, cx = 367.215, cy = 248.375;
    for (int l = 0; l < np; ++l) {
        pt_id[l] = nk + l;
        P[(size_t)l * 3] = -1.0 + 2.0 * ((l * 37) % 101) / 101.0;
        P[(size_t)l * 3 + 1] = -0.8 + 1.6 * ((l * 53) % 97) / 97.0;
        P[(size_t)l * 3 + 2] = 4.0 + 3.0 * ((l * 29) % 89) / 89.0;
        for (int o = 0; o < 2; ++o) {
            const int e = 2 * l + o, k = (l + o) % nk;
            elm[e] = l;
            ekf[e] = k;
            const double x = P[(size_t)l * 3] + T[(size_t)k * 12 + 3], y = P[(size_t)l * 3 + 1], z = P[(size_t)l * 3 + 2];
            eobs[(size_t)e * 2] = fx * x / z + cx + 0.3;
            eobs[(size_t)e * 2 + 1] = fy * y / z + cy - 0.2;
        }
    }
    for (int l = 0; l < nl; ++l) {
        ln_id[l] = nk + np + 1 + l;
        L[(size_t)l * 4] = 0.3 + 0.001 * l;
        L[(size_t)l * 4 + 1] = -0.2;
        L[(size_t)l * 4 + 2] = 0.4;
        L[(size_t)l * 4 + 3] = 0.5;
        for (int o = 0; o < 2; ++o) {
            const int e = 2 * l + o;
            llm[e] = l;
            lkf[e] = (l + o) % nk;
            const double q[4] = {300.0 + l % 7, 200.0 + o, 420.0, 260.0 + l % 5};
            for (int c = 0; c < 4; ++c) lobs[(size_t)e * 4 + c] = q[c];
        }
    }
    plba_graph g{};
    g.n_kf = nk; g.n_pt = np; g.n_ln = nl; g.n_ept = nep; g.n_eln = nel;
    g.fx = fx; g.fy = fy; g.cx = cx; g.cy = cy;
    g.kf_Tcw = T.data(); g.kf_fixed = fixed.data(); g.kf_id = kf_id.data();
    g.pt_xyz = P.data(); g.pt_id = pt_id.data(); g.ln_orth = L.data(); g.ln_id = ln_id.data();
    g.ept_lm = elm.data(); g.ept_kf = ekf.data(); g.ept_obs = eobs.data(); g.ept_info = einfo.data();
    g.eln_lm = llm.data(); g.eln_kf = lkf.data(); g.eln_obs = lobs.data(); g.eln_info = linfo.data();
    g.huber_pt = g.huber_ln = (double)(float)2.4476519360399;
    int rc = plba_upload(ctx, &g);
    if (rc) return rc;
    std::vector<double> Tout((size_t)nk * 12);
    plba_result res{};
    res.kf_Tcw = Tout.data();
    rc = plba_lba_plucker(ctx, &res);
    ctx->uploaded = false;  // no window: calls before the caller's own upload stay PLBA_E_STATE
    ctx->initialized = false;
    ctx->no_bcr = false;    // (a diagnostic forcing BCR timeouts must not carry over to real windows)
    ctx->bcr_fallbacks = 0;
    return rc;
}

int plba_create(plba_ctx **out, const plba_opts *opts) {
    if (!out) return PLBA_E_INVALID;
    *out = nullptr;
    plba_ctx *ctx = new (std::nothrow) plba_ctx();
    if (!ctx) return PLBA_E_NOMEM;
    if (opts) ctx->opts = *opts;
    else plba_default_opts(&ctx->opts);
    if (ctx->opts.max_trials <= 0) ctx->opts.max_trials = 10;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        delete ctx;
        return PLBA_E_DEVICE;
    }
    if (ctx->opts.device < 0 || ctx->opts.device >= ndev || hipSetDevice(ctx->opts.device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_ctrl, sizeof(Ctrl), hipHostMallocDefault) != hipSuccess) {
        delete ctx;
        return PLBA_E_DEVICE;
    }
    std::memset(ctx->h_ctrl, 0, sizeof(Ctrl));
    *out = ctx;
    // Pre-warm (PLBA_NO_PREWARM=1 skips it): the first window of a process otherwise pays the
    // code-object load, the first rocPRIM sorts of the device window build and the first pinned
    // staging (C3: first upload 38 ms against 1.2 ms warm) on the LBA thread's first keyframe.
    const char *npw = getenv("PLBA_NO_PREWARM");
    // A failed pre-warm (a diagnostic switch in the caller's environment, say) is not fatal: the
    // context is returned without a window, as it would be without the pre-warm, and the reason is
    // kept in plba_last_error and printed once. A device that cannot run a kernel fails the caller's
    // own first upload or solve instead.
    if (!(npw && npw[0] == '1')) {
        const int rc = prewarm(ctx);
        if (rc) {
            (void)hipGetLastError();
            (void)hipStreamSynchronize(ctx->stream);
            ctx->uploaded = false;
            ctx->initialized = false;
            ctx->no_bcr = false;
            ctx->bcr_fallbacks = 0;
            ctx->set_error("pre-warm failed (%d): %s (continuing without it)", rc, ctx->err.c_str());
            fprintf(stderr, "[plba] %s\n", ctx->err.c_str());
        }
    }
    return PLBA_OK;
}

int plba_destroy(plba_ctx *ctx) {
    if (!ctx) return PLBA_OK;
    (void)hipSetDevice(ctx->opts.device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    ctx->free_all();
    destroy_graphs(ctx);
    if (ctx->arena) (void)hipFreeAsync(ctx->arena, ctx->stream);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->staging) (void)hipHostFree(ctx->staging);
    for (void *p : ctx->retired) (void)hipHostFree(p);
    for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->h_ctrl) (void)hipHostFree(ctx->h_ctrl);
    if (ctx->pgo_mem) (void)hipFreeAsync(ctx->pgo_mem, ctx->stream);
    ctx->bmemA.release(ctx->stream);
    ctx->bmemB.release(ctx->stream);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->pgo_hout) (void)hipHostFree(ctx->pgo_hout);
    if (ctx->h_out) (void)hipHostFree(ctx->h_out);
    if (ctx->comm.hbuf) (void)hipHostFree(ctx->comm.hbuf);
    if (ctx->comm.nccl) (void)ncclCommDestroy(ctx->comm.nccl);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    pool_hold(ctx, false);
    delete ctx;
    return PLBA_OK;
}

const char *plba_last_error(const plba_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int plba_upload(plba_ctx *ctx, const plba_graph *g) {
    if (!ctx) return PLBA_E_INVALID;
    (void)hipSetDevice(ctx->opts.device);
    ctx->robust = 1;
    ctx->trace.clear();
    return do_upload(ctx, g);
}

int plba_reset_estimates(plba_ctx *ctx) {
    if (!ctx || !ctx->uploaded) return ctx ? PLBA_E_STATE : PLBA_E_INVALID;
    Dev &d = ctx->d;
    ctx->cur = ctx->last_ok = ctx->chi_src = 0;
    PLBA_CHECK(hipMemcpyAsync(d.Tb[0], d.T_init, sizeof(double) * (size_t)d.n_kf * 12, hipMemcpyDeviceToDevice, ctx->stream));
    PLBA_CHECK(hipMemcpyAsync(d.Xb[0], d.X_init, sizeof(double) * (size_t)d.n_lm * 4, hipMemcpyDeviceToDevice, ctx->stream));
    PLBA_CHECK(hipMemsetAsync(&d.ctrl->cur, 0, sizeof(int32_t), ctx->stream));
    PLBA_CHECK(hipMemsetAsync(&d.ctrl->last_ok, 0, 2 * sizeof(int32_t), ctx->stream));  // last_ok, chi_src
    PLBA_CHECK(hipMemsetAsync(d.e_level, 0, std::max(d.E, 1), ctx->stream));
    for (int b = 0; b < d.nbx; ++b) {
        PLBA_CHECK(hipMemsetAsync(d.xpb[b], 0, sizeof(double) * std::max(d.n, 1), ctx->stream));
        PLBA_CHECK(hipMemsetAsync(d.xlb[b], 0, sizeof(double) * std::max((size_t)d.n_lm * 4, (size_t)1), ctx->stream));
        PLBA_CHECK(hipMemsetAsync(d.chi2b[b], 0, sizeof(double) * std::max(d.E, 1), ctx->stream));
    }
    std::fill(ctx->h_level.begin(), ctx->h_level.end(), 0);
    ctx->robust = 1;
    ctx->initialized = false;
    ctx->trace.clear();
    return PLBA_OK;
}

int plba_set_edge_levels(plba_ctx *ctx, const uint8_t *ept_level, const uint8_t *eln_level) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    const int E = ctx->d.E;
    std::vector<uint8_t> lv(E, 0);
    for (int e = 0; e < E; ++e) {
        int o = ctx->e_orig[e];
        bool is_pt = e < ctx->d.Ep;
        lv[e] = is_pt ? (ept_level ? ept_level[o] : 0) : (eln_level ? eln_level[o] : 0);
    }
    ctx->h_level = lv;
    // on the solver stream (ordered after a pending plba_reset_estimates memset), then wait:
    // lv is a local buffer
    if (E) {
        PLBA_CHECK(hipMemcpyAsync(ctx->d.e_level, lv.data(), E, hipMemcpyHostToDevice, ctx->stream));
        PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    }
    ctx->initialized = false;
    return PLBA_OK;
}

int plba_set_robust(plba_ctx *ctx, int32_t robust) {
    if (!ctx) return PLBA_E_INVALID;
    ctx->robust = robust ? 1 : 0;
    return PLBA_OK;
}

int plba_initialize_optimization(plba_ctx *ctx, int32_t level) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    ctx->level = level;  // activation runs on the device at the start of the next optimize()
    ctx->initialized = true;
    return PLBA_OK;
}

int plba_optimize(plba_ctx *ctx, int32_t iterations, int32_t *iters_done, double *final_chi2) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded || !ctx->initialized) return PLBA_E_STATE;
    (void)hipSetDevice(ctx->opts.device);
    ctx->trace.clear();
    return do_optimize(ctx, iterations, iters_done, final_chi2);
}

int plba_refresh_edge_errors(plba_ctx *ctx, int32_t level) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    return launch_edges(ctx, k_refresh, level);
}

int plba_get_edge_chi2(plba_ctx *ctx, double *ept_chi2, uint8_t *ept_depth_ok, double *eln_chi2) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    Dev &d = ctx->d;
    if (d.sharded) {
        std::vector<double> gv;
        int rc = gather_outputs(ctx, gv);
        if (rc) return rc;
        const double *o = gv.data() + (size_t)d.n_lm_g * 4;
        for (int e = 0; e < ctx->Ep; ++e) {
            if (ept_chi2) ept_chi2[e] = o[e];
            if (ept_depth_ok) ept_depth_ok[e] = (uint8_t)o[(size_t)d.E_g + e];
        }
        for (int e = 0; e < ctx->El && eln_chi2; ++e) eln_chi2[e] = o[ctx->Ep + e];
        return PLBA_OK;
    }
    return download_outputs(ctx, nullptr, nullptr, nullptr, ept_chi2, ept_depth_ok, eln_chi2, nullptr, nullptr);
}

int plba_download(plba_ctx *ctx, double *kf_Tcw, double *pt_xyz, double *ln_orth) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    Dev &d = ctx->d;
    if (d.sharded) {  // poses are replicated; landmarks come from the gather
        std::vector<double> gv;
        int rc = gather_outputs(ctx, gv);
        if (rc) return rc;
        if (kf_Tcw && d.n_kf)
            PLBA_CHECK(d2h(ctx, kf_Tcw, d.Tb[ctx->cur], sizeof(double) * (size_t)d.n_kf * 12));
        for (int p = 0; p < ctx->n_pt && pt_xyz; ++p)
            for (int k = 0; k < 3; ++k) pt_xyz[3 * p + k] = gv[(size_t)p * 4 + k];
        for (int l = 0; l < ctx->n_ln && ln_orth; ++l)
            for (int k = 0; k < 4; ++k) ln_orth[4 * l + k] = gv[(size_t)(ctx->n_pt + l) * 4 + k];
        return PLBA_OK;
    }
    return download_outputs(ctx, kf_Tcw, pt_xyz, ln_orth, nullptr, nullptr, nullptr, nullptr, nullptr);
}

// The whole schedule of src/mapHandler.cpp:6119-6160 (stage 1, classification, stage 2,
// level-1 refresh) with no host round trip except the per-trial control read.
int plba_lba_plucker(plba_ctx *ctx, plba_result *res) {
    if (!ctx) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    (void)hipSetDevice(ctx->opts.device);
    Dev &d = ctx->d;
    ctx->trace.clear();
    for (int k = 0; k < K_COUNT; ++k) { ctx->k_ms[k] = 0; ctx->k_n[k] = 0; }
    auto t0 = std::chrono::steady_clock::now();
    int rc;
    // stage 1: level 0, Huber; classification; stage 2: level 0, no kernel
    Ctrl c = schedule_init(ctx, 2);
    c.max_iters[0] = 5;
    c.max_iters[1] = 10;
    c.stage_robust[0] = 1;
    c.stage_robust[1] = 0;
    c.stage_level[0] = 0;
    c.stage_level[1] = 0;
    c.stage_classify[0] = 0;
    c.stage_classify[1] = 1;
    if ((rc = run_schedule(ctx, c))) return rc;
    // computeError() on the level-1 edges at the final state
    if ((rc = launch_edges(ctx, k_refresh, 1))) return rc;
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    auto t1 = std::chrono::steady_clock::now();
    if ((rc = collect_timing(ctx))) return rc;
    ctx->robust = 0;
    ctx->level = 0;
    if (res) {
        res->iters[0] = ctx->h_ctrl->iters_done[0];
        res->iters[1] = ctx->h_ctrl->iters_done[1];
        res->chi2[0] = ctx->h_ctrl->chi2_final[0];
        res->chi2[1] = ctx->h_ctrl->chi2_final[1];
        res->solve_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (d.sharded) {  // one gather for every output
            std::vector<double> gv;
            if ((rc = gather_outputs(ctx, gv))) return rc;
            if (res->kf_Tcw && d.n_kf)
                PLBA_CHECK(d2h(ctx, res->kf_Tcw, d.Tb[ctx->cur], sizeof(double) * (size_t)d.n_kf * 12));
            for (int p = 0; p < ctx->n_pt && res->pt_xyz; ++p)
                for (int k = 0; k < 3; ++k) res->pt_xyz[3 * p + k] = gv[(size_t)p * 4 + k];
            for (int l = 0; l < ctx->n_ln && res->ln_orth; ++l)
                for (int k = 0; k < 4; ++k) res->ln_orth[4 * l + k] = gv[(size_t)(ctx->n_pt + l) * 4 + k];
            const double *o = gv.data() + (size_t)d.n_lm_g * 4;
            const size_t Eg = d.E_g;
            for (int e = 0; e < ctx->Ep; ++e) {
                if (res->ept_chi2) res->ept_chi2[e] = o[e];
                if (res->ept_depth_ok) res->ept_depth_ok[e] = (uint8_t)o[Eg + e];
                if (res->ept_level) res->ept_level[e] = (uint8_t)o[2 * Eg + e];
            }
            for (int e = 0; e < ctx->El; ++e) {
                if (res->eln_chi2) res->eln_chi2[e] = o[ctx->Ep + e];
                if (res->eln_level) res->eln_level[e] = (uint8_t)o[2 * Eg + ctx->Ep + e];
            }
            return PLBA_OK;
        }
        if ((rc = download_outputs(ctx, res->kf_Tcw, res->pt_xyz, res->ln_orth, res->ept_chi2, res->ept_depth_ok,
                                   res->eln_chi2, res->ept_level, res->eln_level)))
            return rc;
    }
    return PLBA_OK;
}

void plba_hlm_default_params(plba_hlm_params *p) {
    if (!p) return;
    p->lambda0 = 1e-5;          // src/slamConfig.cpp:65
    p->lambda_k = 10.0;         // :66
    p->homog_th = 1e-7;         // src2/config.cpp:80
    p->min_error = 1e-7;        // :84
    p->min_error_change = 1e-7; // :85
    p->max_iters = 15;          // src/slamConfig.cpp:67
    p->err_per_obs = 0;
    p->variant = PLBA_HLM_LBA_PLUCKER;
    p->pad = 0;
}

// MapHandler::levMarquardtOptimizationLBAForPluker (src/mapHandler.cpp:1618-2332) on the uploaded
// window: the captured step graph with the Ctrl::hlm variants of each kernel, one step per
// iteration (linearise -> [stop] -> Schur solve -> decide), no host round trip inside a batch.
int plba_hlm_lba(plba_ctx *ctx, const plba_hlm_state *st, const plba_hlm_params *p, plba_hlm_result *res) {
    if (!ctx || !st || (ctx->n_kf && !st->kf_x) || (ctx->n_ln && !st->ln_pluker)) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    (void)hipSetDevice(ctx->opts.device);
    plba_hlm_params prm;
    if (p) prm = *p;
    else plba_hlm_default_params(&prm);
    if (prm.max_iters < 1 || (prm.variant != PLBA_HLM_LBA_PLUCKER && prm.variant != PLBA_HLM_GBA)) {
        ctx->set_error("max_iters must be >= 1 and variant PLBA_HLM_LBA_PLUCKER or PLBA_HLM_GBA");
        return PLBA_E_INVALID;
    }
    const bool gba = prm.variant == PLBA_HLM_GBA;
    if (gba && ctx->n_ln && !st->ln_line3d) {
        ctx->set_error("the GBA variant needs state ln_line3d");
        return PLBA_E_INVALID;
    }
    if (gba && ctx->d.sharded) {
        ctx->set_error("the GBA variant runs on unsharded windows only");
        return PLBA_E_STATE;
    }
    int rc = plba_reset_estimates(ctx);
    if (rc) return rc;
    Dev &d = ctx->d;
    ctx->trace.clear();
    // X_aux pose blocks and the map's NDw (in this rank's device landmark order)
    std::vector<double> Lm((size_t)std::max(d.n_ln, 1) * 8, 0.0);
    for (int i = 0; i < d.n_ln && !gba; ++i) {
        const int gl = ctx->lm_gpos[d.n_pt + i] - ctx->n_pt;
        for (int k = 0; k < 6; ++k) Lm[(size_t)i * 8 + k] = st->ln_pluker[(size_t)gl * 6 + k];
    }
    if (d.n_kf) PLBA_CHECK(hipMemcpyAsync(d.xk[0], st->kf_x, sizeof(double) * (size_t)d.n_kf * 6, hipMemcpyHostToDevice, ctx->stream));
    if (d.n_ln && !gba)
        PLBA_CHECK(hipMemcpyAsync(d.Lpb[0], Lm.data(), sizeof(double) * Lm.size(), hipMemcpyHostToDevice, ctx->stream));
    if (ctx->n_ln && gba)
        PLBA_CHECK(hipMemcpyAsync(d.XL[0], st->ln_line3d, sizeof(double) * (size_t)ctx->n_ln * 6, hipMemcpyHostToDevice,
                                  ctx->stream));
    auto t0 = std::chrono::steady_clock::now();
    Ctrl c = schedule_init(ctx, 1);
    c.max_iters[0] = prm.max_iters;
    c.stage_robust[0] = 0;
    c.stage_level[0] = 0;
    c.hlm = gba ? 2 : 1;
    c.hlm_lambda0 = prm.lambda0;
    c.hlm_k = prm.lambda_k;
    c.hlm_homog = prm.homog_th;
    c.hlm_minerr = prm.min_error;
    c.hlm_minchg = prm.min_error_change;
    c.hlm_nobs = prm.err_per_obs ? (double)(ctx->Ep + ctx->El) : 0.0;
    c.err_prev = 999999999.9;  // :1634
    rc = run_schedule(ctx, c);
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    auto t1 = std::chrono::steady_clock::now();
    if (rc) return rc;
    if ((rc = collect_timing(ctx))) return rc;
    ctx->robust = 1;
    ctx->level = 0;
    ctx->initialized = false;
    if (!res) return PLBA_OK;
    const Ctrl &h = *ctx->h_ctrl;
    res->linearizations = h.hlm_lin;
    res->solves = h.hlm_solves;
    res->accepted = h.hlm_acc;
    res->pad = 0;
    res->err = h.currentChi;
    res->lambda = h.lambda;
    res->dx_norm = std::sqrt(h.dx2);
    res->solve_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (res->kf_x && d.n_kf) {
        PLBA_CHECK(d2h(ctx, res->kf_x, d.xk[ctx->cur], sizeof(double) * (size_t)d.n_kf * 6));
        // KFs outside kf_list keep the caller's x (the device copy carries them through unchanged)
    }
    if (gba && res->ln_line3d && ctx->n_ln)
        PLBA_CHECK(d2h(ctx, res->ln_line3d, d.XL[ctx->cur], sizeof(double) * (size_t)ctx->n_ln * 6));
    return plba_download(ctx, res->kf_Tcw, res->pt_xyz, gba ? nullptr : res->ln_orth);
}

int plba_get_trace(plba_ctx *ctx, plba_iter_trace *out, int32_t cap, int32_t *n) {
    if (!ctx) return PLBA_E_INVALID;
    if (n) *n = (int32_t)ctx->trace.size();
    if (out)
        for (int i = 0; i < (int)ctx->trace.size() && i < cap; ++i) out[i] = ctx->trace[i];
    return PLBA_OK;
}

int plba_synchronize(plba_ctx *ctx) {
    if (!ctx) return PLBA_E_INVALID;
    PLBA_CHECK(hipStreamSynchronize(ctx->stream));
    return PLBA_OK;
}

int plba_kernel_times(plba_ctx *ctx, const char **names, double *ms, int32_t *launches, int32_t cap, int32_t *n) {
    if (!ctx) return PLBA_E_INVALID;
    if (n) *n = K_COUNT;
    for (int k = 0; k < K_COUNT && k < cap; ++k) {
        if (names) names[k] = kKernelNames[k];
        if (ms) ms[k] = ctx->k_ms[k];
        if (launches) launches[k] = ctx->k_n[k];
    }
    return PLBA_OK;
}

// Diagnostic build only: per-wave, per-phase cycle sums of the banded factorisation.
int plba_debug_stamps(plba_ctx *ctx, unsigned long long *out /* [17][8] */) {
#if defined(PLBA_STAMPS) || defined(PLBA_PHASE_STAMPS) || defined(PLBA_LMS_STAMPS)
    if (!ctx || !ctx->d.stamps) return PLBA_E_STATE;
    PLBA_CHECK(d2h(ctx, out, ctx->d.stamps, 17 * 8 * sizeof(unsigned long long)));
    return PLBA_OK;
#else
    (void)ctx; (void)out;
    return PLBA_E_STATE;
#endif
}

// Diagnostics only (PLBA_DIAG bit 8): per-workgroup phase timestamps of the last block-cyclic-
// reduction launch, [bcr_rows][32] s_memrealtime ticks (100 MHz).
int plba_debug_bcr_stamps(plba_ctx *ctx, unsigned long long *out, int32_t cap, int32_t *rows) {
    if (!ctx || !out || !rows) return PLBA_E_INVALID;
    if (!ctx->uploaded || !ctx->d.bcr_stamps) return PLBA_E_STATE;  // BCR rows, or 1 row (dense path)
    const int rows_ = std::max(ctx->d.bcr_N, 1);
    const int n = std::min(cap / kBcrStamps, rows_);
    *rows = rows_;
    PLBA_CHECK(d2h(ctx, out, ctx->d.bcr_stamps, sizeof(unsigned long long) * (size_t)n * kBcrStamps));
    return PLBA_OK;
}

int plba_structure_stats(plba_ctx *ctx, int64_t *out, int32_t cap) {
    if (!ctx || !out) return PLBA_E_INVALID;
    if (!ctx->uploaded) return PLBA_E_STATE;
    const int64_t v[22] = {ctx->d.nf, ctx->d.bw, ctx->d.nblk, (int64_t)ctx->n_triples, ctx->d.E, ctx->d.n_lm,
                           ctx->d.band_mode, ctx->d.nch, ctx->n_free_edges, ctx->d.Ep,
                           ctx->step_exec != nullptr, ctx->d.sharded, ctx->d.twisted, ctx->d.cl, ctx->d.bcr_N,
                           ctx->d.dense_mfma, ctx->bcr_fallbacks, ctx->d.spec_max, ctx->d.spec_policy,
                           ctx->h_ctrl ? ctx->h_ctrl->steps : 0, 0, ctx->dev_build};  // [20]: unused
    for (int i = 0; i < cap && i < 22; ++i) out[i] = v[i];
    return PLBA_OK;
}

int plba_shard_plan(const plba_graph *g, int32_t nranks, int32_t *pt_owner, int32_t *ln_owner) {
    if (!g || nranks < 1 || (g->n_pt && !pt_owner) || (g->n_ln && !ln_owner)) return PLBA_E_INVALID;
    if ((g->n_ept && (!g->ept_lm || !g->ept_kf)) || (g->n_eln && (!g->eln_lm || !g->eln_kf)) ||
        (g->n_kf && !g->kf_id))
        return PLBA_E_INVALID;
    for (int e = 0; e < g->n_ept; ++e)
        if (g->ept_lm[e] < 0 || g->ept_lm[e] >= g->n_pt || g->ept_kf[e] < 0 || g->ept_kf[e] >= g->n_kf)
            return PLBA_E_INVALID;
    for (int e = 0; e < g->n_eln; ++e)
        if (g->eln_lm[e] < 0 || g->eln_lm[e] >= g->n_ln || g->eln_kf[e] < 0 || g->eln_kf[e] >= g->n_kf)
            return PLBA_E_INVALID;
    shard_plan(g, nranks, pt_owner, ln_owner);
    return PLBA_OK;
}

int plba_comm_unique_id(uint8_t id[128]) {
    if (!id) return PLBA_E_INVALID;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PLBA_E_COMM;
    std::memcpy(id, &u, sizeof(u));
    return PLBA_OK;
}

int plba_comm_init_rccl(plba_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return PLBA_E_INVALID;
    if (ctx->comm.kind != plba_ctx::Comm::NONE || ctx->uploaded) return PLBA_E_STATE;
    (void)hipSetDevice(ctx->opts.device);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&ctx->comm.nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->set_error("ncclCommInitRank(%d ranks, rank %d): %s", nranks, rank, ncclGetErrorString(r));
        ctx->comm.nccl = nullptr;
        return PLBA_E_COMM;
    }
    ctx->comm.kind = plba_ctx::Comm::RCCL;
    ctx->comm.nranks = nranks;
    ctx->comm.rank = rank;
    return PLBA_OK;
}

int plba_comm_init_host(plba_ctx *ctx, int32_t nranks, int32_t rank, plba_host_allreduce_fn fn, void *user) {
    if (!ctx || !fn || nranks < 1 || rank < 0 || rank >= nranks) return PLBA_E_INVALID;
    if (ctx->comm.kind != plba_ctx::Comm::NONE || ctx->uploaded) return PLBA_E_STATE;
    ctx->comm.kind = plba_ctx::Comm::HOST;
    ctx->comm.nranks = nranks;
    ctx->comm.rank = rank;
    ctx->comm.fn = fn;
    ctx->comm.user = user;
    return PLBA_OK;
}

int plba_comm_info(plba_ctx *ctx, int32_t *out, int32_t cap) {
    if (!ctx || (cap > 0 && !out)) return PLBA_E_INVALID;
    (void)hipSetDevice(ctx->opts.device);
    const auto &c = ctx->comm;
    int32_t v[8] = {c.kind == plba_ctx::Comm::RCCL ? 1 : c.kind == plba_ctx::Comm::HOST ? 2 : 0,
                    c.kind == plba_ctx::Comm::NONE ? 1 : c.nranks, c.rank, ctx->opts.device, -1, -1, -1, -1};
    if (c.kind == plba_ctx::Comm::RCCL && c.nccl) {
        int n = 0, r = 0, dv = 0;
        if (ncclCommCount(c.nccl, &n) != ncclSuccess || ncclCommUserRank(c.nccl, &r) != ncclSuccess ||
            ncclCommCuDevice(c.nccl, &dv) != ncclSuccess) {
            ctx->set_error("RCCL communicator query failed");
            return PLBA_E_COMM;
        }
        v[1] = n;
        v[2] = r;
        v[3] = dv;
    }
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        ctx->set_error("hipGetDevice failed");
        return PLBA_E_DEVICE;
    }
    v[4] = dev;
    int a = 0;
    if (hipDeviceGetAttribute(&a, hipDeviceAttributePciDomainID, dev) == hipSuccess) v[5] = a;
    if (hipDeviceGetAttribute(&a, hipDeviceAttributePciBusId, dev) == hipSuccess) v[6] = a;
    if (hipDeviceGetAttribute(&a, hipDeviceAttributePciDeviceId, dev) == hipSuccess) v[7] = a;
    (void)hipGetLastError();
    for (int i = 0; i < cap && i < 8; ++i) out[i] = v[i];
    return PLBA_OK;
}

// Extension: enable per-kernel HIP-event timing for subsequent plba_lba_plucker calls.
int plba_enable_kernel_timing(plba_ctx *ctx, int32_t on) {
    if (!ctx) return PLBA_E_INVALID;
    ctx->timing = on != 0;
    return PLBA_OK;
}

// ---------------------------------------------------------------- loop-closure pose graph
// MapHandler::loopClosureOptimization{EssGraph,CovGraph}G2O (src/mapHandler.cpp:5070-5531):
// g2o SparseOptimizer::initializeOptimization / computeInitialGuess / optimize over VertexSE3 +
// EdgeSE3 with OptimizationAlgorithmLevenberg (setUserLambdaInit) — device kernels in
// csrc/plba_pgo.hpp, Levenberg decisions here.
namespace {
#pragma clang fp contract(off)
struct HIso {
    double R[9], t[3];
};
HIso hiso_load(const double *T) {
    HIso a;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) a.R[3 * r + c] = T[4 * r + c];
        a.t[r] = T[4 * r + 3];
    }
    return a;
}
void hiso_store(const HIso &a, double *T) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = a.R[3 * r + c];
        T[4 * r + 3] = a.t[r];
    }
}
HIso hiso_mul(const HIso &a, const HIso &b) {
    HIso o;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s = s + a.R[3 * r + k] * b.R[3 * k + c];
            o.R[3 * r + c] = s;
        }
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s = s + a.R[3 * r + k] * b.t[k];
        o.t[r] = s + a.t[r];
    }
    return o;
}
HIso hiso_inv(const HIso &a) {
    HIso o;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) o.R[3 * r + c] = a.R[3 * c + r];
    for (int r = 0; r < 3; ++r) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s = s + o.R[3 * r + k] * a.t[k];
        o.t[r] = -s;
    }
    return o;
}
}  // namespace

void plba_pgo_default_params(plba_pgo_params *p) {
    if (!p) return;
    p->user_lambda_init = 1e-10;  // src/mapHandler.cpp:5085
    p->max_iters = 100;           // SlamConfig::maxItersPGO(), src/slamConfig.cpp:79
    p->initial_guess = 1;         // optimizer.computeInitialGuess(), :5183
    p->max_trials = 10;           // g2o maxTrialsAfterFailure
    p->pad = 0;
}

int plba_pgo_optimize(plba_ctx *ctx, const plba_pgo_graph *g, const plba_pgo_params *pp, plba_pgo_result *res) {
#pragma clang fp contract(off)
    if (!ctx || !g || !res || g->n_v < 0 || g->n_e < 0) return PLBA_E_INVALID;
    if ((g->n_v && (!g->v_id || !g->v_T || !g->v_fixed)) || (g->n_e && (!g->e_v || !g->e_Z))) return PLBA_E_INVALID;
    plba_pgo_params prm;
    if (pp) prm = *pp;
    else plba_pgo_default_params(&prm);
    if (prm.max_iters < 0 || prm.max_trials < 1) {
        ctx->set_error("max_iters must be >= 0 and max_trials >= 1");
        return PLBA_E_INVALID;
    }
    const int nv = g->n_v, ne = g->n_e;
    for (int e = 0; e < 2 * ne; ++e)
        if (g->e_v[e] < 0 || g->e_v[e] >= nv) {
            ctx->set_error("pose-graph edge %d references vertex %d (n_v %d)", e / 2, g->e_v[e], nv);
            return PLBA_E_INVALID;
        }
    {
        std::vector<int32_t> ids(g->v_id, g->v_id + nv);
        std::sort(ids.begin(), ids.end());
        if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) {
            ctx->set_error("duplicate pose-graph vertex id");
            return PLBA_E_INVALID;
        }
    }
    (void)hipSetDevice(ctx->opts.device);
    const auto t0 = std::chrono::steady_clock::now();
    // ---- SparseOptimizer::initializeOptimization(): active edges (not all vertices fixed) in
    //      creation order; Hessian index of the active free vertices in id order
    std::vector<HIso> X(nv), Z(ne), Zinv(ne);
    for (int v = 0; v < nv; ++v) X[v] = hiso_load(g->v_T + 12 * (size_t)v);
    for (int e = 0; e < ne; ++e) {
        Z[e] = hiso_load(g->e_Z + 12 * (size_t)e);
        Zinv[e] = hiso_inv(Z[e]);  // EdgeSE3::setMeasurement keeps the inverse
    }
    std::vector<int32_t> act;
    std::vector<uint8_t> is_act(ne, 0);
    std::vector<int> nact_v(nv, 0);
    for (int e = 0; e < ne; ++e) {
        const int a = g->e_v[2 * e], b = g->e_v[2 * e + 1];
        if (g->v_fixed[a] && g->v_fixed[b]) continue;
        act.push_back(e);
        is_act[e] = 1;
        ++nact_v[a];
        ++nact_v[b];
    }
    std::vector<int> order(nv);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return g->v_id[a] < g->v_id[b]; });
    std::vector<int32_t> hidx(nv, -1);
    int nfree = 0;
    for (int v : order)
        if (nact_v[v] > 0 && !g->v_fixed[v]) hidx[v] = nfree++;
    // ---- computeInitialGuess(): EstimatePropagator from the fixed vertices of the active edges
    //      (std::set<Vertex*>: creation order), unit edge cost, multimap frontier (smallest
    //      distance first, FIFO among equals), EdgeSE3::initialEstimate on each first reach
    if (prm.initial_guess) {
        std::vector<std::vector<int>> vedges(nv);
        for (int e = 0; e < ne; ++e) {
            vedges[g->e_v[2 * e]].push_back(e);
            vedges[g->e_v[2 * e + 1]].push_back(e);
        }
        std::vector<int> roots;
        std::vector<uint8_t> isroot(nv, 0);
        for (int e : act)
            for (int sd = 0; sd < 2; ++sd) {
                const int v = g->e_v[2 * e + sd];
                if (g->v_fixed[v] && !isroot[v]) { isroot[v] = 1; roots.push_back(v); }
            }
        std::sort(roots.begin(), roots.end());
        const double inf = std::numeric_limits<double>::max();
        std::vector<double> dist(nv, inf);
        std::vector<int> level(nv, 0), pedge(nv, -1), parent(nv, -1);
        std::multimap<double, int> frontier;
        std::vector<std::multimap<double, int>::iterator> qit(nv);
        std::vector<uint8_t> inq(nv, 0);
        auto push = [&](int v) {
            if (inq[v]) frontier.erase(qit[v]);
            qit[v] = frontier.insert(frontier.upper_bound(dist[v]), {dist[v], v});
            inq[v] = 1;
        };
        for (int r : roots) { dist[r] = 0.0; push(r); }
        while (!frontier.empty()) {
            const auto it = frontier.begin();
            const int u = it->second;
            frontier.erase(it);
            inq[u] = 0;
            if (level[u] > 0 && !g->v_fixed[u]) {
                const int e = pedge[u];
                if (parent[u] == g->e_v[2 * e]) X[u] = hiso_mul(X[g->e_v[2 * e]], Z[e]);
                else X[u] = hiso_mul(X[g->e_v[2 * e + 1]], hiso_inv(Z[e]));
            }
            for (int e : vedges[u]) {
                if (!is_act[e]) continue;
                int maxf = -1;
                for (int sd = 0; sd < 2; ++sd) {
                    const int z = g->e_v[2 * e + sd];
                    if (dist[z] != inf) maxf = std::max(maxf, level[z]);
                }
                for (int sd = 0; sd < 2; ++sd) {
                    const int z = g->e_v[2 * e + sd];
                    if (z == u) continue;
                    const double zd = dist[u] + 1.0;
                    if (zd < dist[z]) {
                        dist[z] = zd;
                        parent[z] = u;
                        pedge[z] = e;
                        level[z] = maxf + 1;
                        push(z);
                    }
                }
            }
        }
    }
    // ---- Hessian order: Cholmod orders H by AMD before its supernodal factorisation; here the
    //      free vertices are reordered by reverse Cuthill–McKee when that narrows the band (loop
    //      edges couple vertices far apart in id order), and the dense factorisation runs over the
    //      envelope only (tile_first / tile_last). Any symmetric order gives the same exact solve.
    std::vector<int32_t> first_h(nfree);
    auto envelope_of = [&](const std::vector<int32_t> &hx, std::vector<int32_t> &fh) {
        for (int h = 0; h < nfree; ++h) fh[h] = h;
        for (int e : act) {
            const int a = hx[g->e_v[2 * e]], b = hx[g->e_v[2 * e + 1]];
            if (a < 0 || b < 0) continue;
            fh[std::max(a, b)] = std::min(fh[std::max(a, b)], std::min(a, b));
        }
        int w = 0;
        for (int h = 0; h < nfree; ++h) w = std::max(w, h - fh[h]);
        return w;
    };
    {
        int bwp = envelope_of(hidx, first_h);
        if (bwp > 1 && nfree > 2 && !env_flag("PLBA_NO_RCM")) {
            std::vector<std::vector<int32_t>> adj(nfree);
            for (int e : act) {
                const int a = hidx[g->e_v[2 * e]], b = hidx[g->e_v[2 * e + 1]];
                if (a < 0 || b < 0 || a == b) continue;
                adj[a].push_back(b);
                adj[b].push_back(a);
            }
            const std::vector<int32_t> rcm = rcm_from_adj(adj);
            std::vector<int32_t> pos(nfree), h2(nv, -1), fh2(nfree);
            for (int i = 0; i < nfree; ++i) pos[rcm[i]] = i;
            for (int v = 0; v < nv; ++v) h2[v] = hidx[v] >= 0 ? pos[hidx[v]] : -1;
            if (envelope_of(h2, fh2) < bwp) {
                hidx = h2;
                first_h = fh2;
            }
        }
    }
    // ---- blocks of H (lower triangle) and their contributions in edge order
    std::map<std::pair<int, int>, std::vector<int32_t>> blocks;  // (col, row) -> contributions
    for (int h = 0; h < nfree; ++h) blocks[{h, h}];
    for (int e : act) {
        const int hi = hidx[g->e_v[2 * e]], hj = hidx[g->e_v[2 * e + 1]];
        if (hi >= 0) blocks[{hi, hi}].push_back(e << 2 | 0);
        if (hj >= 0) blocks[{hj, hj}].push_back(e << 2 | 1);
        if (hi >= 0 && hj >= 0 && hi != hj) {
            if (hi > hj) blocks[{hj, hi}].push_back(e << 2 | 2);  // row block = vertex i
            else blocks[{hi, hj}].push_back(e << 2 | 3);          // row block = vertex j
        }
    }
    std::vector<int32_t> blk_r, blk_c, blk_off{0}, blk_con;
    for (auto &kv : blocks) {
        blk_c.push_back(kv.first.first);
        blk_r.push_back(kv.first.second);
        for (int32_t c : kv.second) blk_con.push_back(c);
        blk_off.push_back((int32_t)blk_con.size());
    }
    const int n = 6 * nfree, nblk = (int)blk_r.size(), ntiles = (n + kTile - 1) / kTile;
    const int nact = (int)act.size();
    // ---- device block (grow-only)
    struct Slot {
        void **p;
        size_t bytes;
    };
    PgoDev P{};
    Dev dd{};
    double *T0, *T1, *Ad;
    int32_t *e_v_d, *act_d, *hidx_d, *blk_r_d, *blk_c_d, *blk_off_d, *blk_con_d, *tf_d, *tl_d;
    double *Zinv_d, *info_d;
    Ctrl *ctrl_d;
    std::vector<Slot> slots = {
        {(void **)&e_v_d, sizeof(int32_t) * 2 * (size_t)ne}, {(void **)&act_d, sizeof(int32_t) * (size_t)nact},
        {(void **)&hidx_d, sizeof(int32_t) * (size_t)nv}, {(void **)&blk_r_d, sizeof(int32_t) * (size_t)nblk},
        {(void **)&blk_c_d, sizeof(int32_t) * (size_t)nblk}, {(void **)&blk_off_d, sizeof(int32_t) * (size_t)(nblk + 1)},
        {(void **)&blk_con_d, sizeof(int32_t) * blk_con.size()}, {(void **)&tf_d, sizeof(int32_t) * (size_t)ntiles},
        {(void **)&tl_d, sizeof(int32_t) * (size_t)ntiles}, {(void **)&Zinv_d, sizeof(double) * 12 * (size_t)ne},
        {(void **)&info_d, sizeof(double) * 36 * (size_t)ne}, {(void **)&T0, sizeof(double) * 12 * (size_t)nv},
        {(void **)&T1, sizeof(double) * 12 * (size_t)nv}, {(void **)&P.eH, sizeof(double) * 144 * (size_t)ne},
        {(void **)&P.eg, sizeof(double) * 12 * (size_t)ne}, {(void **)&P.echi, sizeof(double) * (size_t)ne},
        {(void **)&P.Hd, sizeof(double) * (size_t)n * n}, {(void **)&Ad, sizeof(double) * (size_t)n * n},
        {(void **)&P.b, sizeof(double) * (size_t)n}, {(void **)&P.x, sizeof(double) * (size_t)n},
        {(void **)&dd.Wbuf, sizeof(double) * (size_t)std::max(n, 1) * (kTile + 1)}, {(void **)&P.out, sizeof(double) * 4},
        {(void **)&ctrl_d, sizeof(Ctrl)}};
    size_t tot = 0;
    for (auto &sl : slots) tot += (std::max(sl.bytes, (size_t)128) + 255) & ~(size_t)255;
    if (tot > ctx->pgo_cap) {
        if (ctx->pgo_mem) (void)hipFreeAsync(ctx->pgo_mem, ctx->stream);  // stream-ordered (see commit_plan)
        ctx->pgo_mem = nullptr;
        ctx->pgo_cap = 0;
        if (hipMallocAsync((void **)&ctx->pgo_mem, tot, ctx->stream) != hipSuccess) {
            (void)hipGetLastError();
            ctx->set_error("pose graph: cannot allocate %zu bytes", tot);
            return PLBA_E_NOMEM;
        }
        ctx->pgo_cap = tot;
    }
    if (!ctx->pgo_hout) PLBA_CHECK(hipHostMalloc((void **)&ctx->pgo_hout, sizeof(double) * 4));
    {
        size_t off = 0;
        for (auto &sl : slots) {
            *sl.p = ctx->pgo_mem + off;
            off += (std::max(sl.bytes, (size_t)128) + 255) & ~(size_t)255;
        }
    }
    hipStream_t s = ctx->stream;
    std::vector<double> Tv(12 * (size_t)nv), Zi(12 * (size_t)ne), Om(36 * (size_t)ne);
    for (int v = 0; v < nv; ++v) hiso_store(X[v], &Tv[12 * (size_t)v]);
    for (int e = 0; e < ne; ++e) {
        hiso_store(Zinv[e], &Zi[12 * (size_t)e]);
        for (int k = 0; k < 36; ++k) Om[36 * (size_t)e + k] = g->e_info ? g->e_info[36 * (size_t)e + k] : (k % 7 == 0 ? 1.0 : 0.0);
    }
    std::vector<int32_t> tf(std::max(ntiles, 1), 0), tl(std::max(ntiles, 1), 0);
    for (int I = 0; I < ntiles; ++I) {
        int f = I;
        for (int r = I * kTile; r < std::min(n, (I + 1) * kTile); ++r) f = std::min(f, (6 * first_h[r / 6]) / kTile);
        tf[I] = f;
    }
    for (int K = 0; K < ntiles; ++K) {
        int last = K;
        for (int I = K; I < ntiles; ++I)
            if (tf[I] <= K) last = I;
        tl[K] = last;
    }
    auto up = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
        return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
    };
    PLBA_CHECK(up(e_v_d, g->e_v, sizeof(int32_t) * 2 * (size_t)ne));
    PLBA_CHECK(up(act_d, act.data(), sizeof(int32_t) * act.size()));
    PLBA_CHECK(up(hidx_d, hidx.data(), sizeof(int32_t) * hidx.size()));
    PLBA_CHECK(up(blk_r_d, blk_r.data(), sizeof(int32_t) * blk_r.size()));
    PLBA_CHECK(up(blk_c_d, blk_c.data(), sizeof(int32_t) * blk_c.size()));
    PLBA_CHECK(up(blk_off_d, blk_off.data(), sizeof(int32_t) * blk_off.size()));
    PLBA_CHECK(up(blk_con_d, blk_con.data(), sizeof(int32_t) * blk_con.size()));
    PLBA_CHECK(up(tf_d, tf.data(), sizeof(int32_t) * tf.size()));
    PLBA_CHECK(up(tl_d, tl.data(), sizeof(int32_t) * tl.size()));
    PLBA_CHECK(up(Zinv_d, Zi.data(), sizeof(double) * Zi.size()));
    PLBA_CHECK(up(info_d, Om.data(), sizeof(double) * Om.size()));
    PLBA_CHECK(up(T0, Tv.data(), sizeof(double) * Tv.size()));
    PLBA_CHECK(hipMemsetAsync(P.x, 0, sizeof(double) * std::max(n, 1), s));  // g2o's _x starts at zero
    PLBA_CHECK(hipMemsetAsync(ctrl_d, 0, sizeof(Ctrl), s));
    P.nv = nv; P.ne = ne; P.nact = nact; P.nfree = nfree; P.n = n; P.nblk = nblk;
    P.e_v = e_v_d; P.act = act_d; P.Zinv = Zinv_d; P.info = info_d; P.hidx = hidx_d;
    P.T[0] = T0; P.T[1] = T1;
    P.blk_r = blk_r_d; P.blk_c = blk_c_d; P.blk_off = blk_off_d; P.blk_con = blk_con_d;
    dd.n = n; dd.ntiles = ntiles; dd.Ad = Ad; dd.bs = P.b; dd.xp = P.x; dd.ctrl = ctrl_d;
    dd.solve_lds_n = solve_lds_limit();
    dd.tile_first = tf_d; dd.tile_last = tl_d;
    double *hout = ctx->pgo_hout;
    auto fetch = [&]() -> int {
        PLBA_CHECK(hipMemcpyAsync(hout, P.out, sizeof(double) * 4, hipMemcpyDeviceToHost, s));
        PLBA_CHECK(hipStreamSynchronize(s));
        return PLBA_OK;
    };
    const int eb = std::max((nact + kPgoNT - 1) / kPgoNT, 1);
    int cur = 0;
    // computeActiveErrors() after the initial guess
    hipLaunchKernelGGL(k_pgo_linearize<false>, dim3(eb), dim3(kPgoNT), 0, s, P, cur); PLBA_LAUNCHED(ctx, "k_pgo_linearize");
    hipLaunchKernelGGL(k_pgo_sum, dim3(1), dim3(64), 0, s, P, (const Ctrl *)ctrl_d, 0, 0.0); PLBA_LAUNCHED(ctx, "k_pgo_sum");
    PLBA_CHECK(hipGetLastError());
    if (int rc = fetch()) return rc;
    res->chi2_initial = hout[0];
    res->n_free = nfree;
    res->iterations = res->trials = res->solve_fails = 0;
    res->n_trace = 0;
    double lambda = 0.0, ni = 2.0, currentChi = hout[0];
    for (int it = 0; it < prm.max_iters && nfree > 0; ++it) {
        // OptimizationAlgorithmLevenberg::solve: computeActiveErrors, buildSystem
        hipLaunchKernelGGL(k_pgo_linearize<true>, dim3(eb), dim3(kPgoNT), 0, s, P, cur); PLBA_LAUNCHED(ctx, "k_pgo_linearize");
        hipLaunchKernelGGL(k_pgo_sum, dim3(1), dim3(64), 0, s, P, (const Ctrl *)ctrl_d, 0, 0.0); PLBA_LAUNCHED(ctx, "k_pgo_sum");
        PLBA_CHECK(hipMemsetAsync(P.Hd, 0, sizeof(double) * (size_t)n * n, s));
        hipLaunchKernelGGL(k_pgo_assemble, dim3((nblk * 42 + kPgoNT - 1) / kPgoNT), dim3(kPgoNT), 0, s, P); PLBA_LAUNCHED(ctx, "k_pgo_assemble");
        if (it == 0 && prm.user_lambda_init <= 0.0) hipLaunchKernelGGL(k_pgo_maxdiag, dim3(1), dim3(64), 0, s, P); PLBA_LAUNCHED(ctx, "k_pgo_maxdiag");
        PLBA_CHECK(hipGetLastError());
        if (int rc = fetch()) return rc;
        currentChi = hout[0];
        const double chiStart = currentChi;
        if (it == 0) {  // computeLambdaInit
            lambda = prm.user_lambda_init > 0.0 ? prm.user_lambda_init : ctx->opts.tau * hout[2];
            ni = 2.0;
        }
        const double lambdaStart = lambda;
        double rho = 0.0;
        int qmax = 0;
        do {
            // setLambda + solve (dense LDLᵀ, Cholmod's positive-definite test) + update
            hipLaunchKernelGGL(k_pgo_damp, dim3((unsigned)(((size_t)n * n + 255) / 256)), dim3(256), 0, s, P, Ad, lambda); PLBA_LAUNCHED(ctx, "k_pgo_damp");
            for (int K = 0; K < ntiles; ++K) {  // the envelope's row tiles K..tl[K] only
                const int m = tl[K] - K;
                hipLaunchKernelGGL(k_dense_panel, dim3((m + 2) / 2), dim3(kDensePanelNT), 0, s, dd, K); PLBA_LAUNCHED(ctx, "k_dense_panel");
                if (m > 0) hipLaunchKernelGGL(k_dense_update, dim3(m * (m + 1) / 2), dim3(64), 0, s, dd, K); PLBA_LAUNCHED(ctx, "k_dense_update");
            }
            hipLaunchKernelGGL(k_pgo_check, dim3(1), dim3(256), 0, s, dd); PLBA_LAUNCHED(ctx, "k_pgo_check");
            hipLaunchKernelGGL(k_pgo_solve, dim3(1), dim3(kFacThreads),
                               n <= dd.solve_lds_n ? sizeof(double) * (size_t)n : 0, s, dd); PLBA_LAUNCHED(ctx, "k_pgo_solve");
            hipLaunchKernelGGL(k_pgo_update, dim3((nv + kPgoNT - 1) / kPgoNT), dim3(kPgoNT), 0, s, P, cur); PLBA_LAUNCHED(ctx, "k_pgo_update");
            // restoreDiagonal (Hd is untouched), computeActiveErrors at the trial state
            hipLaunchKernelGGL(k_pgo_linearize<false>, dim3(eb), dim3(kPgoNT), 0, s, P, cur ^ 1); PLBA_LAUNCHED(ctx, "k_pgo_linearize");
            hipLaunchKernelGGL(k_pgo_sum, dim3(1), dim3(64), 0, s, P, (const Ctrl *)ctrl_d, 1, lambda); PLBA_LAUNCHED(ctx, "k_pgo_sum");
            PLBA_CHECK(hipGetLastError());
            if (int rc = fetch()) return rc;
            const bool ok = hout[3] != 0.0;
            double tempChi = hout[1];
            if (!ok) {
                tempChi = std::numeric_limits<double>::max();
                ++res->solve_fails;
            }
            const double scale = hout[2] + 1e-3;
            rho = (currentChi - tempChi) / scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
                cur ^= 1;  // discardTop: the trial state becomes current
            } else {
                lambda *= ni;
                ni *= 2;
                if (!std::isfinite(lambda)) break;  // (pop: the current state is untouched)
            }
            ++qmax;
            ++res->trials;
        } while (rho < 0 && qmax < prm.max_trials);
        const int result = (qmax == prm.max_trials || rho == 0 || !std::isfinite(lambda)) ? 1 : 0;
        if (res->trace && res->n_trace < res->trace_cap)
            res->trace[res->n_trace++] = plba_iter_trace{0, it, qmax, result, chiStart, currentChi, lambdaStart, lambda};
        ++res->iterations;
        if (result != 0) break;
    }
    res->chi2_final = currentChi;
    res->lambda_final = lambda;
    if (res->v_T) {
        PLBA_CHECK(hipMemcpyAsync(res->v_T, P.T[cur], sizeof(double) * 12 * (size_t)nv, hipMemcpyDeviceToHost, s));
        PLBA_CHECK(hipStreamSynchronize(s));
    }
    res->solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return PLBA_OK;
}

}  // extern "C"
