// plba_build.hip — device-side window build (see plba_build.hpp). One thread per edge /
// landmark; rocPRIM radix sorts (stable, LSD) and scans; three small read-backs per window (the
// envelope, the triple count, the block offsets) that size the next allocation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "plba_build.hpp"

namespace plba {

namespace {

constexpr int kNT = 256;
constexpr int32_t kBig = 0x7F7F7F7F;  // hipMemset(0x7F) sentinel, above any index

inline unsigned grid(int64_t n) { return (unsigned)std::max<int64_t>((n + kNT - 1) / kNT, 1); }
inline unsigned bits_for(int64_t maxkey) {  // keys in [0, maxkey]
    unsigned b = 1;
    while (b < 31 && ((int64_t)1 << b) <= maxkey) ++b;
    return b;
}

// bump allocator over BuildMem (measuring pass with base == nullptr)
struct Carver {
    char *base;
    size_t off = 0;
    template <class T>
    T *take(size_t n) {
        const size_t bytes = std::max(n * sizeof(T), (size_t)256);
        T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
        off = (off + bytes + 255) & ~(size_t)255;
        return p;
    }
};

struct Raw {  // the caller's graph, on the device
    const int32_t *ept_lm, *ept_kf, *eln_lm, *eln_kf, *kf_hidx, *kpos;
    const double *ept_obs, *ept_info, *eln_obs, *eln_info, *pt_xyz, *ln_orth;
    int n_kf, n_pt, n_ln, Ep, El;
};
// (vertex ids are validated by k_b_edges, reported at the stage's final read-back; the clamps keep
// a broken input from ever addressing outside the arrays in the kernels that run before that)
__device__ __forceinline__ void edge_of(const Raw &r, int e, int &lm, int &kf) {
    if (e < r.Ep) {
        lm = min(max(r.ept_lm[e], 0), max(r.n_pt - 1, 0));
        kf = r.ept_kf[e];
    } else {
        lm = r.n_pt + min(max(r.eln_lm[e - r.Ep], 0), max(r.n_ln - 1, 0));
        kf = r.eln_kf[e - r.Ep];
    }
    kf = min(max(kf, 0), max(r.n_kf - 1, 0));
}

// validity, first observation, observation count, lowest free pose of every landmark
__global__ void k_b_edges(Raw r, int32_t *first_e, int32_t *cnt, int32_t *lmin, int32_t *err) {
    const int e = blockIdx.x * kNT + threadIdx.x;
    if (e >= r.Ep + r.El) return;
    const bool pt = e < r.Ep;
    const int lml = pt ? r.ept_lm[e] : r.eln_lm[e - r.Ep], kf = pt ? r.ept_kf[e] : r.eln_kf[e - r.Ep];
    if (lml < 0 || lml >= (pt ? r.n_pt : r.n_ln) || kf < 0 || kf >= r.n_kf) {
        atomicMin(err, e);
        return;
    }
    const int lm = pt ? lml : r.n_pt + lml;
    atomicMin(&first_e[lm], e);
    atomicAdd(&cnt[lm], 1);
    const int h = r.kf_hidx[kf];
    if (h >= 0) atomicMin(&lmin[lm], h);
}
// envelope over the WHOLE window (every rank of a sharded window needs one layout)
// envelope: first_blk[h] = min over the edges at free pose h of lmin[landmark]. Thousands of edges
// share a pose, so the minimum is taken in LDS first (one copy per workgroup, a grid-stride run of
// edges each) and each workgroup folds its copy into the global one: a few global atomics per
// pose instead of one per edge (min is order-independent: the result is the same).
constexpr int kFirstBlkLds = 8192;
__global__ void k_b_first_blk(Raw r, const int32_t *lmin, int32_t *first_blk, int nf) {
    __shared__ int32_t sm[kFirstBlkLds];
    const int E = r.Ep + r.El;
    const bool lds = nf <= kFirstBlkLds;
    if (lds) {
        for (int h = threadIdx.x; h < nf; h += kNT) sm[h] = INT32_MAX;
        __syncthreads();
    }
    for (int e = blockIdx.x * kNT + threadIdx.x; e < E; e += gridDim.x * kNT) {
        int lm, kf;
        edge_of(r, e, lm, kf);
        const int h = r.kf_hidx[kf];
        if (h < 0) continue;
        if (lds) atomicMin(&sm[h], lmin[lm]);
        else atomicMin(&first_blk[h], lmin[lm]);
    }
    if (lds) {
        __syncthreads();
        for (int h = threadIdx.x; h < nf; h += kNT)
            if (sm[h] != INT32_MAX) atomicMin(&first_blk[h], sm[h]);
    }
}
// off[b] = number of keys < b in a sorted key array (b = 0..nb): the exclusive scan of the
// per-key counts, by binary search instead of one atomic per element
__global__ void k_b_lbound(const uint32_t *key, int64_t n, int nb, int32_t *off) {
    const int b = blockIdx.x * kNT + threadIdx.x;
    if (b > nb) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (key[mid] < (uint32_t)b) lo = mid + 1;
        else hi = mid;
    }
    off[b] = (int32_t)lo;
}
__global__ void k_b_iota(int32_t *a, int n) {
    const int i = blockIdx.x * kNT + threadIdx.x;
    if (i < n) a[i] = i;
}
// landmark key: id rank of the keyframe of its first observation (n_kf: never observed)
__global__ void k_b_key(Raw r, const int32_t *first_e, uint32_t *key, int32_t *idx) {
    const int l = blockIdx.x * kNT + threadIdx.x;
    if (l >= r.n_pt + r.n_ln) return;
    const int e = first_e[l];
    int k = r.n_kf;
    if (e < r.Ep + r.El) {
        int lm, kf;
        edge_of(r, e, lm, kf);
        k = r.kpos[kf];
    }
    key[l] = (uint32_t)k;
    idx[l] = l;
}
__global__ void k_b_gather_cnt(const int32_t *ord, const int32_t *cnt, int32_t *out, int n) {
    const int i = blockIdx.x * kNT + threadIdx.x;
    if (i < n) out[i] = cnt[ord[i]];
}
// owner of each landmark (plba_shard_plan: contiguous runs of ~equal edge count in key order) and
// the point / line ownership flags of this rank
__global__ void k_b_owner(const int32_t *ord, const int32_t *cs, const int32_t *acc, int n, int n_pt, int64_t total,
                          int R, int rank, int32_t *fp, int32_t *fl) {
    const int i = blockIdx.x * kNT + threadIdx.x;
    if (i >= n) return;
    int r = 0;
    if (R > 1) {
        const int64_t mid2 = 2 * (int64_t)acc[i] + cs[i];
        r = total > 0 ? (int)((mid2 * R) / (2 * total)) : 0;
        r = std::min(std::max(r, 0), R - 1);
    }
    const bool own = r == rank, pt = ord[i] < n_pt;
    fp[i] = own && pt ? 1 : 0;
    fl[i] = own && !pt ? 1 : 0;
}
// local landmark order: owned points in key order, then owned lines in key order
__global__ void k_b_local(const int32_t *ord, const int32_t *fp, const int32_t *fl, const int32_t *sp,
                          const int32_t *sl, int n, int32_t *lm_gpos, int32_t *loc, int32_t *info) {
    const int i = blockIdx.x * kNT + threadIdx.x;
    if (i >= n) return;
    const int NP = sp[n - 1] + fp[n - 1];
    if (i == n - 1) {
        info[0] = NP;
        info[1] = sl[n - 1] + fl[n - 1];
    }
    int pos = -1;
    if (fp[i]) pos = sp[i];
    else if (fl[i]) pos = NP + sl[i];
    if (pos >= 0) {
        lm_gpos[pos] = ord[i];
        loc[ord[i]] = pos;
    }
}
__global__ void k_b_lmcnt(const int32_t *lm_gpos, const int32_t *cnt, const int32_t *info, int n, int32_t *lc) {
    const int l = blockIdx.x * kNT + threadIdx.x;
    if (l > n) return;
    const int NL = info[0] + info[1];
    lc[l] = l < NL ? cnt[lm_gpos[l]] : 0;
}
__global__ void k_b_ekey(Raw r, const int32_t *loc, uint32_t *key, int32_t *val) {
    const int e = blockIdx.x * kNT + threadIdx.x;
    if (e >= r.Ep + r.El) return;
    int lm, kf;
    edge_of(r, e, lm, kf);
    const int l = loc[lm];
    key[e] = l >= 0 ? (uint32_t)l : (uint32_t)(r.n_pt + r.n_ln);
    val[e] = e;
}
// landmark-major CSR edge arrays (points first: local point landmarks precede local lines)
__global__ void k_b_gather(Raw r, const uint32_t *skey, const int32_t *se, const int32_t *lm_off, const int32_t *info,
                           int32_t *e_lm, int32_t *e_kf, int32_t *e_hidx, int32_t *e_orig, int32_t *e_gpos,
                           double *e_obs, double *e_info) {
    const int i = blockIdx.x * kNT + threadIdx.x;
    const int NL = info[0] + info[1];
    if (i >= lm_off[NL]) return;
    const int e = se[i];
    const bool pt = e < r.Ep;
    int lm, kf;
    edge_of(r, e, lm, kf);
    e_lm[i] = (int32_t)skey[i];
    e_kf[i] = kf;
    e_hidx[i] = r.kf_hidx[kf];
    e_orig[i] = pt ? e : e - r.Ep;
    e_gpos[i] = e;
    double o[4];
    if (pt) {
        o[0] = r.ept_obs[2 * (size_t)e];
        o[1] = r.ept_obs[2 * (size_t)e + 1];
        o[2] = o[3] = 0.0;
        e_info[i] = r.ept_info[e];
    } else {
        const size_t q = (size_t)(e - r.Ep);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = r.eln_obs[4 * q + k];
        e_info[i] = r.eln_info[q];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e_obs[4 * (size_t)i + k] = o[k];
}
__global__ void k_b_states(Raw r, const int32_t *lm_gpos, const int32_t *info, double *X) {
    const int l = blockIdx.x * kNT + threadIdx.x;
    if (l >= info[0] + info[1]) return;
    const int gp = lm_gpos[l];
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if (gp < r.n_pt) {
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] = r.pt_xyz[3 * (size_t)gp + k];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = r.ln_orth[4 * (size_t)(gp - r.n_pt) + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) X[4 * (size_t)l + k] = v[k];
}
// free-pose-major edge lists: key = Hessian index (nf: fixed pose or not an edge of this rank)
__global__ void k_b_pekey(const int32_t *e_hidx, const int32_t *lm_off, const int32_t *info, int n, int nf,
                          uint32_t *key, int32_t *val, int32_t *pcnt) {
    const int i = blockIdx.x * kNT + threadIdx.x;
    if (i >= n) return;
    const int E = lm_off[info[0] + info[1]];
    const int h = i < E ? e_hidx[i] : -1;
    key[i] = h >= 0 ? (uint32_t)h : (uint32_t)nf;
    val[i] = i;
    (void)pcnt;
}
__global__ void k_b_summary(const int32_t *info, const int32_t *lm_off, const int32_t *pe_off, int nf, int32_t *out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int NP = info[0], NLn = info[1];
    out[0] = NP;
    out[1] = NLn;
    out[2] = lm_off[NP + NLn];
    out[3] = lm_off[NP];
    out[4] = pe_off[nf];
}
// Schur triples of one landmark: (a, b) over its edges in CSR order, i1 = hidx[a] >= 0,
// i2 = hidx[b] >= i1 (the host build's for_pairs)
__global__ void k_b_tcnt(const int32_t *lm_off, const int32_t *e_hidx, int NL, int n, int64_t *tc) {
    const int l = blockIdx.x * kNT + threadIdx.x;
    if (l > n) return;
    int64_t c = 0;
    if (l < NL) {
        const int a0 = lm_off[l], a1 = lm_off[l + 1];
        for (int a = a0; a < a1; ++a) {
            const int i1 = e_hidx[a];
            if (i1 < 0) continue;
            for (int b = a0; b < a1; ++b) c += e_hidx[b] >= i1 ? 1 : 0;
        }
    }
    tc[l] = c;
}
__global__ void k_b_tfill(const int32_t *lm_off, const int32_t *e_hidx, const int64_t *toff, const int64_t *blk_base,
                          const int32_t *first_blk, int NL, uint32_t *key, uint64_t *val) {
    const int l = blockIdx.x * kNT + threadIdx.x;
    if (l >= NL) return;
    const int a0 = lm_off[l], a1 = lm_off[l + 1];
    int64_t t = toff[l];
    for (int a = a0; a < a1; ++a) {
        const int i1 = e_hidx[a];
        if (i1 < 0) continue;
        for (int b = a0; b < a1; ++b) {
            const int i2 = e_hidx[b];
            if (i2 < i1) continue;
            key[t] = (uint32_t)(blk_base[i2] + (i1 - first_blk[i2]));
            val[t] = ((uint64_t)(uint32_t)b << 32) | (uint32_t)a;  // little-endian int32 pair (a, b)
            ++t;
        }
    }
}

#define BCHECK(expr)                                                                                 \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess) {                                                                      \
            (void)hipGetLastError();                                                                 \
            snprintf(err, errlen, "window build: %s at %s:%d: %s", hipGetErrorString(_e), __FILE__, __LINE__, #expr); \
            return PLBA_E_DEVICE;                                                                    \
        }                                                                                            \
    } while (0)

template <class T>
hipError_t h2d(T *dst, const T *src, size_t n, hipStream_t s) {
    return n ? hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, s) : hipSuccess;
}

}  // namespace

// Stream-ordered (hipMallocAsync / hipFreeAsync on the solver stream): a device-synchronising
// hipFree would fail while another context of the process captures its step graphs.
void BuildMem::release(hipStream_t s) {
    if (base) (void)hipFreeAsync(base, s);
    base = nullptr;
    cap = 0;
}
int BuildMem::reserve(size_t bytes, hipStream_t s) {
    if (bytes <= cap) return PLBA_OK;
    release(s);
    const size_t want = bytes + bytes / 4;
    if (hipMallocAsync((void **)&base, want, s) != hipSuccess) {
        (void)hipGetLastError();
        base = nullptr;
        return PLBA_E_NOMEM;
    }
    cap = want;
    return PLBA_OK;
}

// stage-1 layout of BuildMem A (also kept for stage 2: lm_off, e_hidx, first_blk, blk_off, ...)
struct Stage1 {
    int32_t *ept_lm, *ept_kf, *eln_lm, *eln_kf, *kf_hidx, *kpos;
    double *ept_obs, *ept_info, *eln_obs, *eln_info, *pt_xyz, *ln_orth;
    int32_t *first_e, *cnt, *lmin, *err, *first_blk;
    uint32_t *key, *key2;
    int32_t *idx, *ord, *cs, *acc, *fp, *fl, *sp, *sl, *loc, *lm_gpos, *info, *lc, *lm_off;
    uint32_t *ekey, *ekey2;
    int32_t *eval, *eval2;
    int32_t *e_lm, *e_kf, *e_hidx, *e_orig, *e_gpos;
    double *e_obs, *e_info, *X;
    uint32_t *pkey, *pkey2;
    int32_t *pval, *pval2, *pcnt, *pe_off, *summary;
    int64_t *blk_base, *tc, *toff;
    int32_t *bcnt, *blk_off;
    void *temp;
    size_t temp_bytes;
};

static Stage1 carve1(char *base, const plba_graph *g, int nf, size_t temp_bytes, size_t &total) {
    Carver c{base};
    Stage1 s{};
    const size_t Ep = g->n_ept, El = g->n_eln, E = Ep + El, L = (size_t)g->n_pt + g->n_ln, nk = g->n_kf;
    s.ept_lm = c.take<int32_t>(Ep); s.ept_kf = c.take<int32_t>(Ep);
    s.eln_lm = c.take<int32_t>(El); s.eln_kf = c.take<int32_t>(El);
    s.kf_hidx = c.take<int32_t>(nk); s.kpos = c.take<int32_t>(nk);
    s.ept_obs = c.take<double>(2 * Ep); s.ept_info = c.take<double>(Ep);
    s.eln_obs = c.take<double>(4 * El); s.eln_info = c.take<double>(El);
    s.pt_xyz = c.take<double>(3 * (size_t)g->n_pt); s.ln_orth = c.take<double>(4 * (size_t)g->n_ln);
    s.first_e = c.take<int32_t>(L); s.cnt = c.take<int32_t>(L); s.lmin = c.take<int32_t>(L);
    s.err = c.take<int32_t>(1); s.first_blk = c.take<int32_t>(nf + 1);
    s.key = c.take<uint32_t>(L); s.key2 = c.take<uint32_t>(L);
    s.idx = c.take<int32_t>(L); s.ord = c.take<int32_t>(L); s.cs = c.take<int32_t>(L); s.acc = c.take<int32_t>(L);
    s.fp = c.take<int32_t>(L); s.fl = c.take<int32_t>(L); s.sp = c.take<int32_t>(L); s.sl = c.take<int32_t>(L);
    s.loc = c.take<int32_t>(L); s.lm_gpos = c.take<int32_t>(L); s.info = c.take<int32_t>(4);
    s.lc = c.take<int32_t>(L + 1); s.lm_off = c.take<int32_t>(L + 1);
    s.ekey = c.take<uint32_t>(E); s.ekey2 = c.take<uint32_t>(E); s.eval = c.take<int32_t>(E); s.eval2 = c.take<int32_t>(E);
    s.e_lm = c.take<int32_t>(E); s.e_kf = c.take<int32_t>(E); s.e_hidx = c.take<int32_t>(E);
    s.e_orig = c.take<int32_t>(E); s.e_gpos = c.take<int32_t>(E);
    s.e_obs = c.take<double>(4 * E); s.e_info = c.take<double>(E); s.X = c.take<double>(4 * L);
    s.pkey = c.take<uint32_t>(E); s.pkey2 = c.take<uint32_t>(E); s.pval = c.take<int32_t>(E); s.pval2 = c.take<int32_t>(E);
    s.pcnt = c.take<int32_t>(nf + 1); s.pe_off = c.take<int32_t>(nf + 1); s.summary = c.take<int32_t>(8);
    s.blk_base = c.take<int64_t>(nf + 1); s.tc = c.take<int64_t>(L + 1); s.toff = c.take<int64_t>(L + 1);
    // (block counts / offsets are sized in stage 2: nblk <= nf * (nf + 1) / 2 is unknown here)
    s.temp = c.take<char>(temp_bytes);
    s.temp_bytes = temp_bytes;
    total = c.off;
    return s;
}

static size_t stage1_temp_bytes(const plba_graph *g, int nf, hipStream_t st) {
    const size_t E = (size_t)g->n_ept + g->n_eln, L = (size_t)g->n_pt + g->n_ln;
    size_t need = 0, b = 0;
    (void)rocprim::radix_sort_pairs(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, (int32_t *)nullptr,
                                    (int32_t *)nullptr, std::max(L, E), 0, 32, st);
    need = std::max(need, b);
    (void)rocprim::exclusive_scan(nullptr, b, (int32_t *)nullptr, (int32_t *)nullptr, 0, std::max(L + 1, (size_t)nf + 1),
                                  rocprim::plus<int32_t>(), st);
    need = std::max(need, b);
    (void)rocprim::exclusive_scan(nullptr, b, (int64_t *)nullptr, (int64_t *)nullptr, (int64_t)0, L + 1,
                                  rocprim::plus<int64_t>(), st);
    need = std::max(need, b);
    return need + 1024;
}

static_assert(sizeof(Stage1) <= sizeof(WindowBuild::s1), "stage-1 layout fits WindowBuild::s1");

int build_stage1(BuildMem &A, WindowBuild &wb, char *err, size_t errlen) {
    const plba_graph *g = wb.g;
    hipStream_t st = wb.stream;
    // PLBA_TIMING: phase marks of the stage (each waits for the stream: timing runs only)
    const bool tmg = getenv("PLBA_TIMING") != nullptr;
    auto tlast = std::chrono::steady_clock::now();
    auto tmark = [&](const char *what) {
        if (!tmg) return;
        (void)hipStreamSynchronize(st);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[plba stage1] %-24s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - tlast).count());
        tlast = t;
    };
    const int nf = wb.nf, n_kf = g->n_kf, np = g->n_pt, nl = g->n_ln, Ep = g->n_ept, El = g->n_eln;
    const int E = Ep + El, L = np + nl;
    size_t total = 0;
    const size_t temp = stage1_temp_bytes(g, nf, st);
    (void)carve1(nullptr, g, nf, temp, total);
    if (A.reserve(total, st)) {
        snprintf(err, errlen, "window build: cannot allocate %zu bytes", total);
        return PLBA_E_NOMEM;
    }
    Stage1 s = carve1(A.base, g, nf, temp, total);
    // ---- the caller's arrays (pageable; the copies complete before plba_upload returns)
    BCHECK(h2d(s.ept_lm, g->ept_lm, Ep, st));
    BCHECK(h2d(s.ept_kf, g->ept_kf, Ep, st));
    BCHECK(h2d(s.eln_lm, g->eln_lm, El, st));
    BCHECK(h2d(s.eln_kf, g->eln_kf, El, st));
    BCHECK(h2d(s.kf_hidx, wb.kf_hidx, n_kf, st));
    BCHECK(h2d(s.kpos, wb.kpos, n_kf, st));
    BCHECK(h2d(s.ept_obs, g->ept_obs, 2 * (size_t)Ep, st));
    BCHECK(h2d(s.ept_info, g->ept_info, Ep, st));
    BCHECK(h2d(s.eln_obs, g->eln_obs, 4 * (size_t)El, st));
    BCHECK(h2d(s.eln_info, g->eln_info, El, st));
    BCHECK(h2d(s.pt_xyz, g->pt_xyz, 3 * (size_t)np, st));
    BCHECK(h2d(s.ln_orth, g->ln_orth, 4 * (size_t)nl, st));
    tmark("h2d caller arrays");
    BCHECK(hipMemsetAsync(s.first_e, 0x7F, sizeof(int32_t) * std::max(L, 1), st));
    BCHECK(hipMemsetAsync(s.lmin, 0x7F, sizeof(int32_t) * std::max(L, 1), st));
    BCHECK(hipMemsetAsync(s.cnt, 0, sizeof(int32_t) * std::max(L, 1), st));
    BCHECK(hipMemsetAsync(s.err, 0x7F, sizeof(int32_t), st));
    BCHECK(hipMemsetAsync(s.loc, 0xFF, sizeof(int32_t) * std::max(L, 1), st));
    BCHECK(hipMemsetAsync(s.pcnt, 0, sizeof(int32_t) * (nf + 1), st));
    BCHECK(hipMemsetAsync(s.info, 0, sizeof(int32_t) * 4, st));
    Raw r{s.ept_lm, s.ept_kf, s.eln_lm, s.eln_kf, s.kf_hidx, s.kpos, s.ept_obs, s.ept_info, s.eln_obs, s.eln_info,
          s.pt_xyz, s.ln_orth, n_kf, np, nl, Ep, El};
    if (E) hipLaunchKernelGGL(k_b_edges, dim3(grid(E)), dim3(kNT), 0, st, r, s.first_e, s.cnt, s.lmin, s.err);
    BCHECK(hipGetLastError());
    // An invalid edge is reported at the final read-back: every later kernel reads vertex ids
    // through edge_of's clamps, so a broken input never addresses outside the arrays (its build is
    // discarded); no round trip to the host in the middle of the stage.
    hipLaunchKernelGGL(k_b_iota, dim3(grid(nf)), dim3(kNT), 0, st, s.first_blk, nf);
    if (E && nf)
        hipLaunchKernelGGL(k_b_first_blk, dim3((unsigned)std::min<int64_t>(grid(E), 64)), dim3(kNT), 0, st, r, s.lmin,
                           s.first_blk, nf);
    BCHECK(hipGetLastError());
    tmark("memsets + edges + first_blk");
    size_t tb = s.temp_bytes;
    if (L > 0) {
        // ---- landmark order: stable sort by key = first-observing keyframe's id rank
        hipLaunchKernelGGL(k_b_key, dim3(grid(L)), dim3(kNT), 0, st, r, s.first_e, s.key, s.idx);
        BCHECK(hipGetLastError());
        BCHECK(rocprim::radix_sort_pairs(s.temp, tb, s.key, s.key2, s.idx, s.ord, (size_t)L, 0, bits_for(n_kf), st));
        hipLaunchKernelGGL(k_b_gather_cnt, dim3(grid(L)), dim3(kNT), 0, st, s.ord, s.cnt, s.cs, L);
        BCHECK(hipGetLastError());
        tb = s.temp_bytes;
        BCHECK(rocprim::exclusive_scan(s.temp, tb, s.cs, s.acc, 0, (size_t)L, rocprim::plus<int32_t>(), st));
        hipLaunchKernelGGL(k_b_owner, dim3(grid(L)), dim3(kNT), 0, st, s.ord, s.cs, s.acc, L, np, (int64_t)E,
                           wb.nranks, wb.rank, s.fp, s.fl);
        BCHECK(hipGetLastError());
        tb = s.temp_bytes;
        BCHECK(rocprim::exclusive_scan(s.temp, tb, s.fp, s.sp, 0, (size_t)L, rocprim::plus<int32_t>(), st));
        tb = s.temp_bytes;
        BCHECK(rocprim::exclusive_scan(s.temp, tb, s.fl, s.sl, 0, (size_t)L, rocprim::plus<int32_t>(), st));
        hipLaunchKernelGGL(k_b_local, dim3(grid(L)), dim3(kNT), 0, st, s.ord, s.fp, s.fl, s.sp, s.sl, L, s.lm_gpos,
                           s.loc, s.info);
        BCHECK(hipGetLastError());
    }
    tmark("landmark order");
    hipLaunchKernelGGL(k_b_lmcnt, dim3(grid(L + 1)), dim3(kNT), 0, st, s.lm_gpos, s.cnt, s.info, L, s.lc);
    BCHECK(hipGetLastError());
    tb = s.temp_bytes;
    BCHECK(rocprim::exclusive_scan(s.temp, tb, s.lc, s.lm_off, 0, (size_t)L + 1, rocprim::plus<int32_t>(), st));
    if (E) {
        // ---- landmark-major CSR: stable sort of the edges by local landmark (insertion order inside)
        hipLaunchKernelGGL(k_b_ekey, dim3(grid(E)), dim3(kNT), 0, st, r, s.loc, s.ekey, s.eval);
        BCHECK(hipGetLastError());
        tb = s.temp_bytes;
        BCHECK(rocprim::radix_sort_pairs(s.temp, tb, s.ekey, s.ekey2, s.eval, s.eval2, (size_t)E, 0, bits_for(L), st));
        hipLaunchKernelGGL(k_b_gather, dim3(grid(E)), dim3(kNT), 0, st, r, s.ekey2, s.eval2, s.lm_off, s.info, s.e_lm,
                           s.e_kf, s.e_hidx, s.e_orig, s.e_gpos, s.e_obs, s.e_info);
        hipLaunchKernelGGL(k_b_pekey, dim3(grid(E)), dim3(kNT), 0, st, s.e_hidx, s.lm_off, s.info, E, nf, s.pkey,
                           s.pval, s.pcnt);
        BCHECK(hipGetLastError());
        // ---- free-pose-major edge lists (ascending CSR index inside a pose)
        tb = s.temp_bytes;
        BCHECK(rocprim::radix_sort_pairs(s.temp, tb, s.pkey, s.pkey2, s.pval, s.pval2, (size_t)E, 0, bits_for(nf), st));
    }
    tmark("edge CSR + pose sort");
    if (L) hipLaunchKernelGGL(k_b_states, dim3(grid(L)), dim3(kNT), 0, st, r, s.lm_gpos, s.info, s.X);
    // free-pose CSR offsets from the sorted pose keys (non-free edges carry key nf, sorted last)
    if (E) hipLaunchKernelGGL(k_b_lbound, dim3(grid((int64_t)nf + 1)), dim3(kNT), 0, st, s.pkey2, (int64_t)E, nf, s.pe_off);
    else BCHECK(hipMemsetAsync(s.pe_off, 0, sizeof(int32_t) * (nf + 1), st));
    BCHECK(hipGetLastError());
    hipLaunchKernelGGL(k_b_summary, dim3(1), dim3(64), 0, st, s.info, s.lm_off, s.pe_off, nf, s.summary);
    BCHECK(hipGetLastError());
    // ---- read back the counts, the first invalid edge and the envelope
    int32_t sum[8] = {0};
    int32_t bad = kBig;
    wb.first_blk.assign(nf, 0);
    BCHECK(hipMemcpyAsync(sum, s.summary, sizeof(int32_t) * 5, hipMemcpyDeviceToHost, st));
    BCHECK(hipMemcpyAsync(&bad, s.err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (nf) BCHECK(hipMemcpyAsync(wb.first_blk.data(), s.first_blk, sizeof(int32_t) * nf, hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    tmark("states + summary + readback");
    if (bad != kBig) {
        wb.invalid = true;
        snprintf(err, errlen, "%s edge %d references a missing vertex", bad < Ep ? "point" : "line", bad < Ep ? bad : bad - Ep);
        return PLBA_E_INVALID;
    }
    wb.n_pt = sum[0];
    wb.n_ln = sum[1];
    wb.n_lm = sum[0] + sum[1];
    wb.E = sum[2];
    wb.Ep = sum[3];
    wb.El = sum[2] - sum[3];
    wb.n_free_edges = sum[4];
    wb.e_lm = s.e_lm; wb.e_kf = s.e_kf; wb.e_hidx = s.e_hidx; wb.e_orig = s.e_orig; wb.e_gpos = s.e_gpos;
    wb.e_obs = s.e_obs; wb.e_info = s.e_info; wb.X = s.X;
    wb.lm_off = s.lm_off; wb.lm_gpos = s.lm_gpos; wb.pe_off = s.pe_off; wb.pe_list = s.pval2;
    std::memcpy(wb.s1, &s, sizeof s);
    return PLBA_OK;
}

int build_stage2(BuildMem &A, BuildMem &B, WindowBuild &wb, const std::vector<int64_t> &blk_base, int nblk,
                 char *err, size_t errlen) {
    (void)A;
    Stage1 s;
    std::memcpy(&s, wb.s1, sizeof s);
    hipStream_t st = wb.stream;
    const int nf = wb.nf, NL = wb.n_lm, L = wb.g->n_pt + wb.g->n_ln;
    // first_blk back to the device is already there (s.first_blk); blk_base up
    BCHECK(h2d(s.blk_base, blk_base.data(), (size_t)nf + 1, st));
    hipLaunchKernelGGL(k_b_tcnt, dim3(grid(L + 1)), dim3(kNT), 0, st, s.lm_off, s.e_hidx, NL, L, s.tc);
    BCHECK(hipGetLastError());
    size_t tb = s.temp_bytes;
    BCHECK(rocprim::exclusive_scan(s.temp, tb, s.tc, s.toff, (int64_t)0, (size_t)L + 1, rocprim::plus<int64_t>(), st));
    int64_t T = 0;
    BCHECK(hipMemcpyAsync(&T, s.toff + L, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    if (T > INT32_MAX) {
        snprintf(err, errlen, "window build: %lld Schur triples exceed the int32 index range", (long long)T);
        return PLBA_E_INVALID;
    }
    wb.n_triples = T;
    // ---- B: keys / packed (a, b) pairs, sorted copies, block counts / offsets, sort temp
    size_t sort_tmp = 0, scan_tmp = 0;
    (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint64_t *)nullptr,
                                    (uint64_t *)nullptr, (size_t)std::max<int64_t>(T, 1), 0, 32, st);
    (void)rocprim::exclusive_scan(nullptr, scan_tmp, (int32_t *)nullptr, (int32_t *)nullptr, 0, (size_t)nblk + 1,
                                  rocprim::plus<int32_t>(), st);
    const size_t tmp = std::max(sort_tmp, scan_tmp) + 1024;
    Carver c{nullptr};
    auto layout = [&](Carver &cv, uint32_t *&k1, uint32_t *&k2, uint64_t *&v1, uint64_t *&v2, int32_t *&bc, int32_t *&bo,
                      void *&tp) {
        k1 = cv.take<uint32_t>((size_t)T); k2 = cv.take<uint32_t>((size_t)T);
        v1 = cv.take<uint64_t>((size_t)T); v2 = cv.take<uint64_t>((size_t)T);
        bc = cv.take<int32_t>((size_t)nblk + 1); bo = cv.take<int32_t>((size_t)nblk + 1);
        tp = cv.take<char>(tmp);
    };
    uint32_t *k1, *k2;
    uint64_t *v1, *v2;
    int32_t *bc, *bo;
    void *tp;
    layout(c, k1, k2, v1, v2, bc, bo, tp);
    if (B.reserve(c.off, st)) {
        snprintf(err, errlen, "window build: cannot allocate %zu bytes for the Schur triples", c.off);
        return PLBA_E_NOMEM;
    }
    Carver c2{B.base};
    layout(c2, k1, k2, v1, v2, bc, bo, tp);
    if (T > 0) {
        hipLaunchKernelGGL(k_b_tfill, dim3(grid(NL)), dim3(kNT), 0, st, s.lm_off, s.e_hidx, s.toff, s.blk_base,
                           s.first_blk, NL, k1, v1);
        BCHECK(hipGetLastError());
        tb = tmp;
        BCHECK(rocprim::radix_sort_pairs(tp, tb, k1, k2, v1, v2, (size_t)T, 0, bits_for(nblk), st));
    }
    // block offsets from the sorted block keys
    if (T > 0) hipLaunchKernelGGL(k_b_lbound, dim3(grid((int64_t)nblk + 1)), dim3(kNT), 0, st, k2, T, nblk, bo);
    else BCHECK(hipMemsetAsync(bo, 0, sizeof(int32_t) * ((size_t)nblk + 1), st));
    BCHECK(hipGetLastError());
    (void)bc;
    wb.h_blk_off.assign((size_t)nblk + 1, 0);
    BCHECK(hipMemcpyAsync(wb.h_blk_off.data(), bo, sizeof(int32_t) * ((size_t)nblk + 1), hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    wb.trip = reinterpret_cast<int32_t *>(v2);
    wb.blk_off = bo;
    return PLBA_OK;
}

}  // namespace plba
