// MapHandler::localBundleAdjustmentForPlukerWithG2O host logic (src/mapHandler.cpp:5851-6323)
// around the MI355X solve of plba.h. See plslam_map.hpp.
#include "plslam_map.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include <omp.h>

namespace plslam {

// Threads for the per-element passes of one LBA call (gather copies, remaps, write-back), when the
// pass is long enough to pay for the fork/join (the pool persists across calls): up to 8
// (PLSLAM_THREADS overrides; 1 = serial). C3 window in a C5-sized map on the GPU box's host:
// gather 0.66 -> 0.43 ms, write-back 1.09 -> 0.28 ms with 8.
static int pass_threads(size_t n) {
    static const int cap = [] {
        const char *e = getenv("PLSLAM_THREADS");
        return e ? std::max(1, atoi(e)) : 8;
    }();
    if (cap == 1 || n < 32768) return 1;
    return std::max(1, std::min(cap, omp_get_max_threads()));
}

// ----------------------------------------------------------------------------- helpers
int hamming(const Desc &a, const Desc &b) {  // cv::norm(a, b, NORM_HAMMING)
    const size_t n = std::min(a.size(), b.size());
    int d = 0;
    for (size_t i = 0; i < n; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

// General 4x4 inverse by cofactors (what Matrix4d::inverse() computes for the pose matrices,
// src/mapHandler.cpp:5940,5959,6302).
Mat4 inverse4(const Mat4 &m) {
    Mat4 inv;
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] +
             m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] -
             m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] +
             m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] -
              m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] -
             m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] +
             m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] -
             m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] +
              m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] +
             m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] -
             m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] +
              m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] -
              m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] -
             m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] +
             m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] -
              m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] +
              m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    const double r = 1.0 / det;
    for (double &v : inv) v *= r;
    return inv;
}

// ----------------------------------------------------------------------------- incremental window
// Per landmark slot: its observations flattened into an arena (observer kf_idx, observation,
// (float)(1/σ²) as the reference's const float& reads it, index in the landmark's lists), its
// position as the gather hands it over (point3D; changePlukerToOrth(NDw) for lines) and whether it
// is in the local registry. Runs are rewritten (appended) when the landmark changes and the arena
// is compacted when garbage exceeds the live edges.
struct LmEntry {
    int32_t off = -1, n = 0, idx = -1;  // arena run; the object's idx field
    uint8_t dirty = 0, local = 0;
    double pos[4] = {0, 0, 0, 0};
};
struct LmSide {
    int ow;                              // observation doubles per edge (2 points, 4 lines)
    std::vector<LmEntry> e;
    std::vector<int32_t> a_kf, a_oi;
    std::vector<double> a_obs, a_info;
    size_t live = 0;
    std::vector<int32_t> reg;            // local registry (slot indices; sorted + filtered lazily)
    bool reg_sorted = true;
    explicit LmSide(int w) : ow(w) {}
    LmEntry &at(int idx) {
        if ((int)e.size() <= idx) e.resize((size_t)idx + 1);
        return e[idx];
    }
    void clear() {
        e.clear(); a_kf.clear(); a_oi.clear(); a_obs.clear(); a_info.clear(); reg.clear();
        live = 0;
        reg_sorted = true;
    }
};
struct LandmarkStore {
    bool active = true;
    LmSide pt{2}, ln{4};
    std::vector<std::pair<int8_t, int32_t>> log;  // changed landmarks since the last gather
    LmSide &side(int kind) { return kind == 1 ? pt : ln; }
};
void landmark_changed(LandmarkStore *s, int kind, int idx) {
    if (!s || !s->active || idx < 0 || (kind != 1 && kind != 2)) return;
    LmEntry &en = s->side(kind).at(idx);
    if (!en.dirty) {
        en.dirty = 1;
        s->log.push_back({(int8_t)kind, idx});
    }
}

// ----------------------------------------------------------------------------- MapPoint
MapPoint::MapPoint(int idx_, const Vec3 &p, const Desc &desc, int kf_obs, const Vec2 &obs, const Vec3 &dir,
                   double sigma2)
    : idx(idx_), inlier(true), point3D(p) {  // src/mapFeatures.cpp:38-50
    desc_list.push_back(desc);
    obs_list.push_back(obs);
    kf_obs_list.push_back(kf_obs);
    dir_list.push_back(dir);
    sigma_list.push_back(sigma2);
    med_obs_dir = dir;
    med_desc = desc;
}

void MapPoint::addMapPointObservation(const Desc &desc, int kf_obs, const Vec2 &obs, const Vec3 &dir,
                                      double sigma2) {  // src/mapFeatures.cpp:52-60
    desc_list.push_back(desc);
    obs_list.push_back(obs);
    kf_obs_list.push_back(kf_obs);
    dir_list.push_back(dir);
    sigma_list.push_back(sigma2);
    updateAverageDescDir();
    landmark_changed(store, 1, idx);
}

// Index of the descriptor with the smallest median Hamming distance to the others
// (src/mapFeatures.cpp:57-86). The reference reads dist_idx[int(1+0.5*(n-1))], one past the
// end when n == 1; that single-observation case is clamped to the only descriptor here.
static int median_descriptor(const std::vector<Desc> &desc_list) {
    const int n = (int)desc_list.size();
    std::vector<int> conf((size_t)n * n, 0);
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            const int d = hamming(desc_list[i], desc_list[j]);
            conf[(size_t)i * n + j] = d;
            conf[(size_t)j * n + i] = d;
        }
    int max_dist = 99999, max_idx = 0;
    std::vector<int> dist_idx(n);
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) dist_idx[j] = conf[(size_t)i * n + j];
        std::sort(dist_idx.begin(), dist_idx.end());
        const int k = std::min(int(1 + 0.5 * (n - 1)), n - 1);
        const int idx_median = dist_idx[k];
        if (idx_median < max_dist) {
            max_dist = idx_median;
            max_idx = i;
        }
    }
    return max_idx;
}

void MapPoint::updateAverageDescDir() {
    const int n = (int)desc_list.size();
    if (n == 0) return;
    med_desc = desc_list[median_descriptor(desc_list)];
    // direction: mean of the observation directions (the reference sums into an
    // uninitialised Vector3d, src/mapFeatures.cpp:89-92; zero-initialised here)
    Vec3 s{0.0, 0.0, 0.0};
    for (int i = 0; i < (int)dir_list.size() && i < n; ++i)
        for (int k = 0; k < 3; ++k) s[k] += dir_list[i][k];
    for (int k = 0; k < 3; ++k) med_obs_dir[k] = s[k] / n;
}

// ----------------------------------------------------------------------------- MapLine
MapLine::MapLine(int idx_, const Vec6 &NDw_, const Desc &desc, int kf_obs, const Vec4 &obs, double sigma2)
    : idx(idx_), inlier(true), NDw(NDw_) {  // src/mapFeatures.cpp:114-122
    desc_list.push_back(desc);
    NDw_obs_list.push_back(obs);
    kf_obs_list.push_back(kf_obs);
    sigma_list.push_back(sigma2);
    med_desc = desc;
}

void MapLine::addMapLineObservation(const Desc &desc, int kf_obs, const Vec4 &obs, double sigma2) {
    desc_list.push_back(desc);  // src/mapFeatures.cpp:132-138
    NDw_obs_list.push_back(obs);
    sigma_list.push_back(sigma2);
    kf_obs_list.push_back(kf_obs);
    updateAverageDescDir();
    landmark_changed(store, 2, idx);
}

void MapLine::updateAverageDescDir() {  // src/mapFeatures.cpp:140-184 (USE_LINE_PLUKER)
    if (desc_list.empty()) return;
    med_desc = desc_list[median_descriptor(desc_list)];
}

static inline double norm3(const double *v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// changePlukerToOrth with getOrhtRFromPluker / getOrthWFromPluker (src/mapFeatures.cpp:186-249)
Vec4 MapLine::changePlukerToOrth(const Vec6 &L) {
    const double *n = L.data(), *d = L.data() + 3;
    const double nn = norm3(n), dn = norm3(d);
    double c[3] = {n[1] * d[2] - n[2] * d[1], n[2] * d[0] - n[0] * d[2], n[0] * d[1] - n[1] * d[0]};
    const double cn = norm3(c);
    const double u1[3] = {n[0] / nn, n[1] / nn, n[2] / nn};
    const double u2[3] = {d[0] / dn, d[1] / dn, d[2] / dn};
    const double u3[3] = {c[0] / cn, c[1] / cn, c[2] / cn};
    const double f = std::sqrt(nn * nn + dn * dn);
    Vec4 o;
    o[0] = std::atan2(u2[2], u3[2]);
    o[1] = std::asin(-u1[2]);
    o[2] = std::atan2(u1[1], u1[0]);
    o[3] = std::asin(dn / f);
    return o;
}

// changeOrthToPluker (src/mapFeatures.cpp:203-221): [w1·R.col(0); w2·R.col(1)]
Vec6 MapLine::changeOrthToPluker(const Vec4 &o) {
    const double s1 = std::sin(o[0]), c1 = std::cos(o[0]);
    const double s2 = std::sin(o[1]), c2 = std::cos(o[1]);
    const double s3 = std::sin(o[2]), c3 = std::cos(o[2]);
    const double w1 = std::cos(o[3]), w2 = std::sin(o[3]);
    Vec6 L;
    L[0] = w1 * (c2 * c3);
    L[1] = w1 * (c2 * s3);
    L[2] = w1 * (-s2);
    L[3] = w2 * (s1 * s2 * c3 - c1 * s3);
    L[4] = w2 * (s1 * s2 * s3 + c1 * c3);
    L[5] = w2 * (s1 * c2);
    return L;
}

// ----------------------------------------------------------------------------- Window
void Window::clear() {
    nofix_kfs.clear(); fix_kfs.clear(); local_pt.clear(); local_ls.clear();
    max_kf_id = maxPointId = 0;
    kf_Tcw.clear(); pt_xyz.clear(); ln_orth.clear(); ept_obs.clear(); ept_info.clear(); eln_obs.clear(); eln_info.clear();
    kf_fixed.clear();
    kf_id.clear(); pt_id.clear(); ln_id.clear(); ept_lm.clear(); ept_kf.clear(); eln_lm.clear(); eln_kf.clear();
    ept_kfp.clear(); eln_kfp.clear(); ept_obs_idx.clear(); eln_obs_idx.clear();
}

plba_graph Window::graph(double fx, double fy, double cx, double cy) const {
    plba_graph g{};
    g.n_kf = (int32_t)kf_id.size();
    g.n_pt = (int32_t)pt_id.size();
    g.n_ln = (int32_t)ln_id.size();
    g.n_ept = (int32_t)ept_lm.size();
    g.n_eln = (int32_t)eln_lm.size();
    g.fx = fx; g.fy = fy; g.cx = cx; g.cy = cy;
    g.kf_Tcw = kf_Tcw.data(); g.kf_fixed = kf_fixed.data(); g.kf_id = kf_id.data();
    g.pt_xyz = pt_xyz.data(); g.pt_id = pt_id.data();
    g.ln_orth = ln_orth.data(); g.ln_id = ln_id.data();
    g.ept_lm = ept_lm.data(); g.ept_kf = ept_kf.data(); g.ept_obs = ept_obs.data(); g.ept_info = ept_info.data();
    g.eln_lm = eln_lm.data(); g.eln_kf = eln_kf.data(); g.eln_obs = eln_obs.data(); g.eln_info = eln_info.data();
    // const float thHuberMono = sqrt(5.991)  (src/mapHandler.cpp:5978, 6035)
    g.huber_pt = (double)(float)std::sqrt(5.991);
    g.huber_ln = (double)(float)std::sqrt(5.991);
    return g;
}

// ----------------------------------------------------------------------------- MapHandler
MapHandler::MapHandler(double fx, double fy, double cx, double cy, const plba_opts *opts)
    : store_(new LandmarkStore()), fx_(fx), fy_(fy), cx_(cx), cy_(cy) {
    if (opts) {
        opts_ = *opts;
        have_opts_ = true;
    }
}

MapHandler::~MapHandler() {
    if (ctx_) plba_destroy(ctx_);
    for (auto *k : map_keyframes) delete k;
    for (auto *p : map_points) delete p;
    for (auto *l : map_lines) delete l;
}

void MapHandler::setError(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    err_ = buf;
}

static bool has_duplicate_id(const Window &w);

// A1 + A1b: window gather (src/mapHandler.cpp:5868-5921) and graph marshalling (:5923-6117).
// Same sets, orders, ids and error behaviour as the reference's std::map-keyed gather, in one
// pass over the observations: the per-edge arrays are written with observer ids while the ids
// are validated and the observers marked; the map is mutated (fixed observers become local) only
// once every observation is known valid, and the ids are then remapped to kf positions.
// The landmark pass scans the map (gatherScan, as the reference) or walks the local registry and
// copies each landmark's cached run (gatherIncremental); both produce the same arrays.
int MapHandler::gatherWindow(Window &w) {
    const auto t0 = std::chrono::steady_clock::now();
    w.clear();
    std::vector<uint8_t> observer(map_keyframes.size(), 0);
    int dirty = 0;
    const int rc = incremental ? gatherIncremental(w, observer, &dirty) : gatherScan(w, observer);
    last_dirty_ = dirty;
    if (rc) {
        w.clear();
        return rc;
    }
    const auto t1 = std::chrono::steady_clock::now();
    const int rc2 = finishGather(w, observer);
    if (getenv("PLSLAM_TIMING"))
        fprintf(stderr, "[plslam gather] landmarks %.3f ms, keyframes + remap %.3f ms\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    return rc2;
}

int MapHandler::gatherScan(Window &w, std::vector<uint8_t> &observer) {
    const int nkf_map = (int)map_keyframes.size();
    std::vector<uint8_t> valid(nkf_map, 0);
    for (int o = 0; o < nkf_map; ++o) valid[o] = map_keyframes[o] && map_keyframes[o]->kf_idx == o;
    std::vector<size_t> pt_off(1, 0), ln_off(1, 0);  // edge offsets per local landmark
    for (auto *p : map_points)
        if (p && p->local) {
            w.local_pt.push_back(p);  // :5877-5881
            pt_off.push_back(pt_off.back() + p->kf_obs_list.size());
        }
    for (auto *l : map_lines)
        if (l && l->local) {
            w.local_ls.push_back(l);  // :5882-5886
            ln_off.push_back(ln_off.back() + l->kf_obs_list.size());
        }
    const size_t npt = w.local_pt.size(), nln = w.local_ls.size(), n_ept = pt_off.back(), n_eln = ln_off.back();
    w.pt_id.resize(npt);
    w.pt_xyz.resize(npt * 3);
    w.ept_lm.resize(n_ept);
    w.ept_kf.resize(n_ept);
    w.ept_obs.resize(n_ept * 2);
    w.ept_info.resize(n_ept);
    w.ept_obs_idx.resize(n_ept);
    w.ln_id.resize(nln);
    w.ln_orth.resize(nln * 4);
    w.eln_lm.resize(n_eln);
    w.eln_kf.resize(n_eln);
    w.eln_obs.resize(n_eln * 4);
    w.eln_info.resize(n_eln);
    w.eln_obs_idx.resize(n_eln);
    // The landmark passes read the map only: an invalid observation ends the gather before the
    // map is touched (the reference exit(0)s, :5891-5895, 5907-5911).
    // point vertices + edges (:5976-6027); ept_kf holds the observer id until the remap below
    for (size_t li = 0, e = 0; li < npt; ++li) {
        MapPoint *p = w.local_pt[li];
        w.pt_id[li] = p->idx;  // + max_kf_id + 1 below
        for (int k = 0; k < 3; ++k) w.pt_xyz[li * 3 + k] = p->point3D[k];
        const size_t no = p->kf_obs_list.size();
        for (size_t i = 0; i < no; ++i, ++e) {
            const int kf_id = p->kf_obs_list[i];
            if (kf_id < 0 || kf_id >= nkf_map || !valid[kf_id]) {
                setError("[Wrong index in the map_keyframes and MapPoint obs] point %d obs kf %d", p->idx, kf_id);
                return PLBA_E_INVALID;
            }
            observer[kf_id] = 1;
            w.ept_lm[e] = (int32_t)li;
            w.ept_kf[e] = kf_id;
            w.ept_obs[2 * e] = p->obs_list[i][0];
            w.ept_obs[2 * e + 1] = p->obs_list[i][1];
            const float invSigma2 = 1.0 / p->sigma_list[i];  // const float& (:6009)
            w.ept_info[e] = (double)invSigma2;
            w.ept_obs_idx[e] = (int)i;
        }
    }
    // line vertices + edges (:6029-6117)
    for (size_t li = 0, e = 0; li < nln; ++li) {
        MapLine *l = w.local_ls[li];
        w.ln_id[li] = l->idx;  // + maxPointId + 1 below
        const size_t no = l->kf_obs_list.size();
        for (size_t i = 0; i < no; ++i, ++e) {
            const int kf_id = l->kf_obs_list[i];
            if (kf_id < 0 || kf_id >= nkf_map || !valid[kf_id]) {
                setError("[Wrong index in the map_keyframes and MapLine obs] line %d obs kf %d", l->idx, kf_id);
                return PLBA_E_INVALID;
            }
            observer[kf_id] = 1;
            w.eln_lm[e] = (int32_t)li;
            w.eln_kf[e] = kf_id;
            for (int k = 0; k < 4; ++k) w.eln_obs[4 * e + k] = l->NDw_obs_list[i][k];
            const float invSigma2 = 1.0 / l->sigma_list[i];  // (:6073)
            w.eln_info[e] = (double)invSigma2;
            w.eln_obs_idx[e] = (int)i;
        }
        const Vec4 o = MapLine::changePlukerToOrth(l->NDw);
        for (int k = 0; k < 4; ++k) w.ln_orth[li * 4 + k] = o[k];
    }
    return PLBA_OK;
}

// Rewrites one landmark's cached run from its object (or clears it: slot empty).
static void flatten(LandmarkStore &S, int kind, int idx, MapPoint *p, MapLine *l) {
    LmSide &sd = S.side(kind);
    LmEntry &en = sd.at(idx);
    en.dirty = 0;
    sd.live -= (size_t)en.n;
    en.off = -1;
    en.n = 0;
    if (!p && !l) {
        en.local = 0;
        return;
    }
    const std::vector<int> &kfl = p ? p->kf_obs_list : l->kf_obs_list;
    const std::vector<double> &sig = p ? p->sigma_list : l->sigma_list;
    const int n = (int)kfl.size();
    en.off = (int32_t)sd.a_kf.size();
    en.n = n;
    en.idx = p ? p->idx : l->idx;
    for (int i = 0; i < n; ++i) {
        sd.a_kf.push_back(kfl[i]);
        sd.a_oi.push_back(i);
        const float invSigma2 = 1.0 / sig[i];  // const float& (:6009, :6073)
        sd.a_info.push_back((double)invSigma2);
        if (p) {
            sd.a_obs.push_back(p->obs_list[i][0]);
            sd.a_obs.push_back(p->obs_list[i][1]);
        } else {
            for (int k = 0; k < 4; ++k) sd.a_obs.push_back(l->NDw_obs_list[i][k]);
        }
    }
    sd.live += (size_t)n;
    if (p) {
        for (int k = 0; k < 3; ++k) en.pos[k] = p->point3D[k];
    } else {
        const Vec4 o = MapLine::changePlukerToOrth(l->NDw);
        for (int k = 0; k < 4; ++k) en.pos[k] = o[k];
    }
}

// arena garbage (runs rewritten since) above the live edges: copy the live runs, slot order
static void compact(LmSide &sd) {
    if (sd.a_kf.size() <= 2 * sd.live + (1u << 16)) return;
    std::vector<int32_t> kf, oi;
    std::vector<double> obs, info;
    kf.reserve(sd.live); oi.reserve(sd.live); info.reserve(sd.live); obs.reserve(sd.live * sd.ow);
    for (LmEntry &en : sd.e) {
        if (en.off < 0) continue;
        const int32_t off = (int32_t)kf.size();
        kf.insert(kf.end(), sd.a_kf.begin() + en.off, sd.a_kf.begin() + en.off + en.n);
        oi.insert(oi.end(), sd.a_oi.begin() + en.off, sd.a_oi.begin() + en.off + en.n);
        info.insert(info.end(), sd.a_info.begin() + en.off, sd.a_info.begin() + en.off + en.n);
        obs.insert(obs.end(), sd.a_obs.begin() + (size_t)en.off * sd.ow, sd.a_obs.begin() + (size_t)(en.off + en.n) * sd.ow);
        en.off = off;
    }
    sd.a_kf.swap(kf); sd.a_oi.swap(oi); sd.a_obs.swap(obs); sd.a_info.swap(info);
}

int MapHandler::gatherIncremental(Window &w, std::vector<uint8_t> &observer, int *dirty) {
    LandmarkStore &S = *store_;
    const int nkf_map = (int)map_keyframes.size();
    std::vector<uint8_t> valid(nkf_map, 0);
    for (int o = 0; o < nkf_map; ++o) valid[o] = map_keyframes[o] && map_keyframes[o]->kf_idx == o;
    // the landmarks that changed since the last gather (and local ones never cached)
    int nd = 0;
    auto obj = [&](int kind, int idx, MapPoint *&p, MapLine *&l) {
        p = nullptr;
        l = nullptr;
        if (kind == 1 && idx < (int)map_points.size()) p = map_points[idx];
        if (kind == 2 && idx < (int)map_lines.size()) l = map_lines[idx];
    };
    for (const auto &c : S.log) {
        MapPoint *p;
        MapLine *l;
        obj(c.first, c.second, p, l);
        flatten(S, c.first, c.second, p, l);
        ++nd;
    }
    S.log.clear();
    for (int kind = 1; kind <= 2; ++kind) {
        LmSide &sd = S.side(kind);
        if (!sd.reg_sorted) {
            std::sort(sd.reg.begin(), sd.reg.end());
            sd.reg.erase(std::unique(sd.reg.begin(), sd.reg.end()), sd.reg.end());
            sd.reg_sorted = true;
        }
        size_t o = 0;
        for (int32_t idx : sd.reg) {
            MapPoint *p;
            MapLine *l;
            obj(kind, idx, p, l);
            LmEntry &en = sd.at(idx);
            if ((!p && !l) || !en.local) {
                en.local = 0;
                continue;
            }
            if (en.off < 0) {
                flatten(S, kind, idx, p, l);
                ++nd;
            }
            sd.reg[o++] = idx;
        }
        sd.reg.resize(o);
        compact(sd);
    }
    *dirty = nd;
    size_t n_ept = 0, n_eln = 0;
    for (int32_t idx : S.pt.reg) n_ept += (size_t)S.pt.e[idx].n;
    for (int32_t idx : S.ln.reg) n_eln += (size_t)S.ln.e[idx].n;
    const size_t npt = S.pt.reg.size(), nln = S.ln.reg.size();
    w.local_pt.resize(npt);
    w.local_ls.resize(nln);
    w.pt_id.resize(npt);
    w.pt_xyz.resize(npt * 3);
    w.ept_lm.resize(n_ept);
    w.ept_kf.resize(n_ept);
    w.ept_obs.resize(n_ept * 2);
    w.ept_info.resize(n_ept);
    w.ept_obs_idx.resize(n_ept);
    w.ln_id.resize(nln);
    w.ln_orth.resize(nln * 4);
    w.eln_lm.resize(n_eln);
    w.eln_kf.resize(n_eln);
    w.eln_obs.resize(n_eln * 4);
    w.eln_info.resize(n_eln);
    w.eln_obs_idx.resize(n_eln);
    // point vertices + edges (:5976-6027) then line vertices + edges (:6029-6117), from the cached
    // runs (memcpy per run; raw pointers: the vectors' storage does not move in the loop);
    // ept_kf / eln_kf hold the observer ids until finishGather
    // edge offset of every registered landmark (the runs are copied in parallel)
    std::vector<size_t> pt_e0(npt + 1, 0), ln_e0(nln + 1, 0);
    for (size_t li = 0; li < npt; ++li) pt_e0[li + 1] = pt_e0[li] + (size_t)S.pt.e[S.pt.reg[li]].n;
    for (size_t li = 0; li < nln; ++li) ln_e0[li + 1] = ln_e0[li] + (size_t)S.ln.e[S.ln.reg[li]].n;
    auto pass = [&](LmSide &sd, int ow, int pw, const std::vector<int32_t> &reg, const std::vector<size_t> &e0,
                    auto *objs, auto &local_out, int32_t *ids, double *pos, int32_t *lm, int32_t *kfo, double *obs,
                    double *info, int *oidx, const char *what) -> int {
        const int32_t *a_kf = sd.a_kf.data(), *a_oi = sd.a_oi.data();
        const double *a_obs = sd.a_obs.data(), *a_info = sd.a_info.data();
        const LmEntry *ent = sd.e.data();
        const uint8_t *vld = valid.data();
        uint8_t *obsr = observer.data();
        std::atomic<int64_t> first_bad{INT64_MAX};  // (landmark << 32 | observation) of the first invalid one
        const int64_t nreg = (int64_t)reg.size();
#pragma omp parallel for schedule(static) num_threads(pass_threads(e0.back()))
        for (int64_t li = 0; li < nreg; ++li) {
            const int32_t idx = reg[li];
            const LmEntry &en = ent[idx];
            local_out[li] = objs[idx];
            ids[li] = en.idx;
            for (int k = 0; k < pw; ++k) pos[li * pw + k] = en.pos[k];
            const size_t a = (size_t)en.off, n = (size_t)en.n, e = e0[li];
            // (runs are ~5 edges: element loops, a memcpy call per run costs more than the copy)
            for (size_t i = 0; i < n; ++i) {
                const int kf_id = a_kf[a + i];
                if (kf_id < 0 || kf_id >= nkf_map || !vld[kf_id]) {
                    int64_t cur = first_bad.load(std::memory_order_relaxed), mine = (li << 32) | (int64_t)i;
                    while (mine < cur && !first_bad.compare_exchange_weak(cur, mine)) {}
                    break;
                }
                if (!__atomic_load_n(&obsr[kf_id], __ATOMIC_RELAXED))  // (written once per KF: no line ping-pong)
                    __atomic_store_n(&obsr[kf_id], (uint8_t)1, __ATOMIC_RELAXED);
                lm[e + i] = (int32_t)li;
                kfo[e + i] = kf_id;
                info[e + i] = a_info[a + i];
                oidx[e + i] = a_oi[a + i];
                for (int k = 0; k < ow; ++k) obs[(e + i) * ow + k] = a_obs[(a + i) * ow + k];
            }
        }
        const int64_t bad = first_bad.load();
        if (bad != INT64_MAX) {  // the scan gather's message: the first invalid observation in map order
            const LmEntry &en = ent[reg[bad >> 32]];
            setError("[Wrong index in the map_keyframes and %s obs] %s %d obs kf %d", what, ow == 2 ? "point" : "line",
                     en.idx, a_kf[(size_t)en.off + (bad & 0xffffffff)]);
            return PLBA_E_INVALID;
        }
        return PLBA_OK;
    };
    int rc = pass(S.pt, 2, 3, S.pt.reg, pt_e0, map_points.data(), w.local_pt, w.pt_id.data(), w.pt_xyz.data(),
                  w.ept_lm.data(), w.ept_kf.data(), w.ept_obs.data(), w.ept_info.data(), w.ept_obs_idx.data(), "MapPoint");
    if (!rc)
        rc = pass(S.ln, 4, 4, S.ln.reg, ln_e0, map_lines.data(), w.local_ls, w.ln_id.data(), w.ln_orth.data(),
                  w.eln_lm.data(), w.eln_kf.data(), w.eln_obs.data(), w.eln_info.data(), w.eln_obs_idx.data(), "MapLine");
    return rc;
}

void MapHandler::adoptLandmark(int kind, int idx) {
    if (kind == 1 && idx >= 0 && idx < (int)map_points.size() && map_points[idx]) map_points[idx]->store = store_.get();
    if (kind == 2 && idx >= 0 && idx < (int)map_lines.size() && map_lines[idx]) map_lines[idx]->store = store_.get();
    if (!store_->active) return;
    LmSide &sd = store_->side(kind);
    LmEntry &en = sd.at(idx);
    const bool loc = kind == 1 ? map_points[idx] && map_points[idx]->local : map_lines[idx] && map_lines[idx]->local;
    if (loc && !en.local) {
        sd.reg.push_back(idx);
        sd.reg_sorted = false;
    }
    en.local = loc ? 1 : 0;
    landmark_changed(store_.get(), kind, idx);
}

void MapHandler::markLandmarkChanged(int kind, int idx) { landmark_changed(store_.get(), kind, idx); }

int MapHandler::setLandmarkLocal(int kind, int idx, bool local) {
    if (kind == 1) {
        if (idx < 0 || idx >= (int)map_points.size() || !map_points[idx]) return PLBA_E_INVALID;
        map_points[idx]->local = local;
    } else if (kind == 2) {
        if (idx < 0 || idx >= (int)map_lines.size() || !map_lines[idx]) return PLBA_E_INVALID;
        map_lines[idx]->local = local;
    } else {
        return PLBA_E_INVALID;
    }
    if (!store_->active) return PLBA_OK;
    LmSide &sd = store_->side(kind);
    LmEntry &en = sd.at(idx);
    if (local && !en.local) {
        sd.reg.push_back(idx);
        sd.reg_sorted = false;
    }
    en.local = local ? 1 : 0;  // (a cleared entry leaves the registry at the next gather)
    return PLBA_OK;
}

// The store rebuilt from the map: every landmark adopted, the registry = the local flags.
void MapHandler::rebuildLocalRegistry() {
    LandmarkStore &S = *store_;
    S.pt.clear();
    S.ln.clear();
    S.log.clear();
    S.active = incremental;
    for (size_t i = 0; i < map_points.size(); ++i)
        if (map_points[i]) adoptLandmark(1, (int)i);
    for (size_t i = 0; i < map_lines.size(); ++i)
        if (map_lines[i]) adoptLandmark(2, (int)i);
}

// Tests: the landmark pass of the scan gather and of the incremental gather, compared array by
// array (the map is not mutated: the KF part is not run).
int MapHandler::checkIncrementalGather(std::string *why) {
    Window a, b;
    std::vector<uint8_t> oa(map_keyframes.size(), 0), ob(map_keyframes.size(), 0);
    const int ra = gatherScan(a, oa);
    int nd = 0;
    const int rb = gatherIncremental(b, ob, &nd);
    auto fail = [&](const char *what) {
        if (why) *why = what;
        return 1;
    };
    if (ra != rb) return fail("status");
    if (ra) return PLBA_OK;
    if (oa != ob) return fail("observers");
    if (a.local_pt != b.local_pt || a.local_ls != b.local_ls) return fail("landmark sets");
    if (a.pt_id != b.pt_id || a.ln_id != b.ln_id) return fail("ids");
    if (a.pt_xyz != b.pt_xyz || a.ln_orth != b.ln_orth) return fail("positions");
    if (a.ept_lm != b.ept_lm || a.ept_kf != b.ept_kf || a.ept_obs != b.ept_obs || a.ept_info != b.ept_info ||
        a.ept_obs_idx != b.ept_obs_idx)
        return fail("point edges");
    if (a.eln_lm != b.eln_lm || a.eln_kf != b.eln_kf || a.eln_obs != b.eln_obs || a.eln_info != b.eln_info ||
        a.eln_obs_idx != b.eln_obs_idx)
        return fail("line edges");
    return PLBA_OK;
}

int MapHandler::finishGather(Window &w, const std::vector<uint8_t> &observer) {
    const int nkf_map = (int)map_keyframes.size();
    const size_t npt = w.local_pt.size(), n_ept = w.ept_lm.size(), n_eln = w.eln_lm.size();
    std::map<int, KeyFrame *> idx_fix_kfs, idx_nofix_kfs, idx_all_kfs;  // one entry per KF (~100)
    for (auto *k : map_keyframes)  // :5870-5875
        if (k && k->local) {
            idx_nofix_kfs.insert({k->kf_idx, k});
            idx_all_kfs.insert({k->kf_idx, k});
        }
    // observers outside the local set become fixed — and local, as a side effect (:5888-5919)
    for (int o = 0; o < nkf_map; ++o)
        if (observer[o]) {
            KeyFrame *k = map_keyframes[o];
            if (!k->local) {
                idx_fix_kfs.insert({o, k});
                idx_all_kfs.insert({o, k});
                k->local = true;
            }
        }

    // pose vertices: free KFs (id 0 fixed), then the fixed observers (:5931-5967)
    const size_t nkf = idx_nofix_kfs.size() + idx_fix_kfs.size();
    w.kf_Tcw.reserve(nkf * 12);
    w.kf_fixed.reserve(nkf);
    w.kf_id.reserve(nkf);
    std::map<int, int> kf_pos;  // kf_idx -> position in the kf arrays
    auto add_pose = [&](KeyFrame *k, bool fixed) {
        const Mat4 Tcw = inverse4(k->T_kf_w);
        kf_pos[k->kf_idx] = (int)w.kf_id.size();
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) w.kf_Tcw.push_back(Tcw[r * 4 + c]);
        w.kf_fixed.push_back(fixed ? 1 : 0);
        w.kf_id.push_back(k->kf_idx);
        if (w.max_kf_id < k->kf_idx + 1) w.max_kf_id = k->kf_idx + 1;
    };
    for (auto &kv : idx_nofix_kfs) {
        w.nofix_kfs.push_back(kv.second);
        add_pose(kv.second, kv.first == 0);
    }
    for (auto &kv : idx_fix_kfs) {
        w.fix_kfs.push_back(kv.second);
        add_pose(kv.second, true);
    }
    // observer id -> (kf_pos.at(id), idx_all_kfs.at(id)); every observer is in both maps
    std::vector<int> pos_of(nkf_map, -1);
    std::vector<KeyFrame *> kf_of(nkf_map, nullptr);
    for (int o = 0; o < nkf_map; ++o)
        if (observer[o]) {
            pos_of[o] = kf_pos.at(o);
            kf_of[o] = idx_all_kfs.at(o);
        }
    w.ept_kfp.resize(n_ept);
#pragma omp parallel for schedule(static) num_threads(pass_threads(n_ept))
    for (size_t i = 0; i < n_ept; ++i) {
        const int o = w.ept_kf[i];
        w.ept_kf[i] = pos_of[o];
        w.ept_kfp[i] = kf_of[o];
    }
    w.eln_kfp.resize(n_eln);
#pragma omp parallel for schedule(static) num_threads(pass_threads(n_eln))
    for (size_t i = 0; i < n_eln; ++i) {
        const int o = w.eln_kf[i];
        w.eln_kf[i] = pos_of[o];
        w.eln_kfp[i] = kf_of[o];
    }
    // vertex ids: point idx + max_kf_id + 1; line idx + maxPointId + 1 with maxPointId = the last
    // point's id + 1 (`if (maxPointId < id + 1);` — the condition is a no-op, :6025-6026)
    w.maxPointId = w.max_kf_id;
    for (auto &id : w.pt_id) id += w.max_kf_id + 1;
    if (npt) w.maxPointId = w.pt_id[npt - 1] + 1;
    for (auto &id : w.ln_id) id += w.maxPointId + 1;
    // g2o::SparseOptimizer::addVertex refuses a duplicate id; refuse the window instead
    if (has_duplicate_id(w)) {
        setError("duplicate g2o vertex id in the window");
        return PLBA_E_INVALID;
    }
    return PLBA_OK;
}

// any id shared by two vertices of the window: a bitmap over [min, max] when the range is
// comparable to the vertex count, a sort otherwise
static bool has_duplicate_id(const Window &w) {
    const wvector<int32_t> *lists[3] = {&w.kf_id, &w.pt_id, &w.ln_id};
    size_t n = 0;
    long long lo = 0, hi = -1;
    for (auto *v : lists)
        for (int32_t id : *v) {
            if (n++ == 0) lo = hi = id;
            lo = std::min<long long>(lo, id);
            hi = std::max<long long>(hi, id);
        }
    if (n < 2) return false;
    if (hi - lo + 1 <= (long long)(16 * n + 4096)) {
        std::vector<uint8_t> seen((size_t)(hi - lo + 1), 0);
        for (auto *v : lists)
            for (int32_t id : *v) {
                uint8_t &s = seen[(size_t)(id - lo)];
                if (s) return true;
                s = 1;
            }
        return false;
    }
    std::vector<int32_t> ids;
    ids.reserve(n);
    for (auto *v : lists) ids.insert(ids.end(), v->begin(), v->end());
    std::sort(ids.begin(), ids.end());
    return std::adjacent_find(ids.begin(), ids.end()) != ids.end();
}

int MapHandler::ensureCtx() {
    if (!ctx_) {
        plba_opts o;
        if (have_opts_) o = opts_;
        else plba_default_opts(&o);
        const int rc = plba_create(&ctx_, &o);
        if (rc) {
            setError("plba_create failed (%d): no usable MI355X device", rc);
            ctx_ = nullptr;
            return rc;
        }
    }
    return PLBA_OK;
}

int MapHandler::solve(const plba_graph &g, plba_result &r) {
    if (solve_fn_) {
        const int rc = solve_fn_(solve_user_, &g, &r);
        if (rc) setError("solver hook returned %d", rc);
        return rc;
    }
    if (!ctx_) {
        plba_opts o;
        if (have_opts_) o = opts_;
        else plba_default_opts(&o);
        const int rc = plba_create(&ctx_, &o);
        if (rc) {
            setError("plba_create failed (%d): no usable MI355X device", rc);
            ctx_ = nullptr;
            return rc;
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    int rc = plba_upload(ctx_, &g);
    last_upload_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (!rc) rc = plba_lba_plucker(ctx_, &r);
    if (rc) setError("plba: %s", plba_last_error(ctx_));
    return rc;
}

void MapHandler::storePosition(int kind, int idx, const double *pos) {
    if (!incremental || !store_->active || idx < 0) return;
    LmSide &sd = store_->side(kind);
    if (idx >= (int)sd.e.size()) return;
    LmEntry &en = sd.e[idx];
    if (en.dirty || en.off < 0) return;  // (re-read from the object at the next gather anyway)
    for (int k = 0; k < (kind == 1 ? 3 : 4); ++k) en.pos[k] = pos[k];
}

// A1d: post-solve outlier bookkeeping (src/mapHandler.cpp:6154-6293), edges in reverse order.
int MapHandler::outlierPass(Window &w, const std::vector<double> &ept_chi2, const std::vector<uint8_t> &ept_depth_ok,
                            const std::vector<uint8_t> &ept_level, const std::vector<double> &eln_chi2,
                            const std::vector<uint8_t> &eln_level, LbaStats &st) {
    (void)ept_level;
    (void)eln_level;  // level-1 errors were already refreshed by the solver (:6158-6160, 6226-6228)
    auto graph_dec = [&](int a, int b) -> bool {
        if (a < 0 || b < 0 || a >= (int)full_graph.size() || b >= (int)full_graph.size() ||
            b >= (int)full_graph[a].size() || a >= (int)full_graph[b].size()) {
            setError("full_graph has no entry (%d, %d)", a, b);
            return false;
        }
        full_graph[a][b]--;  // unsigned, as the reference's vector<vector<unsigned int>>
        full_graph[b][a]--;
        return true;
    };
    // first observation removed: re-base the landmark (push only — the reference never erases
    // it from the old KF's list; lines use map_points_kf_idx too, :6239-6251)
    auto rebase = [&](int kf_obs, int lm_idx_map, int new_kf_base) -> bool {
        auto it = map_points_kf_idx.find(kf_obs);
        if (it == map_points_kf_idx.end()) {
            setError("map_points_kf_idx.at(%d): no such key", kf_obs);
            return false;
        }
        for (int v : it->second)
            if (v == lm_idx_map) {
                auto jt = map_points_kf_idx.find(new_kf_base);
                if (jt == map_points_kf_idx.end()) {
                    setError("map_points_kf_idx.at(%d): no such key", new_kf_base);
                    return false;
                }
                jt->second.push_back(v);
                break;
            }
        return true;
    };

    for (int i = (int)w.ept_lm.size() - 1; i >= 0; --i) {  // points (:6157-6214)
        if (!(ept_chi2[i] > 5.991 || !ept_depth_ok[i])) continue;
        st.bad_point_obs++;
        KeyFrame *kf = w.ept_kfp[i];
        MapPoint *pMP = w.local_pt[w.ept_lm[i]];
        if (pMP->obs_list.size() > 1) {
            st.actually_bad_point_obs++;
            const int kf_obs = kf->kf_idx, lm_idx_map = pMP->idx, lm_idx_obs = w.ept_obs_idx[i];
            if (lm_idx_obs == 0 && !rebase(kf_obs, lm_idx_map, pMP->kf_obs_list[1])) return PLBA_E_STATE;
            pMP->desc_list.erase(pMP->desc_list.begin() + lm_idx_obs);
            pMP->obs_list.erase(pMP->obs_list.begin() + lm_idx_obs);
            pMP->dir_list.erase(pMP->dir_list.begin() + lm_idx_obs);
            pMP->kf_obs_list.erase(pMP->kf_obs_list.begin() + lm_idx_obs);
            for (int &f : kf->stereo_frame.stereo_pt_idx)
                if (f == lm_idx_map) {
                    f = -1;
                    break;
                }
            pMP->updateAverageDescDir();
            markLandmarkChanged(1, lm_idx_map);
            for (int idx : pMP->kf_obs_list)
                if (kf_obs != idx && !graph_dec(kf_obs, idx)) return PLBA_E_STATE;
        } else {
            pMP->inlier = false;
        }
    }
    for (int i = (int)w.eln_lm.size() - 1; i >= 0; --i) {  // lines (:6220-6288)
        if (!(eln_chi2[i] > 5.991)) continue;
        st.bad_line_obs++;
        KeyFrame *kf = w.eln_kfp[i];
        MapLine *lML = w.local_ls[w.eln_lm[i]];
        if (lML->NDw_obs_list.size() > 1) {
            st.actually_bad_line_obs++;
            const int kf_obs = kf->kf_idx, lm_idx_map = lML->idx, lm_idx_obs = w.eln_obs_idx[i];
            if (lm_idx_obs == 0 && !rebase(kf_obs, lm_idx_map, lML->kf_obs_list[1])) return PLBA_E_STATE;
            lML->desc_list.erase(lML->desc_list.begin() + lm_idx_obs);
            lML->NDw_obs_list.erase(lML->NDw_obs_list.begin() + lm_idx_obs);
            lML->kf_obs_list.erase(lML->kf_obs_list.begin() + lm_idx_obs);
            for (int &f : kf->stereo_frame.stereo_ls_idx)
                if (f == lm_idx_map) {
                    f = -1;
                    break;
                }
            lML->updateAverageDescDir();
            markLandmarkChanged(2, lm_idx_map);
            for (int idx : lML->kf_obs_list)
                if (kf_obs != idx && !graph_dec(kf_obs, idx)) return PLBA_E_STATE;
        } else {
            lML->inlier = false;
        }
    }
    return PLBA_OK;
}

int MapHandler::localBundleAdjustmentForPlukerWithG2O(LbaStats *stats) {
    using clk = std::chrono::steady_clock;
    LbaStats st;
    const auto t0 = clk::now();
    Window &w = win_;
    int rc = gatherWindow(w);
    if (rc) return rc;
    const plba_graph g = w.graph(fx_, fy_, cx_, cy_);
    st.n_free_kf = (int)w.nofix_kfs.size();
    st.n_fixed_kf = (int)w.fix_kfs.size();
    st.n_pt = g.n_pt; st.n_ln = g.n_ln; st.n_ept = g.n_ept; st.n_eln = g.n_eln;

    std::vector<double> &Tcw = out_Tcw_, &xyz = out_xyz_, &orth = out_orth_, &ept_chi2 = out_ept_chi2_,
                        &eln_chi2 = out_eln_chi2_;
    std::vector<uint8_t> &ept_depth = out_ept_depth_, &ept_level = out_ept_level_, &eln_level = out_eln_level_;
    Tcw.resize(w.kf_Tcw.size()); xyz.resize(w.pt_xyz.size()); orth.resize(w.ln_orth.size());
    ept_chi2.resize(g.n_ept); eln_chi2.resize(g.n_eln);
    ept_depth.resize(g.n_ept); ept_level.resize(g.n_ept); eln_level.resize(g.n_eln);
    plba_result r{};
    r.kf_Tcw = Tcw.data(); r.pt_xyz = xyz.data(); r.ln_orth = orth.data();
    r.ept_chi2 = ept_chi2.data(); r.ept_depth_ok = ept_depth.data(); r.ept_level = ept_level.data();
    r.eln_chi2 = eln_chi2.data(); r.eln_level = eln_level.data();
    const auto t1 = clk::now();
    rc = solve(g, r);  // A1c (:6119-6152) on the device
    if (rc) return rc;
    const auto t2 = clk::now();
    st.upload_ms = solve_fn_ ? 0.0 : last_upload_ms_;
    st.dirty_landmarks = last_dirty_;
    st.iters[0] = r.iters[0]; st.iters[1] = r.iters[1];
    st.chi2[0] = r.chi2[0]; st.chi2[1] = r.chi2[1];
    for (uint8_t l : eln_level) st.bad_line_stage1 += l == 1;  // "Bad Obs" (:6137-6147)

    rc = outlierPass(w, ept_chi2, ept_depth, ept_level, eln_chi2, eln_level, st);
    if (rc) return rc;

    // A1e: write-back (:6296-6319). Free KFs (KF 0 included — it is in idx_nofix_kfs even though
    // its vertex is fixed) get T_kf_w = estimate().inverse(); the vertex estimate is the 4x4
    // inverse taken at graph build with R|t replaced by the solver's.
    for (size_t k = 0; k < w.nofix_kfs.size(); ++k) {
        KeyFrame *kf = w.nofix_kfs[k];
        Mat4 est = inverse4(kf->T_kf_w);
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 4; ++b) est[a * 4 + b] = Tcw[k * 12 + a * 4 + b];
        kf->T_kf_w = inverse4(est);
    }
    const size_t nwp = w.local_pt.size(), nwl = w.local_ls.size();
#pragma omp parallel for schedule(static) num_threads(pass_threads(nwp))
    for (size_t p = 0; p < nwp; ++p) {
        for (int k = 0; k < 3; ++k) w.local_pt[p]->point3D[k] = xyz[p * 3 + k];
        storePosition(1, w.local_pt[p]->idx, &xyz[p * 3]);
    }
#pragma omp parallel for schedule(static) num_threads(pass_threads(16 * nwl))
    for (size_t l = 0; l < nwl; ++l) {
        Vec4 o{orth[l * 4], orth[l * 4 + 1], orth[l * 4 + 2], orth[l * 4 + 3]};
        w.local_ls[l]->NDw = MapLine::changeOrthToPluker(o);
        if (incremental) {  // the next gather's changePlukerToOrth(NDw) (not o: the round trip rounds)
            const Vec4 o2 = MapLine::changePlukerToOrth(w.local_ls[l]->NDw);
            storePosition(2, w.local_ls[l]->idx, o2.data());
        }
    }
    const auto t3 = clk::now();
    st.gather_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    st.solve_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    st.bookkeeping_ms = std::chrono::duration<double, std::milli>(t3 - t2).count();
    if (stats) *stats = st;
    return PLBA_OK;
}

// ------------------------------------------------------------------ hand-rolled LM LBA (§8f row 1)
Mat4 inverse_se3(const Mat4 &T) {  // src2/auxiliar.cpp:113-122
    Mat4 Ti{};
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Ti[i * 4 + j] = T[j * 4 + i];
        Ti[i * 4 + 3] = -(T[0 * 4 + i] * T[3] + T[1 * 4 + i] * T[7] + T[2 * 4 + i] * T[11]);
    }
    Ti[15] = 1.0;
    return Ti;
}
static void skew3(const double *v, double *M) {
    M[0] = 0;     M[1] = -v[2]; M[2] = v[1];
    M[3] = v[2];  M[4] = 0;     M[5] = -v[0];
    M[6] = -v[1]; M[7] = v[0];  M[8] = 0;
}
static void mul3(const double *A, const double *B, double *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
Mat4 expmap_se3(const Vec6 &x) {  // src2/auxiliar.cpp:124-141
    const double w[3] = {x[3], x[4], x[5]};
    double t[3] = {x[0], x[1], x[2]};
    const double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(theta < 0.000001)) {
        double s[9], ss[9], V[9];
        skew3(w, s);
        for (double &v : s) v /= theta;
        mul3(s, s, ss);
        const double st = std::sin(theta), ct = 1.0 - std::cos(theta);
        for (int i = 0; i < 9; ++i) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            R[i] = (I + s[i] * st) + ss[i] * ct;
            V[i] = (I + s[i] * ct / theta) + ss[i] * (theta - st) / theta;
        }
        const double t0 = t[0], t1 = t[1], t2 = t[2];
        for (int i = 0; i < 3; ++i) t[i] = V[i * 3] * t0 + V[i * 3 + 1] * t1 + V[i * 3 + 2] * t2;
    }
    Mat4 T{};
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[i * 4 + j] = R[i * 3 + j];
        T[i * 4 + 3] = t[i];
    }
    T[15] = 1.0;
    return T;
}
Vec6 logmap_se3(const Mat4 &T) {  // src2/auxiliar.cpp:143-173
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    double w[3] = {0, 0, 0}, V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double cosine = (R[0] + R[4] + R[8] - 1.0) / 2.0;
    if (cosine > 1.0) cosine = 1.0;
    else if (cosine < -1.0) cosine = -1.0;
    double sine = std::sqrt(1.0 - cosine * cosine);
    if (sine > 1.0) sine = 1.0;
    else if (sine < -1.0) sine = -1.0;
    const double theta = std::acos(cosine);
    if (theta > 0.000001) {
        w[0] = theta * (R[7] - R[5]) / (2.0 * sine);
        w[1] = theta * (R[2] - R[6]) / (2.0 * sine);
        w[2] = theta * (R[3] - R[1]) / (2.0 * sine);
        double s[9], ss[9];
        skew3(w, s);
        for (double &v : s) v /= theta;
        mul3(s, s, ss);
        for (int i = 0; i < 9; ++i) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            V[i] = (I + s[i] * (1.0 - cosine) / theta) + ss[i] * (theta - sine) / theta;
        }
    }
    // t = V⁻¹·Vt (closed-form 3x3 inverse)
    const double c0 = V[4] * V[8] - V[5] * V[7], c1 = V[5] * V[6] - V[3] * V[8], c2 = V[3] * V[7] - V[4] * V[6];
    const double det = V[0] * c0 + V[1] * c1 + V[2] * c2;
    const double Vi[9] = {c0 / det, (V[2] * V[7] - V[1] * V[8]) / det, (V[1] * V[5] - V[2] * V[4]) / det,
                          c1 / det, (V[0] * V[8] - V[2] * V[6]) / det, (V[2] * V[3] - V[0] * V[5]) / det,
                          c2 / det, (V[1] * V[6] - V[0] * V[7]) / det, (V[0] * V[4] - V[1] * V[3]) / det};
    const double Vt[3] = {T[3], T[7], T[11]};
    Vec6 x;
    for (int i = 0; i < 3; ++i) x[i] = Vi[i * 3] * Vt[0] + Vi[i * 3 + 1] * Vt[1] + Vi[i * 3 + 2] * Vt[2];
    x[3] = w[0]; x[4] = w[1]; x[5] = w[2];
    return x;
}

int MapHandler::localBundleAdjustmentForPluker(HlmStats *stats) {
    using clk = std::chrono::steady_clock;
    HlmStats st;
    const auto t0 = clk::now();
    // kf_list: local KFs except KF 0, in map order (:1511-1524)
    std::vector<KeyFrame *> kf_list;
    for (auto *k : map_keyframes)
        if (k && k->local && k->kf_idx != 0) kf_list.push_back(k);
    std::vector<MapPoint *> pts;
    std::vector<MapLine *> lns;
    for (auto *p : map_points)
        if (p && p->local) pts.push_back(p);  // :1527-1565
    for (auto *l : map_lines)
        if (l && l->local) {  // :1567-1607 (orthNDw is written here, a side effect)
            l->orthNDw = MapLine::changePlukerToOrth(l->NDw);
            lns.push_back(l);
        }
    // observations: pt_obs_list / ls_obs_list; an observation whose KF slot is NULL is skipped by
    // the optimiser (:1652, 1741) and so never reaches the graph here
    std::map<int, int> kf_pos;
    std::vector<double> kf_Tcw, kf_x;
    std::vector<uint8_t> kf_fixed;
    std::vector<int32_t> kf_id;
    auto add_kf = [&](KeyFrame *k, bool fixed) {
        kf_pos[k->kf_idx] = (int)kf_id.size();
        const Mat4 Tiw = inverse_se3(k->T_kf_w);  // Tiw = inverse_se3(T_kf_w) (:1657-1659)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) kf_Tcw.push_back(Tiw[r * 4 + c]);
        for (int i = 0; i < 6; ++i) kf_x.push_back(k->x_kf_w[i]);
        kf_fixed.push_back(fixed ? 1 : 0);
        kf_id.push_back(k->kf_idx);
    };
    for (auto *k : kf_list) add_kf(k, false);
    auto observer = [&](int o) -> int {
        if (o < 0 || o >= (int)map_keyframes.size() || !map_keyframes[o]) return -1;
        auto it = kf_pos.find(o);
        if (it != kf_pos.end()) return it->second;
        add_kf(map_keyframes[o], true);
        return (int)kf_id.size() - 1;
    };
    std::vector<double> pt_xyz, ept_obs, ln_orth, ln_plk, eln_obs;
    std::vector<int32_t> pt_id, ln_id, ept_lm, ept_kf, eln_lm, eln_kf;
    for (size_t i = 0; i < pts.size(); ++i) {
        MapPoint *p = pts[i];
        pt_id.push_back(p->idx);
        for (int k = 0; k < 3; ++k) pt_xyz.push_back(p->point3D[k]);
        for (size_t o = 0; o < p->kf_obs_list.size(); ++o) {
            ++st.n_pt_obs;
            const int kp = observer(p->kf_obs_list[o]);
            if (kp < 0) continue;
            ept_lm.push_back((int32_t)i);
            ept_kf.push_back(kp);
            ept_obs.push_back(p->obs_list[o][0]);
            ept_obs.push_back(p->obs_list[o][1]);
        }
    }
    for (size_t i = 0; i < lns.size(); ++i) {
        MapLine *l = lns[i];
        ln_id.push_back(l->idx);
        for (int k = 0; k < 4; ++k) ln_orth.push_back(l->orthNDw[k]);
        for (int k = 0; k < 6; ++k) ln_plk.push_back(l->NDw[k]);
        for (size_t o = 0; o < l->kf_obs_list.size(); ++o) {
            ++st.n_ls_obs;
            const int kp = observer(l->kf_obs_list[o]);
            if (kp < 0) continue;
            eln_lm.push_back((int32_t)i);
            eln_kf.push_back(kp);
            for (int k = 0; k < 4; ++k) eln_obs.push_back(l->NDw_obs_list[o][k]);
        }
    }
    st.n_kf_list = (int)kf_list.size();
    st.n_fixed_kf = (int)kf_id.size() - st.n_kf_list;
    st.n_pt = (int)pts.size();
    st.n_ln = (int)lns.size();
    if (st.n_pt_obs + st.n_ls_obs == 0) {  // :1610-1614
        st.ret = -1;
        if (stats) *stats = st;
        return PLBA_OK;
    }
    std::vector<double> ept_info(ept_lm.size(), 1.0), eln_info(eln_lm.size(), 1.0);
    plba_graph g{};
    g.n_kf = (int32_t)kf_id.size(); g.n_pt = (int32_t)pt_id.size(); g.n_ln = (int32_t)ln_id.size();
    g.n_ept = (int32_t)ept_lm.size(); g.n_eln = (int32_t)eln_lm.size();
    g.fx = fx_; g.fy = fy_; g.cx = cx_; g.cy = cy_;
    g.kf_Tcw = kf_Tcw.data(); g.kf_fixed = kf_fixed.data(); g.kf_id = kf_id.data();
    g.pt_xyz = pt_xyz.data(); g.pt_id = pt_id.data(); g.ln_orth = ln_orth.data(); g.ln_id = ln_id.data();
    g.ept_lm = ept_lm.data(); g.ept_kf = ept_kf.data(); g.ept_obs = ept_obs.data(); g.ept_info = ept_info.data();
    g.eln_lm = eln_lm.data(); g.eln_kf = eln_kf.data(); g.eln_obs = eln_obs.data(); g.eln_info = eln_info.data();
    plba_hlm_state hs{kf_x.data(), ln_plk.data(), nullptr};
    std::vector<double> x_out(kf_x.size()), T_out(kf_Tcw.size()), xyz_out(pt_xyz.size()), orth_out(ln_orth.size());
    plba_hlm_result r{};
    r.kf_x = x_out.data(); r.kf_Tcw = T_out.data(); r.pt_xyz = xyz_out.data(); r.ln_orth = orth_out.data();
    const auto t1 = clk::now();
    int rc;
    if (hlm_fn_) {
        rc = hlm_fn_(hlm_user_, &g, &hs, &hlm_params, &r);
        if (rc) setError("hand-rolled LM solver hook returned %d", rc);
    } else {
        rc = ensureCtx();
        if (!rc) rc = plba_upload(ctx_, &g);
        if (!rc) rc = plba_hlm_lba(ctx_, &hs, &hlm_params, &r);
        if (rc) setError("plba: %s", plba_last_error(ctx_));
    }
    if (rc) return rc;
    const auto t2 = clk::now();
    st.linearizations = r.linearizations; st.solves = r.solves; st.accepted = r.accepted;
    st.err = r.err; st.lambda = r.lambda;
    if (vo_inserting_kf) {  // :2160, 2327-2328
        st.ret = -1;
    } else {
        // :2165-2198. KFs: T_kf_w = expmap_se3(X_i) (x_kf_w itself is not updated)
        for (size_t k = 0; k < kf_list.size(); ++k) {
            Vec6 x;
            for (int i = 0; i < 6; ++i) x[i] = x_out[k * 6 + i];
            kf_list[k]->T_kf_w = expmap_se3(x);
        }
        for (size_t i = 0; i < pts.size(); ++i) {
            double dx[3], n2 = 0;
            for (int k = 0; k < 3; ++k) {
                dx[k] = xyz_out[i * 3 + k] - pts[i]->point3D[k];
                n2 += dx[k] * dx[k];
            }
            if (std::sqrt(n2) > 0.01) {
                pts[i]->inlier = false;
                ++st.pt_outliers;
            }
            for (int k = 0; k < 3; ++k) pts[i]->point3D[k] = xyz_out[i * 3 + k];
            markLandmarkChanged(1, pts[i]->idx);
        }
        for (size_t i = 0; i < lns.size(); ++i) {
            // NDw = changeOrthToPluker(DX) with DX = X − orthNDw: the reference converts the
            // difference, not the new estimate (:2190-2196) — reproduced
            Vec4 dx;
            double n2 = 0;
            for (int k = 0; k < 4; ++k) {
                dx[k] = orth_out[i * 4 + k] - lns[i]->orthNDw[k];
                n2 += dx[k] * dx[k];
            }
            if (std::sqrt(n2) > 0.01) {
                lns[i]->inlier = false;
                ++st.ln_outliers;
            }
            lns[i]->NDw = MapLine::changeOrthToPluker(dx);
            markLandmarkChanged(2, lns[i]->idx);
        }
        // "Remove bad observations" (:2200-2322) acts on observations flagged -1 in column 5,
        // which nothing sets (:1549, 1591): no-op, as in the reference
        st.ret = 0;
    }
    const auto t3 = clk::now();
    st.gather_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    st.solve_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    st.writeback_ms = std::chrono::duration<double, std::milli>(t3 - t2).count();
    if (stats) *stats = st;
    return PLBA_OK;
}

// ----------------------------------------------------------------------------- local mapping
// formLocalMap(KeyFrame*) (src/mapHandler.cpp:1073-1137). The reference dereferences
// map_keyframes[i] and map_points[lm_idx] unchecked; a map on which it would crash is refused
// here before any flag changes.
int MapHandler::formLocalMap(int kf_idx) {
    if (kf_idx < 0 || kf_idx >= (int)map_keyframes.size() || !map_keyframes[kf_idx]) {
        setError("formLocalMap: no keyframe %d", kf_idx);
        return PLBA_E_INVALID;
    }
    const int g_size = (int)full_graph.size() - 1;
    auto in_window = [&](int i) {  // :1117
        return full_graph[g_size][i] >= (unsigned)params.min_lm_cov_graph || std::abs(g_size - i) <= params.min_kf_local_map;
    };
    auto feats_ok = [&](const KeyFrame *k) {
        for (int lm : k->stereo_frame.stereo_pt_idx)
            if (lm < -1 || lm >= (int)map_points.size()) return false;
        for (int lm : k->stereo_frame.stereo_ls_idx)
            if (lm < -1 || lm >= (int)map_lines.size()) return false;
        return true;
    };
    if (!feats_ok(map_keyframes[kf_idx])) {
        setError("formLocalMap: keyframe %d has a feature idx outside the map", kf_idx);
        return PLBA_E_INVALID;
    }
    for (int i = 0; i < g_size; ++i) {
        if ((int)full_graph[g_size].size() <= i) {
            setError("formLocalMap: full_graph row %d too short", g_size);
            return PLBA_E_INVALID;
        }
        if (!in_window(i)) continue;
        if (i >= (int)map_keyframes.size() || !map_keyframes[i] || !feats_ok(map_keyframes[i])) {
            setError("formLocalMap: covisible keyframe %d missing or inconsistent", i);
            return PLBA_E_INVALID;
        }
    }
    // reset local KFs & LMs (:1076-1091). Incremental: only the registered local landmarks are
    // reset (the registry holds every landmark whose flag is set), O(window) instead of O(map).
    for (auto *k : map_keyframes)
        if (k) k->local = false;
    const bool inc = incremental && store_->active;
    if (inc) {
        for (int kind = 1; kind <= 2; ++kind) {
            LmSide &sd = store_->side(kind);
            for (int32_t idx : sd.reg) {
                if (kind == 1 && idx < (int)map_points.size() && map_points[idx]) map_points[idx]->local = false;
                if (kind == 2 && idx < (int)map_lines.size() && map_lines[idx]) map_lines[idx]->local = false;
                sd.at(idx).local = 0;
            }
            sd.reg.clear();
            sd.reg_sorted = true;
        }
    } else {
        for (auto *p : map_points)
            if (p) p->local = false;
        for (auto *l : map_lines)
            if (l) l->local = false;
    }
    auto mark = [&](const KeyFrame *k) {
        for (int lm : k->stereo_frame.stereo_pt_idx)
            if (lm != -1 && map_points[lm]) {
                map_points[lm]->local = true;
                if (inc) {
                    LmEntry &en = store_->pt.at(lm);
                    if (!en.local) {
                        en.local = 1;
                        store_->pt.reg.push_back(lm);
                        store_->pt.reg_sorted = false;
                    }
                }
            }
        for (int lm : k->stereo_frame.stereo_ls_idx)
            if (lm != -1 && map_lines[lm]) {
                map_lines[lm]->local = true;
                if (inc) {
                    LmEntry &en = store_->ln.at(lm);
                    if (!en.local) {
                        en.local = 1;
                        store_->ln.reg.push_back(lm);
                        store_->ln.reg_sorted = false;
                    }
                }
            }
    };
    // the KF itself and its landmarks (:1094-1113)
    map_keyframes[kf_idx]->local = true;
    mark(map_keyframes[kf_idx]);
    // covisible / recent keyframes from the last full_graph row (:1115-1135)
    for (int i = 0; i < g_size; ++i)
        if (in_window(i)) {
            map_keyframes[i]->local = true;
            mark(map_keyframes[i]);
        }
    return PLBA_OK;
}

// removeBadMapLandmarksForPluker (src/mapHandler.cpp:3816-3897). Candidates: non-local
// landmarks whose first observing KF is more than 10 KFs old, that are outliers or have fewer
// than min_lm_obs observations. The KF's feature idx is reset, the first matching entry of
// map_points_kf_idx / map_lines_kf_idx is erased (`.at()`: a missing key is an error here,
// checked before anything is removed) and the landmark is deleted (slot -> NULL).
int MapHandler::removeBadMapLandmarksForPluker(CullStats *cs) {
    CullStats st;
    auto is_bad = [&](bool local, bool inlier, const std::vector<int> &kf_obs, size_t n_obs) {
        return !local && max_kf_idx - kf_obs[0] > 10 && (!inlier || (int)n_obs < params.min_lm_obs);
    };
    auto check = [&](int kf_obs, const std::map<int, std::vector<int>> &kidx, const char *what, int idx) {
        if (kf_obs < 0 || kf_obs >= (int)map_keyframes.size() || !map_keyframes[kf_obs]) {
            setError("removeBadMapLandmarksForPluker: %s %d: no keyframe %d", what, idx, kf_obs);
            return false;
        }
        if (!kidx.count(kf_obs)) {
            setError("removeBadMapLandmarksForPluker: %s %d: %s_kf_idx.at(%d): no such key", what, idx, what, kf_obs);
            return false;
        }
        return true;
    };
    for (auto *p : map_points)
        if (p) {
            if (p->kf_obs_list.empty()) {
                setError("removeBadMapLandmarksForPluker: point %d has no observation", p->idx);
                return PLBA_E_STATE;
            }
            if (is_bad(p->local, p->inlier, p->kf_obs_list, p->obs_list.size()) &&
                !check(p->kf_obs_list[0], map_points_kf_idx, "map_points", p->idx))
                return PLBA_E_STATE;
        }
    for (auto *l : map_lines)
        if (l) {
            if (l->kf_obs_list.empty()) {
                setError("removeBadMapLandmarksForPluker: line %d has no observation", l->idx);
                return PLBA_E_STATE;
            }
            if (is_bad(l->local, l->inlier, l->kf_obs_list, l->NDw_obs_list.size()) &&
                !check(l->kf_obs_list[0], map_lines_kf_idx, "map_lines", l->idx))
                return PLBA_E_STATE;
        }
    auto erase_first = [](std::vector<int> &v, int x) {
        auto it = std::find(v.begin(), v.end(), x);
        if (it != v.end()) v.erase(it);
    };
    for (auto *&p : map_points)
        if (p && is_bad(p->local, p->inlier, p->kf_obs_list, p->obs_list.size())) {
            const int kf_obs = p->kf_obs_list[0], lm_idx = p->idx;
            for (int &f : map_keyframes[kf_obs]->stereo_frame.stereo_pt_idx)
                if (f == lm_idx) {
                    f = -1;
                    break;
                }
            erase_first(map_points_kf_idx.at(kf_obs), lm_idx);
            const int slot = (int)(&p - map_points.data());
            delete p;
            p = nullptr;
            markLandmarkChanged(1, slot);
            st.points_removed++;
        }
    for (auto *&l : map_lines)
        if (l && is_bad(l->local, l->inlier, l->kf_obs_list, l->NDw_obs_list.size())) {
            const int kf_obs = l->kf_obs_list[0], lm_idx = l->idx;
            for (int &f : map_keyframes[kf_obs]->stereo_frame.stereo_ls_idx)
                if (f == lm_idx) {
                    f = -1;
                    break;
                }
            erase_first(map_lines_kf_idx.at(kf_obs), lm_idx);
            const int slot = (int)(&l - map_lines.data());
            delete l;
            l = nullptr;
            markLandmarkChanged(2, slot);
            st.lines_removed++;
        }
    if (cs) *cs = st;
    return PLBA_OK;
}

int MapHandler::localMappingStep(int kf_idx, LbaStats *stats, CullStats *cs) {
    int rc = formLocalMap(kf_idx);  // :1274
    if (rc) return rc;
    rc = localBundleAdjustmentForPlukerWithG2O(stats);  // :1278
    if (rc) return rc;
    return removeBadMapLandmarksForPluker(cs);  // :1279
}

}  // namespace plslam
