// C ABI of the host mirror (include/plslam_host.h) over plslam::MapHandler.
#include "plslam_host.h"

#include <cstring>
#include <string>
#include <new>

#include "plslam_map.hpp"

using namespace plslam;

struct plslam_map {
    MapHandler mh;
    int desc_bytes = 32;
    plslam_map(double fx, double fy, double cx, double cy, const plba_opts *o) : mh(fx, fy, cx, cy, o) {}
};

namespace {
Desc make_desc(const uint8_t *d, int n) { return d ? Desc(d, d + n) : Desc((size_t)n, 0); }

template <typename T>
bool slot_ok(std::vector<T *> &v, int idx) {
    return idx >= 0 && idx < (int)v.size() && v[idx] != nullptr;
}
template <typename T>
void place(std::vector<T *> &v, int idx, T *p) {
    if ((int)v.size() <= idx) v.resize(idx + 1, nullptr);
    delete v[idx];
    v[idx] = p;
}
}  // namespace

extern "C" {

int plslam_map_create(plslam_map **m, double fx, double fy, double cx, double cy, const plba_opts *opts) {
    if (!m) return PLBA_E_INVALID;
    *m = new (std::nothrow) plslam_map(fx, fy, cx, cy, opts);
    return *m ? PLBA_OK : PLBA_E_NOMEM;
}

int plslam_map_destroy(plslam_map *m) {
    delete m;
    return PLBA_OK;
}

const char *plslam_map_last_error(plslam_map *m) { return m ? m->mh.lastError().c_str() : "null map"; }

int plslam_set_solver(plslam_map *m, plslam_solve_fn fn, void *user) {
    if (!m) return PLBA_E_INVALID;
    m->mh.setSolver(fn, user);
    return PLBA_OK;
}

int plslam_add_keyframe(plslam_map *m, int32_t kf_idx, const double T_kf_w[16], int32_t n_pt_feat,
                        const int32_t *pt_idx, int32_t n_ls_feat, const int32_t *ls_idx) {
    if (!m || kf_idx < 0 || !T_kf_w || n_pt_feat < 0 || n_ls_feat < 0) return PLBA_E_INVALID;
    auto *k = new KeyFrame();
    k->kf_idx = kf_idx;
    std::memcpy(k->T_kf_w.data(), T_kf_w, sizeof(double) * 16);
    k->x_kf_w = logmap_se3(k->T_kf_w);  // x_kf_w = logmap_se3(T) at insertion (src/mapHandler.cpp:140,179)
    if (pt_idx) k->stereo_frame.stereo_pt_idx.assign(pt_idx, pt_idx + n_pt_feat);
    if (ls_idx) k->stereo_frame.stereo_ls_idx.assign(ls_idx, ls_idx + n_ls_feat);
    place(m->mh.map_keyframes, kf_idx, k);
    return PLBA_OK;
}

int plslam_add_point(plslam_map *m, int32_t idx, const double xyz[3], const uint8_t *desc, int32_t desc_bytes,
                     int32_t kf, const double obs[2], const double dir[3], double sigma2) {
    if (!m || idx < 0 || !xyz || !obs || desc_bytes <= 0) return PLBA_E_INVALID;
    m->desc_bytes = desc_bytes;
    Vec3 d = dir ? Vec3{dir[0], dir[1], dir[2]} : Vec3{0, 0, 0};
    place(m->mh.map_points, idx,
          new MapPoint(idx, Vec3{xyz[0], xyz[1], xyz[2]}, make_desc(desc, desc_bytes), kf, Vec2{obs[0], obs[1]}, d,
                       sigma2));
    m->mh.adoptLandmark(1, idx);
    return PLBA_OK;
}

int plslam_point_add_observation(plslam_map *m, int32_t idx, const uint8_t *desc, int32_t kf, const double obs[2],
                                 const double dir[3], double sigma2) {
    if (!m || !obs || !slot_ok(m->mh.map_points, idx)) return PLBA_E_INVALID;
    Vec3 d = dir ? Vec3{dir[0], dir[1], dir[2]} : Vec3{0, 0, 0};
    m->mh.map_points[idx]->addMapPointObservation(make_desc(desc, m->desc_bytes), kf, Vec2{obs[0], obs[1]}, d, sigma2);
    return PLBA_OK;
}

int plslam_add_line(plslam_map *m, int32_t idx, const double NDw[6], const uint8_t *desc, int32_t desc_bytes,
                    int32_t kf, const double obs[4], double sigma2) {
    if (!m || idx < 0 || !NDw || !obs || desc_bytes <= 0) return PLBA_E_INVALID;
    m->desc_bytes = desc_bytes;
    Vec6 L;
    std::memcpy(L.data(), NDw, sizeof(double) * 6);
    place(m->mh.map_lines, idx,
          new MapLine(idx, L, make_desc(desc, desc_bytes), kf, Vec4{obs[0], obs[1], obs[2], obs[3]}, sigma2));
    m->mh.adoptLandmark(2, idx);
    return PLBA_OK;
}

int plslam_line_add_observation(plslam_map *m, int32_t idx, const uint8_t *desc, int32_t kf, const double obs[4],
                                double sigma2) {
    if (!m || !obs || !slot_ok(m->mh.map_lines, idx)) return PLBA_E_INVALID;
    m->mh.map_lines[idx]->addMapLineObservation(make_desc(desc, m->desc_bytes), kf,
                                                Vec4{obs[0], obs[1], obs[2], obs[3]}, sigma2);
    return PLBA_OK;
}

int plslam_set_local(plslam_map *m, int32_t kind, int32_t idx, int32_t local) {
    if (!m) return PLBA_E_INVALID;
    switch (kind) {
        case 0:
            if (!slot_ok(m->mh.map_keyframes, idx)) return PLBA_E_INVALID;
            m->mh.map_keyframes[idx]->local = local != 0;
            return PLBA_OK;
        case 1:
        case 2:
            return m->mh.setLandmarkLocal(kind, idx, local != 0);
        default:
            return PLBA_E_INVALID;
    }
}

int plslam_set_inlier(plslam_map *m, int32_t kind, int32_t idx, int32_t inlier) {
    if (!m) return PLBA_E_INVALID;
    if (kind == 1 && slot_ok(m->mh.map_points, idx)) {
        m->mh.map_points[idx]->inlier = inlier != 0;
        return PLBA_OK;
    }
    if (kind == 2 && slot_ok(m->mh.map_lines, idx)) {
        m->mh.map_lines[idx]->inlier = inlier != 0;
        return PLBA_OK;
    }
    return PLBA_E_INVALID;
}

int plslam_set_full_graph(plslam_map *m, int32_t n, const uint32_t *g) {
    if (!m || n < 0 || (n && !g)) return PLBA_E_INVALID;
    m->mh.full_graph.assign(n, std::vector<unsigned int>(n, 0));
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) m->mh.full_graph[i][j] = g[(size_t)i * n + j];
    return PLBA_OK;
}

int plslam_get_full_graph(plslam_map *m, int32_t n, uint32_t *g) {
    if (!m || !g || n != (int)m->mh.full_graph.size()) return PLBA_E_INVALID;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) g[(size_t)i * n + j] = m->mh.full_graph[i][j];
    return PLBA_OK;
}

int plslam_kf_idx_set(plslam_map *m, int32_t kf, const int32_t *lm, int32_t n) {
    if (!m || n < 0 || (n && !lm)) return PLBA_E_INVALID;
    m->mh.map_points_kf_idx[kf].assign(lm, lm + n);
    return PLBA_OK;
}

int plslam_kf_idx_get(plslam_map *m, int32_t kf, int32_t *out, int32_t cap, int32_t *n) {
    if (!m || !n) return PLBA_E_INVALID;
    auto it = m->mh.map_points_kf_idx.find(kf);
    if (it == m->mh.map_points_kf_idx.end()) {
        *n = -1;
        return PLBA_OK;
    }
    *n = (int32_t)it->second.size();
    for (int i = 0; out && i < *n && i < cap; ++i) out[i] = it->second[i];
    return PLBA_OK;
}

static void copy_stats(const LbaStats &st, plslam_lba_stats *stats) {
    if (stats) {
        stats->n_free_kf = st.n_free_kf; stats->n_fixed_kf = st.n_fixed_kf;
        stats->n_pt = st.n_pt; stats->n_ln = st.n_ln; stats->n_ept = st.n_ept; stats->n_eln = st.n_eln;
        stats->bad_line_stage1 = st.bad_line_stage1;
        stats->bad_point_obs = st.bad_point_obs; stats->actually_bad_point_obs = st.actually_bad_point_obs;
        stats->bad_line_obs = st.bad_line_obs; stats->actually_bad_line_obs = st.actually_bad_line_obs;
        stats->iters[0] = st.iters[0]; stats->iters[1] = st.iters[1];
        stats->chi2[0] = st.chi2[0]; stats->chi2[1] = st.chi2[1];
        stats->gather_ms = st.gather_ms; stats->solve_ms = st.solve_ms; stats->bookkeeping_ms = st.bookkeeping_ms;
        stats->upload_ms = st.upload_ms;
        stats->dirty_landmarks = st.dirty_landmarks;
    }
}

int plslam_set_incremental(plslam_map *m, int32_t on) {
    if (!m) return PLBA_E_INVALID;
    m->mh.incremental = on != 0;
    m->mh.rebuildLocalRegistry();
    return PLBA_OK;
}

int plslam_mark_landmark_changed(plslam_map *m, int32_t kind, int32_t idx) {
    if (!m || (kind != 1 && kind != 2) || idx < 0) return PLBA_E_INVALID;
    m->mh.markLandmarkChanged(kind, idx);
    return PLBA_OK;
}

int plslam_check_incremental_gather(plslam_map *m, int32_t *equal) {
    if (!m || !equal) return PLBA_E_INVALID;
    std::string why;
    const int rc = m->mh.checkIncrementalGather(&why);
    *equal = rc == 0 ? 1 : 0;
    if (rc) m->mh.setError("incremental gather differs from the scan gather: %s", why.c_str());
    return PLBA_OK;
}

int plslam_local_ba_plucker_g2o(plslam_map *m, plslam_lba_stats *stats) {
    if (!m) return PLBA_E_INVALID;
    LbaStats st;
    const int rc = m->mh.localBundleAdjustmentForPlukerWithG2O(&st);
    if (rc) return rc;
    copy_stats(st, stats);
    return PLBA_OK;
}

int plslam_set_keyframe_x(plslam_map *m, int32_t kf_idx, const double x[6]) {
    if (!m || !x || !slot_ok(m->mh.map_keyframes, kf_idx)) return PLBA_E_INVALID;
    std::memcpy(m->mh.map_keyframes[kf_idx]->x_kf_w.data(), x, sizeof(double) * 6);
    return PLBA_OK;
}

int plslam_get_keyframe_x(plslam_map *m, int32_t kf_idx, double x[6]) {
    if (!m || !x || !slot_ok(m->mh.map_keyframes, kf_idx)) return PLBA_E_INVALID;
    std::memcpy(x, m->mh.map_keyframes[kf_idx]->x_kf_w.data(), sizeof(double) * 6);
    return PLBA_OK;
}

int plslam_set_hlm_solver(plslam_map *m, plslam_hlm_solve_fn fn, void *user) {
    if (!m) return PLBA_E_INVALID;
    m->mh.setHlmSolver(fn, user);
    return PLBA_OK;
}

int plslam_set_hlm_params(plslam_map *m, const plba_hlm_params *p, int32_t vo_inserting_kf) {
    if (!m) return PLBA_E_INVALID;
    if (p) m->mh.hlm_params = *p;
    else plba_hlm_default_params(&m->mh.hlm_params);
    m->mh.vo_inserting_kf = vo_inserting_kf != 0;
    return PLBA_OK;
}

int plslam_local_ba_plucker(plslam_map *m, plslam_hlm_stats *stats) {
    if (!m) return PLBA_E_INVALID;
    HlmStats st;
    const int rc = m->mh.localBundleAdjustmentForPluker(&st);
    if (rc) return rc;
    if (stats) {
        stats->ret = st.ret;
        stats->n_kf_list = st.n_kf_list; stats->n_fixed_kf = st.n_fixed_kf;
        stats->n_pt = st.n_pt; stats->n_ln = st.n_ln; stats->n_pt_obs = st.n_pt_obs; stats->n_ls_obs = st.n_ls_obs;
        stats->linearizations = st.linearizations; stats->solves = st.solves; stats->accepted = st.accepted;
        stats->pt_outliers = st.pt_outliers; stats->ln_outliers = st.ln_outliers;
        stats->err = st.err; stats->lambda = st.lambda;
        stats->gather_ms = st.gather_ms; stats->solve_ms = st.solve_ms; stats->writeback_ms = st.writeback_ms;
    }
    return PLBA_OK;
}

int plslam_set_loop_closure(plslam_map *m, int32_t n_lc_idxs, const int32_t *lc_idxs, int32_t n_lc_idx_list,
                            const int32_t *lc_idx_list, int32_t n_lc_pose_list, const double *lc_pose_list) {
    if (!m || n_lc_idxs < 0 || n_lc_idx_list < 0 || n_lc_pose_list < 0 || (n_lc_idxs && !lc_idxs) ||
        (n_lc_idx_list && !lc_idx_list) || (n_lc_pose_list && !lc_pose_list))
        return PLBA_E_INVALID;
    MapHandler &mh = m->mh;
    mh.lc_idxs.assign((size_t)n_lc_idxs, Vec3i{});
    for (int i = 0; i < n_lc_idxs; ++i) mh.lc_idxs[i] = Vec3i{lc_idxs[3 * i], lc_idxs[3 * i + 1], lc_idxs[3 * i + 2]};
    mh.lc_idx_list.assign((size_t)n_lc_idx_list, Vec3i{});
    for (int i = 0; i < n_lc_idx_list; ++i)
        mh.lc_idx_list[i] = Vec3i{lc_idx_list[3 * i], lc_idx_list[3 * i + 1], lc_idx_list[3 * i + 2]};
    mh.lc_pose_list.assign((size_t)n_lc_pose_list, Vec6{});
    for (int i = 0; i < n_lc_pose_list; ++i)
        for (int k = 0; k < 6; ++k) mh.lc_pose_list[i][k] = lc_pose_list[6 * i + k];
    return PLBA_OK;
}

int plslam_get_lc_idx_list(plslam_map *m, int32_t *out, int32_t cap, int32_t *n) {
    if (!m) return PLBA_E_INVALID;
    const auto &l = m->mh.lc_idx_list;
    if (n) *n = (int32_t)l.size();
    for (int i = 0; i < (int)l.size() && i < cap && out; ++i)
        for (int k = 0; k < 3; ++k) out[3 * i + k] = l[i][k];
    return PLBA_OK;
}

int plslam_set_pgo_params(plslam_map *m, int32_t min_lm_ess_graph, int32_t max_iters_pgo) {
    if (!m || max_iters_pgo < 0) return PLBA_E_INVALID;
    m->mh.params.min_lm_ess_graph = min_lm_ess_graph;
    m->mh.params.max_iters_pgo = max_iters_pgo;
    return PLBA_OK;
}

int plslam_set_pgo_solver(plslam_map *m, plslam_pgo_solve_fn fn, void *user) {
    if (!m) return PLBA_E_INVALID;
    m->mh.setPgoSolver(fn, user);
    return PLBA_OK;
}

int plslam_loop_closure_optimization(plslam_map *m, int32_t ess, plslam_pgo_stats *stats) {
    if (!m) return PLBA_E_INVALID;
    PgoStats st;
    const int rc = ess ? m->mh.loopClosureOptimizationEssGraphG2O(&st) : m->mh.loopClosureOptimizationCovGraphG2O(&st);
    if (rc) return rc;
    if (stats) {
        stats->kf_prev_idx = st.kf_prev_idx; stats->kf_curr_idx = st.kf_curr_idx;
        stats->n_vertices = st.n_vertices; stats->n_fixed = st.n_fixed; stats->n_edges = st.n_edges;
        stats->n_loop_edges = st.n_loop_edges; stats->iterations = st.iterations; stats->trials = st.trials;
        stats->chi2_initial = st.chi2_initial; stats->chi2_final = st.chi2_final; stats->solve_ms = st.solve_ms;
    }
    return PLBA_OK;
}

int plslam_set_line_geometry(plslam_map *m, int32_t idx, const double line3D[6], const double med_obs_dir[3]) {
    if (!m || idx < 0 || idx >= (int)m->mh.map_lines.size() || !m->mh.map_lines[idx]) return PLBA_E_INVALID;
    MapLine *ml = m->mh.map_lines[idx];
    if (line3D) for (int k = 0; k < 6; ++k) ml->line3D[k] = line3D[k];
    if (med_obs_dir) for (int k = 0; k < 3; ++k) ml->med_obs_dir[k] = med_obs_dir[k];
    return PLBA_OK;
}

int plslam_get_line_geometry(plslam_map *m, int32_t idx, double line3D[6], double med_obs_dir[3]) {
    if (!m || idx < 0 || idx >= (int)m->mh.map_lines.size() || !m->mh.map_lines[idx]) return PLBA_E_INVALID;
    const MapLine *ml = m->mh.map_lines[idx];
    if (line3D) for (int k = 0; k < 6; ++k) line3D[k] = ml->line3D[k];
    if (med_obs_dir) for (int k = 0; k < 3; ++k) med_obs_dir[k] = ml->med_obs_dir[k];
    return PLBA_OK;
}

int plslam_set_params(plslam_map *m, int32_t min_lm_obs, int32_t min_lm_cov_graph, int32_t min_kf_local_map) {
    if (!m) return PLBA_E_INVALID;
    m->mh.params.min_lm_obs = min_lm_obs;
    m->mh.params.min_lm_cov_graph = min_lm_cov_graph;
    m->mh.params.min_kf_local_map = min_kf_local_map;
    return PLBA_OK;
}

int plslam_set_max_kf_idx(plslam_map *m, int32_t max_kf_idx) {
    if (!m) return PLBA_E_INVALID;
    m->mh.max_kf_idx = max_kf_idx;
    return PLBA_OK;
}

int plslam_kf_lines_idx_set(plslam_map *m, int32_t kf, const int32_t *lm, int32_t n) {
    if (!m || n < 0 || (n && !lm)) return PLBA_E_INVALID;
    m->mh.map_lines_kf_idx[kf].assign(lm, lm + n);
    return PLBA_OK;
}

int plslam_kf_lines_idx_get(plslam_map *m, int32_t kf, int32_t *out, int32_t cap, int32_t *n) {
    if (!m || !n) return PLBA_E_INVALID;
    auto it = m->mh.map_lines_kf_idx.find(kf);
    if (it == m->mh.map_lines_kf_idx.end()) {
        *n = -1;
        return PLBA_OK;
    }
    *n = (int32_t)it->second.size();
    for (int i = 0; out && i < *n && i < cap; ++i) out[i] = it->second[i];
    return PLBA_OK;
}

int plslam_form_local_map(plslam_map *m, int32_t kf_idx) {
    if (!m) return PLBA_E_INVALID;
    return m->mh.formLocalMap(kf_idx);
}

int plslam_remove_bad_landmarks_pluker(plslam_map *m, int32_t *n_pt_removed, int32_t *n_ln_removed) {
    if (!m) return PLBA_E_INVALID;
    CullStats cs;
    const int rc = m->mh.removeBadMapLandmarksForPluker(&cs);
    if (rc) return rc;
    if (n_pt_removed) *n_pt_removed = cs.points_removed;
    if (n_ln_removed) *n_ln_removed = cs.lines_removed;
    return PLBA_OK;
}

int plslam_local_mapping_step(plslam_map *m, int32_t kf_idx, plslam_lba_stats *stats, int32_t *n_pt_removed,
                              int32_t *n_ln_removed) {
    if (!m) return PLBA_E_INVALID;
    LbaStats st;
    CullStats cs;
    const int rc = m->mh.localMappingStep(kf_idx, &st, &cs);
    if (rc) return rc;
    copy_stats(st, stats);
    if (n_pt_removed) *n_pt_removed = cs.points_removed;
    if (n_ln_removed) *n_ln_removed = cs.lines_removed;
    return PLBA_OK;
}

int plslam_exists(plslam_map *m, int32_t kind, int32_t idx, int32_t *exists) {
    if (!m || !exists) return PLBA_E_INVALID;
    switch (kind) {
        case 0: *exists = slot_ok(m->mh.map_keyframes, idx); return PLBA_OK;
        case 1: *exists = slot_ok(m->mh.map_points, idx); return PLBA_OK;
        case 2: *exists = slot_ok(m->mh.map_lines, idx); return PLBA_OK;
        default: return PLBA_E_INVALID;
    }
}

int plslam_get_keyframe(plslam_map *m, int32_t kf_idx, double T_kf_w[16], int32_t *local, int32_t *pt_idx,
                        int32_t pt_cap, int32_t *ls_idx, int32_t ls_cap) {
    if (!m || !slot_ok(m->mh.map_keyframes, kf_idx)) return PLBA_E_INVALID;
    const KeyFrame *k = m->mh.map_keyframes[kf_idx];
    if (T_kf_w) std::memcpy(T_kf_w, k->T_kf_w.data(), sizeof(double) * 16);
    if (local) *local = k->local;
    for (int i = 0; pt_idx && i < pt_cap && i < (int)k->stereo_frame.stereo_pt_idx.size(); ++i)
        pt_idx[i] = k->stereo_frame.stereo_pt_idx[i];
    for (int i = 0; ls_idx && i < ls_cap && i < (int)k->stereo_frame.stereo_ls_idx.size(); ++i)
        ls_idx[i] = k->stereo_frame.stereo_ls_idx[i];
    return PLBA_OK;
}

int plslam_get_point(plslam_map *m, int32_t idx, double xyz[3], int32_t *inlier, int32_t *local, int32_t *n_obs,
                     int32_t *kf_obs, double *obs, double *dir, double *sigma, int32_t cap, uint8_t *med_desc,
                     double med_dir[3]) {
    if (!m || !slot_ok(m->mh.map_points, idx)) return PLBA_E_INVALID;
    const MapPoint *p = m->mh.map_points[idx];
    if (xyz) std::memcpy(xyz, p->point3D.data(), sizeof(double) * 3);
    if (inlier) *inlier = p->inlier;
    if (local) *local = p->local;
    if (n_obs) *n_obs = (int32_t)p->kf_obs_list.size();
    for (int i = 0; i < cap && i < (int)p->kf_obs_list.size(); ++i) {
        if (kf_obs) kf_obs[i] = p->kf_obs_list[i];
        if (obs) { obs[2 * i] = p->obs_list[i][0]; obs[2 * i + 1] = p->obs_list[i][1]; }
        if (dir) for (int k = 0; k < 3; ++k) dir[3 * i + k] = p->dir_list[i][k];
    }
    for (int i = 0; sigma && i < cap && i < (int)p->sigma_list.size(); ++i) sigma[i] = p->sigma_list[i];
    if (med_desc) std::memcpy(med_desc, p->med_desc.data(), p->med_desc.size());
    if (med_dir) std::memcpy(med_dir, p->med_obs_dir.data(), sizeof(double) * 3);
    return PLBA_OK;
}

int plslam_get_line(plslam_map *m, int32_t idx, double NDw[6], int32_t *inlier, int32_t *local, int32_t *n_obs,
                    int32_t *kf_obs, double *obs, double *sigma, int32_t cap, uint8_t *med_desc) {
    if (!m || !slot_ok(m->mh.map_lines, idx)) return PLBA_E_INVALID;
    const MapLine *l = m->mh.map_lines[idx];
    if (NDw) std::memcpy(NDw, l->NDw.data(), sizeof(double) * 6);
    if (inlier) *inlier = l->inlier;
    if (local) *local = l->local;
    if (n_obs) *n_obs = (int32_t)l->kf_obs_list.size();
    for (int i = 0; i < cap && i < (int)l->kf_obs_list.size(); ++i) {
        if (kf_obs) kf_obs[i] = l->kf_obs_list[i];
        if (obs) for (int k = 0; k < 4; ++k) obs[4 * i + k] = l->NDw_obs_list[i][k];
    }
    for (int i = 0; sigma && i < cap && i < (int)l->sigma_list.size(); ++i) sigma[i] = l->sigma_list[i];
    if (med_desc) std::memcpy(med_desc, l->med_desc.data(), l->med_desc.size());
    return PLBA_OK;
}

void plslam_pluker_to_orth(const double NDw[6], double orth[4]) {
    Vec6 L;
    std::memcpy(L.data(), NDw, sizeof(double) * 6);
    const Vec4 o = MapLine::changePlukerToOrth(L);
    std::memcpy(orth, o.data(), sizeof(double) * 4);
}

void plslam_orth_to_pluker(const double orth[4], double NDw[6]) {
    const Vec4 o{orth[0], orth[1], orth[2], orth[3]};
    const Vec6 L = MapLine::changeOrthToPluker(o);
    std::memcpy(NDw, L.data(), sizeof(double) * 6);
}

}  // extern "C"
