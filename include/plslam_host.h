/*
 * plslam_host.h — C ABI of the host-side mirror of the reference's map objects and of
 *   void PLSLAM::MapHandler::localBundleAdjustmentForPlukerWithG2O()
 *   (reference: include/mapHandler.h:134, src/mapHandler.cpp:5851-6323)
 *
 * The C++ classes behind it (pl-slam-plucker_amd/host/plslam_map.hpp) restate the state the
 * reference LBA reads and mutates — KeyFrame (include/keyFrame.h:50-71), MapPoint / MapLine
 * (include/mapFeatures.h:39-107), MapHandler::{map_keyframes, map_points, map_lines,
 * map_points_kf_idx, full_graph} (include/mapHandler.h:141-151) — and run the reference's
 * host logic around the solve: window gather (A1, src/mapHandler.cpp:5868-5921), graph
 * marshalling (A1b, :5923-6117), post-solve outlier bookkeeping (A1d, :6154-6293) and
 * write-back (A1e, :6296-6319). The solve itself (A1c) goes through plba.h on the GPU.
 *
 * These entry points exist for bindings and tests; a C++ caller (the reference's own
 * MapHandler) uses the classes directly — see INTEGRATION.md.
 *
 * Status codes are plba.h's (PLBA_OK / PLBA_E_*); nothing throws or exits.
 */
#ifndef PLSLAM_HOST_H
#define PLSLAM_HOST_H

#include <stdint.h>

#include "plba.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct plslam_map plslam_map;

/* Solver hook: solves one marshalled window (plba_graph) into plba_result.
 * NULL (the default) = the MI355X backend of plba.h (one plba context per map, reused across
 * LBA calls). Tests install a stub here to drive the host bookkeeping without a GPU. */
typedef int (*plslam_solve_fn)(void *user, const plba_graph *g, plba_result *r);

/* Statistics of one LBA call (the counters the reference prints, src/mapHandler.cpp:6147,6216,6290). */
typedef struct plslam_lba_stats {
    int32_t n_free_kf, n_fixed_kf;         /* idx_nofix_kfs / idx_fix_kfs sizes                      */
    int32_t n_pt, n_ln, n_ept, n_eln;      /* local landmarks and edges in the window                */
    int32_t bad_line_stage1;               /* "Bad Obs" after optimize(5) (:6147)                     */
    int32_t bad_point_obs, actually_bad_point_obs;   /* (:6216)                                     */
    int32_t bad_line_obs, actually_bad_line_obs;     /* (:6290)                                     */
    int32_t iters[2];
    double  chi2[2];
    double  gather_ms, solve_ms, bookkeeping_ms;
    double  upload_ms;                     /* plba_upload, part of solve_ms (0 with a solver hook)   */
    int32_t dirty_landmarks;               /* landmarks the incremental gather re-read from the map  */
} plslam_lba_stats;

int         plslam_map_create(plslam_map **m, double fx, double fy, double cx, double cy, const plba_opts *opts);
int         plslam_map_destroy(plslam_map *m);
const char *plslam_map_last_error(plslam_map *m);
int         plslam_set_solver(plslam_map *m, plslam_solve_fn fn, void *user);

/* KeyFrame(sf, kf_idx) placed at map_keyframes[kf_idx]; T_kf_w is row-major 4x4 (camera->world).
 * pt_idx / ls_idx are the idx fields of the KF's stereo_frame->stereo_pt / stereo_ls features. */
int plslam_add_keyframe(plslam_map *m, int32_t kf_idx, const double T_kf_w[16], int32_t n_pt_feat,
                        const int32_t *pt_idx, int32_t n_ls_feat, const int32_t *ls_idx);
/* MapPoint(idx, point3D, desc, kf_obs, obs, dir, sigma2) at map_points[idx] (src/mapFeatures.cpp:38-50). */
int plslam_add_point(plslam_map *m, int32_t idx, const double xyz[3], const uint8_t *desc, int32_t desc_bytes,
                     int32_t kf, const double obs[2], const double dir[3], double sigma2);
/* MapPoint::addMapPointObservation (src/mapFeatures.cpp:52-60). */
int plslam_point_add_observation(plslam_map *m, int32_t idx, const uint8_t *desc, int32_t kf, const double obs[2],
                                 const double dir[3], double sigma2);
/* Plücker MapLine(idx, NDw, desc, kf_obs, obs, sigma2) at map_lines[idx] (src/mapFeatures.cpp:114-122). */
int plslam_add_line(plslam_map *m, int32_t idx, const double NDw[6], const uint8_t *desc, int32_t desc_bytes,
                    int32_t kf, const double obs[4], double sigma2);
/* MapLine::addMapLineObservation(desc, kf_obs, obs4, sigma2) (src/mapFeatures.cpp:132-138). */
int plslam_line_add_observation(plslam_map *m, int32_t idx, const uint8_t *desc, int32_t kf, const double obs[4],
                                double sigma2);
/* the `local` flag of a keyframe (kind 0), point (1) or line (2). */
int plslam_set_local(plslam_map *m, int32_t kind, int32_t idx, int32_t local);
/* the `inlier` flag of a point (kind 1) or line (2). */
int plslam_set_inlier(plslam_map *m, int32_t kind, int32_t idx, int32_t inlier);
/* full_graph (n x n, row-major); map_points_kf_idx[kf] = lm[0..n) (creates the key, even empty) */
int plslam_set_full_graph(plslam_map *m, int32_t n, const uint32_t *g);
int plslam_get_full_graph(plslam_map *m, int32_t n, uint32_t *g);
int plslam_kf_idx_set(plslam_map *m, int32_t kf, const int32_t *lm, int32_t n);
int plslam_kf_idx_get(plslam_map *m, int32_t kf, int32_t *out, int32_t cap, int32_t *n);

/* MapHandler::localBundleAdjustmentForPlukerWithG2O() */
int plslam_local_ba_plucker_g2o(plslam_map *m, plslam_lba_stats *stats);

/* Incremental window (default on): the handler keeps every landmark's observations flattened and
 * the local landmarks in a registry, so the LBA gather and formLocalMap cost O(window + changes)
 * instead of scanning the map (the reference's :5877-5886, :1076-1091). Landmarks placed and
 * changed through this ABI are tracked; a caller that writes a landmark's observations or position
 * behind the handler's back reports it with plslam_mark_landmark_changed. on = 0: the scan gather.
 * plslam_check_incremental_gather compares the landmark pass of both gathers (tests). */
int plslam_set_incremental(plslam_map *m, int32_t on);
int plslam_mark_landmark_changed(plslam_map *m, int32_t kind, int32_t idx);
int plslam_check_incremental_gather(plslam_map *m, int32_t *equal);

/* ---- MapHandler::localBundleAdjustmentForPluker() (src/mapHandler.cpp:1505-1615), the hand-rolled
 * LM of levMarquardtOptimizationLBAForPluker (:1618-2332) on the GPU (plba_hlm_lba), and its
 * write-back (:2160-2330: T_kf_w = expmap_se3(X_i); point3D = X with inlier = false when it moved
 * more than 0.01; NDw = changeOrthToPluker(X − orthNDw) — the reference converts the difference).
 * x_kf_w: KeyFrame::x_kf_w; plslam_add_keyframe initialises it to logmap_se3(T_kf_w). */
int plslam_set_keyframe_x(plslam_map *m, int32_t kf_idx, const double x[6]);
int plslam_get_keyframe_x(plslam_map *m, int32_t kf_idx, double x[6]);
typedef int (*plslam_hlm_solve_fn)(void *user, const plba_graph *g, const plba_hlm_state *st,
                                   const plba_hlm_params *p, plba_hlm_result *r);
int plslam_set_hlm_solver(plslam_map *m, plslam_hlm_solve_fn fn, void *user);   /* NULL = plba_hlm_lba */
/* SlamConfig / Config values (NULL = plba_hlm_default_params) and vo_status == VO_INSERTING_KF */
int plslam_set_hlm_params(plslam_map *m, const plba_hlm_params *p, int32_t vo_inserting_kf);
typedef struct plslam_hlm_stats {
    int32_t ret;                            /* the reference's return value: 0 or -1                */
    int32_t n_kf_list, n_fixed_kf, n_pt, n_ln, n_pt_obs, n_ls_obs;
    int32_t linearizations, solves, accepted;
    int32_t pt_outliers, ln_outliers;       /* inlier = false set by the write-back                 */
    double  err, lambda, gather_ms, solve_ms, writeback_ms;
} plslam_hlm_stats;
int plslam_local_ba_plucker(plslam_map *m, plslam_hlm_stats *stats);

/* ---- the rest of the Plücker local-mapping step around the LBA ---- */
/* SlamConfig::minLMObs / minLMCovGraph / minKFLocalMap (src/slamConfig.cpp:48,61-62; defaults
 * 5 / 75 / 3) and MapHandler::max_kf_idx (include/mapHandler.h, src/mapHandler.cpp:135,173). */
int plslam_set_params(plslam_map *m, int32_t min_lm_obs, int32_t min_lm_cov_graph, int32_t min_kf_local_map);
int plslam_set_max_kf_idx(plslam_map *m, int32_t max_kf_idx);
/* map_lines_kf_idx[kf] (include/mapHandler.h:149) */
int plslam_kf_lines_idx_set(plslam_map *m, int32_t kf, const int32_t *lm, int32_t n);
int plslam_kf_lines_idx_get(plslam_map *m, int32_t kf, int32_t *out, int32_t cap, int32_t *n);
/* MapHandler::formLocalMap(KeyFrame*) (src/mapHandler.cpp:1073-1137) */
int plslam_form_local_map(plslam_map *m, int32_t kf_idx);
/* MapHandler::removeBadMapLandmarksForPluker() (src/mapHandler.cpp:3816-3897); counts may be NULL */
int plslam_remove_bad_landmarks_pluker(plslam_map *m, int32_t *n_pt_removed, int32_t *n_ln_removed);
/* localMappingThread's USE_LINE_PLUKER body (src/mapHandler.cpp:1274-1279) after
 * lookForCommonMatches (front-end matching, the caller's): formLocalMap(kf) -> LBA -> culling */
int plslam_local_mapping_step(plslam_map *m, int32_t kf_idx, plslam_lba_stats *stats, int32_t *n_pt_removed,
                              int32_t *n_ln_removed);
/* 1 if map_points[idx] (kind 1) / map_lines[idx] (kind 2) / map_keyframes[idx] (kind 0) is
 * non-NULL, else 0 */
int plslam_exists(plslam_map *m, int32_t kind, int32_t idx, int32_t *exists);

/* State readers (any pointer may be NULL). n_obs receives the observation count; the list
 * outputs are written up to `cap` entries. */
int plslam_get_keyframe(plslam_map *m, int32_t kf_idx, double T_kf_w[16], int32_t *local, int32_t *pt_idx,
                        int32_t pt_cap, int32_t *ls_idx, int32_t ls_cap);
int plslam_get_point(plslam_map *m, int32_t idx, double xyz[3], int32_t *inlier, int32_t *local, int32_t *n_obs,
                     int32_t *kf_obs, double *obs, double *dir, double *sigma, int32_t cap, uint8_t *med_desc,
                     double med_dir[3]);
int plslam_get_line(plslam_map *m, int32_t idx, double NDw[6], int32_t *inlier, int32_t *local, int32_t *n_obs,
                    int32_t *kf_obs, double *obs, double *sigma, int32_t cap, uint8_t *med_desc);

/* ---- loop-closure pose graph ----
 * MapHandler::loopClosureOptimizationEssGraphG2O (src/mapHandler.cpp:5070-5299, ess = 1) and
 * ::loopClosureOptimizationCovGraphG2O (:5301-5531, ess = 0): the g2o VertexSE3 / EdgeSE3 graph of
 * the loop's KFs solved by plba_pgo_optimize (or the hook), then T_kf_w / x_kf_w of those KFs,
 * their landmarks (point3D, med_obs_dir, dir_list; line3D, med_obs_dir, dir_list) and every
 * later KF corrected, lc_idx_list[.][2] = 0, lc_state = LC_IDLE. loopClosureFuseLandmarks()
 * (:5533, descriptor matching) is the caller's. lc_idxs / lc_idx_list: [n][3] int, lc_pose_list:
 * [n][6] ([t; ω], include/mapHandler.h:186-187). */
int plslam_set_loop_closure(plslam_map *m, int32_t n_lc_idxs, const int32_t *lc_idxs, int32_t n_lc_idx_list,
                            const int32_t *lc_idx_list, int32_t n_lc_pose_list, const double *lc_pose_list);
int plslam_get_lc_idx_list(plslam_map *m, int32_t *out, int32_t cap, int32_t *n);
/* SlamConfig::minLMEssGraph (150) and maxItersPGO (100) (src/slamConfig.cpp:60,79) */
int plslam_set_pgo_params(plslam_map *m, int32_t min_lm_ess_graph, int32_t max_iters_pgo);
typedef int (*plslam_pgo_solve_fn)(void *user, const plba_pgo_graph *g, const plba_pgo_params *p,
                                   plba_pgo_result *r);
int plslam_set_pgo_solver(plslam_map *m, plslam_pgo_solve_fn fn, void *user);  /* NULL = plba_pgo_optimize */
typedef struct plslam_pgo_stats {
    int32_t kf_prev_idx, kf_curr_idx, n_vertices, n_fixed, n_edges, n_loop_edges, iterations, trials;
    double  chi2_initial, chi2_final, solve_ms;
} plslam_pgo_stats;
int plslam_loop_closure_optimization(plslam_map *m, int32_t ess, plslam_pgo_stats *stats);
/* MapLine::line3D / med_obs_dir (include/mapFeatures.h:93-94; never set in Plücker mode) */
int plslam_set_line_geometry(plslam_map *m, int32_t idx, const double line3D[6], const double med_obs_dir[3]);
int plslam_get_line_geometry(plslam_map *m, int32_t idx, double line3D[6], double med_obs_dir[3]);

/* MapLine::changePlukerToOrth / changeOrthToPluker (src/mapFeatures.cpp:186-221) */
void plslam_pluker_to_orth(const double NDw[6], double orth[4]);
void plslam_orth_to_pluker(const double orth[4], double NDw[6]);

#ifdef __cplusplus
}
#endif

#endif /* PLSLAM_HOST_H */
