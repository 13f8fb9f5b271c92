// Host-side mirror of the map state the Plücker LBA reads and mutates, and of
// MapHandler::localBundleAdjustmentForPlukerWithG2O (src/mapHandler.cpp:5851-6323).
//
// The classes keep the reference's field names and list semantics (parallel per-observation
// vectors, pointer vectors indexed by id, std::map<int, vector<int>> map_points_kf_idx,
// vector<vector<unsigned>> full_graph) so the bookkeeping reads line-for-line against the
// reference; Eigen/OpenCV types become fixed-size arrays (Matrix4d -> row-major double[16],
// cv::Mat binary descriptor -> byte vector, NORM_HAMMING -> popcount).
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <new>
#include <utility>
#include <string>
#include <vector>

#include "plba.h"

namespace plslam {

// Incremental window state of a MapHandler (map_handler.cpp): landmarks report changes to it.
struct LandmarkStore;
void landmark_changed(LandmarkStore *s, int kind, int idx);  // kind 1 = point, 2 = line

// The marshalled window's arrays: resize() default-initialises (no zero fill) — every element
// is written by the gather. (Page-locked memory for them was measured and did not shorten
// plba_upload: 0.97 vs 0.92-0.96 ms at C3.)
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U> &) {}
    template <class U, class... Args>
    void construct(U *p, Args &&...args) {
        if constexpr (sizeof...(Args) == 0) ::new ((void *)p) U;
        else ::new ((void *)p) U(std::forward<Args>(args)...);
    }
};
template <class T>
using wvector = std::vector<T, DefaultInitAlloc<T>>;

using Vec2 = std::array<double, 2>;
using Vec3 = std::array<double, 3>;
using Vec4 = std::array<double, 4>;
using Vec6 = std::array<double, 6>;
using Mat4 = std::array<double, 16>;  // row-major
using Vec3i = std::array<int, 3>;
using Desc = std::vector<uint8_t>;

// StVO::StereoFrame, reduced to what the LBA touches: the idx of each point / line feature
// (src/mapHandler.cpp:6189-6198, 6262-6271).
struct StereoFrame {
    std::vector<int> stereo_pt_idx;
    std::vector<int> stereo_ls_idx;
};

// include/keyFrame.h:50-71
struct KeyFrame {
    bool local = false;
    int kf_idx = -1;
    Mat4 T_kf_w{};  // camera -> world
    Vec6 x_kf_w{};  // logmap_se3 of T_kf_w at insertion (src/mapHandler.cpp:140,179); the g2o LBA
                    // writes T_kf_w only, so this can be stale — the hand-rolled LBA reads it
    StereoFrame stereo_frame;
};

// include/mapFeatures.h:39-66 and src/mapFeatures.cpp:38-94
struct MapPoint {
    int idx = -1;
    bool inlier = true;
    bool local = false;
    Vec3 point3D{};
    Vec3 med_obs_dir{};
    Desc med_desc;
    std::vector<Desc> desc_list;
    std::vector<Vec2> obs_list;
    std::vector<Vec3> dir_list;
    std::vector<int> kf_obs_list;
    std::vector<double> sigma_list;
    LandmarkStore *store = nullptr;  // the owning MapHandler's incremental window (set when placed)

    MapPoint(int idx_, const Vec3 &p, const Desc &desc, int kf_obs, const Vec2 &obs, const Vec3 &dir, double sigma2);
    void addMapPointObservation(const Desc &desc, int kf_obs, const Vec2 &obs, const Vec3 &dir, double sigma2);
    void updateAverageDescDir();
};

// include/mapFeatures.h:68-107 (Plücker constructor, src/mapFeatures.cpp:114-138, 140-184
// with USE_LINE_PLUKER: no direction average)
struct MapLine {
    int idx = -1;
    bool inlier = true;
    bool local = false;
    Vec6 NDw{};
    Vec4 orthNDw{};  // set by localBundleAdjustmentForPluker (src/mapHandler.cpp:1577)
    Desc med_desc;
    std::vector<Desc> desc_list;
    std::vector<Vec4> NDw_obs_list;
    std::vector<int> kf_obs_list;
    std::vector<double> sigma_list;
    // endpoint geometry (include/mapFeatures.h:93-100): not set by the Plücker constructor
    // (src/mapFeatures.cpp:110-118, left uninitialised there, zero here); the loop-closure
    // write-back transforms it (src/mapHandler.cpp:5224-5238)
    Vec6 line3D{};
    Vec3 med_obs_dir{};
    std::vector<Vec3> dir_list;
    LandmarkStore *store = nullptr;

    MapLine(int idx_, const Vec6 &NDw_, const Desc &desc, int kf_obs, const Vec4 &obs, double sigma2);
    void addMapLineObservation(const Desc &desc, int kf_obs, const Vec4 &obs, double sigma2);
    void updateAverageDescDir();

    static Vec4 changePlukerToOrth(const Vec6 &L);
    static Vec6 changeOrthToPluker(const Vec4 &o);
};

// Marshalled window: the plba_graph SoA arrays plus the back-references the outlier pass and
// the write-back need (vpEdgeKFMono / vpMapPointEdgeMono / vpLmObsIdx, ...).
struct Window {
    std::vector<KeyFrame *> nofix_kfs, fix_kfs;  // idx_nofix_kfs / idx_fix_kfs in id order
    std::vector<MapPoint *> local_pt;
    std::vector<MapLine *> local_ls;
    int max_kf_id = 0, maxPointId = 0;
    // plba_graph arrays
    wvector<double> kf_Tcw, pt_xyz, ln_orth, ept_obs, ept_info, eln_obs, eln_info;
    wvector<uint8_t> kf_fixed;
    wvector<int32_t> kf_id, pt_id, ln_id, ept_lm, ept_kf, eln_lm, eln_kf;
    // per-edge back references
    std::vector<KeyFrame *> ept_kfp, eln_kfp;
    std::vector<int> ept_obs_idx, eln_obs_idx;
    plba_graph graph(double fx, double fy, double cx, double cy) const;
    // empty, keeping every array's capacity (a MapHandler reuses one Window across calls: the
    // arrays of a C3 window are ~6 MB, and fresh pages cost more than filling them)
    void clear();
};

struct LbaStats {
    int n_free_kf = 0, n_fixed_kf = 0, n_pt = 0, n_ln = 0, n_ept = 0, n_eln = 0;
    int bad_line_stage1 = 0, bad_point_obs = 0, actually_bad_point_obs = 0, bad_line_obs = 0,
        actually_bad_line_obs = 0;
    int iters[2] = {0, 0};
    double chi2[2] = {0, 0};
    double gather_ms = 0, solve_ms = 0, bookkeeping_ms = 0;
    double upload_ms = 0;      // plba_upload, part of solve_ms
    int dirty_landmarks = 0;   // landmarks re-read from their objects by the gather (incremental mode)
};

using SolveFn = int (*)(void *user, const plba_graph *g, plba_result *r);
using HlmSolveFn = int (*)(void *user, const plba_graph *g, const plba_hlm_state *st, const plba_hlm_params *p,
                           plba_hlm_result *r);

// One localBundleAdjustmentForPluker call (hand-rolled LM).
struct HlmStats {
    int ret = 0;  // the reference's return value: 0, or -1 (no observations / VO inserting a KF)
    int n_kf_list = 0, n_fixed_kf = 0, n_pt = 0, n_ln = 0, n_pt_obs = 0, n_ls_obs = 0;
    int linearizations = 0, solves = 0, accepted = 0;
    int pt_outliers = 0, ln_outliers = 0;  // inlier = false set by the write-back (|DX| > 0.01)
    double err = 0, lambda = 0, gather_ms = 0, solve_ms = 0, writeback_ms = 0;
};

// The SlamConfig values the local-mapping step reads (src/slamConfig.cpp:48,61-62 defaults).
struct SlamParams {
    int min_lm_obs = 5;         // SlamConfig::minLMObs()
    int min_lm_cov_graph = 75;  // SlamConfig::minLMCovGraph()
    int min_kf_local_map = 3;   // SlamConfig::minKFLocalMap()
    int min_lm_ess_graph = 150; // SlamConfig::minLMEssGraph()  (src/slamConfig.cpp:60)
    int max_iters_pgo = 100;    // SlamConfig::maxItersPGO()    (src/slamConfig.cpp:79)
};

using PgoSolveFn = int (*)(void *user, const plba_pgo_graph *g, const plba_pgo_params *p, plba_pgo_result *r);

// One loopClosureOptimization{EssGraph,CovGraph}G2O call.
struct PgoStats {
    int kf_prev_idx = 0, kf_curr_idx = -1;
    int n_vertices = 0, n_fixed = 0, n_edges = 0, n_loop_edges = 0;
    int iterations = 0, trials = 0;
    double chi2_initial = 0, chi2_final = 0, solve_ms = 0;
};

struct CullStats {
    int points_removed = 0, lines_removed = 0;
};

// include/mapHandler.h:141-151 (the members the LBA uses)
class MapHandler {
  public:
    MapHandler(double fx, double fy, double cx, double cy, const plba_opts *opts = nullptr);
    ~MapHandler();
    MapHandler(const MapHandler &) = delete;
    MapHandler &operator=(const MapHandler &) = delete;

    std::vector<KeyFrame *> map_keyframes;
    std::vector<MapPoint *> map_points;
    std::vector<MapLine *> map_lines;
    std::map<int, std::vector<int>> map_points_kf_idx;
    std::map<int, std::vector<int>> map_lines_kf_idx;
    std::vector<std::vector<unsigned int>> full_graph;
    int max_kf_idx = 0;
    SlamParams params;

    // src/mapHandler.cpp:1073-1137: the local window around `kf` (covisibility >= min_lm_cov_graph
    // landmarks or within min_kf_local_map keyframes of the newest), by the `local` flags.
    int formLocalMap(int kf_idx);
    // src/mapHandler.cpp:3816-3897: delete old non-local landmarks that are outliers or have
    // fewer than min_lm_obs observations (slots become NULL).
    int removeBadMapLandmarksForPluker(CullStats *cs = nullptr);
    // The USE_LINE_PLUKER body of localMappingThread (src/mapHandler.cpp:1264-1280) after
    // lookForCommonMatches (front-end descriptor matching, not part of this library):
    // formLocalMap(kf) -> localBundleAdjustmentForPlukerWithG2O() -> removeBadMapLandmarksForPluker().
    int localMappingStep(int kf_idx, LbaStats *stats = nullptr, CullStats *cs = nullptr);

    // src/mapHandler.cpp:5851. Returns PLBA_OK or a PLBA_E_* status (the reference exit(0)s
    // on an inconsistent map, :5894,5910,5998,6062; here the map is left untouched then).
    int localBundleAdjustmentForPlukerWithG2O(LbaStats *stats = nullptr);

    // src/mapHandler.cpp:1505-1615 + levMarquardtOptimizationLBAForPluker (:1618-2332): the
    // hand-rolled LM LBA of the Plücker map (dead code in the reference's localMappingThread,
    // :1277, kept callable). Returns PLBA_OK (stats->ret carries the reference's 0 / -1).
    int localBundleAdjustmentForPluker(HlmStats *stats = nullptr);
    plba_hlm_params hlm_params{1e-5, 10.0, 1e-7, 1e-7, 1e-7, 15, 0, PLBA_HLM_LBA_PLUCKER, 0};
    bool vo_inserting_kf = false;  // vo_status == VO_INSERTING_KF (:2160): nothing is written back

    // src/mapHandler.cpp:5070-5299 / :5301-5531: the loop-closure pose graph (VertexSE3 per KF from
    // the loop's first to its last KF, EdgeSE3 for covisible / consecutive pairs and for each
    // loop), optimised on the GPU (plba_pgo_optimize), then the KF poses, their landmarks and
    // every later KF corrected, lc_idx_list marked optimised, lc_state = LC_IDLE.
    // loopClosureFuseLandmarks() (:5533, descriptor-matching landmark fusion) is the caller's.
    int loopClosureOptimizationEssGraphG2O(PgoStats *stats = nullptr);
    int loopClosureOptimizationCovGraphG2O(PgoStats *stats = nullptr);
    // include/mapHandler.h:186-200
    std::vector<Vec3i> lc_idxs, lc_idx_list;
    std::vector<Vec6> lc_poses, lc_pose_list;
    int lc_state = 0;  // LC_IDLE = 0

    void setSolver(SolveFn fn, void *user) { solve_fn_ = fn; solve_user_ = user; }
    void setPgoSolver(PgoSolveFn fn, void *user) { pgo_fn_ = fn; pgo_user_ = user; }
    void setHlmSolver(HlmSolveFn fn, void *user) { hlm_fn_ = fn; hlm_user_ = user; }
    const std::string &lastError() const { return err_; }
    void setError(const char *fmt, ...);

    // window gather + marshalling (A1, A1b) — public for tests
    int gatherWindow(Window &w);

    // ---- incremental window (round 6). The handler keeps every landmark's
    // observations flattened into arenas and the set of local landmarks as a registry, so that the
    // gather and formLocalMap cost O(window + changes), not O(map): the reference scans every map
    // landmark (src/mapHandler.cpp:5877-5886, :1076-1091). Landmarks report changes through
    // landmark_changed: placed / replaced (adoptLandmark), observations added (their methods),
    // erased by the outlier pass, deleted by the culling, moved by the loop closure or the hand-rolled
    // LBA. A caller that writes a landmark's fields directly calls markLandmarkChanged, or
    // rebuildLocalRegistry after writing `local` flags, or sets incremental = false (the scan gather).
    bool incremental = true;
    void adoptLandmark(int kind, int idx);
    void markLandmarkChanged(int kind, int idx);
    int setLandmarkLocal(int kind, int idx, bool local);
    void rebuildLocalRegistry();
    // tests: the landmark pass of both gathers on the current map, compared (0 = equal); no mutation
    int checkIncrementalGather(std::string *why = nullptr);

  private:
    int gatherScan(Window &w, std::vector<uint8_t> &observer);
    int gatherIncremental(Window &w, std::vector<uint8_t> &observer, int *dirty);
    int finishGather(Window &w, const std::vector<uint8_t> &observer);
    std::unique_ptr<LandmarkStore> store_;
    int last_dirty_ = 0;
    double last_upload_ms_ = 0;
    void storePosition(int kind, int idx, const double *pos);  // write-back: the cached position
    int solve(const plba_graph &g, plba_result &r);
    int ensureCtx();
    int outlierPass(Window &w, const std::vector<double> &ept_chi2, const std::vector<uint8_t> &ept_depth_ok,
                    const std::vector<uint8_t> &ept_level, const std::vector<double> &eln_chi2,
                    const std::vector<uint8_t> &eln_level, LbaStats &st);
    double fx_, fy_, cx_, cy_;
    plba_opts opts_{};
    bool have_opts_ = false;
    plba_ctx *ctx_ = nullptr;  // reused across LBA calls
    SolveFn solve_fn_ = nullptr;
    void *solve_user_ = nullptr;
    HlmSolveFn hlm_fn_ = nullptr;
    void *hlm_user_ = nullptr;
    PgoSolveFn pgo_fn_ = nullptr;
    void *pgo_user_ = nullptr;
    int loopClosurePGO(bool ess, PgoStats *stats);
    std::string err_;
    // per-call scratch reused across LBA calls (capacity kept; see Window::clear)
    Window win_;
    std::vector<double> out_Tcw_, out_xyz_, out_orth_, out_ept_chi2_, out_eln_chi2_;
    std::vector<uint8_t> out_ept_depth_, out_ept_level_, out_eln_level_;
};

// helpers (host restatements)
Mat4 inverse4(const Mat4 &T);  // Eigen Matrix4d::inverse (general cofactor inverse)
// src2/auxiliar.cpp:113-173 (row-major 4x4, x = [t; ω])
Mat4 inverse_se3(const Mat4 &T);
Mat4 mul4(const Mat4 &A, const Mat4 &B);  // Matrix4d * Matrix4d
Mat4 expmap_se3(const Vec6 &x);
Vec6 logmap_se3(const Mat4 &T);
int hamming(const Desc &a, const Desc &b);

}  // namespace plslam
