/*
 * plba_g2o.hpp — g2o-compatible facade over the plba C ABI (header-only C++17).
 *
 * Lets the graph-build / solve / read-back section of
 *   PLSLAM::MapHandler::localBundleAdjustmentForPlukerWithG2O()   (src/mapHandler.cpp:5923-6319)
 * compile against the MI355X backend with only its includes changed: the reference's
 * g2o::SparseOptimizer / OptimizationAlgorithmLevenberg / BlockSolverX / LinearSolverEigen /
 * RobustKernelHuber and the g2o_types vertex and edge classes (g2o_types/g2o_types.h:28-502:
 * VertexLMPose, VertexLMPointXYZ, VertexLMLineOrth, EdgePosePoint, EdgePoseLine) keep their
 * names and the methods that code calls. Every solve runs on the GPU through libplba.so; nothing
 * here computes a residual, a Jacobian or a linear solve.
 *
 * Mapping (each facade call -> plba call):
 *   SparseOptimizer ctor / dtor          plba_create (lazily, first optimize) / plba_destroy; owns
 *                                        vertices, edges, the algorithm and robust kernels (g2o)
 *   addVertex / addEdge / setEstimate    recorded; marshalled into one plba_graph and uploaded by
 *                                        plba_upload at the next optimize() when the structure or
 *                                        a host-side estimate changed
 *   Edge::setLevel                       plba_set_edge_levels at the next optimize()
 *   Edge::setRobustKernel(Huber | 0)     plba_set_robust at the next optimize() (see Limits)
 *   initializeOptimization(level)        plba_initialize_optimization
 *   optimize(n)                          plba_optimize; returns the iteration count (-1 when no
 *                                        edge is active, as g2o)
 *   Vertex::estimate()                   plba_download (once per optimize, cached)
 *   Edge::chi2() / isDepthPositive()     plba_get_edge_chi2 (last evaluated, g2o semantics A13)
 *   Edge::computeError()                 plba_refresh_edge_errors(level of that edge)
 *
 * Limits (the backend's, checked; violations make optimize() return -1 and set lastError()):
 *   - Ω must be isotropic (info·I), as the reference builds it (src/mapHandler.cpp:6009-6010,
 *     6073-6074);
 *   - the robust kernel is uniform per optimize(): every edge Huber (one δ per edge type) or none —
 *     the reference's two stages (:6004-6007, :6133/:6146);
 *   - SetParams(fx, fy, cx, cy) is the same on every edge (one camera, :6016/:6080);
 *   - Edge::computeError() refreshes every edge of that edge's level (the reference calls it on all
 *     level-1 edges, :6158-6160 / :6226-6228, so the observable chi2() values are identical).
 * Matrix/vector arguments are any type with Eigen-style element access — m(r, c) for matrices,
 * v(i) for vectors — so Eigen types work unchanged; estimate() returns small value types that
 * convert to them.
 */
#ifndef PLBA_G2O_HPP
#define PLBA_G2O_HPP

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "plba.h"

namespace g2o {

template <class T, class... A>
std::unique_ptr<T> make_unique(A &&...a) {
    return std::unique_ptr<T>(new T(std::forward<A>(a)...));
}

// Fixed-size value returned by estimate(): element access like Eigen, converts to any
// default-constructible type with the same element access (Eigen::Vector3d, Matrix4d, ...).
template <int R, int C>
struct Fixed {
    double a[R * C] = {};
    double &operator()(int r, int c = 0) { return a[r * C + c]; }
    double operator()(int r, int c = 0) const { return a[r * C + c]; }
    template <class E>
    operator E() const {
        E e;
        for (int r = 0; r < R; ++r)
            for (int c = 0; c < C; ++c) assign(e, r, c, 0);
        return e;
    }
    // Matrix4d::inverse() of the pose estimate, as the read-back calls it
    // (src/mapHandler.cpp:6302 `pKFi->T_kf_w = vPose->estimate().inverse();`): the general 4x4
    // inverse (adjugate / determinant, Eigen's method for fixed 4x4), not a rigid-body shortcut, so a
    // Tcw whose last row is not exactly (0 0 0 1) inverts the way Eigen would.
    template <int R_ = R, int C_ = C, typename std::enable_if<R_ == 4 && C_ == 4, int>::type = 0>
    Fixed inverse() const {
        const double *m = a;
        double inv[16];
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
        Fixed o;
        for (int i = 0; i < 16; ++i) o.a[i] = inv[i] / det;
        return o;
    }

  private:
    template <class E>
    auto assign(E &e, int r, int c, int) const -> decltype(e(r, c) = 0.0, void()) { e(r, c) = (*this)(r, c); }
    template <class E>
    void assign(E &e, int r, int c, long) const { e(r) = (*this)(r, c); }
};

// Solver-stack types of src/mapHandler.cpp:5924-5928. The choice is fixed by the backend
// (Levenberg–Marquardt, Schur complement, LDLᵀ of the reduced camera system, all on the GPU);
// these only keep that construction code compiling.
struct BlockSolverTraitsX {};
template <class M>
class LinearSolverEigen {
  public:
    LinearSolverEigen() = default;
    virtual ~LinearSolverEigen() = default;
};
class BlockSolverX {
  public:
    typedef BlockSolverTraitsX PoseMatrixType;
    typedef LinearSolverEigen<PoseMatrixType> LinearSolverType;
    explicit BlockSolverX(std::unique_ptr<LinearSolverType> ls) : ls_(std::move(ls)) {}

  private:
    std::unique_ptr<LinearSolverType> ls_;
};
class OptimizationAlgorithm {
  public:
    virtual ~OptimizationAlgorithm() = default;
};
class OptimizationAlgorithmLevenberg : public OptimizationAlgorithm {
  public:
    explicit OptimizationAlgorithmLevenberg(std::unique_ptr<BlockSolverX> s) : solver_(std::move(s)) {}

  private:
    std::unique_ptr<BlockSolverX> solver_;
};

class RobustKernel {
  public:
    virtual ~RobustKernel() = default;
    void setDelta(double d) { delta_ = d; }
    double delta() const { return delta_; }

  protected:
    double delta_ = 1.0;
};
class RobustKernelHuber : public RobustKernel {};

class SparseOptimizer;

struct OptimizableGraph {
    class Vertex {
      public:
        enum Kind { POSE, POINT, LINE };
        virtual ~Vertex() = default;
        void setId(int id) { id_ = id; }
        int id() const { return id_; }
        // g2o applies a changed fixed flag at the next initializeOptimization/optimize: re-marshal
        void setFixed(bool f) {
            if (f != fixed_) structure_changed();
            fixed_ = f;
        }
        bool fixed() const { return fixed_; }
        void setMarginalized(bool m) { marg_ = m; }
        bool marginalized() const { return marg_; }
        virtual Kind kind() const = 0;

      protected:
        friend class g2o::SparseOptimizer;
        void touched();            // a host-side estimate changed: re-upload before the next solve
        void structure_changed();  // fixed flag changed: re-marshal before the next solve
        void sync() const;         // device estimates newer: download
        int id_ = -1, slot_ = -1;  // slot_: index within its kind, assigned by the optimizer
        bool fixed_ = false, marg_ = false;
        SparseOptimizer *opt_ = nullptr;
    };
    class Edge {
      public:
        virtual ~Edge() { delete rk_; }
        void setVertex(int i, Vertex *v) {
            if (v != v_[i & 1]) structure_changed();
            v_[i & 1] = v;
        }
        Vertex *vertex(int i) const { return v_[i & 1]; }
        void setLevel(int l);
        int level() const { return level_; }
        // g2o semantics: the edge owns its kernel and deletes the previous one
        void setRobustKernel(RobustKernel *k) {
            if (k != rk_) delete rk_;
            rk_ = k;
        }
        RobustKernel *robustKernel() const { return rk_; }
        double chi2() const;
        void computeError();
        template <class M>
        void setInformation(const M &m) {
            structure_changed();
            info_ = m(0, 0);
            iso_ = true;
            for (int r = 0; r < dim(); ++r)
                for (int c = 0; c < dim(); ++c)
                    if (m(r, c) != (r == c ? info_ : 0.0)) iso_ = false;
        }
        virtual int dim() const = 0;

      protected:
        friend class g2o::SparseOptimizer;
        // measurement / information / vertices / camera changed after the window was uploaded:
        // re-marshal at the next optimize() (g2o reads them at every linearisation)
        void structure_changed();
        bool depth_ok() const;  // EdgePosePoint::isDepthPositive at the last evaluated state
        Vertex *v_[2] = {nullptr, nullptr};
        RobustKernel *rk_ = nullptr;
        int level_ = 0, slot_ = -1;
        double info_ = 1.0;
        bool iso_ = true;
        double cam_[4] = {0, 0, 0, 0};
        double obs_[4] = {0, 0, 0, 0};
        SparseOptimizer *opt_ = nullptr;
    };
};

class SparseOptimizer {
  public:
    SparseOptimizer() = default;
    SparseOptimizer(const SparseOptimizer &) = delete;
    SparseOptimizer &operator=(const SparseOptimizer &) = delete;
    ~SparseOptimizer() {
        for (auto *e : edges_) delete e;
        for (auto *v : verts_) delete v;
        delete algo_;
        if (ctx_) plba_destroy(ctx_);
    }
    // backend options (not in g2o): device ordinal, the corrected line Jacobian
    void setDevice(int device) { device_ = device; }
    void setCorrectedLineJacobian(bool on) { corrected_ = on; }
    void setVerbose(bool v) { verbose_ = v; }
    void setAlgorithm(OptimizationAlgorithm *a) {
        if (a != algo_) delete algo_;
        algo_ = a;
    }
    OptimizationAlgorithm *algorithm() const { return algo_; }
    const std::string &lastError() const { return err_; }

    bool addVertex(OptimizableGraph::Vertex *v) {
        if (!v || findVertex(v->id()) >= 0) return false;
        v->opt_ = this;
        verts_.push_back(v);
        byid_.clear();
        dirty_struct_ = true;
        return true;
    }
    bool addEdge(OptimizableGraph::Edge *e) {
        if (!e || !e->v_[0] || !e->v_[1]) return false;
        e->opt_ = this;
        edges_.push_back(e);
        dirty_struct_ = true;
        return true;
    }
    OptimizableGraph::Vertex *vertex(int id) {
        const int i = findVertex(id);
        return i < 0 ? nullptr : verts_[i];
    }
    const std::vector<OptimizableGraph::Vertex *> &vertices() const { return verts_; }
    const std::vector<OptimizableGraph::Edge *> &edges() const { return edges_; }

    bool initializeOptimization(int level = 0) {
        level_ = level;
        init_ = true;
        return true;
    }
    // OptimizationAlgorithmLevenberg::solve iterations; -1 when nothing is active (g2o) or the
    // backend refused (lastError()).
    int optimize(int iterations) {
        if (!init_) {
            err_ = "optimize() before initializeOptimization()";
            return -1;
        }
        if (!ensure_uploaded()) return -1;
        int rc = push_levels_and_kernel();
        if (rc) return fail(rc, "plba_set_edge_levels / plba_set_robust");
        if ((rc = plba_initialize_optimization(ctx_, level_))) return fail(rc, "plba_initialize_optimization");
        int32_t it = 0;
        double chi = 0.0;
        if ((rc = plba_optimize(ctx_, iterations, &it, &chi))) return fail(rc, "plba_optimize");
        chi2_ = chi;
        dev_newer_ = true;     // estimates and per-edge chi2 now live on the device
        edge_valid_ = false;
        refreshed_.clear();
        return it;
    }
    double activeRobustChi2() const { return chi2_; }

  private:
    friend struct OptimizableGraph;
    friend class OptimizableGraph::Vertex;
    friend class OptimizableGraph::Edge;

    int fail(int rc, const char *what) {
        err_ = std::string(what) + " failed (" + std::to_string(rc) + "): " + (ctx_ ? plba_last_error(ctx_) : "");
        return -1;
    }
    int findVertex(int id) {
        if (byid_.size() != verts_.size()) {
            byid_.clear();
            for (size_t i = 0; i < verts_.size(); ++i) byid_.push_back({verts_[i]->id(), (int)i});
            std::sort(byid_.begin(), byid_.end());
        }
        auto it = std::lower_bound(byid_.begin(), byid_.end(), std::make_pair(id, -1));
        return it != byid_.end() && it->first == id ? it->second : -1;
    }
    bool ensure_uploaded();
    int push_levels_and_kernel();
    void download() const;
    void fetch_edges() const;
    bool refresh_level(int level);

    std::vector<OptimizableGraph::Vertex *> verts_;
    std::vector<OptimizableGraph::Edge *> edges_;
    std::vector<std::pair<int, int>> byid_;
    OptimizationAlgorithm *algo_ = nullptr;
    plba_ctx *ctx_ = nullptr;
    int device_ = 0, level_ = 0;
    bool corrected_ = false, verbose_ = false, init_ = false;
    bool dirty_struct_ = true, dirty_est_ = false, dirty_levels_ = true;
    mutable bool dev_newer_ = false, edge_valid_ = false;
    double chi2_ = 0.0;
    std::string err_;
    // marshalled window (plba_graph arrays) and per-kind back references
    std::vector<OptimizableGraph::Vertex *> kf_, pt_, ln_;
    std::vector<OptimizableGraph::Edge *> ept_, eln_;
    mutable std::vector<double> kf_T_, pt_x_, ln_o_, ept_obs_, eln_obs_, ept_info_, eln_info_;
    std::vector<uint8_t> kf_fixed_;
    std::vector<int32_t> kf_id_, pt_id_, ln_id_, ept_lm_, ept_kf_, eln_lm_, eln_kf_;
    mutable std::vector<double> ept_chi2_, eln_chi2_;
    mutable std::vector<uint8_t> ept_dep_;
    std::vector<int> refreshed_;
    int robust_ = -1;
};

}  // namespace g2o

// ---- the g2o_types vertex and edge classes (reference: g2o_types/g2o_types.h, global scope)

// VertexLMPose (g2o_types.h:159-204): estimate Tcw (4x4); oplus on the device (pose_oplus).
class VertexLMPose : public g2o::OptimizableGraph::Vertex {
  public:
    Kind kind() const override { return POSE; }
    template <class M>
    void setEstimate(const M &T) {
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) est_(r, c) = T(r, c);
        touched();
    }
    const g2o::Fixed<4, 4> &estimate() const {
        sync();
        return est_;
    }

  private:
    friend class g2o::SparseOptimizer;
    mutable g2o::Fixed<4, 4> est_;
};
// VertexLMPointXYZ (g2o_types.h:28-49)
class VertexLMPointXYZ : public g2o::OptimizableGraph::Vertex {
  public:
    Kind kind() const override { return POINT; }
    template <class V>
    void setEstimate(const V &p) {
        for (int i = 0; i < 3; ++i) est_(i) = p(i);
        touched();
    }
    const g2o::Fixed<3, 1> &estimate() const {
        sync();
        return est_;
    }

  private:
    friend class g2o::SparseOptimizer;
    mutable g2o::Fixed<3, 1> est_;
};
// VertexLMLineOrth (g2o_types.h:52-156): orthonormal (θ1, θ2, θ3, φ)
class VertexLMLineOrth : public g2o::OptimizableGraph::Vertex {
  public:
    Kind kind() const override { return LINE; }
    template <class V>
    void setEstimate(const V &o) {
        for (int i = 0; i < 4; ++i) est_(i) = o(i);
        touched();
    }
    const g2o::Fixed<4, 1> &estimate() const {
        sync();
        return est_;
    }

  private:
    friend class g2o::SparseOptimizer;
    mutable g2o::Fixed<4, 1> est_;
};
// EdgePosePoint (g2o_types.h:206-300): vertex 0 = point, vertex 1 = pose
class EdgePosePoint : public g2o::OptimizableGraph::Edge {
  public:
    int dim() const override { return 2; }
    template <class V>
    void setMeasurement(const V &m) {
        structure_changed();
        obs_[0] = m(0);
        obs_[1] = m(1);
    }
    void SetParams(const double &fx, const double &fy, const double &cx, const double &cy) {
        structure_changed();
        cam_[0] = fx; cam_[1] = fy; cam_[2] = cx; cam_[3] = cy;
    }
    bool isDepthPositive();
};
// EdgePoseLine (g2o_types.h:302-502): vertex 0 = line, vertex 1 = pose
class EdgePoseLine : public g2o::OptimizableGraph::Edge {
  public:
    int dim() const override { return 4; }
    template <class V>
    void setMeasurement(const V &m) {
        structure_changed();
        for (int i = 0; i < 4; ++i) obs_[i] = m(i);
    }
    void SetParams(const double &fx, const double &fy, const double &cx, const double &cy) {
        structure_changed();
        cam_[0] = fx; cam_[1] = fy; cam_[2] = cx; cam_[3] = cy;
    }
};

// the reference's solver typedef (g2o_types/g2o_types.h:16)
typedef g2o::LinearSolverEigen<g2o::BlockSolverX::PoseMatrixType> SlamLinearSolver;

// ------------------------------------------------------------------------ implementation
namespace g2o {

inline void OptimizableGraph::Vertex::touched() {
    if (opt_) opt_->dirty_est_ = true;
}
inline void OptimizableGraph::Vertex::structure_changed() {
    if (opt_) opt_->dirty_struct_ = true;
}
inline void OptimizableGraph::Edge::structure_changed() {
    if (opt_) opt_->dirty_struct_ = true;
}
inline void OptimizableGraph::Vertex::sync() const {
    if (opt_ && opt_->dev_newer_) opt_->download();
}
inline void OptimizableGraph::Edge::setLevel(int l) {
    if (l != level_ && opt_) opt_->dirty_levels_ = true;
    level_ = l;
}
inline double OptimizableGraph::Edge::chi2() const {
    if (!opt_ || slot_ < 0) return 0.0;
    opt_->fetch_edges();
    return dim() == 2 ? opt_->ept_chi2_[slot_] : opt_->eln_chi2_[slot_];
}
inline void OptimizableGraph::Edge::computeError() {
    if (opt_ && slot_ >= 0) opt_->refresh_level(level_);
}
inline bool OptimizableGraph::Edge::depth_ok() const {
    if (!opt_ || slot_ < 0 || dim() != 2) return true;
    opt_->fetch_edges();
    return opt_->ept_dep_[slot_] != 0;
}

// marshal the recorded graph into plba_graph arrays (g2o insertion order within each edge type)
inline bool SparseOptimizer::ensure_uploaded() {
    if (!ctx_) {
        plba_opts o;
        plba_default_opts(&o);
        o.device = device_;
        o.corrected_line_jacobian = corrected_ ? 1 : 0;
        o.verbose = verbose_ ? 1 : 0;
        const int rc = plba_create(&ctx_, &o);
        if (rc) {
            ctx_ = nullptr;
            err_ = "plba_create failed (" + std::to_string(rc) + "): no usable HIP device?";
            return false;
        }
    }
    if (!dirty_struct_ && !dirty_est_) return true;
    if (dev_newer_) download();  // keep the device's estimates for vertices the caller did not set
    kf_.clear(); pt_.clear(); ln_.clear(); ept_.clear(); eln_.clear();
    for (auto *v : verts_) {
        auto &dst = v->kind() == OptimizableGraph::Vertex::POSE ? kf_ : (v->kind() == OptimizableGraph::Vertex::POINT ? pt_ : ln_);
        v->slot_ = (int)dst.size();
        dst.push_back(v);
    }
    const size_t nk = kf_.size(), np = pt_.size(), nl = ln_.size();
    kf_T_.assign(nk * 12, 0.0); kf_fixed_.assign(nk, 0); kf_id_.assign(nk, 0);
    for (size_t i = 0; i < nk; ++i) {
        const auto &T = static_cast<VertexLMPose *>(kf_[i])->est_;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) kf_T_[i * 12 + r * 4 + c] = T(r, c);
        kf_fixed_[i] = kf_[i]->fixed() ? 1 : 0;
        kf_id_[i] = kf_[i]->id();
    }
    pt_x_.assign(np * 3, 0.0); pt_id_.assign(np, 0);
    for (size_t i = 0; i < np; ++i) {
        const auto &p = static_cast<VertexLMPointXYZ *>(pt_[i])->est_;
        for (int k = 0; k < 3; ++k) pt_x_[i * 3 + k] = p(k);
        pt_id_[i] = pt_[i]->id();
    }
    ln_o_.assign(nl * 4, 0.0); ln_id_.assign(nl, 0);
    for (size_t i = 0; i < nl; ++i) {
        const auto &o = static_cast<VertexLMLineOrth *>(ln_[i])->est_;
        for (int k = 0; k < 4; ++k) ln_o_[i * 4 + k] = o(k);
        ln_id_[i] = ln_[i]->id();
    }
    ept_lm_.clear(); ept_kf_.clear(); ept_obs_.clear(); ept_info_.clear();
    eln_lm_.clear(); eln_kf_.clear(); eln_obs_.clear(); eln_info_.clear();
    const double *cam = nullptr;
    double hub[2] = {-1.0, -1.0};
    for (auto *e : edges_) {
        const bool pt = e->dim() == 2;
        OptimizableGraph::Vertex *lm = e->v_[0], *ps = e->v_[1];
        if (!lm || !ps || ps->kind() != OptimizableGraph::Vertex::POSE ||
            lm->kind() != (pt ? OptimizableGraph::Vertex::POINT : OptimizableGraph::Vertex::LINE) || lm->opt_ != this ||
            ps->opt_ != this) {
            err_ = "edge vertices: vertex 0 must be the landmark, vertex 1 the pose, both added to this optimizer";
            return false;
        }
        if (!e->iso_) {
            err_ = "information matrix is not info * I (the backend's edge model)";
            return false;
        }
        if (!cam) cam = e->cam_;
        else if (std::memcmp(cam, e->cam_, sizeof(e->cam_)) != 0) {
            err_ = "SetParams differs between edges (one camera per window)";
            return false;
        }
        if (e->rk_) {
            double &h = hub[pt ? 0 : 1];
            if (h < 0.0) h = e->rk_->delta();
            else if (h != e->rk_->delta()) {
                err_ = "Huber delta differs between edges of one type";
                return false;
            }
        }
        if (pt) {
            e->slot_ = (int)ept_.size();
            ept_.push_back(e);
            ept_lm_.push_back(lm->slot_);
            ept_kf_.push_back(ps->slot_);
            ept_obs_.push_back(e->obs_[0]);
            ept_obs_.push_back(e->obs_[1]);
            ept_info_.push_back(e->info_);
        } else {
            e->slot_ = (int)eln_.size();
            eln_.push_back(e);
            eln_lm_.push_back(lm->slot_);
            eln_kf_.push_back(ps->slot_);
            for (int k = 0; k < 4; ++k) eln_obs_.push_back(e->obs_[k]);
            eln_info_.push_back(e->info_);
        }
    }
    plba_graph g;
    std::memset(&g, 0, sizeof g);
    g.n_kf = (int32_t)nk; g.n_pt = (int32_t)np; g.n_ln = (int32_t)nl;
    g.n_ept = (int32_t)ept_.size(); g.n_eln = (int32_t)eln_.size();
    if (cam) { g.fx = cam[0]; g.fy = cam[1]; g.cx = cam[2]; g.cy = cam[3]; }
    g.kf_Tcw = kf_T_.data(); g.kf_fixed = kf_fixed_.data(); g.kf_id = kf_id_.data();
    g.pt_xyz = pt_x_.data(); g.pt_id = pt_id_.data(); g.ln_orth = ln_o_.data(); g.ln_id = ln_id_.data();
    g.ept_lm = ept_lm_.data(); g.ept_kf = ept_kf_.data(); g.ept_obs = ept_obs_.data(); g.ept_info = ept_info_.data();
    g.eln_lm = eln_lm_.data(); g.eln_kf = eln_kf_.data(); g.eln_obs = eln_obs_.data(); g.eln_info = eln_info_.data();
    g.huber_pt = hub[0] < 0.0 ? 1.0 : hub[0];
    g.huber_ln = hub[1] < 0.0 ? 1.0 : hub[1];
    const int rc = plba_upload(ctx_, &g);
    if (rc) return fail(rc, "plba_upload") == 0;
    dirty_struct_ = dirty_est_ = false;
    dirty_levels_ = true;
    dev_newer_ = false;
    edge_valid_ = false;
    ept_chi2_.assign(ept_.size(), 0.0);
    eln_chi2_.assign(eln_.size(), 0.0);
    ept_dep_.assign(ept_.size(), 1);
    return true;
}

inline int SparseOptimizer::push_levels_and_kernel() {
    if (dirty_levels_) {
        std::vector<uint8_t> lp(ept_.size()), ll(eln_.size());
        for (size_t i = 0; i < ept_.size(); ++i) lp[i] = (uint8_t)ept_[i]->level();
        for (size_t i = 0; i < eln_.size(); ++i) ll[i] = (uint8_t)eln_[i]->level();
        const int rc = plba_set_edge_levels(ctx_, lp.data(), ll.data());
        if (rc) return rc;
        dirty_levels_ = false;
    }
    // the backend applies one kernel state to every edge: Huber iff the active edges carry one
    int with = 0, without = 0;
    for (auto *e : edges_)
        if (e->level() == level_) (e->rk_ ? with : without)++;
    if (with && without) return PLBA_E_INVALID;
    const int robust = with ? 1 : 0;
    if (robust != robust_) {
        const int rc = plba_set_robust(ctx_, robust);
        if (rc) return rc;
        robust_ = robust;
    }
    return PLBA_OK;
}

inline void SparseOptimizer::download() const {
    if (!ctx_ || !dev_newer_) return;
    std::vector<double> T(kf_.size() * 12), P(pt_.size() * 3), O(ln_.size() * 4);
    if (plba_download(ctx_, T.data(), P.data(), O.data())) return;
    for (size_t i = 0; i < kf_.size(); ++i) {
        auto &e = static_cast<VertexLMPose *>(kf_[i])->est_;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) e(r, c) = T[i * 12 + r * 4 + c];
        e(3, 0) = e(3, 1) = e(3, 2) = 0.0;
        e(3, 3) = 1.0;
    }
    for (size_t i = 0; i < pt_.size(); ++i)
        for (int k = 0; k < 3; ++k) static_cast<VertexLMPointXYZ *>(pt_[i])->est_(k) = P[i * 3 + k];
    for (size_t i = 0; i < ln_.size(); ++i)
        for (int k = 0; k < 4; ++k) static_cast<VertexLMLineOrth *>(ln_[i])->est_(k) = O[i * 4 + k];
    const_cast<SparseOptimizer *>(this)->dev_newer_ = false;
}

inline void SparseOptimizer::fetch_edges() const {
    if (!ctx_ || edge_valid_) return;
    if (plba_get_edge_chi2(ctx_, ept_chi2_.data(), ept_dep_.data(), eln_chi2_.data())) return;
    edge_valid_ = true;
}

inline bool SparseOptimizer::refresh_level(int level) {
    if (!ctx_) return false;
    if (std::find(refreshed_.begin(), refreshed_.end(), level) != refreshed_.end()) return true;  // once per solve
    if (plba_refresh_edge_errors(ctx_, level)) return false;
    refreshed_.push_back(level);
    edge_valid_ = false;
    return true;
}

}  // namespace g2o

inline bool EdgePosePoint::isDepthPositive() { return depth_ok(); }

#endif  // PLBA_G2O_HPP
