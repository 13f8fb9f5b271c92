// Host mirror of MapHandler::loopClosureOptimizationEssGraphG2O (src/mapHandler.cpp:5070-5299)
// and MapHandler::loopClosureOptimizationCovGraphG2O (:5301-5531) around the GPU pose-graph
// solve (plba_pgo_optimize), with the g2o SE3Quat conversions the reference goes through
// (SE3Quat::exp / log, SE3Quat <-> Isometry3 via Eigen's quaternion).
#include <chrono>
#include <cmath>
#include <map>

#include "plslam_map.hpp"

namespace plslam {

Mat4 mul4(const Mat4 &A, const Mat4 &B) {
    Mat4 C{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[i * 4 + k] * B[k * 4 + j];
            C[i * 4 + j] = s;
        }
    return C;
}

namespace {

struct Quat {  // Eigen coefficient order is (x, y, z, w)
    double x, y, z, w;
};
// Eigen Quaternion(const Matrix3&)
Quat quat_from_R(const double *m) {
    Quat q;
    double t = m[0] + m[4] + m[8];
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        double v[3];
        v[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[3 * k + j] - m[3 * j + k]) * t;
        v[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        v[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q.x = v[0]; q.y = v[1]; q.z = v[2];
    }
    return q;
}
void R_from_quat(const Quat &q, double *R) {  // QuaternionBase::toRotationMatrix
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}
// g2o::SE3Quat: unit quaternion (w >= 0 after normalizeRotation) + translation
struct SE3Quat {
    Quat r;
    double t[3];
};
SE3Quat make_se3quat(Quat q, const double *t) {  // SE3Quat(q, t): normalizeRotation()
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
    SE3Quat s;
    s.r = q;
    s.t[0] = t[0]; s.t[1] = t[1]; s.t[2] = t[2];
    return s;
}
void skew(const double *v, double *S) {
    S[0] = 0.0;   S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2];  S[4] = 0.0;   S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0];  S[8] = 0.0;
}
void m3mul(const double *A, const double *B, double *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += A[3 * i + k] * B[3 * k + j];
            C[3 * i + j] = s;
        }
}
// SE3Quat::exp(update), update = [ω; υ]
SE3Quat se3quat_exp(const double *u) {
    const double omega[3] = {u[0], u[1], u[2]}, upsilon[3] = {u[3], u[4], u[5]};
    const double theta = std::sqrt(omega[0] * omega[0] + omega[1] * omega[1] + omega[2] * omega[2]);
    double Om[9], Om2[9], R[9], V[9];
    skew(omega, Om);
    m3mul(Om, Om, Om2);
    if (theta < 0.00001) {
        for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0) ? 1.0 : 0.0) + Om[k] + Om2[k];
        for (int k = 0; k < 9; ++k) V[k] = R[k];
    } else {
        const double a = std::sin(theta) / theta, b = (1 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3);
        for (int k = 0; k < 9; ++k) {
            const double I = (k % 4 == 0) ? 1.0 : 0.0;
            R[k] = I + a * Om[k] + b * Om2[k];
            V[k] = I + b * Om[k] + c * Om2[k];
        }
    }
    double t[3];
    for (int i = 0; i < 3; ++i) t[i] = V[3 * i] * upsilon[0] + V[3 * i + 1] * upsilon[1] + V[3 * i + 2] * upsilon[2];
    return make_se3quat(quat_from_R(R), t);
}
// SE3Quat::log() -> [ω; υ]
Vec6 se3quat_log(const SE3Quat &s) {
    double R[9];
    R_from_quat(s.r, R);
    const double d = 0.5 * (R[0] + R[4] + R[8] - 1);
    const double dR[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};  // deltaR
    double omega[3], Om[9], Om2[9], Vinv[9];
    if (std::fabs(d) > 0.99999) {
        for (int i = 0; i < 3; ++i) omega[i] = 0.5 * dR[i];
        skew(omega, Om);
        m3mul(Om, Om, Om2);
        for (int k = 0; k < 9; ++k) Vinv[k] = ((k % 4 == 0) ? 1.0 : 0.0) - 0.5 * Om[k] + (1. / 12.) * Om2[k];
    } else {
        const double theta = std::acos(d);
        for (int i = 0; i < 3; ++i) omega[i] = theta / (2 * std::sqrt(1 - d * d)) * dR[i];
        skew(omega, Om);
        m3mul(Om, Om, Om2);
        const double c = (1 - theta / (2 * std::tan(theta / 2))) / (theta * theta);
        for (int k = 0; k < 9; ++k) Vinv[k] = ((k % 4 == 0) ? 1.0 : 0.0) - 0.5 * Om[k] + c * Om2[k];
    }
    Vec6 res;
    for (int i = 0; i < 3; ++i) res[i] = omega[i];
    for (int i = 0; i < 3; ++i) res[3 + i] = Vinv[3 * i] * s.t[0] + Vinv[3 * i + 1] * s.t[1] + Vinv[3 * i + 2] * s.t[2];
    return res;
}
// (Isometry3) SE3Quat: R = rotation().toRotationMatrix(), t
void se3quat_to_iso(const SE3Quat &s, double *T12) {
    double R[9];
    R_from_quat(s.r, R);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T12[4 * r + c] = R[3 * r + c];
        T12[4 * r + 3] = s.t[r];
    }
}
// internal::toSE3Quat(Isometry3): SE3Quat(Quaternion(R), t)
SE3Quat iso_to_se3quat(const double *T12) {
    const double R[9] = {T12[0], T12[1], T12[2], T12[4], T12[5], T12[6], T12[8], T12[9], T12[10]};
    const double t[3] = {T12[3], T12[7], T12[11]};
    return make_se3quat(quat_from_R(R), t);
}
Vec6 reverse_se3(const Vec6 &x) {  // src2/auxiliar.cpp:199-204
    return Vec6{x[3], x[4], x[5], x[0], x[1], x[2]};
}
Vec3 xform(const Mat4 &T, const Vec3 &p) {  // T.block(0,0,3,3)·p + T.block(0,3,3,1)
    Vec3 o;
    for (int i = 0; i < 3; ++i) o[i] = T[4 * i] * p[0] + T[4 * i + 1] * p[1] + T[4 * i + 2] * p[2] + T[4 * i + 3];
    return o;
}

}  // namespace

int MapHandler::loopClosureOptimizationEssGraphG2O(PgoStats *stats) { return loopClosurePGO(true, stats); }
int MapHandler::loopClosureOptimizationCovGraphG2O(PgoStats *stats) { return loopClosurePGO(false, stats); }

int MapHandler::loopClosurePGO(bool ess, PgoStats *stats) {
    using clk = std::chrono::steady_clock;
    PgoStats st;
    // ---- the KF range (:5087-5097 / :5319-5330; the CovGraph variant then starts at KF 0)
    const std::vector<Vec3i> &range_list = ess ? lc_idxs : lc_idx_list;
    int kf_prev_idx = 2 * max_kf_idx, kf_curr_idx = -1;
    for (const Vec3i &l : range_list) {
        if (l[0] < kf_prev_idx) kf_prev_idx = l[0];
        if (l[1] > kf_curr_idx) kf_curr_idx = l[1];
    }
    if (!ess) kf_prev_idx = 0;
    st.kf_prev_idx = kf_prev_idx;
    st.kf_curr_idx = kf_curr_idx;
    const int nkf = (int)map_keyframes.size();
    if (kf_curr_idx >= nkf || (kf_curr_idx >= 0 && kf_prev_idx < 0)) {
        setError("loop closure: KF range [%d, %d] outside the map (%d KFs)", kf_prev_idx, kf_curr_idx, nkf);
        return PLBA_E_INVALID;
    }
    // ---- vertices (:5099-5141 / :5332-5370); the is_lc test walks the list the range came from
    std::vector<int> kf_list;
    std::vector<double> v_T;
    std::vector<uint8_t> v_fixed;
    std::map<int, int> vpos;
    for (int i = kf_prev_idx; i <= kf_curr_idx; ++i) {
        if (map_keyframes[i] == nullptr) continue;
        bool is_lc_i = false, is_lc_j = false;
        int id = 0;
        for (auto it = range_list.begin(); it != range_list.end(); ++it, ++id) {
            if ((*it)[0] == i) { is_lc_i = true; break; }
            if ((*it)[1] == i) { is_lc_j = true; break; }
        }
        kf_list.push_back(i);
        Vec6 x;
        bool fixed;
        if (is_lc_j) {
            // setFixed(ess); estimate = exp(reverse(log(expmap(lc_pose_list[id]) · T_{kf lc(0)})))
            const int src = range_list[id][0];
            if (id >= (int)lc_pose_list.size() || src < 0 || src >= nkf || map_keyframes[src] == nullptr) {
                setError("loop closure: lc_pose_list / source KF missing for loop %d", id);
                return PLBA_E_INVALID;
            }
            x = reverse_se3(logmap_se3(mul4(expmap_se3(lc_pose_list[id]), map_keyframes[src]->T_kf_w)));
            fixed = ess;
        } else {
            x = reverse_se3(map_keyframes[i]->x_kf_w);
            fixed = ess ? (is_lc_i || i == 0) : (i == 0);
        }
        double T12[12];
        se3quat_to_iso(se3quat_exp(x.data()), T12);
        vpos[i] = (int)v_fixed.size();
        v_T.insert(v_T.end(), T12, T12 + 12);
        v_fixed.push_back(fixed ? 1 : 0);
        st.n_fixed += fixed ? 1 : 0;
    }
    // ---- KF-to-KF edges (:5144-5164 / :5376-5396), then the loop edges (:5166-5179 / :5398-5411)
    std::vector<int32_t> e_v;
    std::vector<double> e_Z;
    auto add_edge = [&](int i, int j, const Vec6 &x) {
        double Z12[12];
        se3quat_to_iso(se3quat_exp(x.data()), Z12);
        e_v.push_back(vpos[i]);
        e_v.push_back(vpos[j]);
        e_Z.insert(e_Z.end(), Z12, Z12 + 12);
    };
    for (int i = kf_prev_idx; i <= kf_curr_idx; ++i)
        for (int j = i + 1; j <= kf_curr_idx; ++j) {
            if (map_keyframes[i] == nullptr || map_keyframes[j] == nullptr) continue;
            const unsigned fg = (size_t)i < full_graph.size() && (size_t)j < full_graph[i].size() ? full_graph[i][j] : 0u;
            const bool conn = ess ? (fg >= (unsigned)params.min_lm_ess_graph || std::abs(i - j) == 1)
                                  : (fg >= (unsigned)params.min_lm_ess_graph || fg >= (unsigned)params.min_lm_cov_graph ||
                                     std::abs(i - j) == 1);
            if (!conn) continue;
            const Mat4 T_ji = mul4(inverse_se3(map_keyframes[i]->T_kf_w), map_keyframes[j]->T_kf_w);
            add_edge(i, j, reverse_se3(logmap_se3(T_ji)));
        }
    st.n_edges = (int)e_v.size() / 2;
    {
        int id = 0;
        for (auto it = lc_idx_list.begin(); it != lc_idx_list.end(); ++it, ++id) {
            // optimizer.vertex() of a KF outside the graph is NULL: g2o refuses the edge
            if (!vpos.count((*it)[0]) || !vpos.count((*it)[1]) || id >= (int)lc_pose_list.size()) continue;
            add_edge((*it)[0], (*it)[1], reverse_se3(lc_pose_list[id]));
            ++st.n_loop_edges;
        }
    }
    st.n_vertices = (int)kf_list.size();
    // ---- initializeOptimization(); computeInitialGuess(); computeActiveErrors(); optimize(maxItersPGO)
    plba_pgo_graph g{};
    std::vector<int32_t> v_id(kf_list.begin(), kf_list.end());
    g.n_v = (int32_t)kf_list.size();
    g.n_e = (int32_t)e_v.size() / 2;
    g.v_id = v_id.data();
    g.v_T = v_T.data();
    g.v_fixed = v_fixed.data();
    g.e_v = e_v.data();
    g.e_Z = e_Z.data();
    g.e_info = nullptr;  // setInformation(Matrix6d::Identity())
    plba_pgo_params p;
    plba_pgo_default_params(&p);
    p.max_iters = params.max_iters_pgo;
    std::vector<double> v_out(v_T.size());
    plba_pgo_result r{};
    r.v_T = v_out.data();
    const auto t0 = clk::now();
    int rc;
    if (pgo_fn_) {
        rc = pgo_fn_(pgo_user_, &g, &p, &r);
        if (rc) setError("pose-graph solver hook returned %d", rc);
    } else {
        rc = ensureCtx();
        if (!rc) rc = plba_pgo_optimize(ctx_, &g, &p, &r);
        if (rc) setError("plba: %s", plba_last_error(ctx_));
    }
    if (rc) return rc;
    st.solve_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    st.iterations = r.iterations;
    st.trials = r.trials;
    st.chi2_initial = r.chi2_initial;
    st.chi2_final = r.chi2_final;
    // ---- recover poses and correct the map (:5187-5240)
    Mat4 Tkfw_corr{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};  // (uninitialised in the reference if no KF)
    auto correct_landmarks = [&](int kf) {
        auto pit = map_points_kf_idx.find(kf);  // .at() in the reference (throws when absent)
        if (pit != map_points_kf_idx.end())
            for (int idx : pit->second) {
                if (idx < 0 || idx >= (int)map_points.size() || map_points[idx] == nullptr) continue;
                MapPoint *mp = map_points[idx];
                mp->point3D = xform(Tkfw_corr, mp->point3D);
                markLandmarkChanged(1, idx);
                mp->med_obs_dir = xform(Tkfw_corr, mp->med_obs_dir);  // directions get the translation too
                for (Vec3 &d : mp->dir_list) d = xform(Tkfw_corr, d);
            }
        auto lit = map_lines_kf_idx.find(kf);
        if (lit != map_lines_kf_idx.end())
            for (int idx : lit->second) {
                if (idx < 0 || idx >= (int)map_lines.size() || map_lines[idx] == nullptr) continue;
                MapLine *ml = map_lines[idx];
                const Vec3 sP{ml->line3D[0], ml->line3D[1], ml->line3D[2]}, eP{ml->line3D[3], ml->line3D[4], ml->line3D[5]};
                const Vec3 sN = xform(Tkfw_corr, sP), eN = xform(Tkfw_corr, eP);
                for (int k = 0; k < 3; ++k) { ml->line3D[k] = sN[k]; ml->line3D[3 + k] = eN[k]; }
                ml->med_obs_dir = xform(Tkfw_corr, ml->med_obs_dir);
                for (Vec3 &d : ml->dir_list) d = xform(Tkfw_corr, d);
            }
    };
    for (size_t q = 0; q < kf_list.size(); ++q) {
        const int kf = kf_list[q];
        const SE3Quat Tiw_corr = iso_to_se3quat(&v_out[12 * q]);  // estimateAsSE3Quat()
        const Mat4 Tkfw = expmap_se3(reverse_se3(se3quat_log(Tiw_corr)));
        const Mat4 Tkfw_prev = map_keyframes[kf]->T_kf_w;
        map_keyframes[kf]->T_kf_w = Tkfw;
        map_keyframes[kf]->x_kf_w = logmap_se3(Tkfw);
        Tkfw_corr = mul4(Tkfw, inverse_se3(Tkfw_prev));
        correct_landmarks(kf);
    }
    // ---- the KFs after the loop (:5243-5287) take the last correction
    for (int i = kf_curr_idx + 1; i < nkf; ++i) {
        if (map_keyframes[i] == nullptr) continue;  // (dereferenced unchecked in the reference)
        map_keyframes[i]->T_kf_w = mul4(Tkfw_corr, map_keyframes[i]->T_kf_w);
        map_keyframes[i]->x_kf_w = logmap_se3(map_keyframes[i]->T_kf_w);
        correct_landmarks(i);
    }
    for (Vec3i &l : lc_idx_list) l[2] = 0;  // mark as optimised (:5290-5292)
    lc_state = 0;                            // LC_IDLE (:5296), after loopClosureFuseLandmarks()
    if (stats) *stats = st;
    return PLBA_OK;
}

}  // namespace plslam
