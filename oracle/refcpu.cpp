// refcpu.cpp — TEST INFRASTRUCTURE ONLY (see refcpu.h). PARITY UNPINNED vs the reference
// (no reference tests / golden vectors exist and the reference cannot be built here);
// pinned instead by the known-answer tests in tests/test_oracle_kat.py.
//
// A single-threaded, bug-compatible CPU restatement of the g2o solve that
// MapHandler::localBundleAdjustmentForPlukerWithG2O() runs (src/mapHandler.cpp:5851-6323),
// structured like g2o so that it doubles as the CPU baseline ("refcpu-g2o"):
//
//   * vertex / edge classes with virtual computeError / linearizeOplus / oplus
//       VertexLMPointXYZ  g2o_types/g2o_types.h:28-49
//       VertexLMLineOrth  g2o_types/g2o_types.h:52-156
//       VertexLMPose      g2o_types/g2o_types.h:159-204
//       EdgePosePoint     g2o_types/g2o_types.h:206-300
//       EdgePoseLine      g2o_types/g2o_types.h:302-502  (incl. the orth-as-Plücker bug, :429-430)
//   * g2o core semantics restated from upstream g2o (not vendored in the reference; SURVEY.md
//     §8a rows A9-A13, evidence libplslam.so symbols):
//       RobustKernelHuber::robustify, BaseBinaryEdge::constructQuadraticForm,
//       BlockSolver<-1,-1> {buildStructure, buildSystem, setLambda, restoreDiagonal, solve}
//       with dynamic-size heap blocks and a PartialPivLU landmark inverse,
//       LinearSolverEigen = block minimum-degree ordering + simplicial LDL^T,
//       OptimizationAlgorithmLevenberg::solve, SparseOptimizer::{initializeOptimization,
//       optimize, computeActiveErrors, activeRobustChi2, push, pop, update}.
//   * the two-stage schedule + classification of src/mapHandler.cpp:6119-6160.

#include "refcpu.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------
// small fixed-size helpers (row-major)
// ------------------------------------------------------------------------------------
inline void vechat(const double v[3], double M[9]) {  // g2o_types.h:18-24
    M[0] = 0;     M[1] = -v[2]; M[2] = v[1];
    M[3] = v[2];  M[4] = 0;     M[5] = -v[0];
    M[6] = -v[1]; M[7] = v[0];  M[8] = 0;
}
inline void mat3mul(const double A[9], const double B[9], double C[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
}
inline void mat3vec(const double A[9], const double v[3], double r[3]) {
    for (int i = 0; i < 3; ++i) r[i] = A[i * 3 + 0] * v[0] + A[i * 3 + 1] * v[1] + A[i * 3 + 2] * v[2];
}
inline void rot_xyz(const double th[3], double R[9]) {  // g2o_types.h:81-91 / :368-378
    double s1 = std::sin(th[0]), c1 = std::cos(th[0]);
    double s2 = std::sin(th[1]), c2 = std::cos(th[1]);
    double s3 = std::sin(th[2]), c3 = std::cos(th[2]);
    R[0] = c2 * c3; R[1] = s1 * s2 * c3 - c1 * s3; R[2] = c1 * s2 * c3 + s1 * s3;
    R[3] = c2 * s3; R[4] = s1 * s2 * s3 + c1 * c3; R[5] = c1 * s2 * s3 - s1 * c3;
    R[6] = -s2;     R[7] = s1 * c2;                R[8] = c1 * c2;
}
inline void orth_to_pluker(const double o[4], double L[6]) {  // g2o_types.h:367-387
    double R[9];
    rot_xyz(o, R);
    double w1 = std::cos(o[3]), w2 = std::sin(o[3]);
    L[0] = w1 * R[0]; L[1] = w1 * R[3]; L[2] = w1 * R[6];
    L[3] = w2 * R[1]; L[4] = w2 * R[4]; L[5] = w2 * R[7];
}
inline double norm3(const double v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
inline void cross3(const double a[3], const double b[3], double c[3]) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
// getOrhtRFromPluker (g2o_types.h:482-495): columns n̂, d̂, (n×d)/|n×d|
inline void orth_R_from_pluker(const double L[6], double U[9]) {
    double n[3] = {L[0], L[1], L[2]}, d[3] = {L[3], L[4], L[5]};
    double nn = norm3(n), dn = norm3(d), c[3];
    cross3(n, d, c);
    double cn = norm3(c);
    for (int i = 0; i < 3; ++i) {
        U[i * 3 + 0] = n[i] / nn;
        U[i * 3 + 1] = d[i] / dn;
        U[i * 3 + 2] = c[i] / cn;
    }
}
// getOrthWFromPluker (g2o_types.h:472-480): returns w1 = W(0,0), w2 = W(1,0)
inline void orth_W_from_pluker(const double L[6], double &w1, double &w2) {
    double nn = norm3(L), dn = norm3(L + 3);
    double f = std::sqrt(nn * nn + dn * dn);
    w1 = nn / f;
    w2 = dn / f;
}
inline void pluker_to_orth(const double L[6], double o[4]) {  // src/mapFeatures.cpp:186-201
    double U[9], w1, w2;
    orth_R_from_pluker(L, U);
    orth_W_from_pluker(L, w1, w2);
    o[0] = std::atan2(U[2 * 3 + 1], U[2 * 3 + 2]);
    o[1] = std::asin(-U[2 * 3 + 0]);
    o[2] = std::atan2(U[1 * 3 + 0], U[0 * 3 + 0]);
    o[3] = std::asin(w2);
}

// VertexLMLineOrth::updateOrthCoord (g2o_types.h:72-130)
inline void update_orth(const double D[4], const double dD[4], double out[4]) {
    double R[9];
    rot_xyz(D, R);
    double w1 = std::cos(D[3]), w2 = std::sin(D[3]);
    double cz = std::cos(dD[2]), sz = std::sin(dD[2]);
    double cy = std::cos(dD[1]), sy = std::sin(dD[1]);
    double cx = std::cos(dD[0]), sx = std::sin(dD[0]);
    double Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    double Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    double T1[9], T2[9], Rn[9];
    mat3mul(R, Rx, T1);   // R = R * Rx * Ry * Rz  (Eigen evaluates left to right)
    mat3mul(T1, Ry, T2);
    mat3mul(T2, Rz, Rn);
    double cp = std::cos(dD[3]), sp = std::sin(dD[3]);
    // W = [[w1,-w2],[w2,w1]] * [[cp,-sp],[sp,cp]];  W(1,0) = w2*cp + w1*sp
    double W10 = w2 * cp + w1 * sp;
    out[0] = std::atan2(Rn[2 * 3 + 1], Rn[2 * 3 + 2]);
    out[1] = std::asin(-Rn[2 * 3 + 0]);
    out[2] = std::atan2(Rn[1 * 3 + 0], Rn[0 * 3 + 0]);
    out[3] = std::asin(W10);
}

// VertexLMPose::oplusImpl (g2o_types.h:172-203): R <- R(q(δω))·R, t <- t + δt.
inline void pose_oplus(double R[9], double t[3], const double d[6]) {
    const double *w = d + 3;
    double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double half = 0.5 * theta;
    double imag, real = std::cos(half);
    if (theta < 1e-10) {
        double tsq = theta * theta, t4 = tsq * tsq;
        imag = 0.5 - 0.0208333 * tsq + 0.000260417 * t4;
    } else {
        imag = std::sin(half) / theta;
    }
    double qw = real, qx = imag * w[0], qy = imag * w[1], qz = imag * w[2];
    // Eigen QuaternionBase::toRotationMatrix
    double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    double twx = tx * qw, twy = ty * qw, twz = tz * qw;
    double txx = tx * qx, txy = ty * qx, txz = tz * qx;
    double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    double dR[9] = {1 - (tyy + tzz), txy - twz,       txz + twy,
                    txy + twz,       1 - (txx + tzz), tyz - twx,
                    txz - twy,       tyz + twx,       1 - (txx + tyy)};
    double Rn[9];
    mat3mul(dR, R, Rn);
    std::memcpy(R, Rn, sizeof Rn);
    t[0] += d[0]; t[1] += d[1]; t[2] += d[2];
}

// ------------------------------------------------------------------------------------
// edge math (shared by the classes and the KAT exports)
// ------------------------------------------------------------------------------------
struct Cam { double fx, fy, cx, cy; };

// EdgePosePoint::computeError / computePc / cam_project (g2o_types.h:224-263)
inline void point_error(const double R[9], const double t[3], const double P[3], const double obs[2],
                        const Cam &c, double e[2], double Pc[3]) {
    mat3vec(R, P, Pc);
    Pc[0] += t[0]; Pc[1] += t[1]; Pc[2] += t[2];
    double u = (Pc[0] / Pc[2]) * c.fx + c.cx;
    double v = (Pc[1] / Pc[2]) * c.fy + c.cy;
    e[0] = obs[0] - u;
    e[1] = obs[1] - v;
}
// EdgePosePoint::linearizeOplus (g2o_types.h:271-296). Ji 2x3, Jj 2x6 row-major.
inline void point_jac(const double R[9], const double t[3], const double P[3], const Cam &c,
                      double Ji[6], double Jj[12]) {
    double Pc[3];
    mat3vec(R, P, Pc);
    Pc[0] += t[0]; Pc[1] += t[1]; Pc[2] += t[2];
    double x = Pc[0], y = Pc[1], z = Pc[2];
    double invz = 1.0 / z, invz2 = invz * invz;
    double J[6] = {c.fx / z, 0, -c.fx * x * invz2, 0, c.fy / z, -c.fy * y * invz2};
    for (int r = 0; r < 2; ++r)
        for (int k = 0; k < 3; ++k)
            Ji[r * 3 + k] = -(J[r * 3 + 0] * R[0 * 3 + k] + J[r * 3 + 1] * R[1 * 3 + k] + J[r * 3 + 2] * R[2 * 3 + k]);
    double RP[3], S[9];
    mat3vec(R, P, RP);
    vechat(RP, S);
    for (int r = 0; r < 2; ++r) {
        for (int k = 0; k < 3; ++k) Jj[r * 6 + k] = -J[r * 3 + k];
        // -J * (-S) = J*S
        for (int k = 0; k < 3; ++k)
            Jj[r * 6 + 3 + k] = -(J[r * 3 + 0] * (-S[0 * 3 + k]) + J[r * 3 + 1] * (-S[1 * 3 + k]) + J[r * 3 + 2] * (-S[2 * 3 + k]));
    }
}

// Plücker line image: l = K_L * n_c  (g2o_types.h:326-336, 349-365)
inline void line_image(const double R[9], const double t[3], const double L[6], const Cam &c, double l[3]) {
    double Rn[3], Rd[3], S[9], tRd[3];
    mat3vec(R, L, Rn);
    mat3vec(R, L + 3, Rd);
    vechat(t, S);
    mat3vec(S, Rd, tRd);
    double nc[3] = {Rn[0] + tRd[0], Rn[1] + tRd[1], Rn[2] + tRd[2]};
    l[0] = c.fy * nc[0];
    l[1] = c.fx * nc[1];
    l[2] = (-c.fy * c.cx) * nc[0] + (-c.fx * c.cy) * nc[1] + (c.fx * c.fy) * nc[2];
}
// EdgePoseLine::computeError (g2o_types.h:320-347)
inline void line_error(const double R[9], const double t[3], const double orth[4], const double obs[4],
                       const Cam &c, double e[4]) {
    double L[6], l[3];
    orth_to_pluker(orth, L);
    line_image(R, t, L, c, l);
    double f = std::sqrt(l[0] * l[0] + l[1] * l[1]);
    e[0] = (l[0] * obs[0] + l[1] * obs[1] + l[2]) / f;
    e[1] = (l[0] * obs[2] + l[1] * obs[3] + l[2]) / f;
    e[2] = 0;
    e[3] = 0;
}
// EdgePoseLine::linearizeOplus (g2o_types.h:389-453). Ji 4x4, Jj 4x6 row-major.
// corrected != 0 replaces the orth vector by the Plücker vector in jac_lc_rt (:429-430).
inline void line_jac(const double R[9], const double t[3], const double orth[4], const double obs[4],
                     const Cam &c, int corrected, double Ji[16], double Jj[24]) {
    double L[6], l[3];
    orth_to_pluker(orth, L);
    line_image(R, t, L, c, l);
    double lx = l[0], ly = l[1], lz = l[2];
    double f = std::sqrt(lx * lx + ly * ly);
    double e0 = (lx * obs[0] + ly * obs[1] + lz) / f;
    double e1 = (lx * obs[2] + ly * obs[3] + lz) / f;
    double j[2][3] = {{-lx * e0 / (f * f) + obs[0] / f, -ly * e0 / (f * f) + obs[1] / f, 1.0 / f},
                      {-lx * e1 / (f * f) + obs[2] / f, -ly * e1 / (f * f) + obs[3] / f, 1.0 / f}};
    const double K[9] = {c.fy, 0, 0, 0, c.fx, 0, -c.fy * c.cx, -c.fx * c.cy, c.fx * c.fy};
    // jk = j * K (1x3)
    double jK[2][3];
    for (int r = 0; r < 2; ++r)
        for (int k = 0; k < 3; ++k)
            jK[r][k] = j[r][0] * K[0 * 3 + k] + j[r][1] * K[1 * 3 + k] + j[r][2] * K[2 * 3 + k];
    // jac_lc_rt top rows: [-[R*a]x , -[R*b]x - [t]x [R*a]x] with a = Lw.tail(3), b = Lw.head(3)
    double a[3], b[3];
    if (!corrected) {
        a[0] = orth[1]; a[1] = orth[2]; a[2] = orth[3];   // Vector4d::tail(3) of the orth estimate
        b[0] = orth[0]; b[1] = orth[1]; b[2] = orth[2];   // Vector4d::head(3)
    } else {
        a[0] = L[3]; a[1] = L[4]; a[2] = L[5];
        b[0] = L[0]; b[1] = L[1]; b[2] = L[2];
    }
    double Ra[3], Rb[3], Sa[9], Sb[9], St[9], StSa[9];
    mat3vec(R, a, Ra);
    mat3vec(R, b, Rb);
    vechat(Ra, Sa);
    vechat(Rb, Sb);
    vechat(t, St);
    mat3mul(St, Sa, StSa);
    double TL[9], TR[9];
    for (int i = 0; i < 9; ++i) {
        TL[i] = -Sa[i];
        TR[i] = -Sb[i] - StSa[i];
    }
    for (int r = 0; r < 2; ++r)
        for (int k = 0; k < 3; ++k) {
            Jj[r * 6 + k] = jK[r][0] * TL[0 * 3 + k] + jK[r][1] * TL[1 * 3 + k] + jK[r][2] * TL[2 * 3 + k];
            Jj[r * 6 + 3 + k] = jK[r][0] * TR[0 * 3 + k] + jK[r][1] * TR[1 * 3 + k] + jK[r][2] * TR[2 * 3 + k];
        }
    for (int k = 0; k < 12; ++k) Jj[12 + k] = 0;
    // jac_lc_lw = [[R, [t]x R],[0,R]];  only its top 3 rows matter (jac_lcPixel_lc = [K, 0])
    double StR[9];
    mat3mul(St, R, StR);
    double U[9], w1, w2;
    orth_R_from_pluker(L, U);
    orth_W_from_pluker(L, w1, w2);
    // jacobianFromPlukerToOrth (g2o_types.h:455-470), 6x4 row-major
    double Jo[24] = {0};
    for (int i = 0; i < 3; ++i) {
        double u1 = U[i * 3 + 0], u2 = U[i * 3 + 1], u3 = U[i * 3 + 2];
        Jo[i * 4 + 1] = -w1 * u3;
        Jo[i * 4 + 2] = w1 * u2;
        Jo[i * 4 + 3] = -w2 * u1;
        Jo[(3 + i) * 4 + 0] = w2 * u3;
        Jo[(3 + i) * 4 + 2] = -w2 * u1;
        Jo[(3 + i) * 4 + 3] = w1 * u2;
    }
    // top rows of jac_lc_lw (3x6) = [R | StR]
    double M[18];
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) {
            M[i * 6 + k] = R[i * 3 + k];
            M[i * 6 + 3 + k] = StR[i * 3 + k];
        }
    for (int r = 0; r < 2; ++r) {
        double v[6];
        for (int k = 0; k < 6; ++k) v[k] = jK[r][0] * M[0 * 6 + k] + jK[r][1] * M[1 * 6 + k] + jK[r][2] * M[2 * 6 + k];
        for (int q = 0; q < 4; ++q) {
            double s = 0;
            for (int k = 0; k < 6; ++k) s += v[k] * Jo[k * 4 + q];
            Ji[r * 4 + q] = s;
        }
    }
    for (int k = 0; k < 8; ++k) Ji[8 + k] = 0;
}

// RobustKernelHuber::robustify (g2o core)
inline void huber(double e, double delta, double rho[3]) {
    double dsqr = delta * delta;
    if (e <= dsqr) {
        rho[0] = e; rho[1] = 1.; rho[2] = 0.;
    } else {
        double sqrte = std::sqrt(e);
        rho[0] = 2 * sqrte * delta - dsqr;
        rho[1] = delta / sqrte;
        rho[2] = -0.5 * rho[1] / e;
    }
}

// ------------------------------------------------------------------------------------
// dynamic-size dense block (Eigen::MatrixXd-like, column-major, heap storage)
// ------------------------------------------------------------------------------------
#ifndef REFCPU_FAST
struct DMat {
    int r = 0, c = 0;
    std::vector<double> a;
    DMat() {}
    DMat(int r_, int c_) : r(r_), c(c_), a((size_t)r_ * c_, 0.0) {}
    double &operator()(int i, int j) { return a[(size_t)i + (size_t)j * r]; }
    double operator()(int i, int j) const { return a[(size_t)i + (size_t)j * r]; }
    void setZero() { std::fill(a.begin(), a.end(), 0.0); }
};
#else
// refcpu-fast (BASELINE.md §2 lower bound): the same blocks with inline fixed-capacity storage
// (every block of this path is at most 6x6) — no heap traffic per block or temporary
struct DMat {
    int r = 0, c = 0;
    double a[36];
    DMat() {}
    DMat(int r_, int c_) : r(r_), c(c_) { setZero(); }
    double &operator()(int i, int j) { return a[i + j * r]; }
    double operator()(int i, int j) const { return a[i + j * r]; }
    void setZero() { for (int k = 0; k < r * c; ++k) a[k] = 0.0; }
};
#endif
inline DMat mul(const DMat &A, const DMat &B) {  // heap temporary, like an Eigen dynamic product
    DMat C(A.r, B.c);
    for (int j = 0; j < B.c; ++j)
        for (int k = 0; k < A.c; ++k) {
            double b = B(k, j);
            for (int i = 0; i < A.r; ++i) C(i, j) += A(i, k) * b;
        }
    return C;
}
inline void sub_mul_transB(DMat &C, const DMat &A, const DMat &B) {  // C -= A * B^T
    for (int j = 0; j < C.c; ++j)
        for (int k = 0; k < A.c; ++k) {
            double b = B(j, k);
            for (int i = 0; i < C.r; ++i) C(i, j) -= A(i, k) * b;
        }
}
// Dinv = D.inverse() for dynamic size -> PartialPivLU(D).inverse()
inline DMat lu_inverse(const DMat &D) {
    int n = D.r;
    DMat LU = D;
    std::vector<int> perm(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = std::fabs(LU(k, k));
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(LU(i, k)) > best) { best = std::fabs(LU(i, k)); p = i; }
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(LU(k, j), LU(p, j));
            std::swap(perm[k], perm[p]);
        }
        double piv = LU(k, k);
        if (piv != 0.0)
            for (int i = k + 1; i < n; ++i) LU(i, k) /= piv;
        for (int j = k + 1; j < n; ++j) {
            double f = LU(k, j);
            for (int i = k + 1; i < n; ++i) LU(i, j) -= LU(i, k) * f;
        }
    }
    DMat X(n, n);
    for (int col = 0; col < n; ++col) {
#ifdef REFCPU_FAST
        double y[6];
#else
        std::vector<double> y(n);
#endif
        for (int i = 0; i < n; ++i) y[i] = (perm[i] == col) ? 1.0 : 0.0;
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < i; ++k) y[i] -= LU(i, k) * y[k];
        for (int i = n - 1; i >= 0; --i) {
            for (int k = i + 1; k < n; ++k) y[i] -= LU(i, k) * y[k];
            y[i] /= LU(i, i);
        }
        for (int i = 0; i < n; ++i) X(i, col) = y[i];
    }
    return X;
}

// ------------------------------------------------------------------------------------
// graph: vertices & edges
// ------------------------------------------------------------------------------------
struct Edge;
struct Vertex {
    int id = -1, dim = 0;
    bool fixed = false, marginalized = false;
    int hidx = -1;                 // g2o hessianIndex
    int col = 0;                   // colInHessian (pose: scalar offset; landmark: offset after poses)
    std::vector<Edge *> edges;
    DMat *H = nullptr;             // diagonal Hessian block in Hpp / Hll
    double b[6] = {0};
    virtual ~Vertex() {}
    virtual void oplus(const double *d) = 0;
    virtual void push() = 0;
    virtual void pop() = 0;
    virtual void discardTop() = 0;
};
struct VertexLMPose : Vertex {  // g2o_types.h:159-204 (estimate Tcw)
    double R[9], t[3];
    std::vector<std::vector<double>> stack;
    VertexLMPose() { dim = 6; }
    void oplus(const double *d) override { pose_oplus(R, t, d); }
    void push() override { std::vector<double> s(12); std::memcpy(s.data(), R, 72); std::memcpy(s.data() + 9, t, 24); stack.push_back(s); }
    void pop() override { std::memcpy(R, stack.back().data(), 72); std::memcpy(t, stack.back().data() + 9, 24); stack.pop_back(); }
    void discardTop() override { stack.pop_back(); }
};
struct VertexLMPointXYZ : Vertex {  // g2o_types.h:28-49
    double p[3];
    std::vector<std::vector<double>> stack;
    VertexLMPointXYZ() { dim = 3; }
    void oplus(const double *d) override { p[0] += d[0]; p[1] += d[1]; p[2] += d[2]; }
    void push() override { stack.push_back(std::vector<double>(p, p + 3)); }
    void pop() override { std::memcpy(p, stack.back().data(), 24); stack.pop_back(); }
    void discardTop() override { stack.pop_back(); }
};
struct VertexLMLineOrth : Vertex {  // g2o_types.h:52-156
    double o[4];
    std::vector<std::vector<double>> stack;
    VertexLMLineOrth() { dim = 4; }
    void oplus(const double *d) override { double n[4]; update_orth(o, d, n); std::memcpy(o, n, 32); }
    void push() override { stack.push_back(std::vector<double>(o, o + 4)); }
    void pop() override { std::memcpy(o, stack.back().data(), 32); stack.pop_back(); }
    void discardTop() override { stack.pop_back(); }
};

struct Edge {
    Vertex *v[2] = {nullptr, nullptr};   // 0 = landmark (Xi), 1 = pose (Xj)
    int D = 2, level = 0, internal_id = 0;
    double info = 1.0;                    // Ω = info * I_D
    bool robust = false;
    double delta = 0.0;
    double err[4] = {0, 0, 0, 0};
    double Ji[16], Jj[24];                // D x dim_i, D x 6 (row-major)
    DMat *hpl = nullptr;                  // Hpl(pose, landmark) block, 6 x dim_i
    Cam cam{};
    virtual ~Edge() {}
    virtual void computeError() = 0;
    virtual void linearizeOplus() = 0;
    double chi2() const {  // _error.dot(information()*_error)
        double s = 0;
        for (int k = 0; k < D; ++k) s += err[k] * (info * err[k]);
        return s;
    }
    bool allVerticesFixed() const { return v[0]->fixed && v[1]->fixed; }
    // BaseBinaryEdge::constructQuadraticForm (g2o core), Ω = info·I
    void constructQuadraticForm() {
#ifdef REFCPU_FAST  // fixed-size blocks: point (3, D 2) and line (4, D 4) edges compiled per shape
        if (v[0]->dim == 3 && D == 2) return quadratic_form<3, 2>();
        if (v[0]->dim == 4 && D == 4) return quadratic_form<4, 4>();
#endif
        quadratic_form<0, 0>();
    }
    template <int DI, int DD>  // 0: runtime size
    void quadratic_form() {
        Vertex *from = v[0], *to = v[1];
        const int di = DI > 0 ? DI : from->dim, dj = 6, D = DD > 0 ? DD : this->D;
        bool fromNotFixed = !from->fixed, toNotFixed = !to->fixed;
        if (!(fromNotFixed || toNotFixed)) return;
        double omega_r[4];
        for (int k = 0; k < D; ++k) omega_r[k] = -(info * err[k]);
        double w = info;  // weightedOmega = rho1 * Ω
        if (robust) {
            double rho[3];
            huber(chi2(), delta, rho);
            w = rho[1] * info;
            for (int k = 0; k < D; ++k) omega_r[k] *= rho[1];
        }
        if (fromNotFixed) {
            for (int a = 0; a < di; ++a) {
                double s = 0;
                for (int k = 0; k < D; ++k) s += Ji[k * di + a] * omega_r[k];
                from->b[a] += s;
                for (int bb = 0; bb < di; ++bb) {
                    double h = 0;
                    for (int k = 0; k < D; ++k) h += Ji[k * di + a] * w * Ji[k * di + bb];
                    (*from->H)(a, bb) += h;
                }
            }
            if (toNotFixed) {  // _hessianTransposed += B^T * Ωw * A   (Hpl = Jp^T Ωw Jl)
                for (int p = 0; p < dj; ++p)
                    for (int a = 0; a < di; ++a) {
                        double h = 0;
                        for (int k = 0; k < D; ++k) h += Jj[k * 6 + p] * w * Ji[k * di + a];
                        (*hpl)(p, a) += h;
                    }
            }
        }
        if (toNotFixed) {
            for (int p = 0; p < dj; ++p) {
                double s = 0;
                for (int k = 0; k < D; ++k) s += Jj[k * 6 + p] * omega_r[k];
                to->b[p] += s;
                for (int q = 0; q < dj; ++q) {
                    double h = 0;
                    for (int k = 0; k < D; ++k) h += Jj[k * 6 + p] * w * Jj[k * 6 + q];
                    (*to->H)(p, q) += h;
                }
            }
        }
    }
};
struct EdgePosePoint : Edge {  // g2o_types.h:206-300
    double obs[2];
    EdgePosePoint() { D = 2; }
    VertexLMPointXYZ *pt() const { return static_cast<VertexLMPointXYZ *>(v[0]); }
    VertexLMPose *pose() const { return static_cast<VertexLMPose *>(v[1]); }
    void computeError() override { double Pc[3]; point_error(pose()->R, pose()->t, pt()->p, obs, cam, err, Pc); }
    void linearizeOplus() override { point_jac(pose()->R, pose()->t, pt()->p, cam, Ji, Jj); }
    bool isDepthPositive() const {
        double Pc[3];
        mat3vec(pose()->R, pt()->p, Pc);
        return Pc[2] + pose()->t[2] > 0.0;
    }
};
struct EdgePoseLine : Edge {  // g2o_types.h:302-502
    double obs[4];
    int corrected = 0;
    EdgePoseLine() { D = 4; }
    VertexLMLineOrth *ln() const { return static_cast<VertexLMLineOrth *>(v[0]); }
    VertexLMPose *pose() const { return static_cast<VertexLMPose *>(v[1]); }
    void computeError() override { line_error(pose()->R, pose()->t, ln()->o, obs, cam, err); }
    void linearizeOplus() override { line_jac(pose()->R, pose()->t, ln()->o, obs, cam, corrected, Ji, Jj); }
};

// ------------------------------------------------------------------------------------
// LinearSolverEigen restatement: block minimum-degree ordering + simplicial LDL^T
// ------------------------------------------------------------------------------------
struct LinearSolverLDLT {
    bool init = true;
    int n = 0;
    std::vector<int> P, Pinv, Parent, Lnz, Lp, Flag, Pattern, Li;
    std::vector<double> Lx, Dg, Y;
    std::vector<int> Ap, Ai;  // full symmetric CSC pattern
    std::vector<double> Ax;

    // block-level minimum degree (exact elimination graph), ties -> lowest index
    static std::vector<int> min_degree(int nb, const std::vector<std::set<int>> &adj0) {
        std::vector<std::set<int>> adj = adj0;
        std::vector<char> done(nb, 0);
        std::vector<int> order;
        order.reserve(nb);
        for (int step = 0; step < nb; ++step) {
            int best = -1;
            size_t bd = 0;
            for (int i = 0; i < nb; ++i)
                if (!done[i] && (best < 0 || adj[i].size() < bd)) { best = i; bd = adj[i].size(); }
            done[best] = 1;
            order.push_back(best);
            std::vector<int> nb_(adj[best].begin(), adj[best].end());
            for (int a : nb_) {
                adj[a].erase(best);
                for (int b : nb_)
                    if (a != b) adj[a].insert(b);
            }
            adj[best].clear();
        }
        return order;
    }

    // blocks: upper block structure (row <= col) with dense col-major 6x6 values
    bool solve(int nblk, const std::vector<std::vector<std::pair<int, DMat *>>> &cols, const double *b, double *x) {
        n = nblk * 6;
        if (n == 0) return true;
        // fill full symmetric CSC (fillSparseMatrix writes the upper part; Eigen's
        // SimplicialLDLT<Upper> symmetrises it under the permutation)
        std::vector<std::vector<std::pair<int, double>>> colv(n);
        for (int cb = 0; cb < nblk; ++cb)
            for (auto &rb : cols[cb]) {
                int rblk = rb.first;
                const DMat &M = *rb.second;
                for (int jj = 0; jj < 6; ++jj)
                    for (int ii = 0; ii < 6; ++ii) {
                        int r = rblk * 6 + ii, c = cb * 6 + jj;
                        if (rblk == cb && ii > jj) continue;  // upper triangle of diagonal block
                        colv[c].push_back({r, M(ii, jj)});
                        if (r != c) colv[r].push_back({c, M(ii, jj)});
                    }
            }
        Ap.assign(n + 1, 0);
        Ai.clear();
        Ax.clear();
        for (int c = 0; c < n; ++c) {
            std::sort(colv[c].begin(), colv[c].end());
            for (auto &e : colv[c]) { Ai.push_back(e.first); Ax.push_back(e.second); }
            Ap[c + 1] = (int)Ai.size();
        }
        if (init) {  // computeSymbolicDecomposition: block ordering, then scalar symbolic
            std::vector<std::set<int>> adj(nblk);
            for (int cb = 0; cb < nblk; ++cb)
                for (auto &rb : cols[cb])
                    if (rb.first != cb) { adj[cb].insert(rb.first); adj[rb.first].insert(cb); }
            std::vector<int> bo = min_degree(nblk, adj);
            P.resize(n);
            Pinv.resize(n);
            for (int i = 0; i < nblk; ++i)
                for (int j = 0; j < 6; ++j) P[i * 6 + j] = bo[i] * 6 + j;
            for (int k = 0; k < n; ++k) Pinv[P[k]] = k;
            Parent.assign(n, -1);
            Lnz.assign(n, 0);
            Flag.assign(n, 0);
            for (int k = 0; k < n; ++k) {  // ldl_symbolic
                Parent[k] = -1;
                Flag[k] = k;
                Lnz[k] = 0;
                int kk = P[k];
                for (int p = Ap[kk]; p < Ap[kk + 1]; ++p) {
                    int i = Pinv[Ai[p]];
                    if (i < k)
                        for (; Flag[i] != k; i = Parent[i]) {
                            if (Parent[i] == -1) Parent[i] = k;
                            Lnz[i]++;
                            Flag[i] = k;
                        }
                }
            }
            Lp.assign(n + 1, 0);
            for (int k = 0; k < n; ++k) Lp[k + 1] = Lp[k] + Lnz[k];
            Li.assign(Lp[n], 0);
            Lx.assign(Lp[n], 0.0);
            init = false;
        }
        // ldl_numeric
        Dg.assign(n, 0.0);
        Y.assign(n, 0.0);
        Pattern.assign(n, 0);
        for (int k = 0; k < n; ++k) {
            Y[k] = 0.0;
            int top = n;
            Flag[k] = k;
            Lnz[k] = 0;
            int kk = P[k];
            for (int p = Ap[kk]; p < Ap[kk + 1]; ++p) {
                int i = Pinv[Ai[p]];
                if (i <= k) {
                    Y[i] += Ax[p];
                    int len = 0;
                    for (; Flag[i] != k; i = Parent[i]) { Pattern[len++] = i; Flag[i] = k; }
                    while (len > 0) Pattern[--top] = Pattern[--len];
                }
            }
            Dg[k] = Y[k];
            Y[k] = 0.0;
            for (; top < n; top++) {
                int i = Pattern[top];
                double yi = Y[i];
                Y[i] = 0.0;
                int p2 = Lp[i] + Lnz[i];
                for (int p = Lp[i]; p < p2; ++p) Y[Li[p]] -= Lx[p] * yi;
                double l_ki = yi / Dg[i];
                Dg[k] -= l_ki * yi;
                Li[p2] = k;
                Lx[p2] = l_ki;
                Lnz[i]++;
            }
            if (Dg[k] == 0.0) return false;  // Eigen SimplicialLDLT NumericalIssue
        }
        std::vector<double> y(n);
        for (int k = 0; k < n; ++k) y[k] = b[P[k]];
        for (int j = 0; j < n; ++j)
            for (int p = Lp[j]; p < Lp[j + 1]; ++p) y[Li[p]] -= Lx[p] * y[j];
        for (int j = 0; j < n; ++j) y[j] /= Dg[j];
        for (int j = n - 1; j >= 0; --j)
            for (int p = Lp[j]; p < Lp[j + 1]; ++p) y[j] -= Lx[p] * y[Li[p]];
        for (int k = 0; k < n; ++k) x[P[k]] = y[k];
        return true;
    }
};

// ------------------------------------------------------------------------------------
// BlockSolver<BlockSolverTraits<-1,-1>> restatement
// ------------------------------------------------------------------------------------
struct BlockSolverX {
    int numPoses = 0, numLandmarks = 0, sizePoses = 0, sizeLandmarks = 0;
    std::vector<std::unique_ptr<DMat>> storage;
    std::vector<DMat *> HppDiag, HllDiag;
    // Hpl in CCS by landmark: sorted (pose row, block)
    std::vector<std::vector<std::pair<int, DMat *>>> HplCCS;
    // Hschur upper structure: column i2 -> sorted (row i1 <= i2, block); and row-major lookup
    std::vector<std::vector<std::pair<int, DMat *>>> schurCols;
    std::vector<std::map<int, DMat *>> schurRow;  // row i1 -> (col i2 >= i1, block)
#ifdef REFCPU_FAST
    std::vector<std::vector<DMat *>> pairBlk;      // per landmark: Hschur block of each (a <= c2) pair
#endif
    std::vector<double> x, b, coeff, bschur;
    std::vector<std::vector<double>> diagBackupP, diagBackupL;
    std::vector<DMat> Dinv;
    LinearSolverLDLT linear;

    DMat *alloc(int r, int c) { storage.emplace_back(new DMat(r, c)); return storage.back().get(); }

    void buildStructure(const std::vector<Vertex *> &ivMap, const std::vector<Edge *> &active) {
        storage.clear();
        numPoses = numLandmarks = sizePoses = sizeLandmarks = 0;
        for (Vertex *v : ivMap) {
            if (!v->marginalized) { v->col = sizePoses; sizePoses += v->dim; numPoses++; }
            else { v->col = sizeLandmarks; sizeLandmarks += v->dim; numLandmarks++; }
        }
        HppDiag.assign(numPoses, nullptr);
        HllDiag.assign(numLandmarks, nullptr);
        for (Vertex *v : ivMap) {
            if (!v->marginalized) { HppDiag[v->hidx] = alloc(6, 6); v->H = HppDiag[v->hidx]; }
            else { int l = v->hidx - numPoses; HllDiag[l] = alloc(v->dim, v->dim); v->H = HllDiag[l]; }
        }
        HplCCS.assign(numLandmarks, {});
        std::vector<std::map<int, DMat *>> hplMap(numLandmarks);
        std::vector<std::set<int>> schurLookup(numLandmarks);
        for (Edge *e : active) {
            Vertex *lm = e->v[0], *ps = e->v[1];
            e->hpl = nullptr;
            if (lm->hidx < 0 || ps->hidx < 0) continue;
            int l = lm->hidx - numPoses;
            auto it = hplMap[l].find(ps->hidx);
            if (it == hplMap[l].end()) it = hplMap[l].emplace(ps->hidx, alloc(6, lm->dim)).first;
            e->hpl = it->second;
            schurLookup[l].insert(ps->hidx);
        }
        for (int l = 0; l < numLandmarks; ++l)
            for (auto &kv : hplMap[l]) HplCCS[l].push_back({kv.first, kv.second});
        // Hschur pattern: Hpp blocks + all pose pairs sharing a landmark (upper)
        schurRow.assign(numPoses, {});
        for (int i = 0; i < numPoses; ++i) schurRow[i][i] = alloc(6, 6);
        for (int l = 0; l < numLandmarks; ++l)
            for (int i1 : schurLookup[l])
                for (int i2 : schurLookup[l])
                    if (i1 <= i2 && !schurRow[i1].count(i2)) schurRow[i1][i2] = alloc(6, 6);
        schurCols.assign(numPoses, {});
        for (int i1 = 0; i1 < numPoses; ++i1)
            for (auto &kv : schurRow[i1]) schurCols[kv.first].push_back({i1, kv.second});
        for (auto &c : schurCols) std::sort(c.begin(), c.end(), [](auto &a, auto &b) { return a.first < b.first; });
#ifdef REFCPU_FAST
        pairBlk.assign(numLandmarks, {});
        for (int l = 0; l < numLandmarks; ++l) {
            const auto &colL = HplCCS[l];
            for (size_t a = 0; a < colL.size(); ++a)
                for (size_t c2 = a; c2 < colL.size(); ++c2) pairBlk[l].push_back(schurRow[colL[a].first].at(colL[c2].first));
        }
#endif
        x.assign(sizePoses + sizeLandmarks, 0.0);
        b.assign(sizePoses + sizeLandmarks, 0.0);
        coeff.assign(sizePoses + sizeLandmarks, 0.0);
        bschur.assign(sizePoses, 0.0);
        Dinv.assign(numLandmarks, DMat());
        linear.init = true;
    }

    void buildSystem(const std::vector<Vertex *> &ivMap, const std::vector<Edge *> &active) {
        for (Vertex *v : ivMap) { std::fill(v->b, v->b + 6, 0.0); v->H->setZero(); }
        for (auto &col : HplCCS) for (auto &kv : col) kv.second->setZero();
        for (Edge *e : active) {
            e->linearizeOplus();
            e->constructQuadraticForm();
        }
        for (Vertex *v : ivMap) {
            double *dst = v->marginalized ? &b[sizePoses + v->col] : &b[v->col];
            for (int k = 0; k < v->dim; ++k) dst[k] = v->b[k];
        }
    }

    void setLambda(double lambda) {
        diagBackupP.assign(numPoses, {});
        diagBackupL.assign(numLandmarks, {});
        for (int i = 0; i < numPoses; ++i) {
            DMat &m = *HppDiag[i];
            diagBackupP[i].resize(6);
            for (int k = 0; k < 6; ++k) { diagBackupP[i][k] = m(k, k); m(k, k) += lambda; }
        }
        for (int i = 0; i < numLandmarks; ++i) {
            DMat &m = *HllDiag[i];
            diagBackupL[i].resize(m.r);
            for (int k = 0; k < m.r; ++k) { diagBackupL[i][k] = m(k, k); m(k, k) += lambda; }
        }
    }
    void restoreDiagonal() {
        for (int i = 0; i < numPoses; ++i)
            for (int k = 0; k < 6; ++k) (*HppDiag[i])(k, k) = diagBackupP[i][k];
        for (int i = 0; i < numLandmarks; ++i)
            for (int k = 0; k < HllDiag[i]->r; ++k) (*HllDiag[i])(k, k) = diagBackupL[i][k];
    }

#ifdef REFCPU_FAST
    // refcpu-fast: one landmark's Schur contribution with compile-time block sizes (same
    // products in the same summation order as the heap-block path below)
    template <int DL>
    void schur_landmark(int l, int base) {
        const DMat &D = *HllDiag[l];
        Dinv[l] = lu_inverse(D);
        const DMat &Di = Dinv[l];
        double db[DL];
        for (int i = 0; i < DL; ++i) {
            double acc = 0.0;
            for (int k = 0; k < DL; ++k) acc += Di(i, k) * b[sizePoses + base + k];
            db[i] = acc;
        }
        auto &colL = HplCCS[l];
        DMat *const *pb = pairBlk[l].data();
        for (size_t a = 0; a < colL.size(); ++a) {
            const int i1 = colL[a].first;
            const double *Bi = colL[a].second->a;  // 6 x DL column-major
            double BD[6 * DL];                     // Bi·Dinv, column-major
            for (int j = 0; j < DL; ++j)
                for (int i = 0; i < 6; ++i) BD[i + 6 * j] = 0.0;
            for (int j = 0; j < DL; ++j)
                for (int k = 0; k < DL; ++k) {
                    const double dkj = Di(k, j);
                    for (int i = 0; i < 6; ++i) BD[i + 6 * j] += Bi[i + 6 * k] * dkj;
                }
            double Bb[6] = {0, 0, 0, 0, 0, 0};
            for (int k = 0; k < DL; ++k)
                for (int i = 0; i < 6; ++i) Bb[i] += Bi[i + 6 * k] * db[k];
            for (int k = 0; k < 6; ++k) coeff[i1 * 6 + k] += Bb[k];
            for (size_t c2 = a; c2 < colL.size(); ++c2) {
                double *C = (*pb++)->a;
                const double *B2 = colL[c2].second->a;
                for (int j = 0; j < 6; ++j)
                    for (int k = 0; k < DL; ++k) {
                        const double bjk = B2[j + 6 * k];
                        for (int i = 0; i < 6; ++i) C[i + 6 * j] -= BD[i + 6 * k] * bjk;
                    }
            }
        }
    }
#endif
    bool solve() {
        // _Hschur = _Hpp (keeping the pattern of _Hschur)
        for (int i = 0; i < numPoses; ++i)
            for (auto &kv : schurRow[i]) {
                if (kv.first == i) *kv.second = *HppDiag[i];
                else kv.second->setZero();
            }
        std::fill(coeff.begin(), coeff.begin() + sizePoses, 0.0);
        std::vector<int> lmBase(numLandmarks);
        {
            int off = 0;
            for (int l = 0; l < numLandmarks; ++l) { lmBase[l] = off; off += HllDiag[l]->r; }
        }
        for (int l = 0; l < numLandmarks; ++l) {
            const DMat &D = *HllDiag[l];
#ifdef REFCPU_FAST
            if (D.r == 3) { schur_landmark<3>(l, lmBase[l]); continue; }
            if (D.r == 4) { schur_landmark<4>(l, lmBase[l]); continue; }
#endif
            Dinv[l] = lu_inverse(D);
            DMat db(D.r, 1);
            for (int j = 0; j < D.r; ++j) db(j, 0) = b[sizePoses + lmBase[l] + j];
            db = mul(Dinv[l], db);
            auto &colL = HplCCS[l];
#ifdef REFCPU_FAST
            DMat *const *pb = pairBlk[l].data();
#endif
            for (size_t a = 0; a < colL.size(); ++a) {
                int i1 = colL[a].first;
                const DMat &Bi = *colL[a].second;
                DMat BDinv = mul(Bi, Dinv[l]);
                DMat Bb = mul(Bi, db);
                for (int k = 0; k < 6; ++k) coeff[i1 * 6 + k] += Bb(k, 0);
#ifdef REFCPU_FAST
                for (size_t c2 = a; c2 < colL.size(); ++c2) sub_mul_transB(**pb++, BDinv, *colL[c2].second);
#else
                auto &row = schurRow[i1];
                for (size_t c2 = a; c2 < colL.size(); ++c2) {
                    int i2 = colL[c2].first;
                    sub_mul_transB(*row.at(i2), BDinv, *colL[c2].second);
                }
#endif
            }
        }
        for (int i = 0; i < sizePoses; ++i) bschur[i] = b[i] - coeff[i];
        bool ok = linear.solve(numPoses, schurCols, bschur.data(), x.data());
        if (!ok) return false;
        // cl = bl - Hpl^T xp ; xl = Dinv * cl
        std::vector<double> cl(sizeLandmarks);
        for (int l = 0; l < numLandmarks; ++l) {
            int d = HllDiag[l]->r;
            for (int j = 0; j < d; ++j) cl[lmBase[l] + j] = b[sizePoses + lmBase[l] + j];
            for (auto &kv : HplCCS[l]) {
                const DMat &Bi = *kv.second;
                for (int j = 0; j < d; ++j) {
                    double s = 0;
                    for (int k = 0; k < 6; ++k) s += Bi(k, j) * (-x[kv.first * 6 + k]);
                    cl[lmBase[l] + j] += s;
                }
            }
            for (int j = 0; j < d; ++j) {
                double s = 0;
                for (int k = 0; k < d; ++k) s += Dinv[l](j, k) * cl[lmBase[l] + k];
                x[sizePoses + lmBase[l] + j] = s;
            }
        }
        return true;
    }
};

// ------------------------------------------------------------------------------------
// SparseOptimizer + OptimizationAlgorithmLevenberg restatement
// ------------------------------------------------------------------------------------
struct Optimizer {
    std::map<int, Vertex *> vertices;
    std::vector<std::unique_ptr<Vertex>> vstore;
    std::vector<std::unique_ptr<Edge>> edges;
    std::vector<Vertex *> activeVertices, ivMap;
    std::vector<Edge *> activeEdges;
    BlockSolverX solver;
    double currentLambda = 0, ni = 2, tau = 1e-5;
    int maxTrials = 10;
    int verbose = 0;
    std::vector<plba_iter_trace> *trace = nullptr;
    int stage = 0;

    void addVertex(Vertex *v) { vstore.emplace_back(v); vertices[v->id] = v; }
    void addEdge(Edge *e) {
        e->internal_id = (int)edges.size();
        edges.emplace_back(e);
        e->v[0]->edges.push_back(e);
        e->v[1]->edges.push_back(e);
    }

    // SparseOptimizer::initializeOptimization(int level)
    bool initializeOptimization(int level) {
        activeVertices.clear();
        activeEdges.clear();
        ivMap.clear();
        std::set<Edge *> aux;
        for (auto &kv : vertices) {
            Vertex *v = kv.second;
            int levelEdges = 0;
            for (Edge *e : v->edges)
                if (level < 0 || e->level == level)
                    if (!e->allVerticesFixed()) { aux.insert(e); levelEdges++; }
            if (levelEdges) activeVertices.push_back(v);
        }
        for (Edge *e : aux) activeEdges.push_back(e);
        std::sort(activeVertices.begin(), activeVertices.end(), [](Vertex *a, Vertex *b) { return a->id < b->id; });
        std::sort(activeEdges.begin(), activeEdges.end(), [](Edge *a, Edge *b) { return a->internal_id < b->internal_id; });
        for (auto &kv : vertices) kv.second->hidx = -1;
        int i = 0;  // buildIndexMapping
        for (int k = 0; k < 2; ++k)
            for (Vertex *v : activeVertices) {
                if (!v->fixed) {
                    if ((int)v->marginalized == k) { v->hidx = i++; ivMap.push_back(v); }
                } else v->hidx = -1;
            }
        return true;
    }
    void computeActiveErrors() { for (Edge *e : activeEdges) e->computeError(); }
    double activeRobustChi2() const {
        double chi = 0.0, rho[3];
        for (Edge *e : activeEdges) {
            if (e->robust) { huber(e->chi2(), e->delta, rho); chi += rho[0]; }
            else chi += e->chi2();
        }
        return chi;
    }
    void push() { for (Vertex *v : activeVertices) v->push(); }
    void pop() { for (Vertex *v : activeVertices) v->pop(); }
    void discardTop() { for (Vertex *v : activeVertices) v->discardTop(); }
    void update(const double *x) {
        for (Vertex *v : ivMap) {
            const double *u = v->marginalized ? x + solver.sizePoses + v->col : x + v->col;
            v->oplus(u);
        }
    }
    double computeLambdaInit() const {
        double maxDiagonal = 0.;
        for (Vertex *v : ivMap)
            for (int j = 0; j < v->dim; ++j) maxDiagonal = std::max(std::fabs((*v->H)(j, j)), maxDiagonal);
        return tau * maxDiagonal;
    }
    double computeScale() const {
        double scale = 0.;
        for (size_t j = 0; j < solver.x.size(); ++j) scale += solver.x[j] * (currentLambda * solver.x[j] + solver.b[j]);
        return scale;
    }
    enum Result { OK = 0, Terminate = 1, Fail = 2 };
    // OptimizationAlgorithmLevenberg::solve(int iteration)
    Result solveIteration(int iteration) {
        if (iteration == 0) solver.buildStructure(ivMap, activeEdges);
        computeActiveErrors();
        double currentChi = activeRobustChi2();
        double tempChi = currentChi;
        double chiStart = currentChi;
        solver.buildSystem(ivMap, activeEdges);
        if (iteration == 0) { currentLambda = computeLambdaInit(); ni = 2; }
        double lambdaStart = currentLambda;
        double rho = 0;
        int qmax = 0;
        do {
            push();
            solver.setLambda(currentLambda);
            bool ok2 = solver.solve();
            update(solver.x.data());  // g2o applies x even when the solve failed (then pops)
            solver.restoreDiagonal();
            computeActiveErrors();
            tempChi = activeRobustChi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            double scale = computeScale();
            scale += 1e-3;
            rho = (currentChi - tempChi) / scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                double scaleFactor = std::max(1. / 3., alpha);
                currentLambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
                discardTop();
            } else {
                currentLambda *= ni;
                ni *= 2;
                pop();
                if (!std::isfinite(currentLambda)) break;
            }
            qmax++;
        } while (rho < 0 && qmax < maxTrials);
        Result r = OK;
        if (qmax == maxTrials || rho == 0 || !std::isfinite(currentLambda)) r = Terminate;
        if (trace) trace->push_back(plba_iter_trace{stage, iteration, qmax, (int)r, chiStart, currentChi, lambdaStart, currentLambda});
        if (verbose)
            std::fprintf(stderr, "[refcpu] stage %d it %d chi2 %.9g -> %.9g lambda %.6g trials %d\n", stage, iteration,
                         chiStart, currentChi, currentLambda, qmax);
        return r;
    }
    // SparseOptimizer::optimize(int iterations)
    int optimize(int iterations, double *finalChi) {
        if (ivMap.empty()) { if (finalChi) *finalChi = 0; return -1; }
        bool ok = true;
        int it_done = 0;
        Result result = OK;
        for (int i = 0; i < iterations && ok; ++i) {
            result = solveIteration(i);
            ok = (result == OK);
            ++it_done;
        }
        if (finalChi) *finalChi = activeRobustChi2();
        if (result == Fail) return 0;
        return it_done;
    }
};

}  // namespace

// ====================================================================================
// C ABI
// ====================================================================================
extern "C" {

void refcpu_default_opts(refcpu_opts *o) {
    o->corrected_line_jacobian = 0;
    o->verbose = 0;
    o->max_trials = 10;
    o->tau = 1e-5;
    o->stage_iters[0] = 5;
    o->stage_iters[1] = 10;
}

static void load_pose(const double *T, double R[9], double t[3]) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = T[i * 4 + j];
        t[i] = T[i * 4 + 3];
    }
}
static void store_pose(double *T, const double R[9], const double t[3]) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[i * 4 + j] = R[i * 3 + j];
        T[i * 4 + 3] = t[i];
    }
}

int refcpu_lba_plucker(const plba_graph *g, const refcpu_opts *o, plba_result *res, plba_iter_trace *trace,
                       int32_t trace_cap, int32_t *n_trace) {
    refcpu_opts dflt;
    if (!o) { refcpu_default_opts(&dflt); o = &dflt; }
    if (!g || g->n_kf < 0 || g->n_pt < 0 || g->n_ln < 0 || g->n_ept < 0 || g->n_eln < 0) return PLBA_E_INVALID;
    for (int e = 0; e < g->n_ept; ++e)
        if (g->ept_lm[e] < 0 || g->ept_lm[e] >= g->n_pt || g->ept_kf[e] < 0 || g->ept_kf[e] >= g->n_kf) return PLBA_E_INVALID;
    for (int e = 0; e < g->n_eln; ++e)
        if (g->eln_lm[e] < 0 || g->eln_lm[e] >= g->n_ln || g->eln_kf[e] < 0 || g->eln_kf[e] >= g->n_kf) return PLBA_E_INVALID;

    Optimizer opt;
    std::vector<plba_iter_trace> tr;
    opt.trace = &tr;
    opt.tau = o->tau;
    opt.maxTrials = o->max_trials;
    opt.verbose = o->verbose;
    Cam cam{g->fx, g->fy, g->cx, g->cy};

    // graph build (src/mapHandler.cpp:5931-6117)
    std::vector<VertexLMPose *> poses(g->n_kf);
    for (int k = 0; k < g->n_kf; ++k) {
        auto *v = new VertexLMPose();
        load_pose(g->kf_Tcw + 12 * k, v->R, v->t);
        v->id = g->kf_id[k];
        v->fixed = g->kf_fixed[k] != 0;
        opt.addVertex(v);
        poses[k] = v;
    }
    std::vector<VertexLMPointXYZ *> pts(g->n_pt);
    for (int p = 0; p < g->n_pt; ++p) {
        auto *v = new VertexLMPointXYZ();
        std::memcpy(v->p, g->pt_xyz + 3 * p, 24);
        v->id = g->pt_id[p];
        v->marginalized = true;
        opt.addVertex(v);
        pts[p] = v;
    }
    std::vector<VertexLMLineOrth *> lns(g->n_ln);
    for (int l = 0; l < g->n_ln; ++l) {
        auto *v = new VertexLMLineOrth();
        std::memcpy(v->o, g->ln_orth + 4 * l, 32);
        v->id = g->ln_id[l];
        v->marginalized = true;
        opt.addVertex(v);
        lns[l] = v;
    }
    std::vector<EdgePosePoint *> ep(g->n_ept);
    for (int e = 0; e < g->n_ept; ++e) {
        auto *ed = new EdgePosePoint();
        ed->v[0] = pts[g->ept_lm[e]];
        ed->v[1] = poses[g->ept_kf[e]];
        ed->obs[0] = g->ept_obs[2 * e];
        ed->obs[1] = g->ept_obs[2 * e + 1];
        ed->info = g->ept_info[e];
        ed->robust = true;
        ed->delta = g->huber_pt;
        ed->cam = cam;
        opt.addEdge(ed);
        ep[e] = ed;
    }
    std::vector<EdgePoseLine *> el(g->n_eln);
    for (int e = 0; e < g->n_eln; ++e) {
        auto *ed = new EdgePoseLine();
        ed->v[0] = lns[g->eln_lm[e]];
        ed->v[1] = poses[g->eln_kf[e]];
        std::memcpy(ed->obs, g->eln_obs + 4 * e, 32);
        ed->info = g->eln_info[e];
        ed->robust = true;
        ed->delta = g->huber_ln;
        ed->cam = cam;
        ed->corrected = o->corrected_line_jacobian;
        opt.addEdge(ed);
        el[e] = ed;
    }

    auto t0 = std::chrono::steady_clock::now();
    // stage 1 (src/mapHandler.cpp:6121-6122)
    opt.stage = 0;
    opt.initializeOptimization(0);
    double chi1 = 0, chi2v = 0;
    int it1 = opt.optimize(o->stage_iters[0], &chi1);
    // classification (src/mapHandler.cpp:6125-6147)
    for (auto *e : ep) {
        if (e->chi2() > 5.991 || !e->isDepthPositive()) e->level = 1;
        e->robust = false;
    }
    for (auto *e : el) {
        if (e->chi2() > 5.991) e->level = 1;
        e->robust = false;
    }
    std::vector<uint8_t> lvl_p(g->n_ept), lvl_l(g->n_eln);
    for (int e = 0; e < g->n_ept; ++e) lvl_p[e] = (uint8_t)ep[e]->level;
    for (int e = 0; e < g->n_eln; ++e) lvl_l[e] = (uint8_t)el[e]->level;
    // stage 2 (src/mapHandler.cpp:6151-6152)
    opt.stage = 1;
    opt.initializeOptimization(0);
    int it2 = opt.optimize(o->stage_iters[1], &chi2v);
    // post-solve refresh of level-1 edges (src/mapHandler.cpp:6158-6160, 6226-6228)
    for (auto *e : ep) if (e->level == 1) e->computeError();
    for (auto *e : el) if (e->level == 1) e->computeError();
    auto t1 = std::chrono::steady_clock::now();

    if (res) {
        res->iters[0] = it1;
        res->iters[1] = it2;
        res->chi2[0] = chi1;
        res->chi2[1] = chi2v;
        res->solve_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (res->kf_Tcw) for (int k = 0; k < g->n_kf; ++k) store_pose(res->kf_Tcw + 12 * k, poses[k]->R, poses[k]->t);
        if (res->pt_xyz) for (int p = 0; p < g->n_pt; ++p) std::memcpy(res->pt_xyz + 3 * p, pts[p]->p, 24);
        if (res->ln_orth) for (int l = 0; l < g->n_ln; ++l) std::memcpy(res->ln_orth + 4 * l, lns[l]->o, 32);
        for (int e = 0; e < g->n_ept; ++e) {
            if (res->ept_chi2) res->ept_chi2[e] = ep[e]->chi2();
            if (res->ept_depth_ok) res->ept_depth_ok[e] = ep[e]->isDepthPositive() ? 1 : 0;
            if (res->ept_level) res->ept_level[e] = lvl_p[e];
        }
        for (int e = 0; e < g->n_eln; ++e) {
            if (res->eln_chi2) res->eln_chi2[e] = el[e]->chi2();
            if (res->eln_level) res->eln_level[e] = lvl_l[e];
        }
    }
    if (n_trace) *n_trace = (int32_t)tr.size();
    if (trace)
        for (int i = 0; i < (int)tr.size() && i < trace_cap; ++i) trace[i] = tr[i];
    return PLBA_OK;
}

void refcpu_point_edge(const double *Tcw, const double *xyz, const double *obs, double fx, double fy, double cx,
                       double cy, double *err, double *Ji, double *Jj) {
    double R[9], t[3], Pc[3];
    load_pose(Tcw, R, t);
    Cam c{fx, fy, cx, cy};
    if (err) point_error(R, t, xyz, obs, c, err, Pc);
    if (Ji && Jj) point_jac(R, t, xyz, c, Ji, Jj);
}
void refcpu_line_edge(const double *Tcw, const double *orth, const double *obs, double fx, double fy, double cx,
                      double cy, int corrected, double *err, double *Ji, double *Jj) {
    double R[9], t[3];
    load_pose(Tcw, R, t);
    Cam c{fx, fy, cx, cy};
    if (err) line_error(R, t, orth, obs, c, err);
    if (Ji && Jj) line_jac(R, t, orth, obs, c, corrected, Ji, Jj);
}
void refcpu_pose_oplus(double *Tcw, const double *d) {
    double R[9], t[3];
    load_pose(Tcw, R, t);
    pose_oplus(R, t, d);
    store_pose(Tcw, R, t);
}
void refcpu_line_oplus(double *orth, const double *d) {
    double n[4];
    update_orth(orth, d, n);
    std::memcpy(orth, n, 32);
}
void refcpu_orth_to_pluker(const double *o, double *L) { orth_to_pluker(o, L); }
void refcpu_pluker_to_orth(const double *L, double *o) { pluker_to_orth(L, o); }

}  // extern "C"
