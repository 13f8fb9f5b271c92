// refhlm.cpp — TEST INFRASTRUCTURE ONLY (see refhlm.h). PARITY UNPINNED vs the reference (no
// reference tests or fixtures exist and it cannot be built here); pinned by the known-answer
// tests of tests/test_hlm_oracle.py.
//
// Single-threaded restatement of the hand-rolled Levenberg–Marquardt LBA of the Plücker map,
//   MapHandler::levMarquardtOptimizationLBAForPluker   src/mapHandler.cpp:1618-2332
// kept bug-compatible with the reference:
//   * one scalar residual r = ‖e‖ per observation; "Jacobians" of r as the reference writes
//     them (:1681-1695 points, :1772-1811 lines) with the max(homogTh, ·) guards;
//   * Cauchy weight w = 1/(1+r²) (src2/auxiliar.cpp:556-559);
//   * H += w·JᵀJ (pose, landmark and coupling blocks), g += w·J·r, err += w·r²;
//   * err /= (Npt_obs + Nls_obs) with both counters never incremented (:1642,1731,1849):
//     err becomes +inf (params.err_per_obs = 1 divides by the observation count instead);
//   * λ = lambdaLbaLM·max|H_ii| once (:1852-1858); Marquardt damping H(i,i) += λ·H(i,i);
//     DX = SimplicialLDLT(H).solve(g) — restated here as an exact block solve (landmark blocks
//     eliminated first, LDLᵀ of the reduced pose system) or, with opts.dense, the literal dense
//     N×N matrix and an unpivoted LDLᵀ;
//   * first step applied unconditionally (:1867-1895); then per iteration: stop if
//     |err−err_prev| < minErrorChange or err < minError (:2111), solve, λ/=k and no update when
//     err > err_prev, else λ*=k and update (:2122-2151), stop if ‖DX‖ < minErrorChange (:2153);
//   * point observations of free KFs use inverse_se3(expmap_se3(X_i)) from the second
//     linearisation on (:1922-1927), every line observation keeps the MAP pose (:2010-2012);
//     the first linearisation reads the map states (point3D, NDw, T_kf_w; :1655-1659,1744-1752);
//   * pose update X_i ← logmap_se3(expmap_se3(X_i)·inverse_se3(expmap_se3(DX_i))) (:1868-1873);
//     lines updateOrthCoord (include/mapHandler.h:252-309), points X += DX.
// The write-back and outlier bookkeeping of :2160-2330 are host-side (host/map_handler.cpp).
// params.variant = PLBA_HLM_GBA restates MapHandler::levMarquardtOptimizationGBA (:3128-3726) the
// same way: 6-dim endpoint lines observed as image line equations (gba_line_obs), the aliased
// Pwj = Qwj = X.block(6Nkf+3Npt+3·j) reads after the first linearisation (:3547-3548), an int
// Hmax (:3386), X += DX for every landmark and the ε stop tests passed in as min_error(_change).

#include "refhlm.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

namespace {

struct Cam {
    double fx, fy, cx, cy;
};

// ---- 3x3 / 4x4 helpers (row-major)
inline void mat3mul(const double A[9], const double B[9], double C[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
inline void mat3vec(const double A[9], const double v[3], double r[3]) {
    for (int i = 0; i < 3; ++i) r[i] = A[i * 3] * v[0] + A[i * 3 + 1] * v[1] + A[i * 3 + 2] * v[2];
}
// skew / vectorHat (src2/auxiliar.cpp:29-45, include/mapHandler.h:224-230)
inline void skew(const double v[3], double M[9]) {
    M[0] = 0;     M[1] = -v[2]; M[2] = v[1];
    M[3] = v[2];  M[4] = 0;     M[5] = -v[0];
    M[6] = -v[1]; M[7] = v[0];  M[8] = 0;
}
inline double norm3(const double v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
inline void cross3(const double a[3], const double b[3], double c[3]) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

// expmap_se3 (src2/auxiliar.cpp:124-141): x = [t; ω], T row-major 4x4
void expmap(const double x[6], double T[16]) {
    const double w[3] = {x[3], x[4], x[5]};
    double t[3] = {x[0], x[1], x[2]};
    const double theta = norm3(w);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(theta < 0.000001)) {
        double s[9], ss[9];
        skew(w, s);
        for (double &v : s) v /= theta;
        mat3mul(s, s, ss);
        const double st = std::sin(theta), ct = 1.0 - std::cos(theta);
        double V[9];
        for (int i = 0; i < 9; ++i) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            R[i] = (I + s[i] * st) + ss[i] * ct;
            V[i] = (I + s[i] * ct / theta) + ss[i] * (theta - st) / theta;
        }
        double tv[3];
        mat3vec(V, t, tv);
        t[0] = tv[0]; t[1] = tv[1]; t[2] = tv[2];
    }
    for (int i = 0; i < 3; ++i) {
        T[i * 4 + 0] = R[i * 3 + 0];
        T[i * 4 + 1] = R[i * 3 + 1];
        T[i * 4 + 2] = R[i * 3 + 2];
        T[i * 4 + 3] = t[i];
    }
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}

// 3x3 inverse by cofactors (Eigen's closed form for fixed 3x3)
void inv3(const double m[9], double r[9]) {
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[5] * m[6] - m[3] * m[8];
    const double c2 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c0 + m[1] * c1 + m[2] * c2;
    r[0] = c0 / det;
    r[3] = c1 / det;
    r[6] = c2 / det;
    r[1] = (m[2] * m[7] - m[1] * m[8]) / det;
    r[4] = (m[0] * m[8] - m[2] * m[6]) / det;
    r[7] = (m[1] * m[6] - m[0] * m[7]) / det;
    r[2] = (m[1] * m[5] - m[2] * m[4]) / det;
    r[5] = (m[2] * m[3] - m[0] * m[5]) / det;
    r[8] = (m[0] * m[4] - m[1] * m[3]) / det;
}

// logmap_se3 (src2/auxiliar.cpp:143-173)
void logmap(const double T[16], double x[6]) {
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    const double Vt[3] = {T[3], T[7], T[11]};
    double w[3] = {0, 0, 0};
    double V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double cosine = (R[0] + R[4] + R[8] - 1.0) / 2.0;
    if (cosine > 1.0) cosine = 1.0;
    else if (cosine < -1.0) cosine = -1.0;
    double sine = std::sqrt(1.0 - cosine * cosine);
    if (sine > 1.0) sine = 1.0;
    else if (sine < -1.0) sine = -1.0;
    const double theta = std::acos(cosine);
    if (theta > 0.000001) {
        // w_hat = θ(R − Rᵀ)/(2 sine); w = skewcoords(w_hat) = (w_hat(2,1), w_hat(0,2), w_hat(1,0))
        w[0] = theta * (R[7] - R[5]) / (2.0 * sine);
        w[1] = theta * (R[2] - R[6]) / (2.0 * sine);
        w[2] = theta * (R[3] - R[1]) / (2.0 * sine);
        double s[9], ss[9];
        skew(w, s);
        for (double &v : s) v /= theta;
        mat3mul(s, s, ss);
        for (int i = 0; i < 9; ++i) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            V[i] = (I + s[i] * (1.0 - cosine) / theta) + ss[i] * (theta - sine) / theta;
        }
    }
    double Vi[9], t[3];
    inv3(V, Vi);
    mat3vec(Vi, Vt, t);
    x[0] = t[0]; x[1] = t[1]; x[2] = t[2];
    x[3] = w[0]; x[4] = w[1]; x[5] = w[2];
}

// inverse_se3 (src2/auxiliar.cpp:113-122)
void inverse_se3(const double T[16], double Ti[16]) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Ti[i * 4 + j] = T[j * 4 + i];
        Ti[i * 4 + 3] = -(T[0 * 4 + i] * T[3] + T[1 * 4 + i] * T[7] + T[2 * 4 + i] * T[11]);
    }
    Ti[12] = 0; Ti[13] = 0; Ti[14] = 0; Ti[15] = 1;
}
void mat4mul(const double A[16], const double B[16], double C[16]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += A[i * 4 + k] * B[k * 4 + j];
            C[i * 4 + j] = s;
        }
}
// Tiw (row-major 3x4 Tcw) of a free KF from its X block: inverse_se3(expmap_se3(x))
void tcw_from_x(const double x[6], double Tcw[12]) {
    double T[16], Ti[16];
    expmap(x, T);
    inverse_se3(T, Ti);
    std::memcpy(Tcw, Ti, 12 * sizeof(double));
}

// updateOrthCoord (include/mapHandler.h:252-309; identical to g2o_types.h:72-130)
void update_orth(const double D[4], const double dD[4], double out[4]) {
    const double s1 = std::sin(D[0]), c1 = std::cos(D[0]);
    const double s2 = std::sin(D[1]), c2 = std::cos(D[1]);
    const double s3 = std::sin(D[2]), c3 = std::cos(D[2]);
    const double R[9] = {c2 * c3, s1 * s2 * c3 - c1 * s3, c1 * s2 * c3 + s1 * s3,
                         c2 * s3, s1 * s2 * s3 + c1 * c3, c1 * s2 * s3 - s1 * c3,
                         -s2,     s1 * c2,                c1 * c2};
    const double w1 = std::cos(D[3]), w2 = std::sin(D[3]);
    const double cz = std::cos(dD[2]), sz = std::sin(dD[2]);
    const double cy = std::cos(dD[1]), sy = std::sin(dD[1]);
    const double cx = std::cos(dD[0]), sx = std::sin(dD[0]);
    const double Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    const double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    const double Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    double T1[9], T2[9], Rn[9];
    mat3mul(R, Rx, T1);
    mat3mul(T1, Ry, T2);
    mat3mul(T2, Rz, Rn);
    const double cp = std::cos(dD[3]), sp = std::sin(dD[3]);
    const double W10 = w2 * cp + w1 * sp;
    out[0] = std::atan2(Rn[7], Rn[8]);
    out[1] = std::asin(-Rn[6]);
    out[2] = std::atan2(Rn[3], Rn[0]);
    out[3] = std::asin(W10);
}
// MapLine::changeOrthToPluker (src/mapFeatures.cpp:203-224)
void orth_to_pluker(const double o[4], double L[6]) {
    const double s1 = std::sin(o[0]), c1 = std::cos(o[0]);
    const double s2 = std::sin(o[1]), c2 = std::cos(o[1]);
    const double s3 = std::sin(o[2]), c3 = std::cos(o[2]);
    const double w1 = std::cos(o[3]), w2 = std::sin(o[3]);
    L[0] = w1 * (c2 * c3); L[1] = w1 * (c2 * s3); L[2] = w1 * (-s2);
    L[3] = w2 * (s1 * s2 * c3 - c1 * s3); L[4] = w2 * (s1 * s2 * s3 + c1 * c3); L[5] = w2 * (s1 * c2);
}

// ---- one point observation (src/mapHandler.cpp:1655-1698 / :1919-1964)
void point_obs(const double Tcw[12], const double X[3], const double obs[2], const Cam &c, double hth, double &r,
               double &w, double Jp[6], double Jl[3]) {
    const double R[9] = {Tcw[0], Tcw[1], Tcw[2], Tcw[4], Tcw[5], Tcw[6], Tcw[8], Tcw[9], Tcw[10]};
    double P[3];
    mat3vec(R, X, P);
    P[0] += Tcw[3]; P[1] += Tcw[7]; P[2] += Tcw[11];
    // cam->projection (src2/pinholeStereoCamera.cpp:235-241)
    const double u = c.cx + c.fx * P[0] / P[2], v = c.cy + c.fy * P[1] / P[2];
    const double dx = obs[0] - u, dy = obs[1] - v;
    r = std::sqrt(dx * dx + dy * dy);
    const double gx = P[0], gy = P[1], gz = P[2];
    const double gz2 = 1.0 / std::max(hth, gz * gz);
    const double fxdx = c.fx * dx, fydy = c.fy * dy;
    const double m = std::max(hth, r);
    Jp[0] = (gz2 * fxdx * gz) / m;
    Jp[1] = (gz2 * fydy * gz) / m;
    Jp[2] = (-gz2 * (fxdx * gx + fydy * gy)) / m;
    Jp[3] = (-gz2 * (fxdx * gx * gy + fydy * gy * gy + fydy * gz * gz)) / m;
    Jp[4] = (gz2 * (fxdx * gx * gx + fxdx * gz * gz + fydy * gx * gy)) / m;
    Jp[5] = (gz2 * (fydy * gx * gz - fxdx * gy * gz)) / m;
    const double j0 = gz2 * fxdx * gz, j1 = gz2 * fydy * gz, j2 = -gz2 * (fxdx * gx + fydy * gy);
    for (int k = 0; k < 3; ++k) Jl[k] = (j0 * R[k] + j1 * R[3 + k] + j2 * R[6 + k]) / m;  // Jᵀ·R
    w = 1.0 / (1.0 + r * r);
}

// ---- one line observation (src/mapHandler.cpp:1744-1811 / :2003-2071)
void line_obs(const double Tcw[12], const double L[6], const double obs[4], const Cam &c, double hth, double &r,
              double &w, double Jp[6], double Jl[4]) {
    const double R[9] = {Tcw[0], Tcw[1], Tcw[2], Tcw[4], Tcw[5], Tcw[6], Tcw[8], Tcw[9], Tcw[10]};
    const double t[3] = {Tcw[3], Tcw[7], Tcw[11]};
    // Rw = getOrhtRFromPluker(NDw), Ww = getOrthWFromPluker(NDw) (src/mapFeatures.cpp:226-249)
    const double n[3] = {L[0], L[1], L[2]}, d[3] = {L[3], L[4], L[5]};
    const double nn = norm3(n), dn = norm3(d);
    double cr[3];
    cross3(n, d, cr);
    const double cn = norm3(cr);
    double u1[3], u2[3], u3[3];
    for (int i = 0; i < 3; ++i) {
        u1[i] = n[i] / nn;
        u2[i] = d[i] / dn;
        u3[i] = cr[i] / cn;
    }
    const double fw = std::sqrt(nn * nn + dn * dn), w1 = nn / fw, w2 = dn / fw;
    // jacobianFromPlukerToOrth (src/mapFeatures.cpp:251-266), 6x4 row-major
    double PO[24] = {0};
    for (int i = 0; i < 3; ++i) {
        PO[i * 4 + 1] = -w1 * u3[i];
        PO[i * 4 + 2] = -w1 * u2[i];
        PO[i * 4 + 3] = -w2 * u1[i];
        PO[(3 + i) * 4 + 0] = w2 * u3[i];
        PO[(3 + i) * 4 + 2] = -w2 * u1[i];
        PO[(3 + i) * 4 + 3] = w1 * u2[i];
    }
    // NDc = TransformForPluker(Tiw, NDw) (include/mapHandler.h:232-240): [R n + [t]x R d; R d]
    double St[9], StR[9], Rn[3], Rd[3], tRd[3];
    skew(t, St);
    mat3mul(St, R, StR);
    mat3vec(R, n, Rn);
    mat3vec(R, d, Rd);
    mat3vec(StR, d, tRd);
    const double nc[3] = {Rn[0] + tRd[0], Rn[1] + tRd[1], Rn[2] + tRd[2]};
    // NDc_pixel = plukerK·NDc.head(3) (src2/pinholeStereoCamera.cpp:123-125)
    const double K[9] = {c.fy, 0, 0, 0, c.fx, 0, -c.fy * c.cx, -c.fx * c.cy, c.fx * c.fy};
    double l[3];
    mat3vec(K, nc, l);
    const double lx = l[0], ly = l[1], lz = l[2];
    const double fenmu = std::sqrt(lx * lx + ly * ly);
    double e[2];
    e[0] = (obs[0] * lx + obs[1] * ly + lz) / fenmu;
    e[1] = (obs[2] * lx + obs[3] * ly + lz) / fenmu;
    r = std::sqrt(e[0] * e[0] + e[1] * e[1]);
    // fai_lineCurr_RT top rows: [ -[R d]x | -[R n]x - [t]x [R d]x ]
    double SRd[9], SRn[9], StSRd[9];
    skew(Rd, SRd);
    skew(Rn, SRn);
    mat3mul(St, SRd, StSRd);
    double jp[2][6], jl[2][4];
    for (int k = 0; k < 2; ++k) {
        const double a = obs[2 * k], b = obs[2 * k + 1];
        const double fe[3] = {a * fenmu - lx * e[k] * fenmu * fenmu, b * fenmu - ly * e[k] * fenmu * fenmu, fenmu};
        double v[3];  // fai_e · K
        for (int j = 0; j < 3; ++j) v[j] = fe[0] * K[j] + fe[1] * K[3 + j] + fe[2] * K[6 + j];
        for (int j = 0; j < 3; ++j) {
            jp[k][j] = v[0] * (-SRd[j]) + v[1] * (-SRd[3 + j]) + v[2] * (-SRd[6 + j]);
            jp[k][3 + j] = v[0] * (-SRn[j] - StSRd[j]) + v[1] * (-SRn[3 + j] - StSRd[3 + j]) +
                           v[2] * (-SRn[6 + j] - StSRd[6 + j]);
        }
        double q[6];  // v · [R | [t]x R]  (top rows of getTransformMatrixForPluker)
        for (int j = 0; j < 3; ++j) {
            q[j] = v[0] * R[j] + v[1] * R[3 + j] + v[2] * R[6 + j];
            q[3 + j] = v[0] * StR[j] + v[1] * StR[3 + j] + v[2] * StR[6 + j];
        }
        for (int j = 0; j < 4; ++j) {
            double s = 0;
            for (int i = 0; i < 6; ++i) s += q[i] * PO[i * 4 + j];
            jl[k][j] = s;
        }
    }
    const double m = std::max(hth, r);
    for (int j = 0; j < 6; ++j) Jp[j] = (jp[0][j] * e[0] + jp[1][j] * e[1]) / m;
    for (int j = 0; j < 4; ++j) Jl[j] = (jl[0][j] * e[0] + jl[1][j] * e[1]) / m;
    w = 1.0 / (1.0 + r * r);
}

// ---- one GBA line observation (src/mapHandler.cpp:3270-3340 / :3545-3619): endpoints P, Q,
// image line l = (a, b, c), e = (l·π(P), l·π(Q)); the Jacobians use fx·e0 and fy·e1 where the
// point rows use fx·dx and fy·dy (lx = l_err(0), ly = l_err(1), :3293-3296)
void gba_line_obs(const double Tcw[12], const double P[3], const double Q[3], const double lo[3], const Cam &c,
                  double hth, double &r, double &w, double Jp[6], double Jl[6]) {
    const double R[9] = {Tcw[0], Tcw[1], Tcw[2], Tcw[4], Tcw[5], Tcw[6], Tcw[8], Tcw[9], Tcw[10]};
    double Pi[3], Qi[3];
    mat3vec(R, P, Pi);
    mat3vec(R, Q, Qi);
    for (int k = 0; k < 3; ++k) {
        Pi[k] += Tcw[4 * k + 3];
        Qi[k] += Tcw[4 * k + 3];
    }
    const double pu = c.cx + c.fx * Pi[0] / Pi[2], pv = c.cy + c.fy * Pi[1] / Pi[2];
    const double qu = c.cx + c.fx * Qi[0] / Qi[2], qv = c.cy + c.fy * Qi[1] / Qi[2];
    const double e0 = lo[0] * pu + lo[1] * pv + lo[2];
    const double e1 = lo[0] * qu + lo[1] * qv + lo[2];
    r = std::sqrt(e0 * e0 + e1 * e1);
    const double fxlx = c.fx * e0, fyly = c.fy * e1;
    const double m = std::max(hth, r);
    double JPi[6], JQi[6];
    auto rows = [&](const double *G, double *Jpose, double *Jlm, double ek) {
        const double gx = G[0], gy = G[1], gz = G[2];
        const double gz2 = 1.0 / std::max(hth, gz * gz);
        Jpose[0] = gz2 * fxlx * gz;
        Jpose[1] = gz2 * fyly * gz;
        Jpose[2] = -gz2 * (fxlx * gx + fyly * gy);
        Jpose[3] = -gz2 * (fxlx * gx * gy + fyly * gy * gy + fyly * gz * gz);
        Jpose[4] = gz2 * (fxlx * gx * gx + fxlx * gz * gz + fyly * gx * gy);
        Jpose[5] = gz2 * (fyly * gx * gz - fxlx * gy * gz);
        const double j0 = gz2 * fxlx * gz, j1 = gz2 * fyly * gz, j2 = -gz2 * (fxlx * gx + fyly * gy);
        for (int k = 0; k < 3; ++k) Jlm[k] = ((j0 * R[k] + j1 * R[3 + k] + j2 * R[6 + k]) * ek) / m;
    };
    rows(Pi, JPi, Jl, e0);
    rows(Qi, JQi, Jl + 3, e1);
    for (int k = 0; k < 6; ++k) Jp[k] = (JPi[k] * e0 + JQi[k] * e1) / m;
    w = 1.0 / (1.0 + r * r);
}

// ---- unpivoted LDLᵀ solve of a dense symmetric system (lower triangle read), in place
bool ldlt_solve(std::vector<double> &A, int n, std::vector<double> &b) {
    std::vector<double> Dv(n);
    for (int j = 0; j < n; ++j) {
        double dj = A[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) dj -= A[(size_t)j * n + k] * A[(size_t)j * n + k] * Dv[k];
        if (dj == 0.0) return false;
        Dv[j] = dj;
        for (int i = j + 1; i < n; ++i) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k] * Dv[k];
            A[(size_t)i * n + j] = s / dj;
        }
    }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < i; ++k) b[i] -= A[(size_t)i * n + k] * b[k];
    for (int i = 0; i < n; ++i) b[i] /= Dv[i];
    for (int i = n - 1; i >= 0; --i)
        for (int k = i + 1; k < n; ++k) b[i] -= A[(size_t)k * n + i] * b[k];
    return true;
}

struct Obs {
    int lm, kf, h;  // landmark (local), keyframe, free-pose index or -1
    double r, w, Jp[6], Jl[6];
};

}  // namespace

extern "C" {

int refhlm_lba(const plba_graph *g, const plba_hlm_state *st, const plba_hlm_params *p, const refhlm_opts *o,
               plba_hlm_result *res, plba_iter_trace *trace, int32_t trace_cap, int32_t *n_trace) {
    if (!g || !st || !p) return -1;
    const auto t0 = std::chrono::steady_clock::now();
    const Cam cam{g->fx, g->fy, g->cx, g->cy};
    const int n_kf = g->n_kf, n_pt = g->n_pt, n_ln = g->n_ln;
    // kf_list: free KFs in id order (map_keyframes order, :1512-1524)
    std::vector<int> korder(n_kf), hidx(n_kf, -1);
    std::iota(korder.begin(), korder.end(), 0);
    std::stable_sort(korder.begin(), korder.end(), [&](int a, int b) { return g->kf_id[a] < g->kf_id[b]; });
    int nf = 0;
    for (int k : korder)
        if (!g->kf_fixed[k]) hidx[k] = nf++;
    // GBA (src/mapHandler.cpp:3128-3726): lines are 6-dim endpoint landmarks line3D = [P; Q]
    const bool gba = p->variant == PLBA_HLM_GBA;
    if (gba && n_ln && !st->ln_line3d) return -1;
    const int LD = gba ? 6 : 4;  // line landmark dimension
    const int N = 6 * nf + 3 * n_pt + LD * n_ln;
    // state X: pose blocks, points, lines (orth, or GBA endpoints)
    std::vector<double> xk((size_t)n_kf * 6), Tcw((size_t)n_kf * 12), Xp((size_t)n_pt * 3), Xl((size_t)n_ln * LD);
    for (size_t i = 0; i < xk.size(); ++i) xk[i] = st->kf_x[i];
    for (size_t i = 0; i < Tcw.size(); ++i) Tcw[i] = g->kf_Tcw[i];  // map poses (first linearisation)
    for (size_t i = 0; i < Xp.size(); ++i) Xp[i] = g->pt_xyz[i];
    for (size_t i = 0; i < Xl.size(); ++i) Xl[i] = gba ? st->ln_line3d[i] : g->ln_orth[i];
    std::vector<double> Lp((size_t)n_ln * 6);
    for (size_t i = 0; i < Lp.size() && !gba; ++i) Lp[i] = st->ln_pluker[i];  // map NDw (first linearisation)
    std::vector<Obs> obs((size_t)g->n_ept + g->n_eln);
    const double nobs = (double)(g->n_ept + g->n_eln);

    double lambda = p->lambda0, err = 0.0, err_prev = 999999999.9, dxn = 0.0;
    int lin = 0, solves = 0, acc = 0, nt = 0;
    std::vector<double> Hpp, gp, Hll, gl, DX(N);
    auto linearize = [&](bool first) {
        err = 0.0;
        Hpp.assign((size_t)nf * 36, 0.0);
        gp.assign((size_t)nf * 6, 0.0);
        Hll.assign((size_t)(n_pt + n_ln) * 36, 0.0);
        gl.assign((size_t)(n_pt + n_ln) * 6, 0.0);
        for (int e = 0; e < g->n_ept + g->n_eln; ++e) {
            Obs &s = obs[e];
            const bool pt = e < g->n_ept;
            const int ee = pt ? e : e - g->n_ept;
            const int kf = pt ? g->ept_kf[ee] : g->eln_kf[ee];
            s.lm = pt ? g->ept_lm[ee] : n_pt + g->eln_lm[ee];
            s.kf = kf;
            s.h = hidx[kf];
            std::fill(s.Jl, s.Jl + 6, 0.0);
            if (pt) {
                // Tiw: map pose on the first linearisation and for KFs outside kf_list (:1657,1925)
                double T[12];
                if (first || s.h < 0) std::memcpy(T, g->kf_Tcw + (size_t)kf * 12, sizeof T);
                else std::memcpy(T, &Tcw[(size_t)kf * 12], sizeof T);
                point_obs(T, &Xp[(size_t)g->ept_lm[ee] * 3], g->ept_obs + 2 * (size_t)ee, cam, p->homog_th, s.r, s.w,
                          s.Jp, s.Jl);
            } else if (gba) {
                // map pose (:3273, 3550); line3D on the first linearisation (:3270-3271), then
                // Pwj = Qwj = X.block(6Nkf+3Npt+3·j) — the 6-dim blocks read at a stride of 3 (:3547-3548)
                const int l = g->eln_lm[ee];
                const double *P = first ? &Xl[(size_t)l * 6] : &Xl[(size_t)l * 3];
                const double *Q = first ? &Xl[(size_t)l * 6 + 3] : &Xl[(size_t)l * 3];
                gba_line_obs(g->kf_Tcw + (size_t)kf * 12, P, Q, g->eln_obs + 4 * (size_t)ee, cam, p->homog_th, s.r,
                             s.w, s.Jp, s.Jl);
            } else {
                // every line observation uses the map pose (:1750,2010); NDw from the map on the
                // first linearisation, changeOrthToPluker(X) afterwards (:2003-2005)
                const int l = g->eln_lm[ee];
                double L[6];
                if (first) std::memcpy(L, &Lp[(size_t)l * 6], sizeof L);
                else orth_to_pluker(&Xl[(size_t)l * 4], L);
                line_obs(g->kf_Tcw + (size_t)kf * 12, L, g->eln_obs + 4 * (size_t)ee, cam, p->homog_th, s.r, s.w, s.Jp,
                         s.Jl);
            }
            const int D = pt ? 3 : LD;
            err += s.r * s.r * s.w;
            double *H = &Hll[(size_t)s.lm * 36];
            for (int i = 0; i < D; ++i) {
                gl[(size_t)s.lm * 6 + i] += s.Jl[i] * s.r * s.w;
                for (int j = 0; j < D; ++j) H[i * 6 + j] += s.Jl[i] * s.Jl[j] * s.w;
            }
            if (s.h >= 0) {
                for (int i = 0; i < 6; ++i) {
                    gp[(size_t)s.h * 6 + i] += s.Jp[i] * s.r * s.w;
                    for (int j = 0; j < 6; ++j) Hpp[(size_t)s.h * 36 + i * 6 + j] += s.Jp[i] * s.Jp[j] * s.w;
                }
            }
        }
        err /= p->err_per_obs ? nobs : 0.0;  // :1849 — (Npt_obs + Nls_obs) == 0 in the reference
        ++lin;
    };
    auto hmax = [&]() {
        double m = 0.0;
        for (int h = 0; h < nf; ++h)
            for (int i = 0; i < 6; ++i) m = std::max(m, std::fabs(Hpp[(size_t)h * 36 + i * 7]));
        for (int l = 0; l < n_pt + n_ln; ++l)
            for (int i = 0; i < 6; ++i) m = std::max(m, std::fabs(Hll[(size_t)l * 36 + i * 7]));
        return m;
    };
    auto dim = [&](int l) { return l < n_pt ? 3 : LD; };
    // DX = (H + λ·diag H)⁻¹ g
    auto solve = [&]() -> bool {
        ++solves;
        std::fill(DX.begin(), DX.end(), 0.0);
        auto col = [&](int l) { return 6 * nf + (l < n_pt ? 3 * l : 3 * n_pt + LD * (l - n_pt)); };
        if (o && o->dense) {  // the reference's dense H, literally
            std::vector<double> A((size_t)N * N, 0.0), b(N, 0.0);
            for (int h = 0; h < nf; ++h)
                for (int i = 0; i < 6; ++i) {
                    b[6 * h + i] = gp[(size_t)h * 6 + i];
                    for (int j = 0; j < 6; ++j) A[(size_t)(6 * h + i) * N + 6 * h + j] = Hpp[(size_t)h * 36 + i * 6 + j];
                }
            for (int l = 0; l < n_pt + n_ln; ++l) {
                const int c0 = col(l), D = dim(l);
                for (int i = 0; i < D; ++i) {
                    b[c0 + i] = gl[(size_t)l * 6 + i];
                    for (int j = 0; j < D; ++j) A[(size_t)(c0 + i) * N + c0 + j] = Hll[(size_t)l * 36 + i * 6 + j];
                }
            }
            for (const Obs &s : obs) {
                if (s.h < 0) continue;
                const int c0 = col(s.lm), D = dim(s.lm);
                for (int i = 0; i < D; ++i)
                    for (int j = 0; j < 6; ++j) {
                        const double v = s.Jl[i] * s.Jp[j] * s.w;
                        A[(size_t)(c0 + i) * N + 6 * s.h + j] += v;
                        A[(size_t)(6 * s.h + j) * N + c0 + i] += v;
                    }
            }
            for (int i = 0; i < N; ++i) A[(size_t)i * N + i] += lambda * A[(size_t)i * N + i];
            if (!ldlt_solve(A, N, b)) return false;
            DX = b;
            return true;
        }
        // block elimination of the landmarks (exact; SimplicialLDLT differs by rounding only)
        const int nl = n_pt + n_ln, n = 6 * nf;
        std::vector<double> Dinv((size_t)nl * 36, 0.0), S((size_t)n * n, 0.0), bs(n, 0.0);
        for (int h = 0; h < nf; ++h)
            for (int i = 0; i < 6; ++i) {
                bs[6 * h + i] = gp[(size_t)h * 6 + i];
                for (int j = 0; j < 6; ++j) S[(size_t)(6 * h + i) * n + 6 * h + j] = Hpp[(size_t)h * 36 + i * 6 + j];
                S[(size_t)(6 * h + i) * n + 6 * h + i] += lambda * Hpp[(size_t)h * 36 + i * 7];
            }
        for (int l = 0; l < nl; ++l) {  // (Hll + λ diag)⁻¹ by LDLᵀ solves of the unit vectors
            const int D = dim(l);
            for (int c = 0; c < D; ++c) {
                std::vector<double> A(D * D), b(D, 0.0);
                for (int i = 0; i < D; ++i)
                    for (int j = 0; j < D; ++j) A[i * D + j] = Hll[(size_t)l * 36 + i * 6 + j];
                for (int i = 0; i < D; ++i) A[i * D + i] += lambda * A[i * D + i];
                b[c] = 1.0;
                if (!ldlt_solve(A, D, b)) return false;
                for (int i = 0; i < D; ++i) Dinv[(size_t)l * 36 + i * 6 + c] = b[i];
            }
        }
        // per landmark: its observations of free KFs, W_e = w Jpᵀ Jl (6 x D)
        std::vector<std::vector<int>> lobs(nl);
        for (int e = 0; e < (int)obs.size(); ++e)
            if (obs[e].h >= 0) lobs[obs[e].lm].push_back(e);
        for (int l = 0; l < nl; ++l) {
            const int D = dim(l);
            const double *Di = &Dinv[(size_t)l * 36];
            // y = D⁻¹ g_l
            double y[6] = {0, 0, 0, 0, 0, 0};
            for (int i = 0; i < D; ++i)
                for (int j = 0; j < D; ++j) y[i] += Di[i * 6 + j] * gl[(size_t)l * 6 + j];
            for (int a : lobs[l]) {
                const Obs &A = obs[a];
                // b_s -= W_a y = Jp_a w_a (Jl_a · y)
                double jy = 0;
                for (int i = 0; i < D; ++i) jy += A.Jl[i] * y[i];
                for (int i = 0; i < 6; ++i) bs[6 * A.h + i] -= A.Jp[i] * A.w * jy;
                double zD[6] = {0, 0, 0, 0, 0, 0};  // Jl_a D⁻¹
                for (int j = 0; j < D; ++j)
                    for (int i = 0; i < D; ++i) zD[j] += A.Jl[i] * Di[i * 6 + j];
                for (int bb : lobs[l]) {
                    const Obs &B = obs[bb];
                    double s = 0;
                    for (int j = 0; j < D; ++j) s += zD[j] * B.Jl[j];
                    s *= A.w * B.w;
                    for (int i = 0; i < 6; ++i)
                        for (int j = 0; j < 6; ++j) S[(size_t)(6 * A.h + i) * n + 6 * B.h + j] -= A.Jp[i] * s * B.Jp[j];
                }
            }
        }
        std::vector<double> xp = bs;
        if (n && !ldlt_solve(S, n, xp)) return false;
        for (int i = 0; i < n; ++i) DX[i] = xp[i];
        for (int l = 0; l < nl; ++l) {  // x_l = D⁻¹(g_l − Σ W_eᵀ x_p)
            const int D = dim(l);
            double rr[6] = {0, 0, 0, 0, 0, 0};
            for (int i = 0; i < D; ++i) rr[i] = gl[(size_t)l * 6 + i];
            for (int a : lobs[l]) {
                const Obs &A = obs[a];
                double jx = 0;
                for (int i = 0; i < 6; ++i) jx += A.Jp[i] * xp[6 * A.h + i];
                for (int i = 0; i < D; ++i) rr[i] -= A.Jl[i] * A.w * jx;
            }
            const double *Di = &Dinv[(size_t)l * 36];
            for (int i = 0; i < D; ++i) {
                double v = 0;
                for (int j = 0; j < D; ++j) v += Di[i * 6 + j] * rr[j];
                DX[col(l) + i] = v;
            }
        }
        return true;
    };
    auto apply = [&]() {
        for (int k = 0; k < n_kf; ++k) {
            const int h = hidx[k];
            if (h < 0) continue;
            double Tp[16], Ed[16], Ei[16], Tc[16];
            expmap(&xk[(size_t)k * 6], Tp);
            expmap(&DX[6 * h], Ed);
            inverse_se3(Ed, Ei);
            mat4mul(Tp, Ei, Tc);
            logmap(Tc, &xk[(size_t)k * 6]);
            tcw_from_x(&xk[(size_t)k * 6], &Tcw[(size_t)k * 12]);
        }
        for (int i = 0; i < 3 * n_pt; ++i) Xp[i] += DX[6 * nf + i];
        for (int l = 0; l < n_ln; ++l) {
            if (gba) {  // GBA: X += DX for every landmark (:3690-3691)
                for (int i = 0; i < 6; ++i) Xl[(size_t)l * 6 + i] += DX[6 * nf + 3 * n_pt + 6 * l + i];
                continue;
            }
            double out[4];
            update_orth(&Xl[(size_t)l * 4], &DX[6 * nf + 3 * n_pt + 4 * l], out);
            for (int i = 0; i < 4; ++i) Xl[(size_t)l * 4 + i] = out[i];
        }
        ++acc;
    };
    auto dxnorm = [&]() {
        double s = 0;
        for (double v : DX) s += v * v;
        return std::sqrt(s);
    };
    auto rec = [&](int it, int result, double l0) {
        if (trace && nt < trace_cap) trace[nt] = plba_iter_trace{0, it, 1, result, err, err, l0, lambda};
        ++nt;
    };
    for (int k = 0; k < n_kf; ++k)  // free KFs: Tiw from X on every later linearisation
        if (hidx[k] >= 0) tcw_from_x(&xk[(size_t)k * 6], &Tcw[(size_t)k * 12]);

    // first iteration (:1639-1895)
    if (N > 0 && !obs.empty()) {
        linearize(true);
        // GBA keeps Hmax in an int (:3386): the maximum truncated toward zero (|H_ii| >= 2^31 would
        // be an undefined conversion in the reference; it is taken as a 64-bit truncation here)
        lambda *= gba ? (double)(long long)hmax() : hmax();
        const double l0 = lambda;
        if (solve()) apply();
        dxn = dxnorm();
        rec(0, 0, l0);
        err_prev = err;
        for (int iters = 1; iters < p->max_iters; ++iters) {  // :1901-2158
            linearize(false);
            const double l0i = lambda;
            if (std::fabs(err - err_prev) < p->min_error_change || err < p->min_error) {
                rec(iters, 3, l0i);
                break;
            }
            const bool ok = solve();
            dxn = dxnorm();
            if (err > err_prev) {
                lambda /= p->lambda_k;
                rec(iters, 1, l0i);
            } else {
                lambda *= p->lambda_k;
                if (ok) apply();
                rec(iters, 0, l0i);
            }
            if (dxn < p->min_error_change) break;
            err_prev = err;
        }
    }
    if (o && o->verbose)
        fprintf(stderr, "[refhlm] %d linearisations, %d solves, %d applied, err %g, lambda %g\n", lin, solves, acc, err,
                lambda);
    if (res) {
        if (res->kf_x) std::memcpy(res->kf_x, xk.data(), xk.size() * sizeof(double));
        if (res->kf_Tcw)
            for (int k = 0; k < n_kf; ++k)
                std::memcpy(res->kf_Tcw + (size_t)k * 12, hidx[k] >= 0 ? &Tcw[(size_t)k * 12] : g->kf_Tcw + (size_t)k * 12,
                            12 * sizeof(double));
        if (res->pt_xyz) std::memcpy(res->pt_xyz, Xp.data(), Xp.size() * sizeof(double));
        if (res->ln_orth && !gba) std::memcpy(res->ln_orth, Xl.data(), Xl.size() * sizeof(double));
        if (res->ln_line3d && gba) std::memcpy(res->ln_line3d, Xl.data(), Xl.size() * sizeof(double));
        res->linearizations = lin;
        res->solves = solves;
        res->accepted = acc;
        res->err = err;
        res->lambda = lambda;
        res->dx_norm = dxn;
        res->solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (n_trace) *n_trace = nt;
    return 0;
}

void refhlm_point_obs(const double *Tcw, const double *xyz, const double *obs, double fx, double fy, double cx,
                      double cy, double homog_th, double *r, double *w, double *Jp, double *Jl) {
    point_obs(Tcw, xyz, obs, Cam{fx, fy, cx, cy}, homog_th, *r, *w, Jp, Jl);
}
void refhlm_line_obs(const double *Tcw, const double *pluker, const double *obs, double fx, double fy, double cx,
                     double cy, double homog_th, double *r, double *w, double *Jp, double *Jl) {
    line_obs(Tcw, pluker, obs, Cam{fx, fy, cx, cy}, homog_th, *r, *w, Jp, Jl);
}
void refhlm_gba_line_obs(const double *Tcw, const double *P, const double *Q, const double *lo, double fx, double fy,
                         double cx, double cy, double homog_th, double *r, double *w, double *Jp, double *Jl) {
    gba_line_obs(Tcw, P, Q, lo, Cam{fx, fy, cx, cy}, homog_th, *r, *w, Jp, Jl);
}
void refhlm_expmap(const double *x, double *T) { expmap(x, T); }
void refhlm_logmap(const double *T, double *x) { logmap(T, x); }
void refhlm_inverse_se3(const double *T, double *Ti) { inverse_se3(T, Ti); }

}  // extern "C"
