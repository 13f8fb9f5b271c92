// plba_math.hpp — device restatement of the g2o_types vertex/edge arithmetic (FP64).
//
// Every function follows the reference formula order so that the GPU path rounds like the
// reference does wherever the data flow allows:
//   vechat                      g2o_types/g2o_types.h:18-24
//   pose oplus (quaternion)     g2o_types/g2o_types.h:172-203  (+ Eigen toRotationMatrix)
//   orth oplus (updateOrthCoord)g2o_types/g2o_types.h:72-130
//   point reprojection error    g2o_types/g2o_types.h:224-263
//   point Jacobians             g2o_types/g2o_types.h:271-296
//   line error (Plücker)        g2o_types/g2o_types.h:320-387
//   line Jacobians              g2o_types/g2o_types.h:389-495 (incl. the orth-as-Plücker pose
//                               block of :429-430 unless `corrected`)
//   Huber robustify             g2o RobustKernelHuber
// Poses are Tcw stored row-major 3x4 [R | t] (12 doubles).
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#define PLBA_HD __host__ __device__ __forceinline__

namespace plba {

typedef double dbl4 __attribute__((ext_vector_type(4)));  // v_mfma_f64_16x16x4 accumulator

// broadcast lane l's value (l must be wave-uniform)
__device__ __forceinline__ double readlane_f64(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}

struct Cam {
    double fx, fy, cx, cy;
};

PLBA_HD void mat3vec(const double *R, const double *v, double *r) {
    r[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    r[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    r[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
}
PLBA_HD void mat3mul(const double *A, const double *B, double *C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3 + 0] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
PLBA_HD void vechat(const double *v, double *M) {
    M[0] = 0;     M[1] = -v[2]; M[2] = v[1];
    M[3] = v[2];  M[4] = 0;     M[5] = -v[0];
    M[6] = -v[1]; M[7] = v[0];  M[8] = 0;
}
PLBA_HD void rot_xyz(const double *th, double *R) {
    double s1 = sin(th[0]), c1 = cos(th[0]);
    double s2 = sin(th[1]), c2 = cos(th[1]);
    double s3 = sin(th[2]), c3 = cos(th[2]);
    R[0] = c2 * c3; R[1] = s1 * s2 * c3 - c1 * s3; R[2] = c1 * s2 * c3 + s1 * s3;
    R[3] = c2 * s3; R[4] = s1 * s2 * s3 + c1 * c3; R[5] = c1 * s2 * s3 - s1 * c3;
    R[6] = -s2;     R[7] = s1 * c2;                R[8] = c1 * c2;
}
// changeOrthToPluker (g2o_types.h:367-387)
PLBA_HD void orth_to_pluker(const double *o, double *L) {
    double R[9];
    rot_xyz(o, R);
    double w1 = cos(o[3]), w2 = sin(o[3]);
    L[0] = w1 * R[0]; L[1] = w1 * R[3]; L[2] = w1 * R[6];
    L[3] = w2 * R[1]; L[4] = w2 * R[4]; L[5] = w2 * R[7];
}

// VertexLMPose::oplusImpl — R <- R(q)·R, t <- t + δt (δ = [δt; δω])
PLBA_HD void pose_oplus(const double *Tin, const double *d, double *Tout) {
    const double wx = d[3], wy = d[4], wz = d[5];
    double theta = sqrt(wx * wx + wy * wy + wz * wz);
    double half = 0.5 * theta;
    double imag, real = cos(half);
    if (theta < 1e-10) {
        double tsq = theta * theta, t4 = tsq * tsq;
        imag = 0.5 - 0.0208333 * tsq + 0.000260417 * t4;
    } else {
        imag = sin(half) / theta;
    }
    double qw = real, qx = imag * wx, qy = imag * wy, qz = imag * wz;
    double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    double twx = tx * qw, twy = ty * qw, twz = tz * qw;
    double txx = tx * qx, txy = ty * qx, txz = tz * qx;
    double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    double dR[9] = {1 - (tyy + tzz), txy - twz,       txz + twy,
                    txy + twz,       1 - (txx + tzz), tyz - twx,
                    txz - twy,       tyz + twx,       1 - (txx + tyy)};
    double R[9] = {Tin[0], Tin[1], Tin[2], Tin[4], Tin[5], Tin[6], Tin[8], Tin[9], Tin[10]};
    double Rn[9];
    mat3mul(dR, R, Rn);
    Tout[0] = Rn[0]; Tout[1] = Rn[1]; Tout[2] = Rn[2];  Tout[3] = Tin[3] + d[0];
    Tout[4] = Rn[3]; Tout[5] = Rn[4]; Tout[6] = Rn[5];  Tout[7] = Tin[7] + d[1];
    Tout[8] = Rn[6]; Tout[9] = Rn[7]; Tout[10] = Rn[8]; Tout[11] = Tin[11] + d[2];
}

// VertexLMLineOrth::updateOrthCoord
PLBA_HD void orth_oplus(const double *D, const double *dD, double *out) {
    double R[9];
    rot_xyz(D, R);
    double w1 = cos(D[3]), w2 = sin(D[3]);
    double cz = cos(dD[2]), sz = sin(dD[2]);
    double cy = cos(dD[1]), sy = sin(dD[1]);
    double cx = cos(dD[0]), sx = sin(dD[0]);
    const double Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    const double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    const double Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    double T1[9], T2[9], Rn[9];
    mat3mul(R, Rx, T1);
    mat3mul(T1, Ry, T2);
    mat3mul(T2, Rz, Rn);
    double cp = cos(dD[3]), sp = sin(dD[3]);
    double W10 = w2 * cp + w1 * sp;
    out[0] = atan2(Rn[7], Rn[8]);
    out[1] = asin(-Rn[6]);
    out[2] = atan2(Rn[3], Rn[0]);
    out[3] = asin(W10);
}

// RobustKernelHuber::robustify -> rho0, rho1
PLBA_HD void huber(double e, double delta, double &rho0, double &rho1) {
    double dsqr = delta * delta;
    if (e <= dsqr) {
        rho0 = e;
        rho1 = 1.0;
    } else {
        double sqrte = sqrt(e);
        rho0 = 2 * sqrte * delta - dsqr;
        rho1 = delta / sqrte;
    }
}

// ---------------- EdgePosePoint ----------------
PLBA_HD void point_pc(const double *T, const double *P, double *Pc) {
    Pc[0] = T[0] * P[0] + T[1] * P[1] + T[2] * P[2] + T[3];
    Pc[1] = T[4] * P[0] + T[5] * P[1] + T[6] * P[2] + T[7];
    Pc[2] = T[8] * P[0] + T[9] * P[1] + T[10] * P[2] + T[11];
}
PLBA_HD void point_error(const double *T, const double *P, const double *obs, const Cam &c, double *e, double &z) {
    double Pc[3];
    point_pc(T, P, Pc);
#ifdef PLBA_EXACT_DIV
    double u = (Pc[0] / Pc[2]) * c.fx + c.cx;
    double v = (Pc[1] / Pc[2]) * c.fy + c.cy;
#else
    const double iz = 1.0 / Pc[2];  // one reciprocal (within ~1 ulp of the two divisions)
    double u = (Pc[0] * iz) * c.fx + c.cx;
    double v = (Pc[1] * iz) * c.fy + c.cy;
#endif
    e[0] = obs[0] - u;
    e[1] = obs[1] - v;
    z = Pc[2];
}
// Jl: 2x3 (row-major), Jp: 2x6
PLBA_HD void point_jac(const double *T, const double *P, const Cam &c, double *Jl, double *Jp) {
    double Pc[3];
    point_pc(T, P, Pc);
    double x = Pc[0], y = Pc[1], z = Pc[2];
    double invz = 1.0 / z, invz2 = invz * invz;
#ifdef PLBA_EXACT_DIV
    const double J[6] = {c.fx / z, 0, -c.fx * x * invz2, 0, c.fy / z, -c.fy * y * invz2};
#else
    const double J[6] = {c.fx * invz, 0, -c.fx * x * invz2, 0, c.fy * invz, -c.fy * y * invz2};
#endif
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            Jl[r * 3 + k] = -(J[r * 3 + 0] * R[k] + J[r * 3 + 1] * R[3 + k] + J[r * 3 + 2] * R[6 + k]);
    double RP[3], S[9];
    mat3vec(R, P, RP);
    vechat(RP, S);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
        for (int k = 0; k < 3; ++k) Jp[r * 6 + k] = -J[r * 3 + k];
#pragma unroll
        for (int k = 0; k < 3; ++k)
            Jp[r * 6 + 3 + k] = -(J[r * 3 + 0] * (-S[k]) + J[r * 3 + 1] * (-S[3 + k]) + J[r * 3 + 2] * (-S[6 + k]));
    }
}

// ---------------- EdgePoseLine ----------------
// l = K_L * (R n + [t]x R d)
PLBA_HD void line_image(const double *T, const double *L, const Cam &c, double *l) {
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    const double t[3] = {T[3], T[7], T[11]};
    double Rn[3], Rd[3], S[9], tRd[3];
    mat3vec(R, L, Rn);
    mat3vec(R, L + 3, Rd);
    vechat(t, S);
    mat3vec(S, Rd, tRd);
    double nc0 = Rn[0] + tRd[0], nc1 = Rn[1] + tRd[1], nc2 = Rn[2] + tRd[2];
    l[0] = c.fy * nc0;
    l[1] = c.fx * nc1;
    l[2] = (-c.fy * c.cx) * nc0 + (-c.fx * c.cy) * nc1 + (c.fx * c.fy) * nc2;
}
PLBA_HD void line_error(const double *T, const double *L, const double *obs, const Cam &c, double *e) {
    double l[3];
    line_image(T, L, c, l);
    double f = sqrt(l[0] * l[0] + l[1] * l[1]);
#ifdef PLBA_EXACT_DIV
    e[0] = (l[0] * obs[0] + l[1] * obs[1] + l[2]) / f;
    e[1] = (l[0] * obs[2] + l[1] * obs[3] + l[2]) / f;
#else
    const double invf = 1.0 / f;
    e[0] = (l[0] * obs[0] + l[1] * obs[1] + l[2]) * invf;
    e[1] = (l[0] * obs[2] + l[1] * obs[3] + l[2]) * invf;
#endif
}
// Jl: 2x4 (row-major), Jp: 2x6 ; also returns the error
PLBA_HD void line_jac(const double *T, const double *orth, const double *L, const double *obs, const Cam &c,
                      int corrected, double *e, double *Jl, double *Jp) {
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    const double t[3] = {T[3], T[7], T[11]};
    double l[3];
    line_image(T, L, c, l);
    double lx = l[0], ly = l[1], lz = l[2];
    double f = sqrt(lx * lx + ly * ly);
#ifdef PLBA_EXACT_DIV
    double e0 = (lx * obs[0] + ly * obs[1] + lz) / f;
    double e1 = (lx * obs[2] + ly * obs[3] + lz) / f;
    e[0] = e0;
    e[1] = e1;
    const double j[2][3] = {{-lx * e0 / (f * f) + obs[0] / f, -ly * e0 / (f * f) + obs[1] / f, 1.0 / f},
                            {-lx * e1 / (f * f) + obs[2] / f, -ly * e1 / (f * f) + obs[3] / f, 1.0 / f}};
#else
    // one reciprocal per distinct denominator (an IEEE division is a ~10-instruction dependent
    // chain, and this edge type is the linearisation's longest wave): within ~1 ulp of a / b
    const double invf = 1.0 / f, invf2 = invf * invf;
    double e0 = (lx * obs[0] + ly * obs[1] + lz) * invf;
    double e1 = (lx * obs[2] + ly * obs[3] + lz) * invf;
    e[0] = e0;
    e[1] = e1;
    const double j[2][3] = {{-lx * e0 * invf2 + obs[0] * invf, -ly * e0 * invf2 + obs[1] * invf, invf},
                            {-lx * e1 * invf2 + obs[2] * invf, -ly * e1 * invf2 + obs[3] * invf, invf}};
#endif
    const double K[9] = {c.fy, 0, 0, 0, c.fx, 0, -c.fy * c.cx, -c.fx * c.cy, c.fx * c.fy};
    double jK[2][3];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) jK[r][k] = j[r][0] * K[k] + j[r][1] * K[3 + k] + j[r][2] * K[6 + k];
    double a[3], b[3];
    if (!corrected) {  // Lw.tail(3) / Lw.head(3) of the 4-vector orth estimate (g2o_types.h:429-430)
        a[0] = orth[1]; a[1] = orth[2]; a[2] = orth[3];
        b[0] = orth[0]; b[1] = orth[1]; b[2] = orth[2];
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
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            Jp[r * 6 + k] = jK[r][0] * (-Sa[k]) + jK[r][1] * (-Sa[3 + k]) + jK[r][2] * (-Sa[6 + k]);
            Jp[r * 6 + 3 + k] = jK[r][0] * (-Sb[k] - StSa[k]) + jK[r][1] * (-Sb[3 + k] - StSa[3 + k]) +
                                jK[r][2] * (-Sb[6 + k] - StSa[6 + k]);
        }
    // U, W recomputed from the Plücker vector (getOrhtRFromPluker / getOrthWFromPluker)
    double nn = sqrt(L[0] * L[0] + L[1] * L[1] + L[2] * L[2]);
    double dn = sqrt(L[3] * L[3] + L[4] * L[4] + L[5] * L[5]);
    double cr[3] = {L[1] * L[5] - L[2] * L[4], L[2] * L[3] - L[0] * L[5], L[0] * L[4] - L[1] * L[3]};
    double cn = sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
    double fw = sqrt(nn * nn + dn * dn);
    double u1[3], u2[3], u3[3];
#ifdef PLBA_EXACT_DIV
    double w1 = nn / fw, w2 = dn / fw;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        u1[i] = L[i] / nn;
        u2[i] = L[3 + i] / dn;
        u3[i] = cr[i] / cn;
    }
#else
    const double ifw = 1.0 / fw, inn = 1.0 / nn, idn = 1.0 / dn, icn = 1.0 / cn;
    double w1 = nn * ifw, w2 = dn * ifw;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        u1[i] = L[i] * inn;
        u2[i] = L[3 + i] * idn;
        u3[i] = cr[i] * icn;
    }
#endif
    double StR[9];
    mat3mul(St, R, StR);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        double v[6];  // jK * [R | [t]x R]
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v[k] = jK[r][0] * R[k] + jK[r][1] * R[3 + k] + jK[r][2] * R[6 + k];
            v[3 + k] = jK[r][0] * StR[k] + jK[r][1] * StR[3 + k] + jK[r][2] * StR[6 + k];
        }
        // jacobianFromPlukerToOrth columns
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            s0 += v[3 + i] * (w2 * u3[i]);
            s1 += v[i] * (-w1 * u3[i]);
            s2 += v[i] * (w1 * u2[i]) + v[3 + i] * (-w2 * u1[i]);
            s3 += v[i] * (-w2 * u1[i]) + v[3 + i] * (w1 * u2[i]);
        }
        Jl[r * 4 + 0] = s0;
        Jl[r * 4 + 1] = s1;
        Jl[r * 4 + 2] = s2;
        Jl[r * 4 + 3] = s3;
    }
}

// ================= hand-rolled LM (MapHandler::levMarquardtOptimizationLBAForPluker) =========
// se(3) maps of src2/auxiliar.cpp:113-173 on row-major 4x4 (x = [t; ω]). No FMA contraction:
// logmap_se3 divides by sin θ, so near θ = π a fused multiply-add in 1 − cos²θ or in R = I + s·sinθ
// + s²(1 − cosθ) moves X_i by ~1e-10 per step relative to the unfused reference arithmetic.
// unfused 3x3 helpers for the se(3) maps below (an inlined callee keeps its own contraction
// setting, so mat3mul / mat3vec would still fuse inside a contract(off) caller)
PLBA_HD void m3mul_nc(const double *A, const double *B, double *C) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3 + 0] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
PLBA_HD void m3vec_nc(const double *R, const double *v, double *r) {
#pragma clang fp contract(off)
    r[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    r[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    r[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
}
PLBA_HD void se3_exp(const double *x, double *T) {  // expmap_se3 (:124-141)
#pragma clang fp contract(off)
    const double w0 = x[3], w1 = x[4], w2 = x[5];
    double t0 = x[0], t1 = x[1], t2 = x[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(theta < 0.000001)) {
        const double w[3] = {w0, w1, w2};
        double s[9], ss[9];
        vechat(w, s);
#pragma unroll
        for (int i = 0; i < 9; ++i) s[i] /= theta;
        m3mul_nc(s, s, ss);
        const double st = sin(theta), ct = 1.0 - cos(theta);
        double V[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            R[i] = (I + s[i] * st) + ss[i] * ct;
            V[i] = (I + s[i] * ct / theta) + ss[i] * (theta - st) / theta;
        }
        const double tv[3] = {t0, t1, t2};
        double r[3];
        m3vec_nc(V, tv, r);
        t0 = r[0]; t1 = r[1]; t2 = r[2];
    }
    T[0] = R[0]; T[1] = R[1]; T[2] = R[2];  T[3] = t0;
    T[4] = R[3]; T[5] = R[4]; T[6] = R[5];  T[7] = t1;
    T[8] = R[6]; T[9] = R[7]; T[10] = R[8]; T[11] = t2;
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}
PLBA_HD void inv3_cof(const double *m, double *r) {  // Eigen's closed-form 3x3 inverse
#pragma clang fp contract(off)
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[5] * m[6] - m[3] * m[8];
    const double c2 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c0 + m[1] * c1 + m[2] * c2;
    r[0] = c0 / det; r[3] = c1 / det; r[6] = c2 / det;
    r[1] = (m[2] * m[7] - m[1] * m[8]) / det;
    r[4] = (m[0] * m[8] - m[2] * m[6]) / det;
    r[7] = (m[1] * m[6] - m[0] * m[7]) / det;
    r[2] = (m[1] * m[5] - m[2] * m[4]) / det;
    r[5] = (m[2] * m[3] - m[0] * m[5]) / det;
    r[8] = (m[0] * m[4] - m[1] * m[3]) / det;
}
PLBA_HD void se3_log(const double *T, double *x) {  // logmap_se3 (:143-173)
#pragma clang fp contract(off)
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    const double Vt[3] = {T[3], T[7], T[11]};
    double w[3] = {0, 0, 0};
    double V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double cosine = (R[0] + R[4] + R[8] - 1.0) / 2.0;
    if (cosine > 1.0) cosine = 1.0;
    else if (cosine < -1.0) cosine = -1.0;
    double sine = sqrt(1.0 - cosine * cosine);
    if (sine > 1.0) sine = 1.0;
    else if (sine < -1.0) sine = -1.0;
    const double theta = acos(cosine);
    if (theta > 0.000001) {
        w[0] = theta * (R[7] - R[5]) / (2.0 * sine);
        w[1] = theta * (R[2] - R[6]) / (2.0 * sine);
        w[2] = theta * (R[3] - R[1]) / (2.0 * sine);
        double s[9], ss[9];
        vechat(w, s);
#pragma unroll
        for (int i = 0; i < 9; ++i) s[i] /= theta;
        m3mul_nc(s, s, ss);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            V[i] = (I + s[i] * (1.0 - cosine) / theta) + ss[i] * (theta - sine) / theta;
        }
    }
    double Vi[9], t[3];
    inv3_cof(V, Vi);
    m3vec_nc(Vi, Vt, t);
    x[0] = t[0]; x[1] = t[1]; x[2] = t[2];
    x[3] = w[0]; x[4] = w[1]; x[5] = w[2];
}
// inverse_se3 (:113-122) of a row-major 4x4 into a row-major 3x4 [Rᵀ | −Rᵀt]
PLBA_HD void se3_inv34(const double *T, double *Ti) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) Ti[i * 4 + j] = T[j * 4 + i];
        Ti[i * 4 + 3] = -(T[0 * 4 + i] * T[3] + T[1 * 4 + i] * T[7] + T[2 * 4 + i] * T[11]);
    }
}
// X_i <- logmap_se3(expmap_se3(X_i) · inverse_se3(expmap_se3(DX_i)))  (src/mapHandler.cpp:1868-1873),
// and the Tiw = inverse_se3(expmap_se3(X_i)) the next linearisation reads (:1922-1927)
PLBA_HD void hlm_pose_update(const double *x, const double *dx, double *xn, double *Tcw) {
#pragma clang fp contract(off)
    double Tp[16], E[16], Ei[12], Tc[16];
    se3_exp(x, Tp);
    se3_exp(dx, E);
    se3_inv34(E, Ei);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += Tp[i * 4 + k] * Ei[k * 4 + j];
            s += Tp[i * 4 + 3] * (j == 3 ? 1.0 : 0.0);
            Tc[i * 4 + j] = s;
        }
    se3_log(Tc, xn);
    double Tn[16];
    se3_exp(xn, Tn);
    se3_inv34(Tn, Tcw);
}

// One point observation as the hand-rolled LM forms it (src/mapHandler.cpp:1655-1698): r = ‖e‖,
// Cauchy weight w (src2/auxiliar.cpp:556-559), the pose row Jp and the landmark row Jl.
PLBA_HD void hlm_point(const double *T, const double *X, const double *obs, const Cam &c, double hth, double &r,
                       double &w, double *Jp, double *Jl) {
    double P[3];
    point_pc(T, X, P);
    const double u = c.cx + c.fx * P[0] / P[2], v = c.cy + c.fy * P[1] / P[2];  // cam->projection
    const double dx = obs[0] - u, dy = obs[1] - v;
    r = sqrt(dx * dx + dy * dy);
    const double gx = P[0], gy = P[1], gz = P[2];
    const double gz2 = 1.0 / fmax(hth, gz * gz);
    const double fxdx = c.fx * dx, fydy = c.fy * dy;
    const double m = fmax(hth, r);
    Jp[0] = (gz2 * fxdx * gz) / m;
    Jp[1] = (gz2 * fydy * gz) / m;
    Jp[2] = (-gz2 * (fxdx * gx + fydy * gy)) / m;
    Jp[3] = (-gz2 * (fxdx * gx * gy + fydy * gy * gy + fydy * gz * gz)) / m;
    Jp[4] = (gz2 * (fxdx * gx * gx + fxdx * gz * gz + fydy * gx * gy)) / m;
    Jp[5] = (gz2 * (fydy * gx * gz - fxdx * gy * gz)) / m;
    const double j0 = gz2 * fxdx * gz, j1 = gz2 * fydy * gz, j2 = -gz2 * (fxdx * gx + fydy * gy);
    Jl[0] = (j0 * T[0] + j1 * T[4] + j2 * T[8]) / m;  // Jᵀ · R
    Jl[1] = (j0 * T[1] + j1 * T[5] + j2 * T[9]) / m;
    Jl[2] = (j0 * T[2] + j1 * T[6] + j2 * T[10]) / m;
    Jl[3] = 0.0;
    w = 1.0 / (1.0 + r * r);
}

// One line observation (src/mapHandler.cpp:1744-1811): NDc = TransformForPluker(Tiw, NDw),
// l = plukerK·NDc.head(3), the pose row from fai_e·[K 0]·fai_lineCurr_RT and the landmark row
// from fai_e·[K 0]·getTransformMatrixForPluker(Tiw)·jacobianFromPlukerToOrth(Rw, Ww)
// (src/mapFeatures.cpp:251-266), both combined as (jac0·e0 + jac1·e1)/max(homogTh, r).
PLBA_HD void hlm_line(const double *T, const double *L, const double *obs, const Cam &c, double hth, double &r,
                      double &w, double *Jp, double *Jl) {
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    const double t[3] = {T[3], T[7], T[11]};
    const double nn = sqrt(L[0] * L[0] + L[1] * L[1] + L[2] * L[2]);
    const double dn = sqrt(L[3] * L[3] + L[4] * L[4] + L[5] * L[5]);
    const double cr[3] = {L[1] * L[5] - L[2] * L[4], L[2] * L[3] - L[0] * L[5], L[0] * L[4] - L[1] * L[3]};
    const double cn = sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
    const double fw = sqrt(nn * nn + dn * dn), w1 = nn / fw, w2 = dn / fw;
    double u1[3], u2[3], u3[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        u1[i] = L[i] / nn;
        u2[i] = L[3 + i] / dn;
        u3[i] = cr[i] / cn;
    }
    double St[9], StR[9], Rn[3], Rd[3], tRd[3];
    vechat(t, St);
    mat3mul(St, R, StR);
    mat3vec(R, L, Rn);
    mat3vec(R, L + 3, Rd);
    mat3vec(StR, L + 3, tRd);
    const double nc[3] = {Rn[0] + tRd[0], Rn[1] + tRd[1], Rn[2] + tRd[2]};
    const double K[9] = {c.fy, 0, 0, 0, c.fx, 0, -c.fy * c.cx, -c.fx * c.cy, c.fx * c.fy};
    double l[3];
    mat3vec(K, nc, l);
    const double lx = l[0], ly = l[1], lz = l[2];
    const double fenmu = sqrt(lx * lx + ly * ly);
    const double e[2] = {(obs[0] * lx + obs[1] * ly + lz) / fenmu, (obs[2] * lx + obs[3] * ly + lz) / fenmu};
    r = sqrt(e[0] * e[0] + e[1] * e[1]);
    double SRd[9], SRn[9], StSRd[9];
    vechat(Rd, SRd);
    vechat(Rn, SRn);
    mat3mul(St, SRd, StSRd);
    double jp[2][6], jl[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double a = obs[2 * k], b = obs[2 * k + 1];
        const double fe[3] = {a * fenmu - lx * e[k] * fenmu * fenmu, b * fenmu - ly * e[k] * fenmu * fenmu, fenmu};
        double v[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) v[j] = fe[0] * K[j] + fe[1] * K[3 + j] + fe[2] * K[6 + j];
        double q[6];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            jp[k][j] = v[0] * (-SRd[j]) + v[1] * (-SRd[3 + j]) + v[2] * (-SRd[6 + j]);
            jp[k][3 + j] = v[0] * (-SRn[j] - StSRd[j]) + v[1] * (-SRn[3 + j] - StSRd[3 + j]) +
                           v[2] * (-SRn[6 + j] - StSRd[6 + j]);
            q[j] = v[0] * R[j] + v[1] * R[3 + j] + v[2] * R[6 + j];
            q[3 + j] = v[0] * StR[j] + v[1] * StR[3 + j] + v[2] * StR[6 + j];
        }
        // q · jacobianFromPlukerToOrth (rows 0-2: n part, rows 3-5: d part)
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            s0 += q[3 + i] * (w2 * u3[i]);
            s1 += q[i] * (-w1 * u3[i]);
            s2 += q[i] * (-w1 * u2[i]) + q[3 + i] * (-w2 * u1[i]);
            s3 += q[i] * (-w2 * u1[i]) + q[3 + i] * (w1 * u2[i]);
        }
        jl[k][0] = s0; jl[k][1] = s1; jl[k][2] = s2; jl[k][3] = s3;
    }
    const double m = fmax(hth, r);
#pragma unroll
    for (int j = 0; j < 6; ++j) Jp[j] = (jp[0][j] * e[0] + jp[1][j] * e[1]) / m;
#pragma unroll
    for (int j = 0; j < 4; ++j) Jl[j] = (jl[0][j] * e[0] + jl[1][j] * e[1]) / m;
    w = 1.0 / (1.0 + r * r);
}

// One GBA line observation (MapHandler::levMarquardtOptimizationGBA, src/mapHandler.cpp:3270-3340 /
// :3545-3619): endpoints P, Q in the world, image line lo = (a, b, c); e = (lo·π(P), lo·π(Q));
// the rows use fx·e0 / fy·e1 (lx = l_err(0), ly = l_err(1), :3293-3296); Jl = [J_P·e0; J_Q·e1]/m.
PLBA_HD void gba_line(const double *T, const double *P, const double *Q, const double *lo, const Cam &c, double hth,
                      double &r, double &w, double *Jp, double *Jl) {
    double Pi[3], Qi[3];
    point_pc(T, P, Pi);
    point_pc(T, Q, Qi);
    const double pu = c.cx + c.fx * Pi[0] / Pi[2], pv = c.cy + c.fy * Pi[1] / Pi[2];
    const double qu = c.cx + c.fx * Qi[0] / Qi[2], qv = c.cy + c.fy * Qi[1] / Qi[2];
    const double e0 = lo[0] * pu + lo[1] * pv + lo[2];
    const double e1 = lo[0] * qu + lo[1] * qv + lo[2];
    r = sqrt(e0 * e0 + e1 * e1);
    const double fxlx = c.fx * e0, fyly = c.fy * e1;
    const double m = fmax(hth, r);
    double JPi[6], JQi[6];
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        const double *G = side ? Qi : Pi;
        double *Jpose = side ? JQi : JPi;
        const double ek = side ? e1 : e0;
        const double gx = G[0], gy = G[1], gz = G[2];
        const double gz2 = 1.0 / fmax(hth, gz * gz);
        Jpose[0] = gz2 * fxlx * gz;
        Jpose[1] = gz2 * fyly * gz;
        Jpose[2] = -gz2 * (fxlx * gx + fyly * gy);
        Jpose[3] = -gz2 * (fxlx * gx * gy + fyly * gy * gy + fyly * gz * gz);
        Jpose[4] = gz2 * (fxlx * gx * gx + fxlx * gz * gz + fyly * gx * gy);
        Jpose[5] = gz2 * (fyly * gx * gz - fxlx * gy * gz);
        const double j0 = gz2 * fxlx * gz, j1 = gz2 * fyly * gz, j2 = -gz2 * (fxlx * gx + fyly * gy);
        Jl[3 * side + 0] = ((j0 * T[0] + j1 * T[4] + j2 * T[8]) * ek) / m;
        Jl[3 * side + 1] = ((j0 * T[1] + j1 * T[5] + j2 * T[9]) * ek) / m;
        Jl[3 * side + 2] = ((j0 * T[2] + j1 * T[6] + j2 * T[10]) * ek) / m;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) Jp[k] = (JPi[k] * e0 + JQi[k] * e1) / m;
    w = 1.0 / (1.0 + r * r);
}

}  // namespace plba
