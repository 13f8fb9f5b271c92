// Loop-closure pose graph on the device (plba_pgo_optimize):
// MapHandler::loopClosureOptimization{EssGraph,CovGraph}G2O (src/mapHandler.cpp:5070-5531) =
// g2o VertexSE3 / EdgeSE3 + OptimizationAlgorithmLevenberg + BlockSolver_6_3 / Cholmod.
//
//   k_pgo_linearize  one thread per active edge: e = toVectorMQT(Z⁻¹·X_i⁻¹·X_j), χ² = eᵀΩe and,
//                    for a linearisation, the 6x6 products J_iᵀΩJ_i, J_jᵀΩJ_j, J_iᵀΩJ_j and
//                    -JᵀΩe of both vertices (per-edge records, no atomics)
//   k_pgo_assemble   one thread per entry of a 6x6 block of H (and of b on diagonal blocks):
//                    the block's edge contributions summed in edge order (host-built CSR) into
//                    the dense column-major lower triangle Hd — deterministic
//   k_pgo_damp       Ad = Hd + λI (g2o setLambda; the undamped Hd is kept: restoreDiagonal)
//   k_dense_panel / k_dense_update   the dense blocked LDLᵀ of plba_dense.hpp (MFMA updates)
//   k_pgo_check      LinearSolverCholmod fails on a non-positive pivot: solve_ok &= all D > 0
//   k_pgo_solve      forward / backward substitution (x keeps its value when the solve failed,
//                    as g2o's _x does)
//   k_pgo_update     trial state X ← X·fromVectorMQT(x_h) (VertexSE3::oplusImpl)
//   k_pgo_sum        χ² (and Σx(λx+b)) summed in edge (index) order by one thread
// The Levenberg decisions run on the host, one read-back per trial (a loop closure is rare;
// the dense factorisation dominates). The edge arithmetic is compiled without FMA contraction,
// like the oracle (oracle/refpgo.cpp), so the two agree to rounding in the solve.
#pragma once

struct PgoDev {
    int32_t nv, ne, nact, nfree, n, nblk;
    const int32_t *e_v;               // [ne][2] vertex positions
    const int32_t *act;               // [nact] active edges, creation order
    const double *Zinv, *info;        // [ne][12] inverse measurement, [ne][36] Ω
    const int32_t *hidx;              // [nv] Hessian block of each vertex (-1: fixed / inactive)
    double *T[2];                     // [nv][12] Isometry3 row-major 3x4: current / trial
    double *eH;                       // [ne][144] J_iᵀΩJ_i | J_jᵀΩJ_j | J_iᵀΩJ_j | J_jᵀΩJ_i (row-major)
    double *eg;                       // [ne][12] -J_iᵀΩe | -J_jᵀΩe
    double *echi;                     // [ne] χ² of each edge at the evaluated state
    const int32_t *blk_r, *blk_c;     // [nblk] block row >= block col (Hessian indices)
    const int32_t *blk_off, *blk_con; // [nblk+1] CSR, contributions (edge << 2 | kind)
    double *Hd;                       // [n][n] column-major lower triangle of H (undamped)
    double *b, *x;                    // [n]
    double *out;                      // [4]: χ² current | χ² trial | scale | solve_ok
};

namespace pgo {
#pragma clang fp contract(off)
struct Iso {
    double R[9], t[3];
};
__device__ __forceinline__ Iso load(const double *T) {
    Iso a;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) a.R[3 * r + c] = T[4 * r + c];
        a.t[r] = T[4 * r + 3];
    }
    return a;
}
__device__ __forceinline__ void store(const Iso &a, double *T) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) T[4 * r + c] = a.R[3 * r + c];
        T[4 * r + 3] = a.t[r];
    }
}
__device__ __forceinline__ Iso mul(const Iso &a, const Iso &b) {
#pragma clang fp contract(off)
    Iso o;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += a.R[3 * r + k] * b.R[3 * k + c];
            o.R[3 * r + c] = s;
        }
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s += a.R[3 * r + k] * b.t[k];
        o.t[r] = s + a.t[r];
    }
    return o;
}
__device__ __forceinline__ Iso inv(const Iso &a) {
#pragma clang fp contract(off)
    Iso o;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) o.R[3 * r + c] = a.R[3 * c + r];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s += o.R[3 * r + k] * a.t[k];
        o.t[r] = -s;
    }
    return o;
}
struct Quat {
    double w, x, y, z;
};
// Eigen Quaternion(Matrix3) (quaternionbase_assign_impl)
__device__ __forceinline__ Quat quat_from_R(const double *m) {
#pragma clang fp contract(off)
    Quat q;
    double t = m[0] + m[4] + m[8];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
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
        t = sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        double v[3];
        v[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[3 * k + j] - m[3 * j + k]) * t;
        v[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        v[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q.x = v[0];
        q.y = v[1];
        q.z = v[2];
    }
    return q;
}
__device__ __forceinline__ void R_from_quat(const Quat &q, double *R) {
#pragma clang fp contract(off)
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}
// g2o internal::normalize: q.normalize(); w >= 0
__device__ __forceinline__ Quat qnormalize(Quat q) {
#pragma clang fp contract(off)
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    if (n > 0.0) { q.w /= n; q.x /= n; q.y /= n; q.z /= n; }
    if (q.w < 0.0) { q.w = -q.w; q.x = -q.x; q.y = -q.y; q.z = -q.z; }
    return q;
}
// internal::fromVectorMQT
__device__ __forceinline__ Iso from_mqt(const double *v) {
#pragma clang fp contract(off)
    Iso a;
    const double w = 1.0 - (v[3] * v[3] + v[4] * v[4] + v[5] * v[5]);
    if (w < 0.0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) a.R[k] = (k % 4 == 0) ? 1.0 : 0.0;
    } else {
        R_from_quat(Quat{sqrt(w), v[3], v[4], v[5]}, a.R);
    }
    a.t[0] = v[0]; a.t[1] = v[1]; a.t[2] = v[2];
    return a;
}
__device__ __forceinline__ void skew(const double *v, double *S) {
    S[0] = 0.0;   S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2];  S[4] = 0.0;   S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0];  S[8] = 0.0;
}
// EdgeSE3::computeError and the derivative EdgeSE3::linearizeOplus evaluates (see
// oracle/refpgo.cpp edge_jacobians for the closed form)
template <bool JAC>
__device__ __forceinline__ void edge(const Iso &Zinv, const Iso &Xi, const Iso &Xj, double *e, double *Ji,
                                     double *Jj) {
#pragma clang fp contract(off)
    const Iso Xii = inv(Xi);
    {   // _inverseMeasurement * from⁻¹ * to, evaluated left to right
        const Iso D = mul(mul(Zinv, Xii), Xj);
        const Quat qd = qnormalize(quat_from_R(D.R));
        e[0] = D.t[0]; e[1] = D.t[1]; e[2] = D.t[2];
        e[3] = qd.x; e[4] = qd.y; e[5] = qd.z;
    }
    if (!JAC) return;
    const Iso B = mul(Xii, Xj);
    const Iso E0 = mul(Zinv, B);
    const Quat q0 = qnormalize(quat_from_R(E0.R));
    const Quat qa = quat_from_R(Zinv.R), qb = quat_from_R(B.R);
    const double sgn = (qa.w * qb.w - (qa.x * qb.x + qa.y * qb.y + qa.z * qb.z)) < 0.0 ? -1.0 : 1.0;
#pragma unroll
    for (int k = 0; k < 36; ++k) Ji[k] = Jj[k] = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) Jj[6 * r + c] = E0.R[3 * r + c];
    {
        const double v0[3] = {q0.x, q0.y, q0.z};
        double S[9];
        skew(v0, S);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) Jj[6 * (3 + r) + 3 + c] = (r == c ? q0.w : 0.0) + S[3 * r + c];
    }
    double Sb[9];
    skew(B.t, Sb);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            Ji[6 * r + c] = -Zinv.R[3 * r + c];
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += Zinv.R[3 * r + k] * Sb[3 * k + c];
            Ji[6 * r + 3 + c] = 2.0 * s;
        }
    const double av[3] = {qa.x, qa.y, qa.z}, bv[3] = {qb.x, qb.y, qb.z};
    double Sa[9], Sq[9];
    skew(av, Sa);
    skew(bv, Sq);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double SaSb = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) SaSb += Sa[3 * r + k] * Sq[3 * k + c];
            const double m = (r == c ? qa.w * qb.w : 0.0) - qa.w * Sq[3 * r + c] - av[r] * bv[c] + qb.w * Sa[3 * r + c] - SaSb;
            Ji[6 * (3 + r) + 3 + c] = -sgn * m;
        }
}
}  // namespace pgo

constexpr int kPgoNT = 64;

// χ² of every active edge at state T[s]; with LIN also the per-edge normal-equation records
template <bool LIN>
__global__ __launch_bounds__(kPgoNT) void k_pgo_linearize(PgoDev p, int s) {
#pragma clang fp contract(off)
    const int a = blockIdx.x * kPgoNT + threadIdx.x;
    if (a >= p.nact) return;
    const int e = p.act[a], vi = p.e_v[2 * e], vj = p.e_v[2 * e + 1];
    const pgo::Iso Zinv = pgo::load(p.Zinv + (size_t)e * 12);
    const pgo::Iso Xi = pgo::load(p.T[s] + (size_t)vi * 12), Xj = pgo::load(p.T[s] + (size_t)vj * 12);
    double r[6], J[2][36];
    pgo::edge<LIN>(Zinv, Xi, Xj, r, J[0], J[1]);
    const double *O = p.info + (size_t)e * 36;
    double Or[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) t += O[6 * q + k] * r[k];
        Or[q] = t;
    }
    {   // χ² = eᵀΩe summed as the oracle does: Σ_a e_a·(Σ_b Ω_ab e_b)
        double c = 0.0;
#pragma unroll
        for (int q = 0; q < 6; ++q) c += r[q] * Or[q];
        p.echi[e] = c;
    }
    if (!LIN) return;
    double OJ[2][36];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 6; ++k) t += O[6 * q + k] * J[sd][6 * k + c];
                OJ[sd][6 * q + c] = t;
            }
    double *H = p.eH + (size_t)e * 144;
    const int pr[4][2] = {{0, 0}, {1, 1}, {0, 1}, {1, 0}};
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                double t = 0.0;
#pragma unroll
                for (int k = 0; k < 6; ++k) t += J[pr[m][0]][6 * k + q] * OJ[pr[m][1]][6 * k + c];
                H[36 * m + 6 * q + c] = t;
            }
#pragma unroll
    for (int sd = 0; sd < 2; ++sd)
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 6; ++k) t += J[sd][6 * k + q] * Or[k];
            p.eg[(size_t)e * 12 + 6 * sd + q] = -t;
        }
}

// one thread per (block, entry): entries 0..35 of the 6x6 block, 36..41 the b rows (diagonal
// blocks). Contributions in edge order: kind 0 J_iᵀΩJ_i (+ b_i), 1 J_jᵀΩJ_j (+ b_j), 2 J_iᵀΩJ_j
// (block row = vertex i), 3 J_jᵀΩJ_i (block row = vertex j)
__global__ __launch_bounds__(kPgoNT) void k_pgo_assemble(PgoDev p) {
#pragma clang fp contract(off)
    const int t = blockIdx.x * kPgoNT + threadIdx.x;
    if (t >= p.nblk * 42) return;
    const int bk = t / 42, en = t % 42;
    const int br = p.blk_r[bk], bc = p.blk_c[bk];
    if (en >= 36 && br != bc) return;
    const int r = en / 6, c = en % 6;
    double s = 0.0;
    for (int q = p.blk_off[bk]; q < p.blk_off[bk + 1]; ++q) {
        const int con = p.blk_con[q], e = con >> 2, kind = con & 3;
        if (en >= 36) {
            s -= -p.eg[(size_t)e * 12 + 6 * kind + (en - 36)];  // b -= JᵀΩe, stored as -JᵀΩe
        } else {
            s += p.eH[(size_t)e * 144 + 36 * kind + 6 * r + c];
        }
    }
    if (en >= 36) p.b[6 * br + (en - 36)] = s;
    else {
        const int row = 6 * br + r, col = 6 * bc + c;
        if (row >= col) p.Hd[(size_t)row + (size_t)col * p.n] = s;
    }
}

// Ad = Hd + λ·I (lower triangle; the strict upper part is never read)
__global__ __launch_bounds__(256) void k_pgo_damp(PgoDev p, double *Ad, double lambda) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, nn = (size_t)p.n * p.n;
    if (i >= nn) return;
    const size_t row = i % p.n, col = i / p.n;
    Ad[i] = p.Hd[i] + (row == col ? lambda : 0.0);
}

// LinearSolverCholmod: not positive definite -> the solve fails
__global__ __launch_bounds__(256) void k_pgo_check(Dev d) {
    __shared__ int s_bad;
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    int bad = 0;
    for (int i = threadIdx.x; i < d.n; i += 256) {
        const double D = d.Ad[(size_t)i + (size_t)i * d.n];
        if (!(D > 0.0)) bad = 1;
    }
    if (bad) s_bad = 1;  // (benign race: every writer stores 1)
    __syncthreads();
    if (threadIdx.x == 0 && s_bad) d.ctrl->solve_ok[0] = 0;
}

__global__ __launch_bounds__(kFacThreads) void k_pgo_solve(Dev d) {
    if (!d.ctrl->solve_ok[0]) return;  // x keeps its previous value (g2o's _x)
    if (d.n <= d.solve_lds_n) dense_solve_wg<true, true>(d);  // forward part done in the factorisation
    else dense_solve_wg<false, true>(d);
}

// trial state: X ← X·fromVectorMQT(x_h) for the Hessian vertices, copy for the others
__global__ __launch_bounds__(kPgoNT) void k_pgo_update(PgoDev p, int cur) {
#pragma clang fp contract(off)
    const int v = blockIdx.x * kPgoNT + threadIdx.x;
    if (v >= p.nv) return;
    const double *src = p.T[cur] + (size_t)v * 12;
    double *dst = p.T[cur ^ 1] + (size_t)v * 12;
    const int h = p.hidx[v];
    if (h < 0) {
#pragma unroll
        for (int k = 0; k < 12; ++k) dst[k] = src[k];
        return;
    }
    pgo::store(pgo::mul(pgo::load(src), pgo::from_mqt(p.x + 6 * (size_t)h)), dst);
}

// out[slot] = Σ χ² over the active edges in edge order; slot 1 also the Levenberg scale
// Σ_k x_k (λ x_k + b_k) and the solve flag
__global__ void k_pgo_sum(PgoDev p, const Ctrl *ctrl, int slot, double lambda) {
#pragma clang fp contract(off)
    if (threadIdx.x != 0) return;
    double c = 0.0;
    for (int a = 0; a < p.nact; ++a) c += p.echi[p.act[a]];
    p.out[slot] = c;
    if (slot == 1) {
        double s = 0.0;
        for (int k = 0; k < p.n; ++k) s += p.x[k] * (lambda * p.x[k] + p.b[k]);
        p.out[2] = s;
        p.out[3] = ctrl->solve_ok[0] ? 1.0 : 0.0;
    }
}

// max |H_ii| (computeLambdaInit without a user λ)
__global__ void k_pgo_maxdiag(PgoDev p) {
    if (threadIdx.x != 0) return;
    double m = 0.0;
    for (int k = 0; k < p.n; ++k) m = fmax(m, fabs(p.Hd[(size_t)k + (size_t)k * p.n]));
    p.out[2] = m;
}
