// refpgo.cpp — TEST INFRASTRUCTURE ONLY (see refpgo.h): CPU restatement of the g2o pose-graph
// optimisation of MapHandler::loopClosureOptimization{EssGraph,CovGraph}G2O
// (src/mapHandler.cpp:5070-5531). Built -ffp-contract=off with refcpu.cpp / refhlm.cpp.
#include "refpgo.h"

#include <chrono>
#include <cmath>
#include <algorithm>
#include <cstring>
#include <limits>
#include <map>
#include <vector>

namespace {

struct Iso {  // Eigen::Isometry3d: R row-major, t
    double R[9];
    double t[3];
};
Iso iso_load(const double *T) {
    Iso a;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) a.R[3 * r + c] = T[4 * r + c];
        a.t[r] = T[4 * r + 3];
    }
    return a;
}
void iso_store(const Iso &a, double *T) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = a.R[3 * r + c];
        T[4 * r + 3] = a.t[r];
    }
}
// Transform<Isometry> * Transform<Isometry>: linear = A.linear * B.linear, t = A.linear * B.t + A.t
Iso iso_mul(const Iso &a, const Iso &b) {
    Iso o;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += a.R[3 * r + k] * b.R[3 * k + c];
            o.R[3 * r + c] = s;
        }
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += a.R[3 * r + k] * b.t[k];
        o.t[r] = s + a.t[r];
    }
    return o;
}
// Isometry3::inverse(): [Rᵀ | -Rᵀt]
Iso iso_inv(const Iso &a) {
    Iso o;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) o.R[3 * r + c] = a.R[3 * c + r];
    for (int r = 0; r < 3; ++r) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += o.R[3 * r + k] * a.t[k];
        o.t[r] = -s;
    }
    return o;
}

struct Quat {  // (w, x, y, z)
    double w, x, y, z;
};
// Eigen quaternionbase_assign_impl<Matrix3>: Quaternion(R)
Quat quat_from_R(const double *m) {
    auto M = [&](int i, int j) { return m[3 * i + j]; };
    Quat q;
    double t = M(0, 0) + M(1, 1) + M(2, 2);
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (M(2, 1) - M(1, 2)) * t;
        q.y = (M(0, 2) - M(2, 0)) * t;
        q.z = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        double v[3];
        v[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (M(k, j) - M(j, k)) * t;
        v[j] = (M(j, i) + M(i, j)) * t;
        v[k] = (M(k, i) + M(i, k)) * t;
        q.x = v[0];
        q.y = v[1];
        q.z = v[2];
    }
    return q;
}
// QuaternionBase::toRotationMatrix
void R_from_quat(const Quat &q, double *R) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}
// g2o internal::normalize(Quaternion&): q.normalize(); if (q.w() < 0) q.coeffs() *= -1
Quat qnormalize(Quat q) {
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    if (n > 0.0) { q.w /= n; q.x /= n; q.y /= n; q.z /= n; }
    if (q.w < 0.0) { q.w = -q.w; q.x = -q.x; q.y = -q.y; q.z = -q.z; }
    return q;
}
// internal::toVectorMQT: [t; compact quaternion (x, y, z) of the normalised q, w >= 0]
void to_mqt(const Iso &a, double *v) {
    const Quat q = qnormalize(quat_from_R(a.R));
    v[0] = a.t[0]; v[1] = a.t[1]; v[2] = a.t[2];
    v[3] = q.x; v[4] = q.y; v[5] = q.z;
}
// internal::fromVectorMQT: R = fromCompactQuaternion(v[3..5]) (w = sqrt(1 - |v|²), identity if
// negative), t = v[0..2]
Iso from_mqt(const double *v) {
    Iso a;
    double w = 1.0 - (v[3] * v[3] + v[4] * v[4] + v[5] * v[5]);
    if (w < 0.0) {
        for (int k = 0; k < 9; ++k) a.R[k] = (k % 4 == 0) ? 1.0 : 0.0;
    } else {
        R_from_quat(Quat{std::sqrt(w), v[3], v[4], v[5]}, a.R);
    }
    a.t[0] = v[0]; a.t[1] = v[1]; a.t[2] = v[2];
    return a;
}

// EdgeSE3::computeError: delta = _inverseMeasurement * from^-1 * to; e = toVectorMQT(delta)
void edge_error(const Iso &Zinv, const Iso &Xi, const Iso &Xj, double *e) {
    to_mqt(iso_mul(iso_mul(Zinv, iso_inv(Xi)), Xj), e);
}

// de/dδ at δ = 0 for X_i <- X_i·Δ(δ_i), X_j <- X_j·Δ(δ_j) (EdgeSE3::linearizeOplus computes the
// same derivative with generated code, internal::computeEdgeSE3Gradient). With A = Z⁻¹,
// B = X_i⁻¹X_j, E0 = A·B, s = sign(w(q_a ⊗ q_b)), q0 = normalised quaternion of E0:
//   ∂t/∂t_j = R_E0        ∂c/∂v_j = w0·I + [q0v]×
//   ∂t/∂t_i = -R_a        ∂t/∂v_i = 2·R_a·[t_b]×
//   ∂c/∂v_i = -s·M,  M = q_aw q_bw I - q_aw [q_bv]× - q_av q_bvᵀ + q_bw [q_av]× - [q_av]×[q_bv]×
void skew(const double *v, double *S) {
    S[0] = 0.0;   S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2];  S[4] = 0.0;   S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0];  S[8] = 0.0;
}
void edge_jacobians(const Iso &Zinv, const Iso &Xi, const Iso &Xj, double *Ji, double *Jj) {
    const Iso B = iso_mul(iso_inv(Xi), Xj);
    const Iso E0 = iso_mul(Zinv, B);
    const Quat q0 = qnormalize(quat_from_R(E0.R));
    const Quat qa = quat_from_R(Zinv.R), qb = quat_from_R(B.R);
    const double sgn = (qa.w * qb.w - (qa.x * qb.x + qa.y * qb.y + qa.z * qb.z)) < 0.0 ? -1.0 : 1.0;
    for (int k = 0; k < 36; ++k) Ji[k] = Jj[k] = 0.0;
    // j
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Jj[6 * r + c] = E0.R[3 * r + c];
    {
        const double v0[3] = {q0.x, q0.y, q0.z};
        double S[9];
        skew(v0, S);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Jj[6 * (3 + r) + 3 + c] = (r == c ? q0.w : 0.0) + S[3 * r + c];
    }
    // i
    {
        double Sb[9];
        skew(B.t, Sb);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                Ji[6 * r + c] = -Zinv.R[3 * r + c];
                double s = 0.0;
                for (int k = 0; k < 3; ++k) s += Zinv.R[3 * r + k] * Sb[3 * k + c];
                Ji[6 * r + 3 + c] = 2.0 * s;
            }
        const double av[3] = {qa.x, qa.y, qa.z}, bv[3] = {qb.x, qb.y, qb.z};
        double Sa[9], Sbq[9];
        skew(av, Sa);
        skew(bv, Sbq);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double SaSb = 0.0;
                for (int k = 0; k < 3; ++k) SaSb += Sa[3 * r + k] * Sbq[3 * k + c];
                const double m = (r == c ? qa.w * qb.w : 0.0) - qa.w * Sbq[3 * r + c] - av[r] * bv[c] +
                                 qb.w * Sa[3 * r + c] - SaSb;
                Ji[6 * (3 + r) + 3 + c] = -sgn * m;
            }
    }
}

// ---------------------------------------------------------------- the optimiser
struct Graph {
    int nv = 0, ne = 0;
    std::vector<int> id;
    std::vector<Iso> X;
    std::vector<uint8_t> fixed;
    std::vector<int> ev;           // [ne][2]
    std::vector<Iso> Z, Zinv;
    std::vector<double> info;      // [ne][36]
    // SparseOptimizer::initializeOptimization(): active edges (not all vertices fixed) in creation
    // order; active vertices (>= 1 active edge) in id order; Hessian index for the free ones
    std::vector<int> active_e, hidx;
    int nfree = 0;
    std::vector<std::vector<int>> vedges;  // all edges of each vertex, creation order

    void load(const plba_pgo_graph *g) {
        nv = g->n_v;
        ne = g->n_e;
        id.assign(g->v_id, g->v_id + nv);
        X.resize(nv);
        fixed.assign(g->v_fixed, g->v_fixed + nv);
        for (int v = 0; v < nv; ++v) X[v] = iso_load(g->v_T + 12 * (size_t)v);
        ev.assign(g->e_v, g->e_v + 2 * (size_t)ne);
        Z.resize(ne);
        Zinv.resize(ne);
        info.assign(36 * (size_t)ne, 0.0);
        for (int e = 0; e < ne; ++e) {
            Z[e] = iso_load(g->e_Z + 12 * (size_t)e);
            Zinv[e] = iso_inv(Z[e]);  // EdgeSE3::setMeasurement stores the inverse too
            for (int k = 0; k < 36; ++k) info[36 * (size_t)e + k] = g->e_info ? g->e_info[36 * (size_t)e + k] : (k % 7 == 0 ? 1.0 : 0.0);
        }
        vedges.assign(nv, {});
        for (int e = 0; e < ne; ++e) {
            vedges[ev[2 * e]].push_back(e);
            vedges[ev[2 * e + 1]].push_back(e);
        }
        active_e.clear();
        std::vector<int> nact(nv, 0);
        for (int e = 0; e < ne; ++e)
            if (!(fixed[ev[2 * e]] && fixed[ev[2 * e + 1]])) {
                active_e.push_back(e);
                ++nact[ev[2 * e]];
                ++nact[ev[2 * e + 1]];
            }
        std::vector<int> order(nv);
        for (int v = 0; v < nv; ++v) order[v] = v;
        std::sort(order.begin(), order.end(), [&](int a, int b) { return id[a] < id[b]; });
        hidx.assign(nv, -1);
        nfree = 0;
        for (int v : order)
            if (nact[v] > 0 && !fixed[v]) hidx[v] = nfree++;
    }
    std::vector<uint8_t> is_active_edge() const {
        std::vector<uint8_t> a(ne, 0);
        for (int e : active_e) a[e] = 1;
        return a;
    }

    // SparseOptimizer::computeInitialGuess with EstimatePropagator (Dijkstra, unit edge cost
    // EdgeSE3::initialEstimatePossible = 1, active edges only). Roots: fixed vertices met while
    // walking the active edges (a std::set<Vertex*>: creation order here). The priority queue is
    // a multimap on distance: pops the smallest distance, FIFO among equal ones. A vertex takes
    // the estimate of the first edge that reached it with its final (smallest) distance, through
    // EdgeSE3::initialEstimate: to = from·Z, or from = to·Z⁻¹.
    void initial_guess() {
        const auto act = is_active_edge();
        std::vector<int> roots;
        std::vector<uint8_t> isroot(nv, 0);
        for (int e : active_e)
            for (int s = 0; s < 2; ++s) {
                const int v = ev[2 * e + s];
                if (fixed[v] && !isroot[v]) { isroot[v] = 1; roots.push_back(v); }
            }
        std::sort(roots.begin(), roots.end());  // pointer order = creation order
        const double inf = std::numeric_limits<double>::max();
        std::vector<double> dist(nv, inf);
        std::vector<int> level(nv, 0), pedge(nv, -1), parent(nv, -1);
        std::multimap<double, int> frontier;
        std::vector<std::multimap<double, int>::iterator> qit(nv);
        std::vector<uint8_t> inq(nv, 0);
        auto push = [&](int v) {
            if (inq[v]) frontier.erase(qit[v]);
            qit[v] = frontier.insert(frontier.upper_bound(dist[v]), {dist[v], v});
            inq[v] = 1;
        };
        for (int r : roots) { dist[r] = 0.0; level[r] = 0; push(r); }
        while (!frontier.empty()) {
            const auto it = frontier.begin();
            const int u = it->second;
            frontier.erase(it);
            inq[u] = 0;
            if (level[u] > 0 && !fixed[u]) {
                const int e = pedge[u];
                if (parent[u] == ev[2 * e]) X[u] = iso_mul(X[ev[2 * e]], Z[e]);
                else X[u] = iso_mul(X[ev[2 * e + 1]], iso_inv(Z[e]));
            }
            for (int e : vedges[u]) {
                if (!act[e]) continue;  // PropagateCost: inactive edge -> max
                int maxf = -1;
                for (int s = 0; s < 2; ++s) {
                    const int z = ev[2 * e + s];
                    if (dist[z] != inf) maxf = std::max(maxf, level[z]);
                }
                for (int s = 0; s < 2; ++s) {
                    const int z = ev[2 * e + s];
                    if (z == u) continue;
                    const double zd = dist[u] + 1.0;
                    if (zd < dist[z]) {
                        dist[z] = zd;
                        parent[z] = u;
                        pedge[z] = e;
                        level[z] = maxf + 1;
                        push(z);
                    }
                }
            }
        }
    }

    double chi2(const std::vector<Iso> &S) const {
        double c = 0.0;
        for (int e : active_e) {
            double r[6];
            edge_error(Zinv[e], S[ev[2 * e]], S[ev[2 * e + 1]], r);
            const double *O = &info[36 * (size_t)e];
            double ce = 0.0;  // eᵀ(Ωe), per edge, then summed in edge order
            for (int a = 0; a < 6; ++a) {
                double s = 0.0;
                for (int b = 0; b < 6; ++b) s += O[6 * a + b] * r[b];
                ce += r[a] * s;
            }
            c += ce;
        }
        return c;
    }
    // BlockSolver::buildSystem: H = Σ JᵀΩJ, b = -Σ JᵀΩe over the free vertices (dense, full)
    void build(std::vector<double> &H, std::vector<double> &b) const {
        const int n = 6 * nfree;
        H.assign((size_t)n * n, 0.0);
        b.assign(n, 0.0);
        for (int e : active_e) {
            const int vi = ev[2 * e], vj = ev[2 * e + 1];
            double r[6], J[2][36];
            edge_error(Zinv[e], X[vi], X[vj], r);
            edge_jacobians(Zinv[e], X[vi], X[vj], J[0], J[1]);
            const double *O = &info[36 * (size_t)e];
            const int h[2] = {hidx[vi], hidx[vj]};
            double OJ[2][36], Or[6];
            for (int s = 0; s < 2; ++s)
                for (int a = 0; a < 6; ++a)
                    for (int c = 0; c < 6; ++c) {
                        double t = 0.0;
                        for (int k = 0; k < 6; ++k) t += O[6 * a + k] * J[s][6 * k + c];
                        OJ[s][6 * a + c] = t;
                    }
            for (int a = 0; a < 6; ++a) {
                double t = 0.0;
                for (int k = 0; k < 6; ++k) t += O[6 * a + k] * r[k];
                Or[a] = t;
            }
            for (int s = 0; s < 2; ++s) {
                if (h[s] < 0) continue;
                for (int a = 0; a < 6; ++a) {
                    double t = 0.0;
                    for (int k = 0; k < 6; ++k) t += J[s][6 * k + a] * Or[k];
                    b[6 * h[s] + a] -= t;
                }
                for (int s2 = 0; s2 < 2; ++s2) {
                    if (h[s2] < 0) continue;
                    for (int a = 0; a < 6; ++a)
                        for (int c = 0; c < 6; ++c) {
                            double t = 0.0;
                            for (int k = 0; k < 6; ++k) t += J[s][6 * k + a] * OJ[s2][6 * k + c];
                            H[(size_t)(6 * h[s] + a) * n + 6 * h[s2] + c] += t;
                        }
                }
            }
        }
    }
};

// LinearSolverCholmod stand-in: dense Cholesky, fails when a pivot is not positive
bool chol_solve(std::vector<double> A, int n, const std::vector<double> &b, std::vector<double> &x) {
    for (int j = 0; j < n; ++j) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / d;
        }
    }
    std::vector<double> y(b);
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < i; ++k) y[i] -= A[(size_t)i * n + k] * y[k];
        y[i] /= A[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        for (int k = i + 1; k < n; ++k) y[i] -= A[(size_t)k * n + i] * y[k];
        y[i] /= A[(size_t)i * n + i];
    }
    x = y;
    return true;
}

}  // namespace

extern "C" {

void refpgo_quat_from_R(const double *R9, double *q) {
    const Quat a = quat_from_R(R9);
    q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w;
}
void refpgo_to_mqt(const double *T12, double *v6) { to_mqt(iso_load(T12), v6); }
void refpgo_from_mqt(const double *v6, double *T12) { iso_store(from_mqt(v6), T12); }
void refpgo_edge_error(const double *Z12, const double *Xi12, const double *Xj12, double *e6) {
    edge_error(iso_inv(iso_load(Z12)), iso_load(Xi12), iso_load(Xj12), e6);
}
void refpgo_edge_jacobians(const double *Z12, const double *Xi12, const double *Xj12, double *Ji, double *Jj) {
    edge_jacobians(iso_inv(iso_load(Z12)), iso_load(Xi12), iso_load(Xj12), Ji, Jj);
}
void refpgo_oplus(const double *X12, const double *d6, double *out12) {
    iso_store(iso_mul(iso_load(X12), from_mqt(d6)), out12);
}

int refpgo_initial_guess(const plba_pgo_graph *g, double *out) {
    Graph G;
    G.load(g);
    G.initial_guess();
    for (int v = 0; v < G.nv; ++v) iso_store(G.X[v], out + 12 * (size_t)v);
    return 0;
}

// SparseOptimizer::optimize(max_iters) with OptimizationAlgorithmLevenberg::solve
int refpgo_optimize(const plba_pgo_graph *g, const plba_pgo_params *p, plba_pgo_result *r) {
    const auto t0 = std::chrono::steady_clock::now();
    Graph G;
    G.load(g);
    if (p->initial_guess) G.initial_guess();
    r->n_free = G.nfree;
    r->chi2_initial = G.chi2(G.X);
    r->iterations = r->trials = r->solve_fails = 0;
    r->n_trace = 0;
    const int n = 6 * G.nfree;
    double lambda = 0.0, ni = 2.0;
    std::vector<double> H, b, x(n, 0.0);
    double currentChi = r->chi2_initial;
    if (G.nfree > 0) {
        for (int it = 0; it < p->max_iters; ++it) {
            currentChi = G.chi2(G.X);  // computeActiveErrors + activeRobustChi2 (no robust kernel)
            const double chiStart = currentChi;
            G.build(H, b);
            if (it == 0) {
                if (p->user_lambda_init > 0.0) lambda = p->user_lambda_init;
                else {
                    double md = 0.0;
                    for (int k = 0; k < n; ++k) md = std::max(md, std::fabs(H[(size_t)k * n + k]));
                    lambda = 1e-5 * md;
                }
                ni = 2.0;
            }
            const double lambdaStart = lambda;
            double rho = 0.0;
            int qmax = 0;
            do {
                std::vector<double> Hd(H);
                for (int k = 0; k < n; ++k) Hd[(size_t)k * n + k] += lambda;
                std::vector<double> xn;
                const bool ok = chol_solve(Hd, n, b, xn);
                if (ok) x = xn;  // a failed Cholmod solve leaves _x as it was; update() still runs
                else ++r->solve_fails;
                std::vector<Iso> S(G.X);
                for (int v = 0; v < G.nv; ++v)
                    if (G.hidx[v] >= 0) S[v] = iso_mul(G.X[v], from_mqt(&x[6 * (size_t)G.hidx[v]]));
                double tempChi = G.chi2(S);
                if (!ok) tempChi = std::numeric_limits<double>::max();
                double scale = 0.0;
                for (int k = 0; k < n; ++k) scale += x[k] * (lambda * x[k] + b[k]);
                scale += 1e-3;
                rho = (currentChi - tempChi) / scale;
                if (rho > 0 && std::isfinite(tempChi)) {
                    double alpha = 1. - std::pow((2 * rho - 1), 3);
                    alpha = std::min(alpha, 2. / 3.);
                    lambda *= std::max(1. / 3., alpha);
                    ni = 2;
                    currentChi = tempChi;
                    G.X = S;
                } else {
                    lambda *= ni;
                    ni *= 2;
                    if (!std::isfinite(lambda)) break;
                }
                ++qmax;
                ++r->trials;
            } while (rho < 0 && qmax < p->max_trials);
            const int res = (qmax == p->max_trials || rho == 0 || !std::isfinite(lambda)) ? 1 : 0;
            if (r->trace && r->n_trace < r->trace_cap)
                r->trace[r->n_trace++] = plba_iter_trace{0, it, qmax, res, chiStart, currentChi, lambdaStart, lambda};
            ++r->iterations;
            if (res != 0) break;
        }
    }
    r->chi2_final = currentChi;
    r->lambda_final = lambda;
    if (r->v_T)
        for (int v = 0; v < G.nv; ++v) iso_store(G.X[v], r->v_T + 12 * (size_t)v);
    r->solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

}  // extern "C"
