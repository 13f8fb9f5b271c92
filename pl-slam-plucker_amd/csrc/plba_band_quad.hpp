// Four-segment column-lane band LDLᵀ of the reduced camera system (LinearSolverEigen, SURVEY.md
// §8a A12; DESIGN §4 "four-segment factorisation"). Bandwidth bw <= kQuadMaxBW pose blocks.
//
// The two-sided kernel (plba_band_cl.hpp) halves the serial chain of block pivots: two workgroups
// eliminate towards one separator from both ends. Here four workgroups eliminate four segments at
// once, which needs three separators (bw block rows each), natural numbering:
//
//   Seg1 [0, a) | S1 [a, a+bw) | Seg2 [a+bw, p) | S2 [p, p+bw) | Seg3 | S3 | Seg4 [.., nf)
//
// * Seg1 top-down and Seg4 bottom-up (the block-reversed band Bd2) end at S1 / S3 exactly like the
//   two-sided kernel's segments (cl_forward).
// * Seg2 sweeps top-down from S1 towards S2, Seg3 bottom-up from S3 towards S2. Their first rows
//   couple to the separator they start from, which is eliminated LATER: that coupling F_i =
//   A_{i,S1} (6 x 6bw, a "spike") fills in down the whole segment. cl_forward_sp carries it: the
//   critical wave additionally yields S_k⁻¹ (six identity lanes in the same Gauss–Jordan), and
//   worker lanes apply each step to the spike window (F_i -= L_ik F_k), accumulate the separator's
//   Schur term SS -= F_kᵀ S_k⁻¹ F_k and right-hand side sb -= F_kᵀ z_k in registers, and store
//   G_k = S_k⁻¹ F_k for the back substitution (x_k -= G_k x_S1). At the end of the sweep the spike
//   rows of S2 are the fill coupling C(S2, S1).
// * The last of {Seg1, Seg2} to finish eliminates S1 (its window + SS), carrying C(S1, S2) as the
//   spike onto S2; the last of {Seg3, Seg4} does the same for S3. The last of those two merges S2
//   (both middle windows, both spike Schur terms) and eliminates it as band steps, then runs the
//   back substitution: x_S2, then x_S1 and x_S3 (spike terms folded into z), then the four
//   segments on four waves.
// Chain at C3 (nf = 90, bw = 7): 17 + 7 + 7 block steps instead of 48 + 7; backward 31 steps
// instead of 55. Exact LDLᵀ in another (symmetric) elimination order: the same solution up to
// rounding, pivots are LDLᵀ pivots (a zero one fails the solve, as SimplicialLDLT).
// Hand-offs are last-arriver counters (no spin), as in the two-sided kernel.

constexpr int kQuadMaxBW = 7;  // 6(bw+1) column lanes + rhs + 6 identity lanes per wave; worker tasks <= 448
constexpr int kQuadNP = 3;     // parts of the spike columns per spike-Schur column (T3 lanes)

// LDS of cl_forward_sp: window [W1][W][36] + rhs [W1][6], pre-pivot [2][W][36],
// X [2][W*36 + 6 + 36] (L blocks, z, S_k⁻¹), spike window [W1][6][6bw], spike Schur [6bw][6bw]
__host__ __device__ constexpr size_t clsp_lds_doubles(int bw) {
    return (size_t)(bw + 2) * (bw + 1) * 36 + (size_t)(bw + 2) * 6 + 2 * (size_t)(bw + 1) * 36 +
           2 * ((size_t)(bw + 1) * 36 + 42) + (size_t)(bw + 2) * 6 * 6 * bw + (size_t)36 * bw * bw;
}
// + x_p staging [nf][6] + two reversed separator copies [bw][6]
__host__ __device__ constexpr size_t quad_lds_doubles(int bw, int nf) {
    return clsp_lds_doubles(bw) + (size_t)nf * 6 + 2 * (size_t)bw * 6;
}
// The record's parts (computed offsets: an array of pointers indexed by a runtime segment would
// live in scratch):
//   win(i)  [4]  separator window left by segment i (cl_store_sep layout)
//   Fout(i) [2]  [bw][6][NS] spike coupling of S2 to S1 (side 0) / to S3 (side 1), separator-major
//   SS(i)   [4]  [NS][NS]: S1 from Seg2, S3 from Seg3, S2 from the S1 / S3 sweeps; sb(i) rhs terms
//   G(i)    [2]  [nf][6][NS] G_k of Seg2 / Seg3;  GS(i) [2] [bw][6][NS] G_k of the S1 / S3 sweeps
struct QuadRec {
    double *b;
    size_t NS, QW, FO, G;
    __device__ QuadRec(double *base, int bw, int nf)
        : b(base), NS(6 * (size_t)bw), QW((size_t)bw * (bw + 1) * 36 + (size_t)bw * 6), FO((size_t)bw * 6 * 6 * bw),
          G((size_t)nf * 6 * 6 * bw) {}
    __device__ double *win(int i) const { return b + i * QW; }
    __device__ double *Fout(int i) const { return b + 4 * QW + i * FO; }
    __device__ double *SS(int i) const { return b + 4 * QW + 2 * FO + i * NS * NS; }
    __device__ double *sb(int i) const { return b + 4 * QW + 2 * FO + 4 * NS * NS + i * NS; }
    __device__ double *Gm(int i) const { return b + 4 * QW + 2 * FO + 4 * NS * NS + 4 * NS + i * G; }
    __device__ double *GS(int i) const { return b + 4 * QW + 2 * FO + 4 * NS * NS + 4 * NS + 2 * G + i * FO; }
};

struct SpikeIO {
    const double *Bd;  // initial spike rows from this band (F0 == nullptr): columns of the separator at sbase
    int sbase;
    const double *F0;  // else: [bw][6][NS] initial spike rows k0.. (separator-major coupling)
    double *G;         // [k1 - k0][6][NS] G_k = S_k⁻¹ F_k
    double *Fout;      // nullable: [bw][6][NS] spike of rows k1.. at the end, separator-major
    double *SS;        // [NS][NS] -Σ F_kᵀ G_k
    double *sb;        // [NS] -Σ F_kᵀ z_k
};

// cl_forward (plba_band_cl.hpp) with a spike: eliminates rows k0..k1-1 of g's band while carrying
// their coupling to the 6·bw columns of a separator eliminated later. Same critical-wave chain;
// the spike work rides on the worker waves one step behind (tasks T2, T3 below).
template <int BW>
__device__ __forceinline__ void cl_forward_sp(const BandSeg &g, int k0, int k1, bool load_window, double *lds, bool &fail,
                                              const SpikeIO &sp) {
    constexpr int W = BW + 1, W1 = BW + 2, NT = kClNT, NW = NT - 64, PD = kClPD, NS = 6 * BW;
    constexpr int XS = W * 36 + 6 + 36;             // X buffer: W blocks + z + S_k⁻¹
    constexpr int NPT6 = (BW - 1) * BW / 2 * 6;     // trailing (block pair, row) tasks
    constexpr int NRHS = (BW - 1) * 6;              // right-hand-side tasks
    constexpr int NROW = W * 36 + 6;                // block row streamed in per step
    constexpr int NFL = BW * 36 + 6;                // L blocks + z flushed per step
    constexpr int NP = kQuadNP, TPP = NS / NP;      // T3: spike-Schur column u, part of the rows
    constexpr int T3_0 = NPT6 + NRHS, T2_0 = T3_0 + NS * NP, NT2 = BW * (NS / 2);
    static_assert(NS % NP == 0 && NP * 2 == 6, "T3 parts also zero two spike rows each");
    static_assert(T2_0 + NT2 <= NW && NROW <= NW && NFL <= NW, "one task of each kind per worker");
    static_assert(6 * W + 7 <= 64, "column lanes + rhs lane + identity lanes must fit one wave");
    const int nrows = g.nrows;
    double *win = lds, *bwin = win + W1 * W * 36, *preA = bwin + W1 * 6, *Xs = preA + 2 * W * 36, *FW = Xs + 2 * XS;
    double *SSl = FW + W1 * 6 * NS;  // [NS][NS] spike Schur term, accumulated in LDS
    const int tid = threadIdx.x, lane = tid & 63, wt = tid - 64;
    const bool crit = tid < 64;
    if (load_window) {
        for (int t = tid; t < W1 * W * 36; t += NT) {
            const int row = k0 + t / (W * 36), rem = t % (W * 36);
            win[(row % W1) * W * 36 + rem] = row < nrows ? g.Bd[(size_t)row * W * 36 + rem] : 0.0;
        }
        for (int t = tid; t < W1 * 6; t += NT) {
            const int row = k0 + t / 6;
            bwin[(row % W1) * 6 + t % 6] = row < nrows ? g.bs[(size_t)row * 6 + t % 6] : 0.0;
        }
    }
    for (int t = tid; t < NS * NS; t += NT) SSl[t] = 0.0;
    // spike window: rows k0..k0+W1-1 (only the first bw rows can couple to the separator)
    for (int t = tid; t < W1 * 6 * NS; t += NT) {
        const int ri = t / (6 * NS), rem = t % (6 * NS), i = k0 + ri;
        double v = 0.0;
        if (ri < BW && i < nrows) {
            if (sp.F0) {
                v = sp.F0[(size_t)ri * 6 * NS + rem];
            } else {
                const int r = rem / NS, col = rem % NS, j = col / 6, c = col % 6, w = i - sp.sbase - j;
                if (w >= 1 && w <= BW) v = sp.Bd[((size_t)i * W + w) * 36 + r * 6 + c];
            }
        }
        FW[(i % W1) * 6 * NS + rem] = v;
    }
    __syncthreads();
    // ---- critical lanes: lane group cs <-> window rows i ≡ cs (mod W), scalar column cc; rhs
    //      lane 6W; identity lanes 6W+1..6W+6 (column il of S_k⁻¹ after the Gauss–Jordan)
    const int cs = lane / 6, cc = lane % 6;
    const bool clane = crit && lane < 6 * W, rlane = crit && lane == 6 * W;
    const int il = lane - 6 * W - 1;
    const bool ilane = crit && il >= 0 && il < 6;
    int sk = k0 % W, lk = k0 % W1;
    double v[6];
    {
        int dw = cs - sk;
        if (dw < 0) dw += W;
        int li = lk + dw;
        if (li >= W1) li -= W1;
        const double *src = clane ? win + (li * W + dw) * 36 + cc * 6 : bwin + lk * 6;
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = src[r];
        if (ilane)
#pragma unroll
            for (int r = 0; r < 6; ++r) v[r] = r == il ? 1.0 : 0.0;
    }
    // ---- worker tasks (static per thread)
    int p_wi = 1 << 20, p_wj = 0, p_a = 0;
    if (!crit && wt < NPT6) {
        const int pr = wt / 6;
        int wi = 2;
        while ((wi - 1) * wi / 2 <= pr) ++wi;
        p_wi = wi;
        p_wj = 2 + pr - (wi - 2) * (wi - 1) / 2;
        p_a = wt % 6;
    }
    int r_wi = 1 << 20, r_a = 0;
    if (!crit && wt >= NPT6 && wt < NPT6 + NRHS) {
        r_wi = 2 + (wt - NPT6) / 6;
        r_a = (wt - NPT6) % 6;
    }
    const int fl = NW - 1 - wt;
    // spike tasks: T3 = (column u, part p3): G_k[.][u], SS[p3 rows][u], sb[u] (p3 == 0), zeroing;
    //              T2 = (row offset w2, column pair q2): F_{k+w2}[.][q2, q2+1] -= L_{k+w2,k} F_k[.][..]
    const int t3 = wt - T3_0, t2 = wt - T2_0;
    const bool is_t3 = !crit && t3 >= 0 && t3 < NS * NP, is_t2 = !crit && t2 >= 0 && t2 < NT2;
    const int u3 = is_t3 ? t3 % NS : 0, p3 = is_t3 ? t3 / NS : 0;
    const int w2 = is_t2 ? 1 + t2 / (NS / 2) : 1, q2 = is_t2 ? 2 * (t2 % (NS / 2)) : 0;
    double sbacc = 0.0;
    double wpf[PD];
    auto prefetch = [&](int k, double &wdst) {
        if (!crit && wt < NROW) {
            const int rr = min(k + 2 + BW, nrows - 1);
            wdst = wt < W * 36 ? g.Bd[(size_t)rr * W * 36 + wt] : g.bs[(size_t)rr * 6 + (wt - W * 36)];
        }
    };
#pragma unroll
    for (int u = 0; u < PD; ++u) prefetch(k0 + u, wpf[u]);
    if (__builtin_amdgcn_readfirstlane(tid) < 64) __builtin_amdgcn_s_setprio(3);
    for (int kb = k0; kb < k1; kb += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const int k = kb + u;
            if (k >= k1) break;
            const int s1 = sk + 1 == W ? 0 : sk + 1;
            const int l1 = lk + 1 == W1 ? 0 : lk + 1;
            double *pA = preA + (u & 1) * W * 36, *X = Xs + (u & 1) * XS;
            if (crit) {
                if (clane) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) pA[cs * 36 + cc * 6 + r] = v[r];
                }
                double a1[36];
                // Gauss–Jordan on block row k across the lanes (identity lanes: S_k⁻¹)
#pragma unroll
                for (int pv = 0; pv < 6; ++pv) {
                    const int pl = 6 * sk + pv;
                    double f[6];
#pragma unroll
                    for (int r = 0; r < 6; ++r) f[r] = readlane_f64(v[r], pl);
                    if (f[pv] == 0.0) fail = true;
                    const double rp = rcp_nr1(f[pv]);
                    const double mp = v[pv] * rp;
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = r == pv ? mp : fma(-f[r], mp, v[r]);
                }
#pragma unroll
                for (int q = 0; q < 36; ++q) a1[q] = pA[s1 * 36 + q];
                __builtin_amdgcn_sched_barrier(0);
                if (clane && cs != sk) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) X[cs * 36 + cc * 6 + r] = v[r];
                }
                if (cs == sk) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = 0.0;
                }
                if (rlane) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) X[W * 36 + r] = v[r];
                }
                if (ilane) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) X[W * 36 + 6 + il * 6 + r] = v[r];
                }
                lds_barrier();
                if (k + 1 < nrows) {
                    int dw = cs - s1;
                    if (dw < 0) dw += W;
                    int li = l1 + dw;
                    if (li >= W1) li -= W1;
                    const double *src = clane ? win + (li * W + dw) * 36 + cc * 6 : bwin + l1 * 6;
                    double o[6];
#pragma unroll
                    for (int r = 0; r < 6; ++r) o[r] = src[r];
                    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int m = 0; m < 6; ++m)
#pragma unroll
                        for (int r = 0; r < 6; ++r) acc[r] = fma(a1[r * 6 + m], v[m], acc[r]);
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = o[r] - acc[r];
                }
                if (ilane)
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = r == il ? 1.0 : 0.0;
            } else {
                lds_barrier();
                // block row k+2+bw enters slot lk (row k is consumed)
                if (wt < NROW) {
                    const double val = k + 2 + BW < nrows ? wpf[u] : 0.0;
                    if (wt < W * 36) win[lk * W * 36 + wt] = val;
                    else bwin[lk * 6 + (wt - W * 36)] = val;
                }
                prefetch(k + PD, wpf[u]);
                // trailing update A_ij -= L_ik A_jkᵀ, k+2 <= j <= i <= k+bw (row p_a of the block)
                if (k + p_wi < nrows) {
                    int si = sk + p_wi, sj = sk + p_wj, li = lk + p_wi;
                    if (si >= W) si -= W;
                    if (sj >= W) sj -= W;
                    if (li >= W1) li -= W1;
                    const double *Lr = X + si * 36 + p_a * 6, *Aj = pA + sj * 36;
                    double L[6];
#pragma unroll
                    for (int m = 0; m < 6; ++m) L[m] = Lr[m];
                    double *dst = win + (li * W + (p_wi - p_wj)) * 36 + p_a * 6;
#pragma unroll
                    for (int b = 0; b < 6; ++b) {
                        double acc = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) acc = fma(L[m], Aj[b * 6 + m], acc);
                        dst[b] -= acc;
                    }
                }
                // b_i -= A_ik z_k, k+2 <= i <= k+bw
                if (k + r_wi < nrows) {
                    int si = sk + r_wi, li = lk + r_wi;
                    if (si >= W) si -= W;
                    if (li >= W1) li -= W1;
                    double acc = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) acc = fma(pA[si * 36 + r_a * 6 + m], X[W * 36 + m], acc);
                    bwin[li * 6 + r_a] -= acc;
                }
                // flush L_{k+w,k} (w = 1..bw) and z_k to HBM
                if (fl < BW * 36) {
                    const int w = 1 + fl / 36, e = fl % 36, i = k + w;
                    if (i < nrows) {
                        int si = sk + w;
                        if (si >= W) si -= W;
                        g.Lband[((size_t)i * W + w) * 36 + e] = X[si * 36 + e];
                    }
                } else if (fl < NFL) {
                    g.zb[(size_t)k * 6 + (fl - BW * 36)] = X[W * 36 + (fl - BW * 36)];
                }
                // ---- spike
                const double *Fk = FW + lk * 6 * NS;
                if (is_t3) {
                    const double *Si = X + W * 36 + 6, *zk = X + W * 36;
                    double fu[6], gv[6];
#pragma unroll
                    for (int q = 0; q < 6; ++q) fu[q] = Fk[q * NS + u3];
#pragma unroll
                    for (int m = 0; m < 6; ++m) {  // G_k[m][u] = Σ_q S_k⁻¹[m][q] F_k[q][u]
                        double a = 0.0;
#pragma unroll
                        for (int q = 0; q < 6; ++q) a = fma(Si[q * 6 + m], fu[q], a);
                        gv[m] = a;
                    }
#pragma unroll 2
                    for (int tt = 0; tt < TPP; ++tt) {  // SS[t][u] -= Σ_m F_k[m][t] G_k[m][u] (own entries)
                        const int t = p3 * TPP + tt;
                        double a = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) a = fma(Fk[m * NS + t], gv[m], a);
                        SSl[t * NS + u3] -= a;
                    }
                    if (p3 == 0) {
                        double a = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) a = fma(fu[m], zk[m], a);
                        sbacc -= a;
                        double *Gk = sp.G + (size_t)(k - k0) * 6 * NS + u3;
#pragma unroll
                        for (int m = 0; m < 6; ++m) Gk[(size_t)m * NS] = gv[m];
                    }
                    // row k-1's slot is row k+1+bw's: it enters with no coupling to the separator
                    double *Fz = FW + (lk == 0 ? W1 - 1 : lk - 1) * 6 * NS;
                    Fz[(2 * p3) * NS + u3] = 0.0;
                    Fz[(2 * p3 + 1) * NS + u3] = 0.0;
                }
                if (is_t2 && k + w2 < nrows) {
                    int si = sk + w2, li = lk + w2;
                    if (si >= W) si -= W;
                    if (li >= W1) li -= W1;
                    const double *L = X + si * 36;
                    double *Fi = FW + li * 6 * NS;
                    double f0[6], f1[6];
#pragma unroll
                    for (int m = 0; m < 6; ++m) {
                        f0[m] = Fk[m * NS + q2];
                        f1[m] = Fk[m * NS + q2 + 1];
                    }
#pragma unroll
                    for (int a = 0; a < 6; ++a) {
                        double a0 = 0.0, a1v = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) {
                            const double l = L[a * 6 + m];
                            a0 = fma(l, f0[m], a0);
                            a1v = fma(l, f1[m], a1v);
                        }
                        Fi[a * NS + q2] -= a0;
                        Fi[a * NS + q2 + 1] -= a1v;
                    }
                }
            }
            sk = s1;
            lk = l1;
        }
    }
    __syncthreads();
    // column k1 (through step k1-1) lives in the critical wave's registers: write it back
    if (k1 < nrows) {
        if (clane) {
            int dw = cs - sk;
            if (dw < 0) dw += W;
            int li = lk + dw;
            if (li >= W1) li -= W1;
            if (dw < BW && k1 + dw < nrows) {
#pragma unroll
                for (int r = 0; r < 6; ++r) win[(li * W + dw) * 36 + cc * 6 + r] = v[r];
            }
        }
        if (rlane) {
#pragma unroll
            for (int r = 0; r < 6; ++r) bwin[lk * 6 + r] = v[r];
        }
    }
    for (int t = tid; t < NS * NS; t += NT) sp.SS[t] = SSl[t];
    if (is_t3 && p3 == 0) sp.sb[u3] = sbacc;
    if (sp.Fout)  // Fout[i][r][6j+c] = F_{k1+j}[c][6i+r]: the next separator's coupling, separator-major
        for (int t = tid; t < BW * 6 * NS; t += NT) {
            const int i = t / (6 * NS), rem = t % (6 * NS), r = rem / NS, col = rem % NS, j = col / 6, c = col % 6;
            sp.Fout[t] = FW[((k1 + j) % W1) * 6 * NS + c * NS + 6 * i + r];
        }
    __syncthreads();
}

// One of two workgroups arriving at a hand-off: drains this workgroup's global stores, publishes its
// fail flag (agent release), counts the arrival. True in the second arriver, which then sees the
// other's stores (agent acquire) and gets s_fail = either flag. The last arriver resets the counter
// for the next launch (exactly two arrivals per launch and counter).
__device__ __forceinline__ bool quad_arrive(int32_t *cnt, int32_t *my_fail, const int32_t *other_fail, bool fail,
                                            int &s_last, int &s_fail) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(my_fail, fail ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == 1 ? 1 : 0;
        if (old == 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_fail = (fail || __hip_atomic_load(other_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 1 : 0;
        }
    }
    __syncthreads();
    return s_last != 0;
}

// a separator window stored by cl_store_sep (rows k1..k1+bw-1) into this workgroup's LDS window
// at rows k1.. (the other slots zeroed: rows past the separator are not part of its sweep)
template <int BW>
__device__ __forceinline__ void cl_load_sep(double *lds, int k1, const double *sep) {
    constexpr int W = BW + 1, W1 = BW + 2;
    double *win = lds, *bwin = win + W1 * W * 36;
    for (int t = threadIdx.x; t < W1 * W * 36; t += kClNT) {
        const int i = t / (W * 36), rem = t % (W * 36);
        win[((k1 + i) % W1) * W * 36 + rem] = i < BW ? sep[t] : 0.0;
    }
    for (int t = threadIdx.x; t < W1 * 6; t += kClNT) {
        const int i = t / 6;
        bwin[((k1 + i) % W1) * 6 + t % 6] = i < BW ? sep[(size_t)BW * W * 36 + t] : 0.0;
    }
}

template <int BW>
__global__ __launch_bounds__(kClNT) void k_rcs_factor_quad_cl(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int s_last, s_fail;
    if constexpr (BW >= 2 && BW <= kQuadMaxBW) {
        constexpr int W = BW + 1, W1 = BW + 2, NS = 6 * BW;
        const int seg = blockIdx.x, tid = threadIdx.x, nf = d.nf;
        const int a = d.q_a, p = d.q_p, n3 = d.q_n3, n4 = d.q_n4, n2 = p - a - BW;
        const QuadRec Q(d.qbuf, BW, nf);
        double *xl = lds + clsp_lds_doubles(BW);          // [nf][6] x_p staging
        double *xs1 = xl + (size_t)nf * 6, *xs2 = xs1 + BW * 6;  // x_S3, x_S2 in reversed order
        bool fail = false;
        // ---- phase 1: the four segments, each in its own numbering (reversed for Seg3 / Seg4)
        const bool rev = seg >= 2;
        const int side = rev ? 1 : 0;
        const double *Bd = rev ? d.Bd2 : d.Bd, *bs = rev ? d.bs2 : d.bs;
        double *Lb = rev ? d.Lband2 : d.Lband, *zb = rev ? d.zb2 : d.zb;
        const int sa = rev ? n4 : a;             // outer separator (S1 / S3) in this numbering
        const int sm = rev ? n4 + BW + n3 : p;   // middle separator S2 in this numbering
        const int outer = rev ? 3 : 0;           // the segment that ends at the outer separator
        if (seg == outer) {
            const BandSeg g{Bd, bs, Lb, nullptr, zb, sa + BW, sa, nullptr};
            cl_forward<BW>(g, 0, sa, true, lds, fail);
            cl_store_sep<BW>(lds, sa, Q.win(seg));
        } else {
            const BandSeg g{Bd, bs, Lb, nullptr, zb, sm + BW, sm, nullptr};
            const SpikeIO sp{Bd, sa, nullptr, Q.Gm(side), Q.Fout(side), Q.SS(side), Q.sb(side)};
            cl_forward_sp<BW>(g, sa + BW, sm, true, lds, fail, sp);
            cl_store_sep<BW>(lds, sm, Q.win(seg));
        }
        // hand-off A (pairs {Seg1, Seg2} and {Seg3, Seg4}): the last eliminates the outer separator
        const int partner = seg ^ 1;
        if (!quad_arrive(d.qcnt + side, d.qfail + seg, d.qfail + partner, fail, s_last, s_fail)) return;
        fail = s_fail != 0;
        // ---- phase 2: outer separator = its window + the middle segment's spike Schur term,
        //      eliminated with its fill coupling to S2 as the spike
        if (seg != outer) cl_load_sep<BW>(lds, sa, Q.win(outer));
        __syncthreads();
        {
            double *win = lds, *bwin = win + W1 * W * 36;
            const double *SS = Q.SS(side), *sb = Q.sb(side);
            for (int t = tid; t < BW * W * 36; t += kClNT) {
                const int i = t / (W * 36), rem = t % (W * 36), w = rem / 36, e = rem % 36;
                if (w > i) continue;
                const int j = i - w, r = e / 6, c = e % 6;
                win[((sa + i) % W1) * W * 36 + rem] += SS[(size_t)(6 * i + r) * NS + 6 * j + c];
            }
            for (int t = tid; t < BW * 6; t += kClNT) bwin[((sa + t / 6) % W1) * 6 + t % 6] += sb[t];
        }
        __syncthreads();
        {
            const BandSeg g{Bd, bs, Lb, nullptr, zb, sa + BW, sa + BW, nullptr};
            const SpikeIO sp{nullptr, 0, Q.Fout(side), Q.GS(side), nullptr, Q.SS(2 + side), Q.sb(2 + side)};
            cl_forward_sp<BW>(g, sa, sa + BW, false, lds, fail, sp);
        }
        // hand-off B (the two outer-separator eliminations): the last merges and eliminates S2
        if (!quad_arrive(d.qcnt + 2, d.qfail + 4 + side, d.qfail + 4 + (side ^ 1), fail, s_last, s_fail)) return;
        fail = s_fail != 0;
        // ---- phase 3: S2 (natural rows p..p+bw-1) = Seg2's window + Seg3's (reversed) − A_S2 + both
        //      spike Schur terms (the S3 sweep's in reversed S2 numbering), eliminated as band steps
        cl_load_sep<BW>(lds, p, Q.win(1));
        __syncthreads();
        {
            double *win = lds, *bwin = win + W1 * W * 36;
            const double *W2 = Q.win(2), *SSa = Q.SS(2), *SSb = Q.SS(3), *sba = Q.sb(2), *sbb = Q.sb(3);
            for (int t = tid; t < BW * W * 36; t += kClNT) {
                const int i = t / (W * 36), rem = t % (W * 36), w = rem / 36, e = rem % 36;
                if (w > i) continue;
                const int j = i - w, r = e / 6, c = e % 6;
                const int ir = BW - 1 - i, jr = BW - 1 - j;
                win[((p + i) % W1) * W * 36 + rem] += W2[((size_t)jr * W + w) * 36 + c * 6 + r] -
                                                      d.Bd[((size_t)(p + i) * W + w) * 36 + e] +
                                                      SSa[(size_t)(6 * i + r) * NS + 6 * j + c] +
                                                      SSb[(size_t)(6 * ir + r) * NS + 6 * jr + c];
            }
            for (int t = tid; t < BW * 6; t += kClNT) {
                const int i = t / 6, r = t % 6;
                bwin[((p + i) % W1) * 6 + r] += W2[(size_t)BW * W * 36 + (BW - 1 - i) * 6 + r] - d.bs[(size_t)(p + i) * 6 + r] +
                                                sba[t] + sbb[6 * (BW - 1 - i) + r];
            }
        }
        __syncthreads();
        {
            bool fail3 = false;
            const BandSeg g{d.Bd, d.bs, d.Lband, nullptr, d.zb, p + BW, p + BW, nullptr};
            cl_forward<BW>(g, p, p + BW, false, lds, fail3);
            if (tid == 0) s_fail = (fail || fail3 || diag_fail(d)) ? 1 : 0;
        }
        __syncthreads();
        const bool failed = s_fail != 0;
        if (tid == 0) *d.solve_okp = failed ? 0 : 1;
        if (!failed) {
            const int lane = tid & 63, wv = tid >> 6;
            // x_S2
            if (wv == 0) band_backward_rl<BW, true>(d.Lband + (size_t)p * W * 36, d.zb + (size_t)p * 6, BW, BW, nullptr,
                                                    xl + (size_t)p * 6, false, nf, lane);
            __syncthreads();
            for (int t = tid; t < BW * 6; t += kClNT) xs2[t] = xl[(size_t)(p + BW - 1 - t / 6) * 6 + t % 6];
            __syncthreads();
            // z of the outer separators -= G x_S2 (their fill coupling to S2)
            for (int t = tid; t < 2 * BW * 6; t += kClNT) {
                const int sd = t / (BW * 6), rr = t % (BW * 6);
                const double *G = Q.GS(sd) + (size_t)rr * NS, *x = sd ? xs2 : xl + (size_t)p * 6;
                double acc = 0.0;
                for (int q = 0; q < NS; ++q) acc = fma(G[q], x[q], acc);
                if (sd == 0) d.zb[(size_t)a * 6 + rr] -= acc;
                else d.zb2[(size_t)n4 * 6 + rr] -= acc;
            }
            __syncthreads();
            // x_S1 (wave 0), x_S3 (wave 1, reversed rows n4..)
            if (wv == 0)
                band_backward_rl<BW, true>(d.Lband + (size_t)a * W * 36, d.zb + (size_t)a * 6, BW, BW, nullptr,
                                           xl + (size_t)a * 6, false, nf, lane);
            else if (wv == 1)
                band_backward_rl<BW, true>(d.Lband2 + (size_t)n4 * W * 36, d.zb2 + (size_t)n4 * 6, BW, BW, nullptr, xl, true,
                                           nf - n4, lane);
            __syncthreads();
            for (int t = tid; t < BW * 6; t += kClNT) xs1[t] = xl[(size_t)(nf - 1 - n4 - t / 6) * 6 + t % 6];
            __syncthreads();
            // z of the middle segments -= G_k x_S1 / G_k x_S3 (their spike)
            for (int t = tid; t < (n2 + n3) * 6; t += kClNT) {
                const int sd = t >= n2 * 6 ? 1 : 0, rr = sd ? t - n2 * 6 : t;
                const double *G = Q.Gm(sd) + (size_t)rr * NS, *x = sd ? xs1 : xl + (size_t)a * 6;
                double acc = 0.0;
                for (int q = 0; q < NS; ++q) acc = fma(G[q], x[q], acc);
                if (sd == 0) d.zb[(size_t)(a + BW) * 6 + rr] -= acc;
                else d.zb2[(size_t)(n4 + BW) * 6 + rr] -= acc;
            }
            __syncthreads();
            // the four segments on four waves
            if (wv == 0)
                band_backward_rl<BW, true>(d.Lband, d.zb, a, a + BW, xl + (size_t)a * 6, xl, false, nf, lane);
            else if (wv == 1)
                band_backward_rl<BW, true>(d.Lband + (size_t)(a + BW) * W * 36, d.zb + (size_t)(a + BW) * 6, n2, n2 + BW,
                                           xl + (size_t)p * 6, xl + (size_t)(a + BW) * 6, false, nf, lane);
            else if (wv == 2)
                band_backward_rl<BW, true>(d.Lband2 + (size_t)(n4 + BW) * W * 36, d.zb2 + (size_t)(n4 + BW) * 6, n3, n3 + BW,
                                           xs2, xl, true, nf - n4 - BW, lane);
            else if (wv == 3)
                band_backward_rl<BW, true>(d.Lband2, d.zb2, n4, n4 + BW, xs1, xl, true, nf, lane);
            __syncthreads();
            for (int t = tid; t < nf * 6; t += kClNT) d.xp[t] = xl[t];
        }
        __syncthreads();
        pose_update_wg<kClNT>(d, failed);  // applied even after a failed solve, with the previous x_p (A13)
    }
}
