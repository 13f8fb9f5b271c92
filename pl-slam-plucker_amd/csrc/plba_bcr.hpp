// Block cyclic reduction (BCR) of the banded reduced camera system, many workgroups.
//
// The column-lane factorisation (plba_band_cl.hpp) is a chain of nf/2 dependent 6x6 pivot
// steps on two workgroups; at C4/C5 that chain is 184/454 steps. Here the band (bandwidth bw
// pose blocks) is grouped into N = ceil(nf/bw) super-rows of S = 6·bw scalars, which makes it
// block TRIDIAGONAL (super-row m couples only to m-1 and m+1). Cyclic reduction then eliminates
// the odd super-rows, then every second remaining one, ... : level l eliminates the rows with
// ctz(m) == l, each against its two neighbours a = m - 2^l and c = m + 2^l, and super-row 0 is
// the root solved last. The chain is ceil(log2 N) + 1 dense eliminations instead of nf/2 6x6
// pivot steps; every elimination of a level runs concurrently on its own workgroup.
//
// Eliminating row m (one workgroup, 512 threads, everything in LDS / registers):
//   block LDLᵀ of D_m with 6x6 pivots, RHS = [U | V | b] = [A(m,a) | A(m,c) | b_m] carried along
//   (right-looking, one 6x6 register tile per thread), and the Gram matrix
//   G = RHSᵀ D_m⁻¹ RHS = Σ_k R'_kᵀ P_k⁻¹ R'_k accumulated in the same loop. Published:
//     D_a -= G_UU, b_a -= G_Ub;  D_c -= G_VV, b_c -= G_Vb;  A(c,a) = F = -G_VU (new coupling).
//   Then, off the critical path, X = D_m⁻¹ RHS (block back substitution), and once x_a and x_c
//   are known: x_m = X_b - X_U x_a - X_V x_c.
// The survivors pick up their neighbours' contributions level by level (fixed order: above,
// then below, level by level — results do not depend on timing).
//
// Two launches per factorisation, each workgroup taking its super-row from a ticket counter:
//   k_rcs_factor_bcr  forward elimination, tickets in increasing level order (level 0 rows, then
//                     level 1, ..., the root last). A row waits only for rows of lower levels, whose
//                     tickets were taken earlier by workgroups that are running and never wait on a
//                     later ticket, so the launch completes whatever the co-residency (a workgroup
//                     that cannot be resident yet holds no ticket anybody waits for). Each row stores
//                     X = D_m⁻¹[U | V | b] for the backward pass; the root solves x_0.
//   k_rcs_bcr_back    back substitution x_m = X_b - X_U x_a - X_V x_c, tickets in decreasing level
//                     order (root first): a row waits only for rows of higher levels (earlier
//                     tickets). Then the pose update of the row's poses.
//
// Hand-offs (MI355X_MICROARCH.md, "Valid forms" table row 1): payload stored write-through
// (sc1, __hip_atomic_store relaxed/agent), every storing wave drains vmcnt, workgroup barrier,
// ONE lane stores the flag (relaxed agent atomic); the consumer polls the flag from one lane,
// barrier, then every load of the payload is an sc1 load (__hip_atomic_load relaxed/agent).
// Flags carry an epoch (factorisation count + 1) kept in bcr_ctl[0], advanced by the last
// workgroup of the backward launch (arrival counter), so nothing has to be cleared between launches
// or graph replays. bcr_ctl: [0] epoch, [1] forward arrivals, [2] forward tickets, [3] backward
// arrivals, [4] backward tickets. Every spin is bounded; a timeout raises Ctrl::dev_error, which
// stops every later kernel of the batch (the guards) and makes the host re-solve the window with
// the column-lane factorisation (plba.hip, run_schedule).
//
// Reference semantics: LinearSolverEigen = SimplicialLDLT fails iff a pivot
// is exactly 0. Every 6x6 pivot block is factorised LDLᵀ without pivoting, so its scalar pivots
// are LDLᵀ pivots of the (reordered) system and a zero one fails the solve; x_p then keeps its
// previous value (g2o still calls update()).
//
// Co-residency of the N workgroups is not required for completion (tickets above); the host
// selects BCR only when the N workgroups fit the device at once (occupancy x CUs), since a
// partly serialised launch loses the log-depth chain it is chosen for.

constexpr int kBcrNT = 512;
constexpr int kBcrMaxBW = 9;
constexpr int kBcrMaxRows = 240;   // co-residency margin below the 256 CUs
constexpr int kBcrParts = 12;      // partial sums per row of the x_m mat-vec
constexpr int kBcrBackNT = 256;    // backward (back substitution + pose update) workgroup
constexpr int kBcrCtl = 8;         // bcr_ctl words

// super-row of a forward ticket: level 0 rows (odd m) in increasing m, then level 1 (m ≡ 2 mod 4),
// ..., the root (m = 0, level L = ceil(log2 N)) last. Level l holds the m = 2^l (2i + 1) < N.
__device__ __forceinline__ int bcr_row_fwd(int t, int N, int L) {
    for (int l = 0; l < L; ++l) {
        const int cnt = (((N - 1) >> l) + 1) >> 1;
        if (t < cnt) return (2 * t + 1) << l;
        t -= cnt;
    }
    return 0;
}
// super-row of a backward ticket: the root first, then level L-1, ..., level 0
__device__ __forceinline__ int bcr_row_bwd(int t, int N, int L) {
    if (t == 0) return 0;
    --t;
    for (int l = L - 1; l >= 0; --l) {
        const int cnt = (((N - 1) >> l) + 1) >> 1;
        if (t < cnt) return (2 * t + 1) << l;
        t -= cnt;
    }
    return 0;
}

__host__ __device__ constexpr int bcr_tri(int bw) { return bw * (bw + 1) / 2; }
// Gram tiles: lower triangle of (2bw+1)x(2bw+1) 6x6 blocks over [U | V | b], minus the (b,b) corner
__host__ __device__ constexpr int bcr_ngram(int bw) { return (2 * bw + 1) * (2 * bw + 2) / 2 - 1; }
// LDS: D_m [S][S] | RHS [S][RS] (RS = 6(2bw+1): U, V, b padded to 6 columns) | W [S][S+RS] |
//      x_a, x_c, x_m [3][S] | pivot factors [2][48] | mat-vec partials [kBcrParts][S] | poses [bw][24] + λ
__host__ __device__ constexpr size_t bcr_lds_doubles(int bw) {
    return (size_t)(6 * bw) * (6 * bw) + (size_t)(6 * bw) * (6 * (2 * bw + 1)) +
           (size_t)(6 * bw) * (6 * bw + 6 * (2 * bw + 1)) + 3 * (size_t)(6 * bw) + 96 + (size_t)kBcrParts * (6 * bw) +
           (size_t)bw * 24 + 2;
}
// published record of an eliminated super-row: its Gram matrix G = Rᵀ D_m⁻¹ R over [U | V | b]
// (RS = 6(2bw+1) columns, b padded to 6) as a grid of 16x16 tiles, each tile row-major (the
// MFMA accumulator layout), only tiles (I, J) with J <= I + 1 written; + 1 failure word
#define BCR_T16(bw) ((6 * (2 * (bw) + 1) + 15) / 16)
__host__ __device__ constexpr size_t bcr_pub_doubles(int bw) { return (size_t)BCR_T16(bw) * BCR_T16(bw) * 256 + 2; }
// index of G(p, q) in a record
__host__ __device__ constexpr size_t bcr_gidx(int bw, int p, int q) {
    return ((size_t)(p / 16) * BCR_T16(bw) + q / 16) * 256 + (p % 16) * 16 + q % 16;
}
// the written tiles: row I, columns J = 0 .. min(I + 1, T16 - 1)
__host__ __device__ constexpr int bcr_gram_tiles(int bw) {
    int n = 0;
    for (int I = 0; I < BCR_T16(bw); ++I) n += (I + 1 < BCR_T16(bw) ? I + 1 : BCR_T16(bw) - 1) + 1;
    return n;
}
__host__ __device__ inline void bcr_gram_tile(int bw, int t, int &I, int &J) {
    const int T = BCR_T16(bw);
    for (I = 0; I < T; ++I) {
        const int cnt = (I + 1 < T ? I + 1 : T - 1) + 1;
        if (t < cnt) {
            J = t;
            return;
        }
        t -= cnt;
    }
    I = J = 0;
}
// solution record of a super-row: x (6 bw), padded
__host__ __device__ constexpr int bcr_xrec(int bw) { return 6 * bw + 2; }
// X = D_m⁻¹ [U | V | b] of an eliminated super-row, [6 bw][12 bw + 1] row-major
__host__ __device__ constexpr size_t bcr_X_doubles(int bw) { return (size_t)(6 * bw) * (12 * bw + 1); }
// backward kernel LDS: X_m | x_a | x_c | x_m | mat-vec partials | poses [bw][24] + λ
__host__ __device__ constexpr size_t bcr_back_lds_doubles(int bw) {
    return bcr_X_doubles(bw) + 3 * (size_t)(6 * bw) + (size_t)kBcrParts * (6 * bw) + (size_t)bw * 24 + 2;
}

// one lane: relaxed poll until the flag carries `epoch`; bounded (~0.3 s), timeout -> *err = 1.
// PLBA_DIAG bit 64 (failure-path test only): every wait times out at once, so the first hand-off
// of a launch raises the error and the host's fallback must take over
__device__ __forceinline__ bool bcr_poll(uint32_t *flag, uint32_t epoch, int32_t *err, int diag) {
    if (diag & 64) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
    }
    for (uint32_t spins = 0;; ++spins) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) return true;
        if (spins >= (1u << 23)) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// every storing wave drains its sc1 stores, then one lane raises the flag
__device__ __forceinline__ void bcr_publish(uint32_t *flag, uint32_t epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tri_decode(int t, int &i, int &j) {
    i = 0;
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    j = t - i * (i + 1) / 2;
}
// 6x6 tile from LDS (row-major, leading dimension ld, 16-B aligned rows)
__device__ __forceinline__ void lds_tile(const double *p, int ld, double (&t)[36]) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const double2 *q = reinterpret_cast<const double2 *>(p + (size_t)r * ld);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double2 v = q[c];
            t[r * 6 + 2 * c] = v.x;
            t[r * 6 + 2 * c + 1] = v.y;
        }
    }
}
__device__ __forceinline__ void lds_tile_store(double *p, int ld, const double (&t)[36]) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        double2 *q = reinterpret_cast<double2 *>(p + (size_t)r * ld);
#pragma unroll
        for (int c = 0; c < 3; ++c) q[c] = make_double2(t[r * 6 + 2 * c], t[r * 6 + 2 * c + 1]);
    }
}
// LDLᵀ of a symmetric 6x6 block (lower triangle of p used): unit-lower l, 1/d; fail iff a pivot is 0
__device__ __forceinline__ void ldl6(const double (&p)[36], double (&l)[36], double (&dinv)[6], bool &fail) {
    double dd[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double w[6];
#pragma unroll
        for (int q = 0; q < j; ++q) w[q] = l[j * 6 + q] * dd[q];
        double s = p[j * 6 + j];
#pragma unroll
        for (int q = 0; q < j; ++q) s = fma(-l[j * 6 + q], w[q], s);
        dd[j] = s;
        if (s == 0.0) fail = true;
        dinv[j] = rcp_nr(s);
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double t = p[i * 6 + j];
#pragma unroll
            for (int q = 0; q < j; ++q) t = fma(-l[i * 6 + q], w[q], t);
            l[i * 6 + j] = t * dinv[j];
        }
    }
}
// v <- P⁻¹ v with P = L D Lᵀ
__device__ __forceinline__ void ldl6_solve(const double (&l)[36], const double (&dinv)[6], double (&v)[6]) {
#pragma unroll
    for (int i = 1; i < 6; ++i)
#pragma unroll
        for (int q = 0; q < i; ++q) v[i] = fma(-l[i * 6 + q], v[q], v[i]);
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] *= dinv[i];
#pragma unroll
    for (int i = 4; i >= 0; --i)
#pragma unroll
        for (int q = i + 1; q < 6; ++q) v[i] = fma(-l[q * 6 + i], v[q], v[i]);
}

// PLBA_DIAG bit 8 (diagnostics only): per-workgroup phase timestamps (s_memrealtime, 100 MHz)
// into bcr_stamps[m][kBcrStamps]; read with plba_debug_bcr_stamps / tools/bcr_stamps.py
constexpr int kBcrStamps = 32;
#define BCR_STAMP(slot)                                                                          \
    do {                                                                                         \
        if ((d.diag & 8) && threadIdx.x == 0)                                                    \
            d.bcr_stamps[(size_t)m * kBcrStamps + (slot)] = __builtin_amdgcn_s_memrealtime();         \
    } while (0)

// tile index of Gram block (u, v), u >= v
__device__ __forceinline__ int gtile(int u, int v) { return u * (u + 1) / 2 + v; }

template <int BW>
__global__ __launch_bounds__(kBcrNT) void k_rcs_factor_bcr(Dev d0) {
    TRIAL_SLOT(blockIdx.y)  // trial slot s: its own band, records, flags and tickets (slot_view)
    if constexpr (BW >= 1 && BW <= kBcrMaxBW) {
        constexpr int NT = kBcrNT, S = 6 * BW, NB = 2 * BW + 1, RS = 6 * NB, WS = S + RS;
        constexpr int TRI = bcr_tri(BW), NRT = BW * NB, NG = bcr_ngram(BW), NX = 2 * S + 1;
        constexpr size_t PUB = bcr_pub_doubles(BW);
        static_assert(TRI + NRT + NG <= NT, "one tile per thread");
        static_assert(S + RS <= NT, "one W column per thread");
        extern __shared__ __attribute__((aligned(16))) double lds[];
        double *Dm = lds, *Rm = Dm + S * S, *Wm = Rm + S * RS, *xv = Wm + S * WS;  // xv: x_a | x_c | x_m
        double *pv = xv + 3 * S;          // [2][48] pivot block factors: unit-lower L (36) + 1/d (6)
        __shared__ uint32_t s_epoch;
        __shared__ int s_fail, s_m;
        const int tid = threadIdx.x, N = d.bcr_N, nf = d.nf;
        int L = 0;
        while ((1 << L) < N) ++L;
        // super-row by ticket in level order (deadlock-free without co-residency, see the top)
        if (tid == 0) {
            const uint32_t t = __hip_atomic_fetch_add(&d.bcr_ctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_m = bcr_row_fwd((int)t, N, L);
            s_epoch = __hip_atomic_load(&d.bcr_ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
            s_fail = 0;
        }
        __syncthreads();
        const int m = s_m;
        const bool root = m == 0;
        const int lm = root ? L : __builtin_ctz(m);
        const bool hasU = !root, hasC = !root && m + (1 << lm) < N;
        BCR_STAMP(0);
        // ---- D_m (lower blocks; diagonal blocks full), b_m and, for odd m, the band couplings
        //      U = A(m, m-1), V = A(m, m+1); rows past nf are identity / zero. Every global load of
        //      a thread is issued before its LDS stores.
        const size_t bstr = (size_t)(BW + 1) * 36;
        const bool odd = (m & 1) != 0;
        {
            constexpr int ND = (S * S + NT - 1) / NT, NR = (S * RS + NT - 1) / NT;
            double vd[ND], vr[NR];
#pragma unroll
            for (int u = 0; u < ND; ++u) {
                const int t = tid + u * NT, r = t / S, c = t % S, bi = r / 6, bj = c / 6, i = m * BW + bi;
                const bool ok = t < S * S && bi >= bj && i < nf;
                // unconditional load from a clamped (always in-bounds) address, then select
                const double g = d.Bd[ok ? (size_t)i * bstr + (bi - bj) * 36 + (r % 6) * 6 + c % 6 : 0];
                vd[u] = ok ? g : (i >= nf && r == c ? 1.0 : 0.0);
            }
#pragma unroll
            for (int u = 0; u < NR; ++u) {
                const int t = tid + u * NT, r = t / RS, c = t % RS, bi = r / 6, bc = c / 6, ra = r % 6, cb = c % 6;
                const int i = m * BW + bi, bj = bc - BW, j = (m + 1) * BW + bj;
                size_t addr = 0;
                int src = 0;  // 1: Bd, 2: bs
                if (t < S * RS && i < nf) {
                    if (bc < BW) {
                        if (odd && bi <= bc) { src = 1; addr = (size_t)i * bstr + (BW + bi - bc) * 36 + ra * 6 + cb; }
                    } else if (bc < 2 * BW) {
                        if (odd && bj <= bi && j < nf) { src = 1; addr = (size_t)j * bstr + (BW + bj - bi) * 36 + cb * 6 + ra; }
                    } else if (cb == 0) {
                        src = 2;
                        addr = (size_t)i * 6 + ra;
                    }
                }
                const double g1 = d.Bd[src == 1 ? addr : 0], g2 = d.bs[src == 2 ? addr : 0];
                vr[u] = src == 1 ? g1 : (src == 2 ? g2 : 0.0);
            }
#pragma unroll
            for (int u = 0; u < ND; ++u)
                if (tid + u * NT < S * S) Dm[tid + u * NT] = vd[u];
#pragma unroll
            for (int u = 0; u < NR; ++u)
                if (tid + u * NT < S * RS) Rm[tid + u * NT] = vr[u];
        }
        for (int t = tid; t < S * WS; t += NT) Wm[t] = 0.0;
        __syncthreads();
        BCR_STAMP(1);
        // ---- survivor phases: contributions of the neighbours eliminated at levels < lm. Every
        //      sc1 load of a phase is issued before the first use (no per-element round trip).
        double fail_in = 0.0;  // failure words flowing in (forward)
        for (int lp = 0; lp < lm; ++lp) {
            const int na = m - (1 << lp), nb = m + (1 << lp);  // above (m is its c) / below (m is its a)
            const bool ha = na >= 0, hb = nb < N;
            if (tid == 0 && ha && !bcr_poll(&d.bcr_flag[2 * na], s_epoch, &d.ctrl->dev_error, d.diag)) s_fail = 1;
            if (tid == 64 && hb && !bcr_poll(&d.bcr_flag[2 * nb], s_epoch, &d.ctrl->dev_error, d.diag)) s_fail = 1;
            __syncthreads();
            const double *pa = d.bcr_pub + (size_t)(ha ? na : 0) * PUB, *pb = d.bcr_pub + (size_t)(hb ? nb : 0) * PUB;
            const bool takeF = lm == lp + 1;  // the coupling created at level lm-1: U from above, V from below
            const bool fU = takeF && ha && !root, fV = takeF && hb && hasC;
            constexpr int KD = (TRI * 36 + NT - 1) / NT, KF = (S * S + NT - 1) / NT;
            double gda[KD], gdb[KD], gfa[KF], gfb[KF], gba = 0.0, gbb = 0.0, fa = 0.0, fb = 0.0;
            // D_m -= G_VV(above) + G_UU(below)   (lower blocks; G entries from the 16x16-tile records)
#pragma unroll
            for (int u = 0; u < KD; ++u) {
                const int t = tid + u * NT, blk = t % TRI, e = t / TRI;
                int bi, bj;
                tri_decode(blk, bi, bj);
                const bool ok = t < TRI * 36;
                const int r = 6 * bi + e / 6, c = 6 * bj + e % 6;
                gda[u] = ok && ha ? ld_sc1(pa + bcr_gidx(BW, S + r, S + c)) : 0.0;
                gdb[u] = ok && hb ? ld_sc1(pb + bcr_gidx(BW, r, c)) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < KF; ++u) {
                const int t = tid + u * NT, blk = t % (BW * BW), e = t / (BW * BW), vb = blk / BW, ub = blk % BW;
                const bool ok = t < S * S;
                const size_t o = bcr_gidx(BW, S + 6 * vb + e / 6, 6 * ub + e % 6);  // F = A(c_n, a_n) = -G_VU
                gfa[u] = ok && fU ? -ld_sc1(pa + o) : 0.0;
                gfb[u] = ok && fV ? -ld_sc1(pb + o) : 0.0;
            }
            if (tid < S) {  // b_m -= g_Vb(above) + g_Ub(below)
                gba = ha ? ld_sc1(pa + bcr_gidx(BW, 2 * S, S + tid)) : 0.0;
                gbb = hb ? ld_sc1(pb + bcr_gidx(BW, 2 * S, tid)) : 0.0;
            }
            if (tid == 0) {
                constexpr size_t FW = (size_t)BCR_T16(BW) * BCR_T16(BW) * 256;
                fa = ha ? ld_sc1(pa + FW) : 0.0;
                fb = hb ? ld_sc1(pb + FW) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < KD; ++u) {
                const int t = tid + u * NT, blk = t % TRI, e = t / TRI;
                if (t < TRI * 36) {
                    int bi, bj;
                    tri_decode(blk, bi, bj);
                    Dm[(6 * bi + e / 6) * S + 6 * bj + e % 6] -= gda[u] + gdb[u];
                }
            }
#pragma unroll
            for (int u = 0; u < KF; ++u) {
                const int t = tid + u * NT, blk = t % (BW * BW), e = t / (BW * BW), vb = blk / BW, ub = blk % BW;
                const int ea = e / 6, eb = e % 6;
                if (t < S * S) {
                    if (fU) Rm[(6 * vb + ea) * RS + 6 * ub + eb] = gfa[u];       // U_m = A(m, a_n), m = c_n
                    if (fV) Rm[(6 * ub + eb) * RS + S + 6 * vb + ea] = gfb[u];   // V_m = A(c_n, m)ᵀ
                }
            }
            if (tid < S) Rm[tid * RS + 2 * S] -= gba + gbb;
            if (tid == 0) fail_in += fa + fb;
            __syncthreads();
            BCR_STAMP(2 + lp);
        }
        // ---- elimination of super-row m: block LDLᵀ of D_m with 6x6 pivots, [U | V | b] carried
        //      as right-hand sides. Step k: W(k, ·) = P_k⁻¹ M(k, ·) (one thread per column), then
        //      the trailing update of D and R in LDS as half-tile tasks (3 rows x 6 columns, K = 6)
        //      spread over waves 0-6, while wave 7 updates the next pivot block first and factors it
        //      (lookahead). Rows of R are final once their block is the pivot (R'), so the Gram
        //      G = R'ᵀ W_R = Rᵀ D_m⁻¹ R is one rank-S product at the end, on the matrix cores.
        bool fail = false;
        auto factor_pivot = [&](const double (&p)[36], double *dst) {
            double l[36], dinv[6];
#pragma unroll
            for (int e = 0; e < 36; ++e) l[e] = 0.0;
            ldl6(p, l, dinv, fail);
#pragma unroll
            for (int e = 0; e < 36; ++e) dst[e] = l[e];
#pragma unroll
            for (int e = 0; e < 6; ++e) dst[36 + e] = dinv[e];
        };
        if (tid == 0) {
            double p0[36];
            lds_tile(Dm, S, p0);
            factor_pivot(p0, pv);  // P_0
        }
        __syncthreads();
        const int nU = hasU ? S : 0, nV = hasC ? S : 0;
        const int nRB = (hasU ? BW : 0) + (hasC ? BW : 0) + 1;  // active R column blocks
        constexpr int NTW = NT - 64;                             // task threads (waves 0-6)
        for (int k = 0; k < BW; ++k) {
            const double *pk = pv + 48 * (k & 1);
            // A2: W(k, col) = P_k⁻¹ M(k, col) for the D columns of later blocks and the active R
            // columns (P_k factors broadcast from LDS)
            const int nWd = S - 6 * (k + 1);
            if (tid < nWd + nU + nV + 1 && !(d.diag & 32)) {  // (diag 32/16: timing experiments only)
                double v[6];
                int col;
                if (tid < nWd) {
                    const int j = 6 * (k + 1) + tid;  // M(k, j) = D(j, k)ᵀ (lower storage)
#pragma unroll
                    for (int q = 0; q < 6; ++q) v[q] = Dm[j * S + 6 * k + q];
                    col = j;
                } else {
                    int cc = tid - nWd;
                    cc = cc < nU ? cc : (cc - nU < nV ? S + (cc - nU) : 2 * S);
#pragma unroll
                    for (int q = 0; q < 6; ++q) v[q] = Rm[(6 * k + q) * RS + cc];
                    col = S + cc;
                }
                double l[36], dinv[6];
#pragma unroll
                for (int e = 0; e < 36; ++e) l[e] = pk[e];
#pragma unroll
                for (int e = 0; e < 6; ++e) dinv[e] = pk[36 + e];
                ldl6_solve(l, dinv, v);
#pragma unroll
                for (int q = 0; q < 6; ++q) Wm[(6 * k + q) * WS + col] = v[q];
            }
            __syncthreads();
            if (k + 1 < BW && !(d.diag & 16)) {
                const double *Wk = Wm + (size_t)(6 * k) * WS;
                if (tid >= NTW) {
                    // lookahead: the next pivot block P_{k+1} = D(k+1,k+1) - D(k+1,k) W(k,k+1), one
                    // entry per lane, then factored by one lane
                    const int lane = tid - NTW;
                    if (lane < 36) {
                        const int r = 6 * (k + 1) + lane / 6, c = 6 * (k + 1) + lane % 6;
                        double sacc = Dm[r * S + c];
#pragma unroll
                        for (int q = 0; q < 6; ++q) sacc = fma(-Dm[r * S + 6 * k + q], Wk[q * WS + c], sacc);
                        Dm[r * S + c] = sacc;
                    }
                    wave_lds_sync();
                    if (lane == 0) {
                        double p1[36];
                        lds_tile(Dm + (6 * (k + 1)) * S + 6 * (k + 1), S, p1);
                        factor_pivot(p1, pv + 48 * ((k + 1) & 1));
                    }
                } else {
                    // A3: half-tile tasks (block row bi > k, rows 6bi + 3h .. + 2, column block cb):
                    // D blocks k < cb <= bi except the pivot block (k+1, k+1), then the R blocks
                    int nD = 0;
                    for (int bi = k + 1; bi < BW; ++bi) nD += bi - k;
                    nD = 2 * (nD - 1);
                    const int nTask = nD + 2 * (BW - 1 - k) * nRB;
                    for (int t = tid; t < nTask; t += NTW) {
                        int bi, cb, h;
                        bool isD = t < nD;
                        if (isD) {
                            int r = t / 2 + 1;  // skip the pivot block, the first D block in this order
                            h = t & 1;
                            bi = k + 1;
                            while (r >= bi - k) {
                                r -= bi - k;
                                ++bi;
                            }
                            cb = k + 1 + r;
                        } else {
                            const int t2 = t - nD;
                            h = t2 & 1;
                            const int rest = t2 >> 1;
                            bi = k + 1 + rest / nRB;
                            int rb = rest % nRB;
                            if (!hasU) rb += BW;
                            if (!hasC && rb >= BW) rb += BW;
                            cb = rb;  // U blocks 0..BW-1, V blocks BW..2BW-1, b block 2BW
                        }
                        const int r0 = 6 * bi + 3 * h;
                        double a[3][6], w[6][6];
#pragma unroll
                        for (int rr = 0; rr < 3; ++rr) {
                            const double2 *src = reinterpret_cast<const double2 *>(Dm + (r0 + rr) * S + 6 * k);
#pragma unroll
                            for (int c = 0; c < 3; ++c) {
                                const double2 v2 = src[c];
                                a[rr][2 * c] = v2.x;
                                a[rr][2 * c + 1] = v2.y;
                            }
                        }
                        const int wc = isD ? 6 * cb : S + 6 * cb;
#pragma unroll
                        for (int q = 0; q < 6; ++q) {
                            const double2 *src = reinterpret_cast<const double2 *>(Wk + q * WS + wc);
#pragma unroll
                            for (int c = 0; c < 3; ++c) {
                                const double2 v2 = src[c];
                                w[q][2 * c] = v2.x;
                                w[q][2 * c + 1] = v2.y;
                            }
                        }
                        double *dst = isD ? Dm + r0 * S + 6 * cb : Rm + r0 * RS + 6 * cb;
                        const int ld = isD ? S : RS;
#pragma unroll
                        for (int rr = 0; rr < 3; ++rr) {
                            double2 *o2 = reinterpret_cast<double2 *>(dst + rr * ld);
#pragma unroll
                            for (int c = 0; c < 3; ++c) {
                                double2 v2 = o2[c];
                                double s0 = v2.x, s1 = v2.y;
#pragma unroll
                                for (int q = 0; q < 6; ++q) {
                                    s0 = fma(-a[rr][q], w[q][2 * c], s0);
                                    s1 = fma(-a[rr][q], w[q][2 * c + 1], s1);
                                }
                                o2[c] = make_double2(s0, s1);
                            }
                        }
                    }
                }
            }
            __syncthreads();
            BCR_STAMP(20 + k);
        }
        if (fail) s_fail = 1;  // (benign race: every writer stores 1)
        BCR_STAMP(12);
        const uint32_t epoch = s_epoch;
        __syncthreads();
        const double fail_fwd = fail_in + (s_fail ? 1.0 : 0.0);  // meaningful on tid 0
        // ---- Gram G = R'ᵀ W_R (RS x RS) on v_mfma_f64_16x16x4f64: 16x16 tiles (I, J) with
        //      J <= I + 1 (every 6x6 block (u, v) with u >= v lies in one), K = S in steps of 4.
        //      Published write-through as 16x16 tiles, each row-major — the MFMA accumulator's own
        //      lane order, so every store instruction is one contiguous 512-B run.
        if (!root) {
            double *pub = d.bcr_pub + (size_t)m * PUB;
            const int wave = tid >> 6, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
            constexpr int NGT = bcr_gram_tiles(BW);
            for (int gtl = wave; gtl < NGT; gtl += NT / 64) {
                int I = 0, J = 0;
                bcr_gram_tile(BW, gtl, I, J);
                dbl4 acc4 = dbl4{0.0, 0.0, 0.0, 0.0};
                const int p = 16 * I + lr, q = 16 * J + lr;
#pragma unroll
                for (int ks = 0; ks < (S + 3) / 4; ++ks) {
                    const int r = 4 * ks + lk;
                    const double av = (r < S && p < RS) ? Rm[r * RS + p] : 0.0;       // A[p][r] = R'(r, p)
                    const double bv = (r < S && q < RS) ? Wm[r * WS + S + q] : 0.0;   // B[r][q] = W(r, S + q)
                    acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc4, 0, 0, 0);
                }
                double *tp = pub + ((size_t)I * BCR_T16(BW) + J) * 256;
#pragma unroll
                for (int i = 0; i < 4; ++i) st_sc1(tp + (lk + 4 * i) * 16 + lr, acc4[i]);
            }
            if (tid == 0) st_sc1(pub + (size_t)BCR_T16(BW) * BCR_T16(BW) * 256, fail_fwd);
            bcr_publish(&d.bcr_flag[2 * m], epoch);
        }
        BCR_STAMP(13);
        // ---- X = D_m⁻¹ RHS (block back substitution, right-looking, into Rm) for the active
        //      columns; x_m = X_b - X_U x_a - X_V x_c once the neighbours are solved
        const int ncol = nU + nV + 1;
        for (int t = tid; t < S * ncol; t += NT) {
            const int r = t / ncol, cc0 = t % ncol;
            const int cc = cc0 < nU ? cc0 : (cc0 - nU < nV ? S + (cc0 - nU) : 2 * S);
            Rm[r * RS + cc] = Wm[r * WS + S + cc];
        }
        __syncthreads();
        for (int j = BW - 1; j >= 1; --j) {
            for (int t = tid; t < 6 * j * ncol; t += NT) {
                const int r = t / ncol, cc0 = t % ncol;
                const int cc = cc0 < nU ? cc0 : (cc0 - nU < nV ? S + (cc0 - nU) : 2 * S);
                double sacc = Rm[r * RS + cc];
#pragma unroll
                for (int p = 0; p < 6; ++p) sacc = fma(-Wm[r * WS + 6 * j + p], Rm[(6 * j + p) * RS + cc], sacc);
                Rm[r * RS + cc] = sacc;
            }
            __syncthreads();
        }
        BCR_STAMP(14);
        // ---- X = D_m⁻¹ [U | V | b] for the backward kernel (split mode); the root holds the solution
        //      x_0 itself. Fused mode (default): X stays in Rm and this workgroup back-substitutes its
        //      own super-row below, so X never goes through memory and the second launch is gone.
        const bool fused = d.bcr_fused != 0;
        const int XR = bcr_xrec(BW);
        if (!root) {
            if (!fused) {
                double *Xg = d.bcr_X + (size_t)m * S * NX;
                for (int t = tid; t < S * NX; t += NT) Xg[t] = Rm[(t / NX) * RS + t % NX];
            }
        } else {
            for (int r = tid; r < S; r += NT) st_sc1(d.bcr_x + r, Rm[r * RS + 2 * S]);
            // every failure word has flowed in (PLBA_DIAG bit 128: the tests' forced failures)
            if (tid == 0) {
                const bool failed0 = fail_fwd != 0.0 || diag_fail(d);
                *d.solve_okp = failed0 ? 0 : 1;
                // fused: the decision travels down the tree in the x records (slot S), so every
                // row's pose update knows it without reading solve_ok across workgroups
                st_sc1(d.bcr_x + S, failed0 ? 1.0 : 0.0);
            }
            bcr_publish(&d.bcr_flag[1], epoch);
        }
        BCR_STAMP(16);
        if (fused) {
            // ---- back substitution of this super-row: x_m = X_b - X_U x_a - X_V x_c once the
            //      neighbours (higher levels: later tickets, co-resident by the selection rule — a
            //      timed-out wait raises Ctrl::dev_error and the host re-solves) are solved; then
            //      the pose update of its poses (as k_rcs_bcr_back).
            constexpr int NPART = NT / S < kBcrParts ? NT / S : kBcrParts;
            double *xa = xv, *xc = xv + S, *xm = xv + 2 * S, *red = pv + 96, *ps = red + kBcrParts * S;
            __shared__ double s_sum[NT / 64];
            __shared__ double s_failed;
            __shared__ int s_kf[BW + 1];
            const int a_row = m - (1 << lm), c_row = m + (1 << lm);
            const double *Tc0 = d.Tc;
            double *Tt0 = d.Tt;
            if (tid < BW) s_kf[tid] = m * BW + tid < nf ? d.h_kf[m * BW + tid] : 0;
            for (int t = tid; t < BW * 24; t += NT) {
                const int i = t / 24, q = t % 24, h = m * BW + i;
                double v = 0.0;
                if (h < nf) {
                    const int kf = d.h_kf[h];
                    v = q < 12 ? Tc0[(size_t)kf * 12 + q] : (q < 18 ? d.bp[(size_t)h * 6 + q - 12] : d.xp_prev[(size_t)h * 6 + q - 18]);
                }
                ps[t] = v;
            }
            const bool hlm0 = d.ctrl->hlm != 0;
            for (int k = m + N * tid; k < d.n_kf; k += N * NT)
                if (d.kf_hidx[k] < 0) {
#pragma unroll
                    for (int q = 0; q < 12; ++q) Tt0[(size_t)k * 12 + q] = Tc0[(size_t)k * 12 + q];
                    if (hlm0)
#pragma unroll
                        for (int q = 0; q < 6; ++q) d.xkt[(size_t)k * 6 + q] = d.xkc[(size_t)k * 6 + q];
                }
            if (!root) {
                if (tid == 0) (void)bcr_poll(&d.bcr_flag[2 * a_row + 1], epoch, &d.ctrl->dev_error, d.diag);
                if (hasC && tid == 64) (void)bcr_poll(&d.bcr_flag[2 * c_row + 1], epoch, &d.ctrl->dev_error, d.diag);
                __syncthreads();
                for (int t = tid; t < S; t += NT) {
                    xa[t] = ld_sc1(d.bcr_x + (size_t)a_row * XR + t);
                    xc[t] = hasC ? ld_sc1(d.bcr_x + (size_t)c_row * XR + t) : 0.0;
                }
                if (tid == 0) s_failed = ld_sc1(d.bcr_x + (size_t)a_row * XR + S);
                __syncthreads();
                if (tid < S * NPART) {  // mat-vec in column slices per row, partials summed in slice order
                    const int r = tid % S, part = tid / S;
                    constexpr int CPP = (2 * S + NPART - 1) / NPART;
                    double sacc = 0.0;
#pragma unroll
                    for (int u = 0; u < CPP; ++u) {
                        const int q = part * CPP + u;
                        if (q < S) sacc = fma(Rm[r * RS + q], xa[q], sacc);
                        else if (q < 2 * S && hasC) sacc = fma(Rm[r * RS + q], xc[q - S], sacc);
                    }
                    red[part * S + r] = sacc;
                }
                __syncthreads();
                for (int r = tid; r < S; r += NT) {
                    double sacc = Rm[r * RS + 2 * S];
                    for (int part = 0; part < NPART; ++part) sacc -= red[part * S + r];
                    xm[r] = sacc;
                    st_sc1(d.bcr_x + (size_t)m * XR + r, sacc);
                }
                if (tid == 0) st_sc1(d.bcr_x + (size_t)m * XR + S, s_failed);
                bcr_publish(&d.bcr_flag[2 * m + 1], epoch);
            } else {
                for (int r = tid; r < S; r += NT) xm[r] = Rm[r * RS + 2 * S];
                if (tid == 0) s_failed = (fail_fwd != 0.0 || diag_fail(d)) ? 1.0 : 0.0;
                __syncthreads();
            }
            // ---- this super-row's poses: x_p (kept from the previous trial if the solve failed, A13),
            //      oplus into the trial state, pose part of Σx(λx+b)
            const bool failed = s_failed != 0.0;
            const double lam = d.lam;
            double sc = 0.0;
            if (tid < BW) {
                const int h = m * BW + tid;
                if (h < nf) {
                    const double *pp = ps + tid * 24;
                    double x[6];
#pragma unroll
                    for (int q = 0; q < 6; ++q) x[q] = failed ? pp[18 + q] : xm[6 * tid + q];
                    if (!failed)
#pragma unroll
                        for (int q = 0; q < 6; ++q) d.xp[6 * h + q] = x[q];
                    if (hlm0) {  // hand-rolled LM: se(3) update, ‖DX‖² part
                        const int kf = s_kf[tid];
                        double xn[6];
#pragma unroll
                        for (int q = 0; q < 6; ++q) sc += x[q] * x[q];
                        hlm_pose_update(d.xkc + (size_t)kf * 6, x, xn, Tt0 + (size_t)kf * 12);
#pragma unroll
                        for (int q = 0; q < 6; ++q) d.xkt[(size_t)kf * 6 + q] = xn[q];
                    } else {
#pragma unroll
                        for (int q = 0; q < 6; ++q) sc += x[q] * (lam * x[q] + pp[12 + q]);
                        pose_oplus(pp, x, Tt0 + (size_t)s_kf[tid] * 12);
                    }
                }
            }
            const double ssum = block_sum<NT>(sc, s_sum);
            if (tid == 0) d.part_ps[m] = ssum;
        }
        BCR_STAMP(18);
        // ---- arrival: the last workgroup resets the ticket counter for the next launch (fused: and
        //      advances the epoch, as the backward launch's last workgroup does in split mode)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const uint32_t old = __hip_atomic_fetch_add(&d.bcr_ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == (uint32_t)(N - 1)) {
                __hip_atomic_store(&d.bcr_ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&d.bcr_ctl[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (fused) __hip_atomic_store(&d.bcr_ctl[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        BCR_STAMP(17);
    }
}

// Backward launch: x of every super-row from the root down, then the pose update (oplus into the
// trial state, x_p kept from the previous trial when the solve failed — A13 — and the pose part of
// Σx(λx+b) per row; fixed poses k ≡ m (mod N) copied to the trial state).
template <int BW>
__global__ __launch_bounds__(kBcrBackNT) void k_rcs_bcr_back(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    if constexpr (BW >= 1 && BW <= kBcrMaxBW) {
        constexpr int NT = kBcrBackNT, S = 6 * BW, NX = 2 * S + 1, XR = bcr_xrec(BW);
        constexpr int NPART = NT / S < kBcrParts ? NT / S : kBcrParts;  // mat-vec slices per row
        extern __shared__ __attribute__((aligned(16))) double lds[];
        double *Xm = lds, *xa = Xm + bcr_X_doubles(BW), *xc = xa + S, *xm = xc + S, *red = xm + S;
        double *ps = red + kBcrParts * S;  // [BW][24] Tcw | b_p | previous x_p of this row's poses, λ
        __shared__ uint32_t s_epoch;
        __shared__ int s_m;
        __shared__ double s_sum[NT / 64];
        __shared__ int s_kf[BW + 1];
        const int tid = threadIdx.x, N = d.bcr_N, nf = d.nf;
        int L = 0;
        while ((1 << L) < N) ++L;
        if (tid == 0) {
            const uint32_t t = __hip_atomic_fetch_add(&d.bcr_ctl[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_m = bcr_row_bwd((int)t, N, L);
            s_epoch = __hip_atomic_load(&d.bcr_ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        }
        __syncthreads();
        const int m = s_m;
        const bool root = m == 0;
        const int lm = root ? L : __builtin_ctz(m);
        const int a_row = m - (1 << lm), c_row = m + (1 << lm);
        const bool hasC = !root && c_row < N;
        const uint32_t epoch = s_epoch;
        // X_m into LDS and this row's poses (current Tcw, b_p, previous x_p, λ), issued before the waits
        if (!root) {
            const double *Xg = d.bcr_X + (size_t)m * S * NX;
            for (int t = tid; t < S * NX; t += NT) Xm[t] = Xg[t];
        }
        const double *Tc0 = d.Tc;  // (slot view: this slot's trial buffer)
        double *Tt0 = d.Tt;
        if (tid < BW) s_kf[tid] = m * BW + tid < nf ? d.h_kf[m * BW + tid] : 0;
        for (int t = tid; t < BW * 24; t += NT) {
            const int i = t / 24, q = t % 24, h = m * BW + i;
            double v = 0.0;
            if (h < nf) {
                const int kf = d.h_kf[h];
                v = q < 12 ? Tc0[(size_t)kf * 12 + q] : (q < 18 ? d.bp[(size_t)h * 6 + q - 12] : d.xp_prev[(size_t)h * 6 + q - 18]);
            }
            ps[t] = v;
        }
        if (tid == 0) ps[BW * 24] = d.lam;
        const bool hlm0 = d.ctrl->hlm != 0;
        for (int k = m + N * tid; k < d.n_kf; k += N * NT)
            if (d.kf_hidx[k] < 0) {
#pragma unroll
                for (int q = 0; q < 12; ++q) Tt0[(size_t)k * 12 + q] = Tc0[(size_t)k * 12 + q];
                if (hlm0)
#pragma unroll
                    for (int q = 0; q < 6; ++q) d.xkt[(size_t)k * 6 + q] = d.xkc[(size_t)k * 6 + q];
            }
        if (!root) {
            // (a timeout raises Ctrl::dev_error: the host discards this schedule and re-solves)
            if (tid == 0) (void)bcr_poll(&d.bcr_flag[2 * a_row + 1], epoch, &d.ctrl->dev_error, d.diag);
            if (hasC && tid == 64) (void)bcr_poll(&d.bcr_flag[2 * c_row + 1], epoch, &d.ctrl->dev_error, d.diag);
            __syncthreads();
            for (int t = tid; t < S; t += NT) {
                xa[t] = ld_sc1(d.bcr_x + (size_t)a_row * XR + t);
                xc[t] = hasC ? ld_sc1(d.bcr_x + (size_t)c_row * XR + t) : 0.0;
            }
            __syncthreads();
            // mat-vec in column slices per row, partials summed in slice order
            if (tid < S * NPART) {
                const int r = tid % S, part = tid / S;
                constexpr int CPP = (2 * S + NPART - 1) / NPART;
                double sacc = 0.0;
#pragma unroll
                for (int u = 0; u < CPP; ++u) {
                    const int q = part * CPP + u;
                    if (q < S) sacc = fma(Xm[r * NX + q], xa[q], sacc);
                    else if (q < 2 * S && hasC) sacc = fma(Xm[r * NX + q], xc[q - S], sacc);
                }
                red[part * S + r] = sacc;
            }
            __syncthreads();
            for (int r = tid; r < S; r += NT) {
                double sacc = Xm[r * NX + 2 * S];
                for (int part = 0; part < NPART; ++part) sacc -= red[part * S + r];
                xm[r] = sacc;
                st_sc1(d.bcr_x + (size_t)m * XR + r, sacc);
            }
            bcr_publish(&d.bcr_flag[2 * m + 1], epoch);
        } else {
            for (int r = tid; r < S; r += NT) xm[r] = d.bcr_x[r];  // solved by the forward root
            __syncthreads();
        }
        // ---- this super-row's poses: x_p (kept from the previous trial if the solve failed, A13),
        //      oplus into the trial state, pose part of Σx(λx+b)
        const bool failed = *d.solve_okp == 0;
        const double lam = ps[BW * 24];
        double sc = 0.0;
        if (tid < BW) {
            const int h = m * BW + tid;
            if (h < nf) {
                const double *pp = ps + tid * 24;
                double x[6];
#pragma unroll
                for (int q = 0; q < 6; ++q) x[q] = failed ? pp[18 + q] : xm[6 * tid + q];
                if (!failed)
#pragma unroll
                    for (int q = 0; q < 6; ++q) d.xp[6 * h + q] = x[q];
                if (d.ctrl->hlm) {  // hand-rolled LM: se(3) update, ‖DX‖² part
                    const int kf = s_kf[tid];
                    double xn[6];
#pragma unroll
                    for (int q = 0; q < 6; ++q) sc += x[q] * x[q];
                    hlm_pose_update(d.xkc + (size_t)kf * 6, x, xn, Tt0 + (size_t)kf * 12);
#pragma unroll
                    for (int q = 0; q < 6; ++q) d.xkt[(size_t)kf * 6 + q] = xn[q];
                } else {
#pragma unroll
                    for (int q = 0; q < 6; ++q) sc += x[q] * (lam * x[q] + pp[12 + q]);
                    pose_oplus(pp, x, Tt0 + (size_t)s_kf[tid] * 12);
                }
            }
        }
        const double ssum = block_sum<NT>(sc, s_sum);
        if (tid == 0) d.part_ps[m] = ssum;
        // ---- arrival: the last workgroup resets the tickets and advances the epoch
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const uint32_t old = __hip_atomic_fetch_add(&d.bcr_ctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == (uint32_t)(N - 1)) {
                __hip_atomic_store(&d.bcr_ctl[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&d.bcr_ctl[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&d.bcr_ctl[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}
