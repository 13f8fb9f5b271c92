// Column-lane banded LDLᵀ of the reduced camera system (envelope bandwidth bw <= 9 pose blocks).
//
// Same factorisation and outputs as band_forward (L_{i,k} in Lband, z_k in zb, the separator
// window for the two-sided variant), restructured around the latency of the serial chain:
//
// * The critical wave holds the whole current block column k of the band in registers, one
//   lane per scalar column of block row k: lane 6s+c carries column c of A_{k,i} (the block of
//   row i ≡ s mod W), lane 6W carries the right-hand side y_k. Eliminating block k: the column
//   is published to LDS (the workers need it anyway), every lane reads the pivot block S_k back,
//   factors it LDLᵀ in its own registers (no cross-lane dependency; v_rcp_f64 + one Newton step
//   per pivot) and solves its own 6-vector. The result is X_i = S_k⁻¹A_{k,i} = L_{i,k}ᵀ for
//   every band block at once, and z_k = S_k⁻¹y_k — no separate S⁻¹ and no separate L product.
//   (Rounds 2-4 broadcast the pivot column of a cross-lane Gauss–Jordan with v_readlane: 72 per
//   step, the largest single cost of the step.)
// * The next column k+1 (the next pivot's block column) is formed by the same wave right after
//   the single workgroup barrier: A_{i,k+1} -= L_{i,k}A_{k+1,k}ᵀ with A_{k+1,k} read from LDS
//   while the X publish and the barrier run.
// * Worker waves apply step k to the rest of the window (blocks (i,j), k+2 <= j <= i <= k+bw,
//   and b_i) one step behind, stream block row k+1+bw in, and flush L/z to HBM: they are off
//   the chain as long as they finish within one Gauss–Jordan.
// One LDS barrier per pose block (two in band_forward); pre-pivot columns and X are
// double-buffered in LDS by step parity so the next step's writes never race the workers.
//
// Reference semantics: src/mapHandler.cpp:5925-5927 solves with LinearSolverEigen =
// SimplicialLDLT: no pivoting, failure iff a pivot is zero. The pivots of the
// lane-local 6x6 LDLᵀ of each pivot block are exactly LDLᵀ pivots of the system, so a zero one
// fails the solve the same way.

constexpr int kClNT = 512;     // 1 critical wave + 7 worker waves (2 waves per SIMD)
constexpr int kClMaxBW = 9;    // 6(bw+1) column lanes + 1 rhs lane must fit one wave
constexpr int kClPD = 4;       // worker prefetch distance in steps (= unroll factor of the step loop)

// LDS: window [bw+2 slots][bw+1 blocks][36] + rhs [bw+2][6], pre-pivot columns [2][bw+1][36],
// X = L blocks + z [2][(bw+1)*36 + 6]. The window has one slot more than the band is wide so
// that block row k+1+bw is already resident when the critical wave forms column k+1.
__host__ __device__ constexpr size_t cl_lds_doubles(int bw) {
    return (size_t)(bw + 2) * (bw + 1) * 36 + (size_t)(bw + 2) * 6 + 2 * (size_t)(bw + 1) * 36 +
           2 * ((size_t)(bw + 1) * 36 + 6);
}

// (rcp_nr1, ltri, ldl6_inplace, ldl6_solve: plba_kernels.hpp, shared with the register-window band kernel)

// Eliminates block rows k0..k1-1 of an nrows-row band (g.nrows). The LDS window (row i in slot
// i mod (bw+2), block (i, i-w) row-major) is loaded for rows k0..k0+bw+1 when load_window is
// set, otherwise it is taken as left by a previous call (plus whatever the caller added to it).
// On return the critical wave's column k1 has been written back into the window, so the window
// holds rows k1..k1+bw-1 updated through step k1-1 (the separator of a two-sided elimination).
// `fail` is uniform on wave 0 (a zero pivot was met). The critical wave issues no global
// memory operation (no vmcnt waits on the chain); workers stream rows bw+2 steps ahead.
template <int BW>
__device__ __forceinline__ void cl_forward(const BandSeg &g, int k0, int k1, bool load_window, double *lds, bool &fail,
                                           unsigned long long *stamps = nullptr) {
    constexpr int W = BW + 1, W1 = BW + 2, NT = kClNT, NW = NT - 64, PD = kClPD;
    constexpr int XS = W * 36 + 6;                  // X buffer: W blocks + z
    constexpr int NPT6 = (BW - 1) * BW / 2 * 6;     // trailing (block pair, row) tasks
    constexpr int NRHS = (BW - 1) * 6;              // right-hand-side tasks
    constexpr int NROW = W * 36 + 6;                // block row streamed in per step
    constexpr int NFL = BW * 36 + 6;                // L blocks + z flushed per step
    constexpr int NWX = NW;
    static_assert(NPT6 + NRHS <= NWX && NROW <= NWX && NFL <= NWX, "one task of each kind per worker");
    static_assert(6 * W + 1 <= 64, "column lanes + rhs lane must fit one wave");
    const int nrows = g.nrows;
    double *win = lds, *bwin = win + W1 * W * 36, *preA = bwin + W1 * 6, *Xs = preA + 2 * W * 36;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wt = tid - 64;
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
        __syncthreads();
    }
    // ---- critical lanes: lane group cs <-> window rows i ≡ cs (mod W), scalar column cc; rhs lane
    const int cs = lane / 6, cc = lane % 6;
    const bool clane = crit && lane < 6 * W, rlane = crit && lane == 6 * W;
    int sk = k0 % W;        // lane group of the pivot block
    int lk = k0 % W1;       // LDS slot of row k
    double v[6];
    {
        int dw = cs - sk;
        if (dw < 0) dw += W;
        int li = lk + dw;
        if (li >= W1) li -= W1;
        const double *src = clane ? win + (li * W + dw) * 36 + cc * 6 : bwin + lk * 6;
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = src[r];  // rows past nrows are zero-filled
    }
    // ---- worker tasks (static per thread)
    int p_wi = 1 << 20, p_wj = 0, p_a = 0;          // trailing pair (k+wi, k+wj), row p_a
    if (!crit && wt < NPT6) {
        const int pr = wt / 6;
        int wi = 2;
        while ((wi - 1) * wi / 2 <= pr) ++wi;
        p_wi = wi;
        p_wj = 2 + pr - (wi - 2) * (wi - 1) / 2;
        p_a = wt % 6;
    }
    int r_wi = 1 << 20, r_a = 0;                    // rhs row k+r_wi, component r_a
    if (!crit && wt >= NPT6 && wt < NPT6 + NRHS) {
        r_wi = 2 + (wt - NPT6) / 6;
        r_a = (wt - NPT6) % 6;
    }
    const int fl = NWX - 1 - wt;                    // flush task (counted from the last worker)
    // ---- worker prefetch ring: block row k+2+bw for step k
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
#ifdef PLBA_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
    for (int kb = k0; kb < k1; kb += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const int k = kb + u;
            if (k >= k1) break;
            const int s1 = sk + 1 == W ? 0 : sk + 1;
            const int l1 = lk + 1 == W1 ? 0 : lk + 1;
            double *pA = preA + (u & 1) * W * 36, *X = Xs + (u & 1) * XS;
            if (crit) {
                // A: publish the pre-pivot column (workers: A_{j,k}; this wave: A_{k+1,k}). LDS
                // operations of one wave complete in order, so the read-back needs no wait.
                if (clane) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) pA[cs * 36 + cc * 6 + r] = v[r];
                }
                double a1[36];
                STAMP(0);
                // B: every lane factors S_k = A_{k,k} (the pivot group's just-published columns) in
                // its own registers and applies S_k⁻¹ to its own column (X_i = L_{i,k}ᵀ, z_k on the
                // rhs lane). Replaces a Gauss–Jordan across the lanes whose 72 v_readlane a step were
                // ~35 % of the step (tools/micro/cl_step.hip): the real kernel's forward step
                // 2,360 -> 2,200 cycles (phase stamps, C3).
                {
                    double s[21], dv[6];
                    const double *Sk = pA + sk * 36;  // entry (r, c) at [c * 6 + r]
#pragma unroll
                    for (int i = 0; i < 6; ++i)
#pragma unroll
                        for (int j = 0; j <= i; ++j) s[ltri(i, j)] = Sk[j * 6 + i];
                    bool zp = false;
                    ldl6_inplace(s, dv, zp);
                    if (zp) fail = true;
                    ldl6_solve(s, dv, v);
                }
                // A_{k+1,k} only feeds E/F: read after the Gauss–Jordan, so B does not wait for
                // 18 broadcast reads (C and the barrier cover their latency; the sched_barrier
                // keeps the scheduler from sinking them to their use): step 2,696 -> 2,570 cycles
#pragma unroll
                for (int q = 0; q < 36; ++q) a1[q] = pA[s1 * 36 + q];
                __builtin_amdgcn_sched_barrier(0);
                STAMP(1);
                // C: publish X_i = L_{i,k}ᵀ (lane 6s+c holds row c of L_{i,k}) and z_k
                if (clane && cs != sk) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) X[cs * 36 + cc * 6 + r] = v[r];
                }
                if (cs == sk) {  // identity columns: the pivot group takes the new bottom block in E/F
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = 0.0;
                }
                if (rlane) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) X[W * 36 + r] = v[r];
                }
                STAMP(2);
                lds_barrier();
                STAMP(3);
                // E/F: column k+1 through step k. Lane group s now stands for row
                // i = k+1 + ((s - s1) mod W); the pivot's group takes the new bottom block
                // (k+1+bw, k+1), resident since the workers' previous step.
                if (k + 1 < nrows) {
                    // Unconditional loads (a predicated load is waited on by itself). Window rows
                    // past nrows are zero-filled and the pivot group's X was zeroed in C, so no
                    // masks: those lanes come out as o - 0 (the new bottom block) or 0.
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
                STAMP(4);
            } else {
                lds_barrier();
                STAMP(3);
                // block row k+2+bw enters slot lk (row k is consumed)
                if (wt < NROW) {
                    const double val = k + 2 + BW < nrows ? wpf[u] : 0.0;
                    if (wt < W * 36) win[lk * W * 36 + wt] = val;
                    else bwin[lk * 6 + (wt - W * 36)] = val;
                }
                prefetch(k + PD, wpf[u]);
                STAMP(4);
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
                STAMP(5);
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
                STAMP(6);
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
                STAMP(7);
            }
            sk = s1;
            lk = l1;
        }
    }
#ifdef PLBA_STAMPS
    if (stamps && (tid & 63) == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&stamps[(tid >> 6) * 8 + q], st_acc[q]);
#endif
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
    __syncthreads();
}

// separator window of a segment after k1 steps: rows k1..k1+bw-1, all W blocks, + rhs
template <int BW>
__device__ __forceinline__ void cl_store_sep(const double *lds, int k1, double *sep) {
    constexpr int W = BW + 1, W1 = BW + 2;
    const double *win = lds, *bwin = win + W1 * W * 36;
    for (int t = threadIdx.x; t < BW * W * 36; t += kClNT) {
        const int i = t / (W * 36), rem = t % (W * 36);
        sep[t] = win[((k1 + i) % W1) * W * 36 + rem];
    }
    for (int t = threadIdx.x; t < BW * 6; t += kClNT) sep[(size_t)BW * W * 36 + t] = bwin[((k1 + t / 6) % W1) * 6 + t % 6];
}

template <int BW>
__global__ __launch_bounds__(kClNT) void k_rcs_factor_band_cl(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int s_fail;
    if constexpr (BW >= 1 && BW <= kClMaxBW) {
        const BandSeg g{d.Bd, d.bs, d.Lband, nullptr, d.zb, d.nf, d.nf, nullptr};
        bool fail = false;
        cl_forward<BW>(g, 0, d.nf, true, lds, fail);
        if (diag_fail(d)) fail = true;
        if (threadIdx.x == 0) {
            s_fail = fail ? 1 : 0;
            *d.solve_okp = fail ? 0 : 1;
        }
        __syncthreads();
        if (!s_fail && threadIdx.x < 64) band_backward_rl<BW>(d.Lband, d.zb, d.nf, d.nf, nullptr, d.xp, false, d.nf, threadIdx.x);
        __syncthreads();
        pose_update_wg<kClNT>(d, s_fail != 0);  // applied even after a failed solve, with the previous x_p (A13)
    }
}

// Two-sided variant. Workgroup 0 eliminates the top segment (rows 0..m-1), workgroup 1 the
// block-reversed bottom segment (rows nf-1 .. m+bw); each publishes its separator window and its
// L / z rows. The workgroup that arrives second (last-arriver counter, no spin: MI355X_MICROARCH.md
// hand-off "counter form") takes over: it puts segment 0's separator window into its LDS window
// (already there when it is workgroup 0), adds the bottom segment's Schur contribution
// W1 - A_sep and keeps eliminating the bw separator rows as ordinary band steps (the separator
// is itself a band of width bw), so no dense separator solve is needed. Back substitution: the
// separator rows first (one wave), then both segments concurrently on two waves.
template <int BW>
__global__ __launch_bounds__(kClNT) void k_rcs_factor_twisted_cl(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int s_fail, s_last;
    if constexpr (BW >= 1 && BW <= kClMaxBW) {
        constexpr int W = BW + 1;
        const int seg = blockIdx.x, tid = threadIdx.x;
        const int m = d.tw_m, n1 = d.nf - BW - d.tw_m;
        const size_t sep_stride = (size_t)BW * W * 36 + (size_t)BW * 6;
        double *sep0 = d.tw_sep, *sep1 = d.tw_sep + sep_stride;
        bool fail = false;
#if defined(PLBA_STAMPS) || defined(PLBA_PHASE_STAMPS)  // (phase marks alone: no per-step stamps)
        unsigned long long t0 = __builtin_readcyclecounter();
#define CL_MARK(q)                                                                       \
    do {                                                                                 \
        const unsigned long long t1 = __builtin_readcyclecounter();                      \
        if (tid == 0) atomicAdd(&d.stamps[16 * 8 + (q)], t1 - t0);                        \
        t0 = t1;                                                                         \
    } while (0)
#else
#define CL_MARK(q) do {} while (0)
#endif
        const BandSeg g = seg == 0 ? BandSeg{d.Bd, d.bs, d.Lband, nullptr, d.zb, m + BW, m, nullptr}
                                   : BandSeg{d.Bd2, d.bs2, d.Lband2, nullptr, d.zb2, n1 + BW, n1, nullptr};
        const int mine = seg == 0 ? m : n1;
        cl_forward<BW>(g, 0, mine, true, lds, fail, seg == 0 ? d.stamps : nullptr);
        CL_MARK(seg);
        cl_store_sep<BW>(lds, mine, seg == 0 ? sep0 : sep1);
        // the separator rows' original band A_sep (the merge subtracts it), loaded while the stores
        // drain, so the last arriver's merge takes one global round trip instead of two or three
        constexpr int NWIN = BW * W * 36, NWT = (NWIN + kClNT - 1) / kClNT;
        double a_sep[NWT], b_sep = 0.0;
#pragma unroll
        for (int u = 0; u < NWT; ++u) {
            const int t = tid + u * kClNT, i = t / (W * 36), rem = t % (W * 36), w = rem / 36;
            a_sep[u] = t < NWIN && w <= i ? d.Bd[((size_t)(m + i) * W + w) * 36 + rem % 36] : 0.0;
        }
        if (tid < BW * 6) b_sep = d.bs[(size_t)(m + tid / 6) * 6 + tid % 6];
        // hand-off: every wave drains its L / z / separator stores, one agent release by lane 0,
        // then the arrival counter; the workgroup whose add returns 1 is last and acquires once
        // before reading the other's data. Exactly two arrivals per launch (both workgroups pass
        // or both skip TRIAL_GUARD), so the last arriver resets the counter for the next launch.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_store(&d.tw_fail[seg], fail ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int old = __hip_atomic_fetch_add(d.tw_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == 1 ? 1 : 0;
            if (old == 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(d.tw_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
                s_fail = (__hip_atomic_load(&d.tw_fail[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                          __hip_atomic_load(&d.tw_fail[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 1 : 0;
            }
        }
        __syncthreads();
        if (!s_last) return;
        const BandSeg g0{d.Bd, d.bs, d.Lband, nullptr, d.zb, m + BW, m, nullptr};
        // merge: separator rows m+i of the top segment's window += the bottom segment's Schur
        // contribution (W1: its separator window, reversed numbering, blocks transposed) - A_sep.
        // As workgroup 1 the last arriver first takes segment 0's window (sep0) from global memory;
        // both loads go out in one round.
        {
            double *win = lds, *bwin = win + (BW + 2) * W * 36;
            const double *W1 = sep1;
            double w1v[NWT], s0v[NWT];
#pragma unroll
            for (int u = 0; u < NWT; ++u) {
                const int t = tid + u * kClNT, i = t / (W * 36), rem = t % (W * 36), w = rem / 36, e = rem % 36;
                const bool ok = t < NWIN && w <= i;
                const int j = i - w, a = e / 6, b = e % 6;
                w1v[u] = ok ? W1[((size_t)(BW - 1 - j) * W + w) * 36 + b * 6 + a] : 0.0;
                s0v[u] = seg == 1 && t < NWIN ? sep0[t] : 0.0;
            }
            double w1b = 0.0, s0b = 0.0;
            if (tid < BW * 6) {
                w1b = W1[(size_t)BW * W * 36 + (BW - 1 - tid / 6) * 6 + tid % 6];
                s0b = seg == 1 ? sep0[(size_t)BW * W * 36 + tid] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < NWT; ++u) {
                const int t = tid + u * kClNT, i = t / (W * 36), rem = t % (W * 36), w = rem / 36;
                if (t >= NWIN) continue;
                double *dst = win + ((m + i) % (BW + 2)) * W * 36 + rem;
                const double base = seg == 1 ? s0v[u] : *dst;
                *dst = w <= i ? base + (w1v[u] - a_sep[u]) : base;
            }
            if (tid < BW * 6) {
                double *dst = bwin + ((m + tid / 6) % (BW + 2)) * 6 + tid % 6;
                *dst = (seg == 1 ? s0b : *dst) + (w1b - b_sep);
            }
            if (seg == 1) {  // window rows m+bw, m+bw+1 (past the separator): zero, as segment 0 left them
                for (int t = tid; t < 2 * W * 36; t += kClNT) win[((m + BW + t / (W * 36)) % (BW + 2)) * W * 36 + t % (W * 36)] = 0.0;
                for (int t = tid; t < 2 * 6; t += kClNT) bwin[((m + BW + t / 6) % (BW + 2)) * 6 + t % 6] = 0.0;
            }
        }
        __syncthreads();
        CL_MARK(2);
        bool fail2 = false;
        cl_forward<BW>(g0, m, m + BW, false, lds, fail2);
        CL_MARK(3);
        if (tid == 0) {
            if (fail2 || diag_fail(d)) s_fail = 1;
            *d.solve_okp = s_fail ? 0 : 1;
        }
        __syncthreads();
        if (!s_fail) {
            double *xl = lds + cl_lds_doubles(BW);       // [nf][6] x_p staging
            double *xsr = lds + (BW + 2) * W * 36 + (BW + 2) * 6;  // reversed separator x (preA is free now)
            if (tid < 64)
                band_backward_rl<BW, true>(d.Lband + (size_t)m * W * 36, d.zb + (size_t)m * 6, BW, BW, nullptr,
                                           xl + (size_t)m * 6, false, d.nf, tid);
            __syncthreads();
            for (int t = tid; t < BW * 6; t += kClNT) xsr[t] = xl[(size_t)(m + BW - 1 - t / 6) * 6 + t % 6];
            __syncthreads();
            if (tid < 64) band_backward_rl<BW, true>(d.Lband, d.zb, m, m + BW, xl + (size_t)m * 6, xl, false, d.nf, tid);
            else if (tid < 128) band_backward_rl<BW, true>(d.Lband2, d.zb2, n1, n1 + BW, xsr, xl, true, d.nf, tid - 64);
            __syncthreads();
            for (int t = tid; t < d.nf * 6; t += kClNT) d.xp[t] = xl[t];
            CL_MARK(4);
            CL_MARK(5);  // (count: one unit of t1 - t0 ~ 0 is not a count; see stamp_diag.py)
        }
        __syncthreads();
        pose_update_wg<kClNT>(d, s_fail != 0);  // applied even after a failed solve, with the previous x_p (A13)
    }
}
