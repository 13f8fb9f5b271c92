// Dense reduced camera system on many workgroups, trailing updates on the FP64 matrix cores.
//
// Windows whose envelope is wider than the band kernels hold (revisits / loop closures: poses
// a loop apart share landmarks) factorise the RCS S (n = 6·nf, column-major
// `Ad`, lower triangle) as a right-looking blocked LDLᵀ with 32×32 tiles, two launches per
// panel K (captured in the step graph like every other kernel):
//   k_dense_panel<K>   one wave per two row tiles I >= K: LDLᵀ of the diagonal tile S_KK in
//                      LDS (every workgroup redundantly — cheaper than a third launch),
//                      then W_IK = S_IK·L_KK⁻ᵀ (= L_IK·D_K) and L_IK = W_IK·D_K⁻¹ (I > K);
//   k_dense_update<K>  one wave per trailing tile (I, J), K < J <= I: S_IJ -= W_IK·L_JKᵀ with
//                      v_mfma_f64_16x16x4_f64 (2×2 blocks of 16×16, eight k-steps of 4), W and
//                      L staged through LDS with coalesced loads.
// Both launches cover only the envelope: row tiles up to tile_last[K], tiles whose row or column
// envelope starts after K skipped (they are exact zeros — LDLᵀ makes no fill outside the
// envelope), so an RCM-ordered matrix costs Σ_K (envelope height)² tiles, not (n/32)³/6.
// The forward substitution L y = b rides along: panel K solves y_K = L_KK⁻¹ b_K on its diagonal
// tile and the diagonal update tile (I, I) of step K subtracts L_IK·y_K from b_I (dense_yd).
// Then k_dense_solve: D⁻¹ and the backward substitution through the factor (one workgroup,
// envelope-aware) and the pose update — the tail of the single-workgroup k_rcs_factor.
// Semantics of LinearSolverEigen (SimplicialLDLT): the solve fails iff a pivot is exactly 0;
// later panels then skip their work and x_p keeps its previous value (A13).
// MFMA operand layout (cdna_hip_programming.md §3): A lane l -> A[l&15][k=l>>4],
// B lane l -> B[k=l>>4][l&15]; C/D (f64 form) reg i -> row (l>>4)+4i, col l&15.
#pragma once

constexpr int kDT = 32;            // tile
constexpr int kDensePanelNT = 64;  // one wave: two row tiles per workgroup
// PLBA_DIAG bit 8 (diagnostics only): phase timestamps of panel / update K = 5, workgroup 0
#define DENSE_STAMP(slot)                                                                                   \
    do {                                                                                                   \
        if ((d.diag & 8) && K == 5 && blockIdx.x == ((slot) < 8 ? 1u : 0u) && threadIdx.x == 0)           \
            d.bcr_stamps[slot] = __builtin_amdgcn_s_memrealtime();                                        \
    } while (0)

// One wave per pair of row tiles (I0 = K + 2·blockIdx.x, I1 = I0 + 1), everything in registers:
// lane l holds row l&31 of the diagonal tile S_KK and factorises it (every workgroup
// redundantly, right-looking, the pivot column broadcast with v_readlane), then row l&31 of the
// off-diagonal tile S_IK (I = I0 + (l>>5)) is solved against it, W = S_IK·L_KK⁻ᵀ by forward
// substitution along the row (L_KK entries broadcast the same way). Fully unrolled: register
// arrays need compile-time indices; no LDS, no barriers.
__global__ __launch_bounds__(kDensePanelNT) void k_dense_panel(Dev d, int K) {
    TRIAL_GUARD
    DENSE_STAMP(0);
    if (K > 0 && d.ctrl->solve_ok[0] == 0) return;  // an earlier panel hit a zero pivot
    DENSE_STAMP(1);
    const int lane = threadIdx.x, r = lane & 31, n = d.n;
    const int k0 = K * kDT, kb = min(kDT, n - k0);
    const int I = K + 2 * (int)blockIdx.x + (lane >> 5);
    const int i0 = I * kDT;
    double *Ad = d.Ad;
    // loads at clamped (always valid) addresses, selected after: no per-element branches
    double t[kDT];
    {
        const double *row = Ad + (size_t)(k0 + min(r, kb - 1)) + (size_t)k0 * n;
#pragma unroll
        for (int c = 0; c < kDT; ++c) t[c] = row[(size_t)min(c, kb - 1) * n];
    }
#pragma unroll
    for (int c = 0; c < kDT; ++c)  // row r, lower part; rows past kb are identity rows
        t[c] = (r < kb && c <= r) ? t[c] : (c == r ? 1.0 : 0.0);
    DENSE_STAMP(2);
    bool ok = true;
#pragma unroll
    for (int j = 0; j < kDT; ++j) {
        const double djj = readlane_f64(t[j], j);  // wave-uniform
        ok = ok && djj != 0.0;
        const double lrj = r > j ? t[j] * (1.0 / djj) : 0.0;
#pragma unroll
        for (int c = j + 1; c < kDT; ++c) {
            const double tcj = readlane_f64(t[j], c);
            if (r >= c) t[c] -= lrj * tcj;
        }
    }
    DENSE_STAMP(3);
    // t[p] (p < r) = L[r][p]·D_p -> L[r][p]; t[r] = D_r
    double D[kDT];
#pragma unroll
    for (int p = 0; p < kDT; ++p) D[p] = readlane_f64(t[p], p);
#pragma unroll
    for (int p = 0; p < kDT; ++p)
        if (p < r) t[p] = t[p] / D[p];
    if (blockIdx.x == 0) {
        if (lane == 0 && (K == 0 || !ok)) d.ctrl->solve_ok[0] = ok ? 1 : 0;
        if (ok && lane < 32 && r < kb) {
#pragma unroll
            for (int c = 0; c < kDT; ++c)
                if (c <= r) Ad[(size_t)(k0 + r) + (size_t)(k0 + c) * n] = t[c];
        }
        if (ok && lane < 32) {  // forward substitution of tile K: y_K = L_KK⁻¹ b_K
            double *yd = dense_yd(d);
            // (rows of tile K first touched here when its envelope starts at K)
            double yi = (d.tile_first[K] == K ? d.bs : yd)[k0 + min(r, kb - 1)];
#pragma unroll
            for (int j = 0; j < kDT; ++j) {
                const double yj = readlane_f64(yi, j);
                if (r > j && r < kb) yi -= t[j] * yj;
            }
            if (r < kb) yd[k0 + r] = yi;
        }
    }
    DENSE_STAMP(4);
    // row tiles outside the envelope of column tile K: S_IK = 0, so W_IK = L_IK = 0 (never read)
    if (!ok || I == K || I > d.tile_last[K] || d.tile_first[I] > K) return;
    const bool live = i0 + r < n;
    double a[kDT];
    {
        const double *row = Ad + (size_t)min(i0 + r, n - 1) + (size_t)k0 * n;
#pragma unroll
        for (int c = 0; c < kDT; ++c) a[c] = row[(size_t)min(c, kb - 1) * n];
    }
#pragma unroll
    for (int c = 0; c < kDT; ++c) a[c] = (live && c < kb) ? a[c] : 0.0;
#pragma unroll
    for (int c = 1; c < kDT; ++c)
#pragma unroll
        for (int p = 0; p < c; ++p) a[c] -= a[p] * readlane_f64(t[p], c);  // L[c][p]
    DENSE_STAMP(5);  // (the compiler sinks part of the solve past this stamp)
    if (!live) return;
    // W_IK = L_IK·D_K into Wbuf column-major ([kTile][n]: a lane per row, coalesced) and L_IK
#pragma unroll
    for (int c = 0; c < kDT; ++c)
        if (c < kb) {
            d.Wbuf[(size_t)c * n + i0 + r] = a[c];
            Ad[(size_t)(i0 + r) + (size_t)(k0 + c) * n] = a[c] / D[c];
        }
    DENSE_STAMP(6);
}

// trailing tile index t -> (I, J) with K < J <= I < nt, row-major over the lower triangle
__device__ __forceinline__ void dense_tile_of(int t, int K, int &I, int &J) {
    // t = (I'·(I'+1))/2 + J' with I' = I-K-1, J' = J-K-1
    int Ip = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((Ip + 1) * (Ip + 2) / 2 <= t) ++Ip;
    while (Ip * (Ip + 1) / 2 > t) --Ip;
    I = K + 1 + Ip;
    J = K + 1 + (t - Ip * (Ip + 1) / 2);
}

__global__ __launch_bounds__(64) void k_dense_update(Dev d, int K) {
    TRIAL_GUARD
    DENSE_STAMP(8);
    if (d.ctrl->solve_ok[0] == 0) return;
    __shared__ double Ws[kDT][kDT + 1];  // W_IK rows
    __shared__ double Ls[kDT][kDT + 1];  // L_JK rows
    const int lane = threadIdx.x, n = d.n;
    int I, J;
    dense_tile_of(blockIdx.x, K, I, J);
    // envelope: L_IK or L_JK is zero — nothing to subtract (the grid covers K < J <= I <= tile_last[K])
    if (d.tile_first[I] > K || d.tile_first[J] > K) return;
    const int k0 = K * kDT, kb = min(kDT, n - k0);
    const int i0 = I * kDT, j0 = J * kDT;
    const double *Ad = d.Ad;
    // stage W_IK (column-major Wbuf) and L_JK (column-major Ad) through LDS: all loads issued
    // first (clamped valid addresses, masked after)
    constexpr int NU = kDT * kDT / 64;
    double wv[NU], lv[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int e = lane + 64 * u, rr = e / kDT, p = e % kDT;  // W: (row rr, col p); L: (row p, col rr)
        // (row index e % kDT along the lanes: both sources are column-major, coalesced)
        wv[u] = d.Wbuf[(size_t)min(rr, kb - 1) * n + min(i0 + p, n - 1)];  // W[i0 + p][rr]
        lv[u] = Ad[(size_t)min(j0 + p, n - 1) + (size_t)(k0 + min(rr, kb - 1)) * n];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int e = lane + 64 * u, rr = e / kDT, p = e % kDT;
        Ws[p][rr] = (i0 + p < n && rr < kb) ? wv[u] : 0.0;
        Ls[p][rr] = (j0 + p < n && rr < kb) ? lv[u] : 0.0;
    }
    __syncthreads();
    DENSE_STAMP(9);
    dbl4 acc[2][2];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < kDT / 4; ++s) {
        const int p = 4 * s + lk;
        const double a0 = Ws[lr][p], a1 = Ws[16 + lr][p];   // A[row][k] = W[row][p]
        const double b0 = Ls[lr][p], b1 = Ls[16 + lr][p];   // B[k][col] = L[col][p]
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    DENSE_STAMP(10);
    if (I == J && lane < kDT && i0 + lane < n) {
        // forward substitution of rows I against tile K: y_I -= L_IK·y_K (Ls holds L_IK here),
        // summed in column order like the single-workgroup solve
        double *yd = dense_yd(d);
        double yk[kDT];
#pragma unroll
        for (int p = 0; p < kDT; ++p) yk[p] = yd[k0 + min(p, kb - 1)];
        double s = 0.0;
#pragma unroll
        for (int p = 0; p < kDT; ++p)
            if (p < kb) s += Ls[lane][p] * yk[p];
        yd[i0 + lane] = (K == d.tile_first[I] ? d.bs : yd)[i0 + lane] - s;  // first update of rows I
    }
    double *Aw = d.Ad;
    double cv[2][2][4];  // the 16 entries of C this lane updates: all loads, then all stores
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = i0 + 16 * bi + lk + 4 * i, col = j0 + 16 * bj + lr;
                cv[bi][bj][i] = Aw[(size_t)min(row, n - 1) + (size_t)min(col, n - 1) * n];
            }
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = i0 + 16 * bi + lk + 4 * i, col = j0 + 16 * bj + lr;
                if (row < n && col < n && col <= row) Aw[(size_t)row + (size_t)col * n] = cv[bi][bj][i] - acc[bi][bj][i];
            }
}

// forward / backward substitution through the dense factor + pose update (one workgroup)
__global__ __launch_bounds__(kFacThreads) void k_dense_solve(Dev d0) {
    TRIAL_SLOT(0)
    SOLVE_STAMP(12);
    const bool ok = *d.solve_okp != 0;
    if (ok) {  // forward substitution done by the panels / updates (dense_yd)
        if (d.n <= d.solve_lds_n) dense_solve_wg<true, true>(d);
        else dense_solve_wg<false, true>(d);
    }
    __syncthreads();
    SOLVE_STAMP(14);
    pose_update_wg<kFacThreads>(d, !ok);  // applied even after a failed solve, with the previous x_p (A13)
    SOLVE_STAMP(15);
}
