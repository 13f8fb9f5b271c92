// Dense reduced camera system on many workgroups, trailing updates on the FP64 matrix cores.
//
// Windows whose envelope is wider than the band kernels hold (revisits / loop closures: poses
// a loop apart share landmarks) factorise the RCS S (n = 6·nf, column-major
// `Ad`, lower triangle) as a right-looking blocked LDLᵀ with 32×32 tiles, two launches per
// panel K (captured in the step graph like every other kernel):
//   k_dense_panel<K>   one workgroup per row tile I >= K: LDLᵀ of the diagonal tile S_KK in LDS
//                      (every workgroup redundantly — 32 steps, cheaper than a third launch),
//                      then W_IK = S_IK·L_KK⁻ᵀ (= L_IK·D_K) and L_IK = W_IK·D_K⁻¹ (I > K);
//   k_dense_update<K>  one wave per trailing tile (I, J), K < J <= I: S_IJ -= W_IK·L_JKᵀ with
//                      v_mfma_f64_16x16x4_f64 (2×2 blocks of 16×16, eight k-steps of 4), W and
//                      L staged through LDS with coalesced loads.
// Then k_dense_solve: forward / backward substitution through the factor (one workgroup,
// envelope-aware) and the pose update — the tail of the single-workgroup k_rcs_factor.
// Semantics of LinearSolverEigen (SimplicialLDLT): the solve fails iff a pivot is exactly 0;
// later panels then skip their work and x_p keeps its previous value (A13).
// MFMA operand layout (cdna_hip_programming.md §3): A lane l -> A[l&15][k=l>>4],
// B lane l -> B[k=l>>4][l&15]; C/D (f64 form) reg i -> row (l>>4)+4i, col l&15.
#pragma once

typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int kDT = 32;          // tile
constexpr int kDensePanelNT = 256;

// LDLᵀ of the kb×kb lower tile T (in LDS, padded rows) in place: strict lower T[r][c] = L·D
// (not yet divided), diagonal = D. Returns false on a zero pivot.
template <int NT>
__device__ __forceinline__ bool dense_tile_ldlt(double (*T)[kDT + 1], int kb, int *s_fail) {
    const int tid = threadIdx.x;
    for (int j = 0; j < kb; ++j) {
        __syncthreads();
        const double djj = T[j][j];
        if (djj == 0.0) {
            if (tid == 0) *s_fail = 1;
        } else {
            for (int e = tid; e < kDT * kDT; e += NT) {
                const int r = e / kDT, c = e % kDT;
                if (r > j && c > j && c <= r && r < kb) T[r][c] -= (T[r][j] / djj) * T[c][j];
            }
        }
    }
    __syncthreads();
    return *s_fail == 0;
}

__global__ __launch_bounds__(kDensePanelNT) void k_dense_panel(Dev d, int K) {
    TRIAL_GUARD
    if (K > 0 && d.ctrl->solve_ok == 0) return;  // an earlier panel hit a zero pivot
    __shared__ double T[kDT][kDT + 1];
    __shared__ double A[kDT][kDT + 1];
    __shared__ double Dk[kDT];
    __shared__ int s_fail;
    const int tid = threadIdx.x, n = d.n;
    const int I = K + blockIdx.x;
    const int k0 = K * kDT, kb = min(kDT, n - k0);
    const int i0 = I * kDT, ib = min(kDT, n - i0);
    double *Ad = d.Ad;
    if (tid == 0) s_fail = 0;
    for (int e = tid; e < kDT * kDT; e += kDensePanelNT) {  // column-major source: c outer, r inner
        const int c = e / kDT, r = e % kDT;
        T[r][c] = (r < kb && c <= r) ? Ad[(size_t)(k0 + r) + (size_t)(k0 + c) * n] : 0.0;
        if (I > K) A[r][c] = (r < ib && c < kb) ? Ad[(size_t)(i0 + r) + (size_t)(k0 + c) * n] : 0.0;
    }
    const bool ok = dense_tile_ldlt<kDensePanelNT>(T, kb, &s_fail);
    if (blockIdx.x == 0) {
        if (tid == 0 && (K == 0 || !ok)) d.ctrl->solve_ok = ok ? 1 : 0;
        if (!ok) return;
        for (int e = tid; e < kDT * kDT; e += kDensePanelNT) {  // L (strict lower) and D
            const int c = e / kDT, r = e % kDT;
            if (r < kb && c <= r)
                Ad[(size_t)(k0 + r) + (size_t)(k0 + c) * n] = r == c ? T[r][r] : T[r][c] / T[c][c];
        }
        return;
    }
    if (!ok) return;
    if (tid < kDT) Dk[tid] = tid < kb ? T[tid][tid] : 1.0;
    __syncthreads();
    // W = A·L⁻ᵀ row by row (L unit lower: L[c][p] = T[c][p]/D_p), 8 threads per row: thread q of
    // row r owns columns c ≡ q (mod 8); column c needs W[r][p<c] — kept in LDS (A is overwritten)
    const int r = tid / 8, q = tid % 8;
    for (int c = 0; c < kb; ++c) {
        if (r < ib && (c & 7) == q) {
            double w = A[r][c];
            for (int p = 0; p < c; ++p) w -= A[r][p] * (T[c][p] / Dk[p]);
            A[r][c] = w;
        }
        __syncthreads();
    }
    for (int e = tid; e < kDT * kDT; e += kDensePanelNT) {
        const int c = e / kDT, rr = e % kDT;
        if (rr < ib && c < kb) {
            const double w = A[rr][c];
            Ad[(size_t)(i0 + rr) + (size_t)(k0 + c) * n] = w / Dk[c];  // L_IK
            d.Wbuf[(size_t)(i0 + rr) * kTile + c] = w;                // W_IK = L_IK·D_K
        }
    }
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
    if (d.ctrl->solve_ok == 0) return;
    __shared__ double Ws[kDT][kDT + 1];  // W_IK rows
    __shared__ double Ls[kDT][kDT + 1];  // L_JK rows
    const int lane = threadIdx.x, n = d.n;
    int I, J;
    dense_tile_of(blockIdx.x, K, I, J);
    const int k0 = K * kDT, kb = min(kDT, n - k0);
    const int i0 = I * kDT, j0 = J * kDT;
    const double *Ad = d.Ad;
    // stage: W rows (row-major Wbuf, coalesced along p) and L_JK (column-major Ad, coalesced along rows)
    for (int e = lane; e < kDT * kDT; e += 64) {
        const int rr = e / kDT, p = e % kDT;
        Ws[rr][p] = (i0 + rr < n && p < kb) ? d.Wbuf[(size_t)(i0 + rr) * kTile + p] : 0.0;
        const int pc = e / kDT, jr = e % kDT;
        Ls[jr][pc] = (j0 + jr < n && pc < kb) ? Ad[(size_t)(j0 + jr) + (size_t)(k0 + pc) * n] : 0.0;
    }
    __syncthreads();
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
    double *Aw = d.Ad;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = i0 + 16 * bi + lk + 4 * i, col = j0 + 16 * bj + lr;
                if (row < n && col < n && col <= row) Aw[(size_t)row + (size_t)col * n] -= acc[bi][bj][i];
            }
}

// forward / backward substitution through the dense factor + pose update (one workgroup)
__global__ __launch_bounds__(kFacThreads) void k_dense_solve(Dev d) {
    TRIAL_GUARD
    if (d.ctrl->solve_ok) dense_solve_wg(d);
    __syncthreads();
    pose_update_wg<kFacThreads>(d);  // applied even after a failed solve, with the previous x_p (A13)
}
