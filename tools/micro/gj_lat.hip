// Microbenchmark (diagnostic only): latency of the 6x6 Gauss-Jordan inverse on one wave,
// the scalar-pivot form (gj_inverse6) vs alternatives, chained 64 times on dependent data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../pl-slam-plucker_amd/csrc/plba_kernels.hpp"
using namespace plba;

__device__ __forceinline__ double readlane_f64(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

__device__ __forceinline__ double gj_inverse6_b3(double M, int lane, bool &fail) {
    const bool mat = lane < 36, rhs = lane >= 36 && lane < 42;
    const int r = mat ? lane / 6 : (rhs ? lane - 36 : 0);
    const int c = mat ? lane % 6 : 0;
    double I = (mat && r == c) ? 1.0 : (rhs ? M : 0.0);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int b = 3 * p;
        double Mp[3], Ip[3], Mr[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            Mp[j] = __shfl(M, (b + j) * 6 + c, 64);
            Ip[j] = __shfl(I, rhs ? 36 + b + j : (b + j) * 6 + c, 64);
            Mr[j] = __shfl(M, r * 6 + b + j, 64);
        }
        double P[3][3];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int e = 0; e < 3; ++e) P[a][e] = readlane_f64(M, (b + a) * 6 + b + e);
        const double a00 = fma(P[1][1], P[2][2], -P[1][2] * P[2][1]);
        const double a01 = fma(P[0][2], P[2][1], -P[0][1] * P[2][2]);
        const double a02 = fma(P[0][1], P[1][2], -P[0][2] * P[1][1]);
        const double a10 = fma(P[1][2], P[2][0], -P[1][0] * P[2][2]);
        const double a11 = fma(P[0][0], P[2][2], -P[0][2] * P[2][0]);
        const double a12 = fma(P[0][2], P[1][0], -P[0][0] * P[1][2]);
        const double a20 = fma(P[1][0], P[2][1], -P[1][1] * P[2][0]);
        const double a21 = fma(P[0][1], P[2][0], -P[0][0] * P[2][1]);
        const double a22 = fma(P[0][0], P[1][1], -P[0][1] * P[1][0]);
        const double det = fma(P[0][0], a00, fma(P[0][1], a10, P[0][2] * a20));
        if (det == 0.0) fail = true;
        const double id = rcp_nr(det);
        const double Q[3][3] = {{a00 * id, a01 * id, a02 * id}, {a10 * id, a11 * id, a12 * id},
                                {a20 * id, a21 * id, a22 * id}};
        double nM[3], nI[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            nM[j] = fma(Q[j][0], Mp[0], fma(Q[j][1], Mp[1], Q[j][2] * Mp[2]));
            nI[j] = fma(Q[j][0], Ip[0], fma(Q[j][1], Ip[1], Q[j][2] * Ip[2]));
        }
        const int rr = r - b;
        if (rr >= 0 && rr < 3) {
            M = rr == 0 ? nM[0] : (rr == 1 ? nM[1] : nM[2]);
            I = rr == 0 ? nI[0] : (rr == 1 ? nI[1] : nI[2]);
        } else {
            M = fma(-Mr[0], nM[0], fma(-Mr[1], nM[1], fma(-Mr[2], nM[2], M)));
            I = fma(-Mr[0], nI[0], fma(-Mr[1], nI[1], fma(-Mr[2], nI[2], I)));
        }
    }
    return I;
}

template <int V>
__global__ __launch_bounds__(64) void k_gj(double *out, unsigned long long *cyc, int reps) {
    const int lane = threadIdx.x;
    // SPD-ish matrix: diag dominant
    double M = 0.0;
    if (lane < 36) M = (lane / 6 == lane % 6) ? 4.0 + lane * 0.01 : 0.1 / (1 + lane);
    else if (lane < 42) M = 1.0 + lane;
    bool fail = false;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int r = 0; r < reps; ++r) {
        double I;
        if constexpr (V == 0) I = gj_inverse6(M, lane, fail);
        else if constexpr (V == 2) I = gj_inverse6_b3(M, lane, fail);
        else if constexpr (V == 3) { I = M;
#pragma unroll
            for (int u = 0; u < 16; ++u) I = fma(I, 1.0000001, 1e-9); }
        else if constexpr (V == 4) { I = M;
#pragma unroll
            for (int u = 0; u < 16; ++u) I = __shfl(I, (lane + 1) & 63, 64); }
        else if constexpr (V == 5) { I = M;
#pragma unroll
            for (int u = 0; u < 16; ++u) I = I * 0.5 + readlane_f64(I, 5); }
        else if constexpr (V == 6) { I = M;
#pragma unroll
            for (int u = 0; u < 16; ++u) I = rcp_nr(I); }
        else { I = M * 1.0000001; }
        // feed back (keep SPD): M' = I for the matrix lanes (inverse of SPD is SPD)
        M = I;
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[lane] = M + (fail ? 1 : 0);
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    double *out; unsigned long long *cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(unsigned long long));
    const int reps = 64;
    for (int it = 0; it < 3; ++it) {
        unsigned long long c;
        hipLaunchKernelGGL(k_gj<0>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("gj_inverse6 scalar: %.1f cycles/inverse\n", (double)c / reps);
        hipLaunchKernelGGL(k_gj<2>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("gj 3x3-block:       %.1f cycles/inverse\n", (double)c / reps);
        const char *nm[] = {"", "", "", "fma chain /16", "bpermute chain /16", "readlane chain /16", "rcp_nr chain /16"};
        for (int v = 3; v <= 6; ++v) {
            if (v == 3) hipLaunchKernelGGL(k_gj<3>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            if (v == 4) hipLaunchKernelGGL(k_gj<4>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            if (v == 5) hipLaunchKernelGGL(k_gj<5>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            if (v == 6) hipLaunchKernelGGL(k_gj<6>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%-20s %.1f cycles\n", nm[v], (double)c / reps / 16);
        }
        hipLaunchKernelGGL(k_gj<1>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("loop overhead:      %.1f cycles/iter\n", (double)c / reps);
    }
    return 0;
}
