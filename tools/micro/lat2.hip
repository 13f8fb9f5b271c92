// Microbenchmark (diagnostic only): cost of broadcast patterns for the column-lane
// Gauss–Jordan of plba_band_cl.hpp, one wave, s_memtime units, chained on dependent data.
//   rl12    12 independent v_readlane_b32 (6 doubles from one lane) then 6 fma using them
//   gj      6-pivot column-lane GJ with readlane broadcast (as in cl_forward)
//   gjlds   6-pivot GJ with the pivot column broadcast through LDS
//   gjdpp   6-pivot GJ, pivot column by ds_bpermute (__shfl)
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ __forceinline__ double rcp_nr1(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(fma(-x, r, 1.0), r, r);
}

constexpr int N = 64;

__global__ void k(double *out, unsigned long long *t, int sk0) {
    __shared__ double sh[1024];
    const int lane = threadIdx.x;
    double v[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[r] = (lane % 6 == r ? 4.0 : 0.1) + 1e-3 * lane + 1e-4 * r;
    unsigned long long t0, t1;
    // rl12
    t0 = now();
    for (int i = 0; i < N; ++i) {
        const int l = (sk0 + i) & 63;
        double f[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) f[r] = readlane_f64(v[r], l);
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = fma(f[r], 1e-9, v[r]);
    }
    t1 = now();
    if (lane == 0) t[0] = t1 - t0;
    // gj (readlane)
    t0 = now();
    for (int i = 0; i < N; ++i) {
        const int sk = (sk0 + i) % 8;
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            const int pl = 6 * sk + p;
            double f[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) f[r] = readlane_f64(v[r], pl);
            const double rp = rcp_nr1(f[p]);
            const double mp = v[p] * rp;
#pragma unroll
            for (int r = 0; r < 6; ++r) v[r] = r == p ? mp : fma(-f[r], mp, v[r]);
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = v[r] * 0.5 + (lane % 6 == r ? 4.0 : 0.1);
    }
    t1 = now();
    if (lane == 0) t[1] = t1 - t0;
    // gj via LDS broadcast of the pivot column
    t0 = now();
    for (int i = 0; i < N; ++i) {
        const int sk = (sk0 + i) % 8;
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            const int pl = 6 * sk + p;
            if (lane == pl) {
#pragma unroll
                for (int r = 0; r < 6; ++r) sh[p * 8 + r] = v[r];
            }
            double f[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) f[r] = sh[p * 8 + r];
            const double rp = rcp_nr1(f[p]);
            const double mp = v[p] * rp;
#pragma unroll
            for (int r = 0; r < 6; ++r) v[r] = r == p ? mp : fma(-f[r], mp, v[r]);
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = v[r] * 0.5 + (lane % 6 == r ? 4.0 : 0.1);
    }
    t1 = now();
    if (lane == 0) t[2] = t1 - t0;
    // gj via pivot from readlane only (2 readlanes) + other 5 by LDS
    t0 = now();
    for (int i = 0; i < N; ++i) {
        const int sk = (sk0 + i) % 8;
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            const int pl = 6 * sk + p;
            const double fp = readlane_f64(v[p], pl);
            const double rp = rcp_nr1(fp);
            if (lane == pl) {
#pragma unroll
                for (int r = 0; r < 6; ++r) sh[p * 8 + r] = v[r];
            }
            double f[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) f[r] = r == p ? fp : sh[p * 8 + r];
            const double mp = v[p] * rp;
#pragma unroll
            for (int r = 0; r < 6; ++r) v[r] = r == p ? mp : fma(-f[r], mp, v[r]);
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = v[r] * 0.5 + (lane % 6 == r ? 4.0 : 0.1);
    }
    t1 = now();
    if (lane == 0) t[3] = t1 - t0;
    // uniform 6x6 LDLt-style inverse per lane from S held in every lane (36 values), then X = S^-1 v
    double S[36];
#pragma unroll
    for (int q = 0; q < 36; ++q) S[q] = (q % 7 == 0 ? 4.0 : 0.1) + 1e-5 * q;
    t0 = now();
    for (int i = 0; i < N; ++i) {
        double M[36];
#pragma unroll
        for (int q = 0; q < 36; ++q) M[q] = S[q] + 1e-9 * v[q % 6];
        // in-place GJ on the uniform copy, applied to v
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            const double rp = rcp_nr1(M[p * 6 + p]);
            const double vp = v[p] * rp;
            double row[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) row[c] = M[p * 6 + c] * rp;
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                if (r == p) continue;
                const double f = M[r * 6 + p];
#pragma unroll
                for (int c = p + 1; c < 6; ++c) M[r * 6 + c] = fma(-f, row[c], M[r * 6 + c]);
                v[r] = fma(-f, vp, v[r]);
            }
            v[p] = vp;
#pragma unroll
            for (int c = p + 1; c < 6; ++c) M[p * 6 + c] = row[c];
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = v[r] * 0.5 + (lane % 6 == r ? 4.0 : 0.1);
    }
    t1 = now();
    if (lane == 0) t[4] = t1 - t0;
    double s = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) s += v[r];
    out[lane] = s;
}

int main() {
    double *out;
    unsigned long long *t;
    (void)hipMalloc(&out, 64 * 8);
    (void)hipMalloc(&t, 8 * 8);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, t, 1);
        (void)hipDeviceSynchronize();
    }
    unsigned long long h[8];
    (void)hipMemcpy(h, t, 8 * 8, hipMemcpyDeviceToHost);
    printf("per iteration (s_memtime units): rl12+6fma %.1f | gj-readlane %.1f | gj-lds %.1f | gj-pivot-rl+lds %.1f | "
           "gj-uniform-copy %.1f\n",
           h[0] / (double)N, h[1] / (double)N, h[2] / (double)N, h[3] / (double)N, h[4] / (double)N);
    return 0;
}
