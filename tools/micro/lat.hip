// Microbenchmark (diagnostic only): basic latencies on one wave of gfx950, in s_memtime units.
//   fma    dependent v_fma_f64 chain
//   fma6   6 independent chains interleaved
//   rl     readlane -> dependent fma (uniform broadcast round trip)
//   lds1   ds_write + ds_read of the same address (one wave), dependent chain
//   lds18  18 broadcast ds_read_b128 (36 doubles), waited together
//   rcp    v_rcp_f64 + 1 Newton step, dependent chain
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

constexpr int N = 256;

__global__ void k(double *out, unsigned long long *t, double seed) {
    __shared__ double sh[4096];
    const int lane = threadIdx.x;
    double x = seed + lane * 1e-3, y = 1.0 + lane * 1e-6;
    for (int i = lane; i < 4096; i += 64) sh[i] = 1.0 + i * 1e-9;
    __syncthreads();
    unsigned long long t0, t1;
    // fma chain
    t0 = now();
#pragma unroll 16
    for (int i = 0; i < N; ++i) x = fma(x, y, 1e-9);
    t1 = now();
    if (lane == 0) t[0] = t1 - t0;
    // 6 interleaved chains
    double a[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) a[r] = x + r;
    t0 = now();
#pragma unroll 4
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int r = 0; r < 6; ++r) a[r] = fma(a[r], y, 1e-9);
    }
    t1 = now();
    if (lane == 0) t[1] = t1 - t0;
    // readlane round trip
    double z = a[0] + a[1] + a[2] + a[3] + a[4] + a[5];
    t0 = now();
#pragma unroll 16
    for (int i = 0; i < N; ++i) z = fma(readlane_f64(z, i & 63), y, 1e-9);
    t1 = now();
    if (lane == 0) t[2] = t1 - t0;
    // LDS write -> read (same address, same wave), dependent
    t0 = now();
#pragma unroll 8
    for (int i = 0; i < N; ++i) {
        sh[lane] = z;
        __builtin_amdgcn_sched_barrier(0);
        z = sh[(lane + 1) & 63] * y;
    }
    t1 = now();
    if (lane == 0) t[3] = t1 - t0;
    // 36 broadcast doubles
    double s = 0;
    t0 = now();
    for (int i = 0; i < N / 8; ++i) {
        double b[36];
        const int base = ((int)z & 7) * 36 + i;
#pragma unroll
        for (int q = 0; q < 36; ++q) b[q] = sh[base + q];
        double acc = 0;
#pragma unroll
        for (int q = 0; q < 36; ++q) acc += b[q];
        z = z * 1e-30 + acc;
    }
    t1 = now();
    if (lane == 0) t[4] = t1 - t0;
    // rcp + 1 NR, dependent
    double r = z + 3.0;
    t0 = now();
#pragma unroll 16
    for (int i = 0; i < N; ++i) {
        const double e = __builtin_amdgcn_rcp(r);
        r = fma(fma(-r, e, 1.0), e, e) + 1.5;
    }
    t1 = now();
    if (lane == 0) t[5] = t1 - t0;
    out[lane] = x + a[0] + a[5] + z + s + r;
}

int main() {
    double *out;
    unsigned long long *t;
    hipMalloc(&out, 64 * 8);
    hipMalloc(&t, 8 * 8);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, t, 1.0);
        hipDeviceSynchronize();
    }
    unsigned long long h[8];
    hipMemcpy(h, t, 8 * 8, hipMemcpyDeviceToHost);
    printf("per op (s_memtime units): fma-chain %.1f | 6 chains (per fma) %.2f | readlane->fma %.1f | "
           "lds write->read %.1f | 36 bcast reads+sum %.1f | rcp+nr1 %.1f\n",
           h[0] / (double)N, h[1] / (6.0 * N), h[2] / (double)N, h[3] / (double)N, h[4] / (N / 8.0), h[5] / (double)N);
    return 0;
}
