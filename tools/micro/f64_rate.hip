// Microbenchmark: FP64 VALU FMA throughput vs independent chains per lane and waves per SIMD
// (gfx950), plus v_mfma_f64_16x16x4_f64. One block per CU (256 blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int C>
__global__ void k_fma(double *out, int iters) {
    double x[C];
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = threadIdx.x * 1e-3 + j;
    const double a = 0.999999, b = 1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = fma(x[j], a, b);
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mfma(double *out, int iters) {
    d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, acc3, 0, 0, 0);
    }
    d4 s = acc0 + acc1 + acc2 + acc3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}
template <typename K>
double run(K k, int nt, int iters, double flop_per_thread_iter) {
    double *out;
    (void)hipMalloc(&out, 256 * 1024 * sizeof(double));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(256), dim3(nt), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    (void)hipFree(out);
    return 256.0 * nt * iters * flop_per_thread_iter / best / 1e9;
}
int main() {
    const int it = 20000;
    for (int nt : {256, 512, 1024}) {
        printf("threads/CU %4d (waves/SIMD %d): fma chains 8: %.1f  16: %.1f  32: %.1f TF   mfma(4 acc): %.1f TF\n", nt, nt / 256,
               run(k_fma<8>, nt, it, 16), run(k_fma<16>, nt, it / 2, 32), run(k_fma<32>, nt, it / 4, 64),
               run(k_mfma, nt, it / 4, 4.0 * 16 * 16 * 4 * 2 / 64));
    }
    return 0;
}
