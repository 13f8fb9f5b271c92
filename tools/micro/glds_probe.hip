// Probe: direct global->LDS loads issued by inline asm (global_load_lds_dwordx4 with M0 = LDS
// byte address), the form band_forward uses to stage entering band rows. Checks the LDS image
// is lane-linear (base + 16 * lane) for a buffer at a nonzero LDS offset and a partial wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(const double *g, double *out, int npieces) {
    __shared__ __attribute__((aligned(16))) double pad[40];
    __shared__ __attribute__((aligned(16))) double stg[2 * 300];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    pad[lane % 40] = 0.0;
    for (int i = threadIdx.x; i < 600; i += blockDim.x) stg[i] = -1.0;
    __syncthreads();
    const int p = wv * 64 + lane;
    if (wv * 64 < npieces && p < npieces) {
        const double *src = g + 2 * p;
        const unsigned dst = __builtin_amdgcn_readfirstlane(
            (unsigned)(size_t)(__attribute__((address_space(3))) double *)(stg + 300 + wv * 128));
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 600; i += blockDim.x) out[i] = stg[i] + 0.0 * pad[0];
}
int main() {
    const int np = 147;  // 294 doubles: 2 full waves + a partial one
    std::vector<double> h(1024);
    for (int i = 0; i < 1024; ++i) h[i] = 1000.0 + i;
    double *g, *o;
    hipMalloc(&g, 1024 * 8);
    hipMalloc(&o, 600 * 8);
    hipMemcpy(g, h.data(), 1024 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, g, o, np);
    std::vector<double> r(600);
    hipMemcpy(r.data(), o, 600 * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 600; ++i) {
        const double want = i < 300 ? -1.0 : (i - 300 < 2 * np ? 1000.0 + (i - 300) : -1.0);
        if (r[i] != want) { if (bad < 10) printf("mismatch at %d: %g want %g\n", i, r[i], want); ++bad; }
    }
    printf("glds probe: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
    return bad ? 1 : 0;
}
