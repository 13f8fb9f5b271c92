// Microbenchmark (diagnostic only): latency of one block step of a lane-local banded LDLᵀ —
// every lane factors the 6x6 pivot block S_k in its own registers (no cross-lane traffic), lane
// (r, c) forms S_{k+1}[r][c] = A[r][c] - (L⁻¹a_r)ᵀ D⁻¹ (L⁻¹a_c), the 36 results go through LDS
// and every lane reads the new S back. Chained `reps` times on dependent data; compared with the
// primitive latencies it is built from.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double rcp_nr1(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(fma(-x, r, 1.0), r, r);
}
constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// lane-local LDLᵀ of the packed lower triangle s (unit L below the diagonal, dinv = 1/d)
__device__ __forceinline__ void ldl6(double (&s)[21], double (&dinv)[6], bool &fail) {
#pragma unroll
    for (int p = 0; p < 6; ++p) {
        const double dp = s[tri(p, p)];
        if (dp == 0.0) fail = true;
        const double rp = rcp_nr1(dp);
        dinv[p] = rp;
        double col[6];
#pragma unroll
        for (int i = p + 1; i < 6; ++i) col[i] = s[tri(i, p)];
#pragma unroll
        for (int i = p + 1; i < 6; ++i) s[tri(i, p)] = col[i] * rp;
#pragma unroll
        for (int i = p + 1; i < 6; ++i)
#pragma unroll
            for (int j = p + 1; j <= i; ++j) s[tri(i, j)] = fma(-s[tri(i, p)], col[j], s[tri(i, j)]);
    }
}
// u = L⁻¹a (unit lower L in s)
__device__ __forceinline__ void lsolve6(const double (&s)[21], const double *a, double (&u)[6]) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double v = a[i];
#pragma unroll
        for (int m = 0; m < i; ++m) v = fma(-s[tri(i, m)], u[m], v);
        u[i] = v;
    }
}

template <int NW>  // waves in the workgroup (1 = critical wave alone, else + idle workers at the barrier)
__global__ __launch_bounds__(64 * NW) void k_ll(double *out, unsigned long long *cyc, int reps) {
    __shared__ __attribute__((aligned(16))) double Sb[2][36], Ar[36], An[36];
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < 36) {
        const int r = tid / 6, c = tid % 6;
        Sb[0][tid] = r == c ? 4.0 + 0.1 * r : 0.2 / (1 + r + c);
        Ar[tid] = (r == c ? 0.5 : 0.05) / (1 + r);
        An[tid] = r == c ? 4.0 + 0.1 * r : 0.2 / (1 + r + c);
    }
    __syncthreads();
    const int r = lane < 36 ? lane / 6 : 0, c = lane < 36 ? lane % 6 : 0;
    bool fail = false;
    unsigned long long t0 = 0, t1 = 0;
    if (tid < 64) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int k = 0; k < reps; ++k) {
        const int par = k & 1;
        if (tid < 64) {
            double s[21], dinv[6], ar[6], ac[6], u[6], v[6];
            const double *S = Sb[par];
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) s[tri(i, j)] = S[i * 6 + j];
#pragma unroll
            for (int m = 0; m < 6; ++m) { ar[m] = Ar[r * 6 + m]; ac[m] = Ar[c * 6 + m]; }
            const double anrc = An[r * 6 + c];
            ldl6(s, dinv, fail);
            lsolve6(s, ar, u);
            lsolve6(s, ac, v);
            double acc = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) acc = fma(u[m] * dinv[m], v[m], acc);
            if (lane < 36) Sb[par ^ 1][lane] = anrc - acc;
        }
        if constexpr (NW == 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
    }
    if (tid < 64) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (tid < 36) out[tid] = Sb[reps & 1][tid] + (fail ? 1.0 : 0.0);
    if (tid == 0) cyc[0] = t1 - t0;
}

// two independent chains in one wave (the two segments of the two-sided elimination): how much of
// one chain's latency does the other chain's work fill?
__global__ __launch_bounds__(64) void k_ll2(double *out, unsigned long long *cyc, int reps) {
    __shared__ __attribute__((aligned(16))) double Sb[2][2][36], Ar[36], An[36];
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < 36) {
        const int r = tid / 6, c = tid % 6;
        Sb[0][0][tid] = Sb[1][0][tid] = r == c ? 4.0 + 0.1 * r : 0.2 / (1 + r + c);
        Ar[tid] = (r == c ? 0.5 : 0.05) / (1 + r);
        An[tid] = r == c ? 4.0 + 0.1 * r : 0.2 / (1 + r + c);
    }
    __syncthreads();
    const int r = lane < 36 ? lane / 6 : 0, c = lane < 36 ? lane % 6 : 0;
    bool fail = false;
    unsigned long long t0 = 0, t1 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int k = 0; k < reps; ++k) {
        const int par = k & 1;
        double s[2][21], dinv[2][6], ar[6], ac[6], u[2][6], v[2][6];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) s[h][tri(i, j)] = Sb[h][par][i * 6 + j];
#pragma unroll
        for (int m = 0; m < 6; ++m) { ar[m] = Ar[r * 6 + m]; ac[m] = Ar[c * 6 + m]; }
        const double anrc = An[r * 6 + c];
#pragma unroll
        for (int h = 0; h < 2; ++h) ldl6(s[h], dinv[h], fail);
#pragma unroll
        for (int h = 0; h < 2; ++h) { lsolve6(s[h], ar, u[h]); lsolve6(s[h], ac, v[h]); }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            double acc = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) acc = fma(u[h][m] * dinv[h][m], v[h][m], acc);
            if (lane < 36) Sb[h][par ^ 1][lane] = anrc - acc;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (tid < 36) out[tid] = Sb[0][reps & 1][tid] + Sb[1][reps & 1][tid] + (fail ? 1.0 : 0.0);
    if (tid == 0) cyc[0] = t1 - t0;
}

__device__ __forceinline__ double rl64(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// the column-lane step of plba_band_cl.hpp (cross-lane Gauss-Jordan on pivot lanes 0..5, then
// v <- o - a1·v with a1, o from LDS), H independent chains interleaved in one wave
template <int H>
__global__ __launch_bounds__(64) void k_gj(double *out, unsigned long long *cyc, int reps) {
    __shared__ __attribute__((aligned(16))) double A1[36], O[64 * 6];
    const int lane = threadIdx.x;
    if (lane < 36) A1[lane] = (lane / 6 == lane % 6 ? 0.3 : 0.01);
    for (int r = 0; r < 6; ++r) O[lane * 6 + r] = (lane % 6 == r ? 4.0 : 0.1);
    __syncthreads();
    double v[H][6];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
        for (int r = 0; r < 6; ++r) v[h][r] = O[lane * 6 + r] + 0.01 * h;
    bool fail = false;
    unsigned long long t0 = 0, t1 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int k = 0; k < reps; ++k) {
#pragma unroll
        for (int p = 0; p < 6; ++p) {
#pragma unroll
            for (int h = 0; h < H; ++h) {
                double f[6];
#pragma unroll
                for (int r = 0; r < 6; ++r) f[r] = rl64(v[h][r], p);
                fail = fail || f[p] == 0.0;
                const double rp = rcp_nr1(f[p]);
                const double mp = v[h][p] * rp;
#pragma unroll
                for (int r = 0; r < 6; ++r) v[h][r] = r == p ? mp : fma(-f[r], mp, v[h][r]);
            }
        }
        double a1[36], o[6];
#pragma unroll
        for (int q = 0; q < 36; ++q) a1[q] = A1[q];
#pragma unroll
        for (int r = 0; r < 6; ++r) o[r] = O[lane * 6 + r];
#pragma unroll
        for (int h = 0; h < H; ++h) {
            double acc[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < 6; ++m)
#pragma unroll
                for (int r = 0; r < 6; ++r) acc[r] = fma(a1[r * 6 + m], v[h][m], acc[r]);
#pragma unroll
            for (int r = 0; r < 6; ++r) v[h][r] = o[r] - acc[r];
        }
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    double sum = 0.0;
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
        for (int r = 0; r < 6; ++r) sum += v[h][r];
    out[lane] = sum + (fail ? 1.0 : 0.0);
    if (lane == 0) cyc[0] = t1 - t0;
}

// primitive latencies, 64 dependent repetitions each
template <int V>
__global__ __launch_bounds__(64) void k_prim(double *out, unsigned long long *cyc, int reps) {
    __shared__ double buf[128];
    const int lane = threadIdx.x;
    double x = 1.0 + lane * 1e-3;
    buf[lane] = x;
    __syncthreads();
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int k = 0; k < reps; ++k) {
        if constexpr (V == 0) x = fma(x, 1.0000001, 1e-9);          // dependent fma
        else if constexpr (V == 1) x = rcp_nr1(x) + 0.5;            // rcp + Newton
        else if constexpr (V == 2) {                                // LDS write -> read round trip
            buf[(lane + k) & 63] = x;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            x = buf[(lane + 1 + k) & 63] * 1.0000001;
        }
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[lane] = x;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(unsigned long long));
    const int reps = 256;
    for (int it = 0; it < 3; ++it) {
        unsigned long long c;
        hipLaunchKernelGGL(k_ll<1>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("lane-local step, 1 wave:        %.1f cycles/step\n", (double)c / reps);
        hipLaunchKernelGGL(k_ll<8>, dim3(1), dim3(512), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("lane-local step, 8 waves + bar: %.1f cycles/step\n", (double)c / reps);
        hipLaunchKernelGGL(k_ll2, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("two chains in one wave:         %.1f cycles/double step\n", (double)c / reps);
        hipLaunchKernelGGL(k_gj<1>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("column-lane GJ step, 1 chain:   %.1f cycles/step\n", (double)c / reps);
        hipLaunchKernelGGL(k_gj<2>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("column-lane GJ step, 2 chains:  %.1f cycles/double step\n", (double)c / reps);
        const char *nm[] = {"dependent fma", "rcp_nr1 + add", "LDS write->read"};
        for (int v = 0; v < 3; ++v) {
            if (v == 0) hipLaunchKernelGGL(k_prim<0>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            if (v == 1) hipLaunchKernelGGL(k_prim<1>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            if (v == 2) hipLaunchKernelGGL(k_prim<2>, dim3(1), dim3(64), 0, 0, out, cyc, reps);
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%-31s %.1f cycles\n", nm[v], (double)c / reps);
        }
    }
    double h[36];
    hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    printf("S[0][0] after chain: %.6f (finite check)\n", h[0]);
    return 0;
}
