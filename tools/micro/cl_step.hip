// Microbenchmark (diagnostic only): where the column-lane factorisation's critical step spends
// its cycles. A copy of cl_forward's critical-wave loop (plba_band_cl.hpp) on a synthetic SPD band,
// one workgroup, with phases switched off by a knob mask (wrong results; timing only). The worker
// waves only take the barriers (their work does not change the step: DESIGN §4, NOWORK A/B).
//   1 no workgroup barrier (wave-local LDS sync)    2 no pre-pivot publish (a1 from a fixed block)
//   4 no X publish                                    8 no o loads (v reused)
//  16 a1 not re-read per step (constant registers)   32 Gauss-Jordan without readlane (lane-local f)
//  64 critical wave launched alone (64 threads)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../pl-slam-plucker_amd/csrc/plba_kernels.hpp"
using namespace plba;

template <int BW, int K>
__global__ __launch_bounds__(512) void k_clx(const double *Bd, int nsteps, double *out, unsigned long long *cyc) {
    constexpr int W = BW + 1, W1 = BW + 2, XS = W * 36 + 6;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double *win = lds, *bwin = win + W1 * W * 36, *preA = bwin + W1 * 6, *Xs = preA + 2 * W * 36;
    const int tid = threadIdx.x, lane = tid & 63, NT = blockDim.x;
    const bool crit = tid < 64;
    for (int t = tid; t < W1 * W * 36; t += NT) win[t] = Bd[t % (W * 36)];
    for (int t = tid; t < W1 * 6; t += NT) bwin[t] = 1.0;
    for (int t = tid; t < 2 * W * 36 + 2 * XS; t += NT) preA[t] = Bd[t % 36] * 0.01;
    __syncthreads();
    const int cs = lane / 6, cc = lane % 6;
    const bool clane = crit && lane < 6 * W, rlane = crit && lane == 6 * W;
    int sk = 0, lk = 0;
    double v[6];
    {
        const double *src = clane ? win + (cs * W + cs) * 36 + cc * 6 : bwin;
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = src[r];
    }
    double a1c[36];
#pragma unroll
    for (int q = 0; q < 36; ++q) a1c[q] = preA[q];
    bool fail = false;
    unsigned long long t0 = 0, t1 = 0;
    if (crit) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int kb = 0; kb < nsteps; kb += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = kb + u;
            if (k >= nsteps) break;
            const int s1 = sk + 1 == W ? 0 : sk + 1;
            const int l1 = lk + 1 == W1 ? 0 : lk + 1;
            double *pA = preA + (u & 1) * W * 36, *X = Xs + (u & 1) * XS;
            if (crit) {
                if (!(K & 2) && clane) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) pA[cs * 36 + cc * 6 + r] = v[r];
                }
                double a1[36];
                if constexpr ((K & 128) != 0) {  // lane-local LDLᵀ of S_k from the published column
                    double s[21], dv[6];
                    const double *Sk = pA + sk * 36;
#pragma unroll
                    for (int i = 0; i < 6; ++i)
#pragma unroll
                        for (int j = 0; j <= i; ++j) s[ltri(i, j)] = Sk[j * 6 + i];
                    if constexpr ((K & 512) != 0) {  // a1 loads issued with S_k's, under the factor
#pragma unroll
                        for (int q = 0; q < 36; ++q) a1[q] = pA[s1 * 36 + q];
                    }
                    bool zp = false;
                    ldl6_inplace(s, dv, zp);
                    if (zp) fail = true;
                    ldl6_solve(s, dv, v);
                } else
#pragma unroll
                for (int p = 0; p < 6; ++p) {
                    const int pl = 6 * sk + p;
                    double f[6];
#pragma unroll
                    for (int r = 0; r < 6; ++r) f[r] = (K & 32) ? v[r] : readlane_f64(v[r], pl);
                    if (f[p] == 0.0) fail = true;
                    const double rp = rcp_nr1(f[p]);
                    const double mp = v[p] * rp;
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = r == p ? mp : fma(-f[r], mp, v[r]);
                }
                if constexpr ((K & 256) != 0) {  // X published before the a1 loads
                    if (clane && cs != sk) {
#pragma unroll
                        for (int r = 0; r < 6; ++r) X[cs * 36 + cc * 6 + r] = v[r];
                    }
                    if (rlane) {
#pragma unroll
                        for (int r = 0; r < 6; ++r) X[W * 36 + r] = v[r];
                    }
                }
                if constexpr ((K & 512) == 0) {
#pragma unroll
                    for (int q = 0; q < 36; ++q) a1[q] = (K & 16) ? a1c[q] : pA[s1 * 36 + q];
                }
                __builtin_amdgcn_sched_barrier(0);
                if (!(K & (4 | 256))) {
                    if (clane && cs != sk) {
#pragma unroll
                        for (int r = 0; r < 6; ++r) X[cs * 36 + cc * 6 + r] = v[r];
                    }
                    if (rlane) {
#pragma unroll
                        for (int r = 0; r < 6; ++r) X[W * 36 + r] = v[r];
                    }
                }
                if (cs == sk) {
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = 0.0;
                }
                if (K & (1 | 64)) wave_lds_sync();
                else lds_barrier();
                {
                    int dw = cs - s1;
                    if (dw < 0) dw += W;
                    int li = l1 + dw;
                    if (li >= W1) li -= W1;
                    const double *src = clane ? win + (li * W + dw) * 36 + cc * 6 : bwin + l1 * 6;
                    double o[6];
#pragma unroll
                    for (int r = 0; r < 6; ++r) o[r] = (K & 8) ? v[r] * 0.5 + 1.0 : src[r];
                    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int m = 0; m < 6; ++m)
#pragma unroll
                        for (int r = 0; r < 6; ++r) acc[r] = fma(a1[r * 6 + m], v[m], acc[r]);
#pragma unroll
                    for (int r = 0; r < 6; ++r) v[r] = o[r] - 1e-3 * acc[r];
                }
            } else if (!(K & 1)) {
                lds_barrier();
            }
            sk = s1;
            lk = l1;
        }
    }
    if (crit) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (crit) out[lane] = v[0] + v[5] + (fail ? 1.0 : 0.0);
    if (tid == 0) cyc[0] = t1 - t0;
}

template <int K>
void run(const double *Bd, double *out, unsigned long long *cyc, int nsteps, const char *name) {
    constexpr int BW = 7;
    const size_t lds = cl_lds_doubles(BW) * sizeof(double);
    hipFuncSetAttribute((const void *)k_clx<BW, K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int nt = (K & 64) ? 64 : 512;
    unsigned long long c = 0;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((k_clx<BW, K>), dim3(1), dim3(nt), lds, 0, Bd, nsteps, out, cyc);
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    }
    printf("%-44s %7.1f cycles/step\n", name, (double)c / nsteps);
}

int main() {
    constexpr int BW = 7, W = BW + 1;
    std::vector<double> h(W * 36);
    for (int w = 0; w < W; ++w)
        for (int e = 0; e < 36; ++e) h[w * 36 + e] = (w == 0 && e / 6 == e % 6) ? 10.0 : 0.01 * ((e * 7 + w) % 5);
    double *Bd, *out;
    unsigned long long *cyc;
    (void)hipMalloc(&Bd, h.size() * sizeof(double));
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&cyc, 8);
    (void)hipMemcpy(Bd, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice);
    const int n = 96;
    run<0>(Bd, out, cyc, n, "copy of cl_forward's critical step");
    run<1>(Bd, out, cyc, n, "- barrier");
    run<2>(Bd, out, cyc, n, "- pre-pivot publish");
    run<4>(Bd, out, cyc, n, "- X publish");
    run<8>(Bd, out, cyc, n, "- o loads");
    run<16>(Bd, out, cyc, n, "- a1 loads");
    run<32>(Bd, out, cyc, n, "- readlanes");
    run<64>(Bd, out, cyc, n, "critical wave alone (64 threads)");
    run<1 | 2 | 4>(Bd, out, cyc, n, "- barrier - publishes");
    run<1 | 2 | 4 | 8 | 16>(Bd, out, cyc, n, "- barrier - publishes - loads");
    run<1 | 2 | 4 | 8 | 16 | 32>(Bd, out, cyc, n, "arithmetic only");
    run<128>(Bd, out, cyc, n, "lane-local LDLT pivot (PLBA_CL_LL)");
    run<128 | 4>(Bd, out, cyc, n, "lane-local LDLT pivot - X publish");
    run<128 | 1 | 2 | 4 | 8 | 16>(Bd, out, cyc, n, "lane-local LDLT, arithmetic only");
    run<256>(Bd, out, cyc, n, "GJ, X published before the a1 loads");
    run<128 | 256>(Bd, out, cyc, n, "LL, X published before the a1 loads");
    run<128 | 512>(Bd, out, cyc, n, "LL, a1 loads with S_k's");
    run<128 | 512 | 256>(Bd, out, cyc, n, "LL, a1 with S_k, X before barrier");
    return 0;
}
