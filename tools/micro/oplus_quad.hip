// Diagnostic: orth_oplus + orth_to_pluker vs orth_oplus_quad on random lines (one quad per line).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../pl-slam-plucker_amd/csrc/plba_kernels.hpp"
using namespace plba;
__global__ void k(const double *D, const double *dD, double *o1, double *o2, int n) {
    const int gt = blockIdx.x * blockDim.x + threadIdx.x, l = gt / 4, q = gt % 4;
    if (l >= n) return;
    double a[4], b[4], X[4], L1[6], L2[6];
    for (int i = 0; i < 4; ++i) { a[i] = D[4 * l + i]; b[i] = dD[4 * l + i]; }
    orth_oplus(a, b, X);
    orth_to_pluker(X, L1);
    double xq = -1.0;
    for (int i = 0; i < 6; ++i) L2[i] = -1.0;
    if ((l % 3) != 0) {   // mixed "point" and "line" quads in one wave, divergent like k_lm_solve
        xq = orth_oplus_quad(a, b, q, L2);
    } else {
        xq = X[q];
        for (int i = 0; i < 6; ++i) L2[i] = L1[i];
    }
    o1[l * 10 + q] = X[q];
    o2[l * 10 + q] = xq;
    if (q == 0) for (int i = 0; i < 6; ++i) { o1[l * 10 + 4 + i] = L1[i]; o2[l * 10 + 4 + i] = L2[i]; }
}
int main() {
    const int n = 1000;
    double *D, *dD, *o1, *o2;
    hipMallocManaged(&D, n * 32); hipMallocManaged(&dD, n * 32);
    hipMallocManaged(&o1, n * 80); hipMallocManaged(&o2, n * 80);
    srand(1);
    for (int i = 0; i < 4 * n; ++i) { D[i] = (rand() / (double)RAND_MAX - 0.5) * 6.2; dD[i] = (rand() / (double)RAND_MAX - 0.5) * 2.0; }
    hipLaunchKernelGGL(k, dim3((4 * n + 255) / 256), dim3(256), 0, 0, D, dD, o1, o2, n);
    hipDeviceSynchronize();
    double m = 0; int at = -1;
    for (int i = 0; i < 10 * n; ++i) { double e = fabs(o1[i] - o2[i]); if (e > m) { m = e; at = i; } }
    printf("max |diff| %.3e at %d (line %d comp %d): %.17g vs %.17g\n", m, at, at / 10, at % 10, o1[at], o2[at]);
    return 0;
}
