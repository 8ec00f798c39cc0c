// Cycle cost of the chi^2 tail sum variants (exact_sum.h), one workgroup:
// mode 0 the one-lane loop, mode 1 the one-wave scan (wave_seq_sum),
// mode 2 the workgroup-wide segmented scan (block_exact_sum, 256 threads).
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../mcmc-in-tonga_amd/csrc/exact_sum.h"
using namespace tdstar;

__global__ __launch_bounds__(256) void k(const double *t, int cnt, double C0, double *out, long long *cyc,
                                         double *res, int mode, int reps) {
    __shared__ double lt[1024], lo[1024];
    __shared__ ExactSumLds xs;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < cnt; i += 256) lt[i] = t[i];
    __syncthreads();
    long long best = 1ll << 60;
    double C = 0.0;
    int okc = 0;
    for (int r = 0; r < reps; ++r) {
        __syncthreads();
        const long long t0 = clock64();
        if (mode == 0) {
            if (tid == 0) {
                C = C0;
                for (int k = 0; k < cnt; ++k) { C = C + lt[k]; lo[k] = C; }
            }
        } else if (mode == 1) {
            if (tid < 64) {
                bool st = false;
                C = wave_seq_sum(lt, cnt, C0, lo, lane, nullptr, &st);
            }
        } else {
            okc += block_exact_sum<256>(lt, cnt, C0, lo, &C, xs) ? 1 : 0;
        }
        __syncthreads();
        const long long t1 = clock64();
        best = min(best, t1 - t0);
    }
    if (tid == 0) { *cyc = best; *res = mode == 2 && okc != reps ? -1.0 : C; }
    for (int i = tid; i < cnt; i += 256) out[i] = lo[i];
}

int main() {
    srand(1);
    std::vector<double> base(1000);
    for (auto &x : base) x = -36.0 * std::log((rand() + 1.0) / (RAND_MAX + 2.0));
    double *dt, *dout, *dres; long long *dcyc;
    (void)hipMalloc(&dt, 8 * 1024); (void)hipMalloc(&dout, 8 * 1024); (void)hipMalloc(&dres, 8); (void)hipMalloc(&dcyc, 8);
    for (int n : {381, 1000}) {
        for (int k0 : {0, 10, 100, 190, 300, 370}) {
            double C0 = 0.0;
            for (int i = 0; i < k0; ++i) C0 = C0 + base[i];
            const int cnt = n - k0;
            (void)hipMemcpy(dt, base.data() + k0, 8 * cnt, hipMemcpyHostToDevice);
            printf("n %4d k0 %3d cnt %4d C0 %9.1f:", n, k0, cnt, C0);
            double ref = 0;
            for (int mode = 0; mode < 3; ++mode) {
                hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, dt, cnt, C0, dout, dcyc, dres, mode, 20);
                long long cyc; double res;
                (void)hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
                (void)hipMemcpy(&res, dres, 8, hipMemcpyDeviceToHost);
                if (mode == 0) ref = res;
                printf("  mode%d %6lld cyc%s", mode, cyc, res == ref ? "" : (res == -1.0 ? " (no fast path)" : " MISMATCH"));
            }
            printf("\n");
        }
    }
    return 0;
}
