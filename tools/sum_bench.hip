// Cycle cost of the chi^2 tail sum variants on one wave (exact_sum.h):
// the one-lane loop, the run-per-scan loop and the chunked segmented sum.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../mcmc-in-tonga_amd/csrc/exact_sum.h"
using namespace tdstar;

__global__ void k(const double *t, int cnt, double C0, double *out, long long *cyc, double *res, int mode, int reps) {
    __shared__ double lt[1024], lo[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < cnt; i += 64) lt[i] = t[i];
    __syncthreads();
    long long best = 1ll << 60;
    double C = 0.0;
    for (int r = 0; r < reps; ++r) {
        __syncthreads();
        const long long t0 = clock64();
        if (mode == 0) {
            if (lane == 0) {
                C = C0;
                for (int k = 0; k < cnt; ++k) { C = C + lt[k]; lo[k] = C; }
            }
        } else {
            bool st = false;
            C = wave_seq_sum(lt, cnt, C0, lo, lane, nullptr, &st);
        }
        __syncthreads();
        const long long t1 = clock64();
        best = min(best, t1 - t0);
    }
    if (lane == 0) { *cyc = best; *res = C; }
    for (int i = lane; i < cnt; i += 64) out[i] = lo[i];
}

int main() {
    srand(1);
    std::vector<double> base(381);
    for (auto &x : base) x = -36.0 * std::log((rand() + 1.0) / (RAND_MAX + 2.0));
    double *dt, *dout, *dres; long long *dcyc;
    (void)hipMalloc(&dt, 8 * 1024); (void)hipMalloc(&dout, 8 * 1024); (void)hipMalloc(&dres, 8); (void)hipMalloc(&dcyc, 8);
    for (int k0 : {0, 10, 100, 190, 300, 370}) {
        double C0 = 0.0;
        for (int i = 0; i < k0; ++i) C0 = C0 + base[i];
        const int cnt = 381 - k0;
        (void)hipMemcpy(dt, base.data() + k0, 8 * cnt, hipMemcpyHostToDevice);
        printf("k0 %3d cnt %3d C0 %9.1f:", k0, cnt, C0);
        double ref = 0;
        for (int mode = 0; mode < 2; ++mode) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dt, cnt, C0, dout, dcyc, dres, mode, 20);
            long long cyc; double res;
            (void)hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(&res, dres, 8, hipMemcpyDeviceToHost);
            if (mode == 0) ref = res;
            printf("  mode%d %6lld cyc%s", mode, cyc, res == ref ? "" : " MISMATCH");
        }
        printf("\n");
    }
    return 0;
}
