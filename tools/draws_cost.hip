// Diagnostic: cycles one wave spends on draw_iteration (the chain's 64-iteration
// draw refill, chain_kernels.hip) -- 64 lanes, one iteration each.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../mcmc-in-tonga_amd/csrc/chain_logic.h"

__global__ void k(unsigned long long seed, double *sink, long long *cyc) {
    const int lane = threadIdx.x;
    double acc = 0.0;
    long long t0 = clock64();
    for (int rep = 0; rep < 4; ++rep) {
        const tdchain::Draws d = tdchain::draw_iteration(seed + rep, 7, (uint64_t)(1000 + lane));
        acc += d.z_a + d.z_b + d.z_c + d.z_zeta + d.log_u + d.u_index;
    }
    long long t1 = clock64();
    sink[lane] = acc;
    if (lane == 0) cyc[0] = (t1 - t0) / 4;
}

int main() {
    double *sink;
    long long *cyc, h = 0;
    (void)hipMalloc(&sink, 64 * sizeof(double));
    (void)hipMalloc(&cyc, sizeof(long long));
    for (int i = 0; i < 3; ++i) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, 12345ull + i, sink, cyc);
        (void)hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("draw_iteration, one wave (64 iterations): %lld cycles\n", h);
    }
    return 0;
}
