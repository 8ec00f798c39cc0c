// barrier_bench.hip -- cost of a workgroup barrier vs workgroup size on
// gfx950 (feeds the chain kernel's design).
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 8192;

template <int T>
__global__ __launch_bounds__(T) void k_bar(long long *out) {
    __shared__ int x[T];
    x[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < kIters; ++it) {
        __builtin_amdgcn_s_barrier();
    }
    const long long t1 = clock64();
    int v = x[(threadIdx.x + 1) % T];
    for (int it = 0; it < kIters; ++it) {
        x[threadIdx.x] = v + it;
        __syncthreads();
        v = x[(threadIdx.x + 1) % T];
    }
    const long long t2 = clock64();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = t2 - t1 + (v & 1);
    }
}

template <int T>
void run(long long *d) {
    long long best[2] = {-1, -1};
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_bar<T>, dim3(1), dim3(T), 0, 0, d);
        long long h[2];
        (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        for (int k = 0; k < 2; ++k)
            if (best[k] < 0 || h[k] < best[k]) best[k] = h[k];
    }
    std::printf("threads %5d: s_barrier %6.1f cycles, LDS write + __syncthreads + read %6.1f cycles\n", T,
                (double)best[0] / kIters, (double)best[1] / kIters);
}

int main() {
    long long *d;
    (void)hipMalloc(&d, 2 * sizeof(long long));
    run<64>(d);
    run<128>(d);
    run<256>(d);
    run<512>(d);
    run<1024>(d);
    return 0;
}
