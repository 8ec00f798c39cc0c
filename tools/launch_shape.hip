// Dispatch cost of a launch shape with no work: how long an empty kernel of
// B workgroups x T threads with D bytes of dynamic LDS takes (HIP events over
// back-to-back launches), to separate k_nn_tile's fixed cost at config 3 from
// its scan.  Build: hipcc --offload-arch=gfx950 -O2 tools/launch_shape.hip -o tools/launch_shape
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                    \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

// touches its LDS once so the allocation is real; writes one word per workgroup
__global__ void k_empty(int *out) {
    extern __shared__ int lds[];
    lds[threadIdx.x] = (int)threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = lds[blockDim.x - 1];
}

// the same plus a global round trip per thread (a staging load) before the barrier
__global__ void k_load(const double *in, int *out) {
    extern __shared__ int lds[];
    lds[threadIdx.x] = (int)in[blockIdx.x * blockDim.x + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = lds[blockDim.x - 1];
}

int main() {
    int *out = nullptr;
    double *in = nullptr;
    CHECK(hipMalloc(&out, 1 << 20));
    CHECK(hipMalloc(&in, 64 << 20));
    CHECK(hipMemset(in, 0, 64 << 20));
    CHECK(hipFuncSetAttribute((const void *)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute((const void *)k_load, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    struct Shape { int blocks, threads, lds; };
    const Shape shapes[] = {{1, 64, 4096},        {1, 1024, 4096},      {256, 1024, 83 * 1024},
                            {256, 1024, 4096},    {1024, 256, 4096},    {1024, 256, 40 * 1024},
                            {2048, 128, 4096},    {512, 512, 4096},     {256, 512, 83 * 1024}};
    for (int kind = 0; kind < 2; ++kind)
        for (const Shape &s : shapes) {
            for (int w = 0; w < 20; ++w) {
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(s.blocks), dim3(s.threads), s.lds, 0, out);
                else hipLaunchKernelGGL(k_load, dim3(s.blocks), dim3(s.threads), s.lds, 0, in, out);
            }
            CHECK(hipDeviceSynchronize());
            const int n = 200;
            float ms_one = 0.0f;
            double sum_one = 0.0;
            for (int i = 0; i < n; ++i) {  // one launch between two events (the bench's measurement)
                CHECK(hipEventRecord(a, 0));
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(s.blocks), dim3(s.threads), s.lds, 0, out);
                else hipLaunchKernelGGL(k_load, dim3(s.blocks), dim3(s.threads), s.lds, 0, in, out);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                CHECK(hipEventElapsedTime(&ms_one, a, b));
                sum_one += ms_one;
            }
            CHECK(hipEventRecord(a, 0));
            for (int i = 0; i < n; ++i) {
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(s.blocks), dim3(s.threads), s.lds, 0, out);
                else hipLaunchKernelGGL(k_load, dim3(s.blocks), dim3(s.threads), s.lds, 0, in, out);
            }
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0.0f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            std::printf("%s blocks %5d x %4d threads, LDS %6d B: %.2f us alone, %.2f us back to back\n",
                        kind ? "load " : "empty", s.blocks, s.threads, s.lds, sum_one / n * 1e3, ms / n * 1e3);
        }
    return 0;
}
