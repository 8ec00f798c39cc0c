// microbench.hip -- cost model of the primitives the persistent chain
// workgroup is built from (one 512-thread workgroup, like k_chain_run):
// barriers with and without pending stores, dependent L2 / LDS round trips,
// wave reductions.  Prints shader cycles per iteration (s_memtime).
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench.hip -o /tmp/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kT = 512;
constexpr int kIters = 4096;

__global__ __launch_bounds__(kT) void k_bench(int mode, int *chase, double *gbuf, long long *out) {
    __shared__ int lchase[1024];
    __shared__ double ldsd[kT];
    __shared__ int cnt;
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += kT) lchase[i] = (i * 97 + 13) & 1023;
    if (tid == 0) cnt = 0;
    __syncthreads();
    int idx = tid;
    double acc = tid;
    const long long t0 = clock64();
    for (int it = 0; it < kIters; ++it) {
        switch (mode) {
            case 0:  // barrier only
                __syncthreads();
                break;
            case 1:  // every thread stores to global, then barrier
                gbuf[it % 64 * kT + tid] = acc;
                __syncthreads();
                break;
            case 2:  // every thread stores to LDS, then barrier
                ldsd[tid] = acc;
                __syncthreads();
                acc += ldsd[(tid + 1) & (kT - 1)];
                break;
            case 3:  // tid 0: one dependent global load (L2-resident chase), then barrier
                if (tid == 0) idx = chase[idx];
                __syncthreads();
                break;
            case 4:  // tid 0: one dependent LDS load, then barrier
                if (tid == 0) idx = lchase[idx & 1023];
                __syncthreads();
                break;
            case 5:  // tid 0: 8 dependent global loads, no barrier
                if (tid == 0)
                    for (int k = 0; k < 8; ++k) idx = chase[idx];
                break;
            case 6:  // tid 0: 8 dependent LDS loads, no barrier
                if (tid == 0)
                    for (int k = 0; k < 8; ++k) idx = lchase[idx & 1023];
                break;
            case 7: {  // wave 0: 6-step double shfl_xor min reduction, no barrier
                if (tid < 64) {
                    for (int off = 32; off >= 1; off >>= 1) acc = fmin(acc, __shfl_xor(acc, off, 64));
                    acc += 1.0;
                }
                break;
            }
            case 8:  // LDS atomicAdd by every thread + barrier
                atomicAdd(&cnt, 1);
                __syncthreads();
                break;
            case 9:  // tid 0: 8 dependent FP64 adds
                if (tid == 0)
                    for (int k = 0; k < 8; ++k) acc = acc + 1.000001;
                break;
            case 10:  // tid 0: one global store + barrier (only one lane stores)
                if (tid == 0) gbuf[it % 64] = acc;
                __syncthreads();
                break;
            case 11:  // all threads: one independent global load each (L2), then barrier
                acc += gbuf[(it % 64) * kT + tid];
                __syncthreads();
                break;
        }
    }
    const long long t1 = clock64();
    if (tid == 0) out[0] = (t1 - t0) + (idx & 1) + (long long)(acc * 0.0);
    if (tid == 1) out[1] = (long long)acc;
}

int main() {
    int *chase;
    double *gbuf;
    long long *out;
    const int N = 1 << 16;
    std::vector<int> h(N);
    for (int i = 0; i < N; ++i) h[i] = (int)(((long long)i * 40503 + 977) % N);
    hipMalloc(&chase, sizeof(int) * N);
    hipMemcpy(chase, h.data(), sizeof(int) * N, hipMemcpyHostToDevice);
    hipMalloc(&gbuf, sizeof(double) * 64 * kT);
    hipMemset(gbuf, 0, sizeof(double) * 64 * kT);
    hipMalloc(&out, sizeof(long long) * 2);
    const char *names[] = {"barrier",
                           "global store/thread + barrier",
                           "LDS store/thread + barrier",
                           "tid0 dependent global load + barrier",
                           "tid0 dependent LDS load + barrier",
                           "tid0 dependent global load (x8, per load)",
                           "tid0 dependent LDS load (x8, per load)",
                           "wave0 6-step double shfl reduction",
                           "LDS atomicAdd/thread + barrier",
                           "tid0 dependent FP64 add (x8, per add)",
                           "tid0 global store + barrier",
                           "global load/thread (L2) + barrier"};
    for (int mode = 0; mode < 12; ++mode) {
        long long best = -1;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k_bench, dim3(1), dim3(kT), 0, 0, mode, chase, gbuf, out);
            long long r[2];
            hipMemcpy(r, out, sizeof r, hipMemcpyDeviceToHost);
            if (best < 0 || r[0] < best) best = r[0];
        }
        double per = (double)best / kIters;
        if (mode == 5 || mode == 6 || mode == 9) per /= 8.0;
        std::printf("%-45s %8.1f cycles\n", names[mode], per);
    }
    return 0;
}
