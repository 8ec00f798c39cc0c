// Round-trip latency of a host <-> resident-kernel mailbox, two placements of
// the host -> device command word:
//   A: pinned host memory (the kernel polls it across PCIe; what the td_evaluate server does today)
//   B: fine-grained device memory the host writes through the BAR (the kernel polls its own HBM)
// The answer always goes to pinned host memory (the host polls its own memory).
// A one-workgroup kernel echoes seq -> done; the host times N round trips.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mailbox_latency.hip -o /tmp/mailbox_latency
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
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

__device__ long long ld_sys(const long long *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ void st_sys(long long *p, long long v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// echo: wait for cmd[0] != last, write done = cmd[0]; quit on a negative seq or 2 s of silence.
// mode bit 0: s_sleep between polls; bit 1: after seeing the seq, read a 24-word payload in a
// second round trip (the chain server's command read); bit 2: write a result word and wait for
// its acknowledgment before done (the server's answer); bit 3: every poll reads the 24 words
__global__ void k_echo_full(const long long *cmd, long long *done, int mode) {
    const int lane = threadIdx.x;
    long long last = 0;
    long long t0 = (long long)wall_clock64();
    long long sink = 0;
    while (true) {
        long long w = 0;
        if (mode & 8) w = lane < 24 ? ld_sys(cmd + lane) : 0;
        else w = ld_sys(cmd);
        const long long s = __shfl(w, 0);
        if (s != last) {
            if (s < 0) break;
            last = s;
            if (mode & 2) {
                const long long p = lane < 24 ? ld_sys(cmd + lane) : 0;
                sink += p;
            }
            if (lane == 0) {
                if (mode & 4) {
                    st_sys(done + 2, s + sink);
                    __builtin_amdgcn_s_waitcnt(0);
                }
                st_sys(done, s);
            }
            t0 = (long long)wall_clock64();
            continue;
        }
        if ((long long)wall_clock64() - t0 > 200000000ll) break;
        if (mode & 1) __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0 && sink == 42) st_sys(done + 3, sink);
}

__global__ void k_echo(const long long *cmd, long long *done, int sleep_mode) {
    if (threadIdx.x != 0) return;
    long long last = 0;
    long long t0 = (long long)wall_clock64();
    while (true) {
        const long long s = ld_sys(cmd);
        if (s != last) {
            if (s < 0) return;
            last = s;
            st_sys(done, s);
            t0 = (long long)wall_clock64();
            continue;
        }
        if ((long long)wall_clock64() - t0 > 200000000ll) return;  // 2 s
        if (sleep_mode) __builtin_amdgcn_s_sleep(2);
    }
}

double run(long long *cmd_host_view, const long long *cmd_dev, long long *done_host, long long *done_dev, int n,
           int sleep_mode) {
    *(volatile long long *)cmd_host_view = 0;
    *(volatile long long *)done_host = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (sleep_mode >= 16) hipLaunchKernelGGL(k_echo_full, dim3(1), dim3(64), 0, 0, cmd_dev, done_dev, sleep_mode - 16);
    else hipLaunchKernelGGL(k_echo, dim3(1), dim3(64), 0, 0, cmd_dev, done_dev, sleep_mode);
    // warm
    for (int i = 1; i <= 100; ++i) {
        *(volatile long long *)cmd_host_view = i;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        while (*(volatile long long *)done_host != i) {}
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 101; i <= 100 + n; ++i) {
        *(volatile long long *)cmd_host_view = i;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        const auto ts = std::chrono::steady_clock::now();
        while (*(volatile long long *)done_host != i)
            if (std::chrono::steady_clock::now() - ts > std::chrono::seconds(1)) {
                std::printf("timeout\n");
                std::exit(2);
            }
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    *(volatile long long *)cmd_host_view = -1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    CHECK(hipDeviceSynchronize());
    return us;
}

int main() {
    long long *done_host = nullptr, *done_dev = nullptr;
    CHECK(hipHostMalloc(&done_host, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer((void **)&done_dev, done_host, 0));
    // A: command in pinned host memory
    long long *cmdA = nullptr, *cmdA_dev = nullptr;
    CHECK(hipHostMalloc(&cmdA, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer((void **)&cmdA_dev, cmdA, 0));
    for (int sm = 0; sm < 2; ++sm)
        std::printf("A pinned host command, sleep %d: %.3f us per round trip\n", sm,
                    run(cmdA, cmdA_dev, done_host, done_dev, 2000, sm));
    for (int mode : {16, 16 + 2, 16 + 4, 16 + 6, 16 + 8, 16 + 12})
        std::printf("A pinned host command, server-like mode %d (2: payload read, 4: acked result, 8: wide poll): %.3f us\n",
                    mode - 16, run(cmdA, cmdA_dev, done_host, done_dev, 2000, mode));
    // B: command in fine-grained device memory, written by the host
    long long *cmdB = nullptr;
    hipError_t e = hipExtMallocWithFlags((void **)&cmdB, 4096, hipDeviceMallocFinegrained);
    std::printf("fine-grained device alloc: %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
        hipPointerAttribute_t at{};
        CHECK(hipPointerGetAttributes(&at, cmdB));
        std::printf("  type %d host ptr %p dev ptr %p\n", (int)at.type, at.hostPointer, at.devicePointer);
        if (at.hostPointer)
            for (int sm = 0; sm < 2; ++sm)
                std::printf("B device command (host writes through the BAR), sleep %d: %.3f us per round trip\n", sm,
                            run((long long *)at.hostPointer, cmdB, done_host, done_dev, 2000, sm));
    }
    return 0;
}
