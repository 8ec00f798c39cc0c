// Host cost of issuing td_evaluate's three kernels (fill, search, ray sums) with a CellGrid-sized
// argument block, four ways: three hipLaunchKernelGGL calls; one hipGraphLaunch of the three captured
// as a graph; the graph with two of its kernel nodes' arguments updated per call
// (hipGraphExecKernelNodeSetParams, what a per-call grid geometry would need); and one launch.
// Per way: host issue time (the calls alone) and issue-to-done wall time (+ hipStreamSynchronize),
// medians over 2000 calls.  Build: hipcc --offload-arch=gfx950 -O2 tools/issue_cost.hip -o /tmp/issue_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                    \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

struct Geo {  // about the size of CellGrid
    double v[20];
    int g[8];
};

__global__ void k_a(Geo G, double *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = G.v[blockIdx.x % 20];
}
__global__ void k_b(Geo G, const double *in, double *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = in[blockIdx.x] + G.v[3];
}
__global__ void k_c(const double *in, double *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i % 2048];
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    double *a = nullptr, *b = nullptr, *c = nullptr;
    CHECK(hipMalloc(&a, 1 << 20));
    CHECK(hipMalloc(&b, 1 << 20));
    CHECK(hipMalloc(&c, 1 << 20));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Geo G{};
    const int reps = 2000;
    auto three = [&](const Geo &g) {
        hipLaunchKernelGGL(k_a, dim3(20), dim3(256), 0, s, g, a);
        hipLaunchKernelGGL(k_b, dim3(2106), dim3(256), 0, s, g, a, b);
        hipLaunchKernelGGL(k_c, dim3(96), dim3(256), 0, s, b, c, 381 * 64);
    };
    // graph of the same three
    hipGraph_t graph;
    hipGraphExec_t exec;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    three(G);
    CHECK(hipStreamEndCapture(s, &graph));
    CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    size_t nn = 0;
    CHECK(hipGraphGetNodes(graph, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    CHECK(hipGraphGetNodes(graph, nodes.data(), &nn));
    const char *names[] = {"3 launches", "graph", "graph + 2 node updates", "1 launch"};
    for (int way = 0; way < 4; ++way) {
        std::vector<double> issue, wall;
        for (int r = 0; r < reps + 100; ++r) {
            G.v[r % 20] = r;
            const double t0 = now_us();
            if (way == 0) {
                three(G);
            } else if (way == 1) {
                CHECK(hipGraphLaunch(exec, s));
            } else if (way == 2) {
                for (int k = 0; k < 2 && k < (int)nn; ++k) {
                    hipKernelNodeParams p{};
                    CHECK(hipGraphKernelNodeGetParams(nodes[k], &p));
                    CHECK(hipGraphExecKernelNodeSetParams(exec, nodes[k], &p));
                }
                CHECK(hipGraphLaunch(exec, s));
            } else {
                hipLaunchKernelGGL(k_b, dim3(2106), dim3(256), 0, s, G, a, b);
            }
            const double t1 = now_us();
            CHECK(hipStreamSynchronize(s));
            const double t2 = now_us();
            if (r >= 100) {
                issue.push_back(t1 - t0);
                wall.push_back(t2 - t0);
            }
        }
        std::printf("%-24s issue %.2f us, issue-to-done %.2f us\n", names[way], median(issue), median(wall));
    }
    return 0;
}
