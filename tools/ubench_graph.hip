// ubench_graph.hip -- what a hipGraph replay costs against direct launches on this ROCm, for the
// micro-batch shape (gd_microbatch_run: two dependent kernels, then a stream synchronize).
// Empty-bodied kernels, so the numbers are launch + completion-signal overhead alone:
//   eager   K1<<<64 x 64>>>, K2<<<8 x 1024>>>, hipStreamSynchronize
//   graph   the same two launches captured once, hipGraphLaunch, hipStreamSynchronize
//   graph1  a one-node graph (K1 only) replayed, for the per-graph fixed cost
// Prints p50 / p99 microseconds over 20,000 iterations each.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_graph.hip -o /tmp/ubench_graph && /tmp/ubench_graph
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void k1(uint32_t* p) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }
__global__ void k2(uint32_t* p) { if (p && threadIdx.x == 0 && blockIdx.x == 0) p[1] += 1; }

template <class F>
void timeit(const char* name, F f, hipStream_t s) {
    std::vector<double> us;
    for (int i = 0; i < 2000; ++i) f();
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < 20000; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        f();
        CK(hipStreamSynchronize(s));
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(us.begin(), us.end());
    std::printf("%-8s p50 %6.2f us   p99 %6.2f us\n", name, us[us.size() / 2], us[us.size() * 99 / 100]);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* p = nullptr;
    CK(hipMalloc(&p, 64));
    CK(hipMemset(p, 0, 64));
    auto eager = [&] {
        hipLaunchKernelGGL(k1, dim3(64), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k2, dim3(8), dim3(1024), 0, s, p);
    };
    hipGraph_t g2, g1;
    hipGraphExec_t e2, e1;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    eager();
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&e2, g2, nullptr, nullptr, 0));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k1, dim3(64), dim3(64), 0, s, p);
    CK(hipStreamEndCapture(s, &g1));
    CK(hipGraphInstantiate(&e1, g1, nullptr, nullptr, 0));
    timeit("eager", eager, s);
    timeit("graph", [&] { CK(hipGraphLaunch(e2, s)); }, s);
    timeit("eager1", [&] { hipLaunchKernelGGL(k1, dim3(64), dim3(64), 0, s, p); }, s);
    timeit("graph1", [&] { CK(hipGraphLaunch(e1, s)); }, s);
    CK(hipGraphExecDestroy(e2));
    CK(hipGraphExecDestroy(e1));
    CK(hipGraphDestroy(g2));
    CK(hipGraphDestroy(g1));
    CK(hipFree(p));
    CK(hipStreamDestroy(s));
    return 0;
}
