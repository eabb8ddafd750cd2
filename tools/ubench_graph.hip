// ubench_graph.hip -- what a hipGraph replay costs against direct launches on this ROCm, for the
// micro-batch shape (gd_microbatch_run: two dependent kernels, then a stream synchronize).
// Empty-bodied kernels, so the numbers are launch + completion-signal overhead alone:
//   eager   K1<<<64 x 64>>>, K2<<<8 x 1024>>>, hipStreamSynchronize
//   graph   the same two launches captured once, hipGraphLaunch, hipStreamSynchronize
//   graph1  a one-node graph (K1 only) replayed, for the per-graph fixed cost
//   fusedE  one kernel, 64 x 1024, whose workgroups meet at a grid barrier (agent-scope ticket counter
//           in device memory) before workgroups 0..7 run a second phase -- the two launches as one
//   fusedG  the same kernel as a one-node graph
// Environment knobs of the runtime can be A/B'd around it (DEBUG_HIP_FORCE_GRAPH_QUEUES,
// DEBUG_CLR_GRAPH_PACKET_CAPTURE, ...).
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

// ticket barrier: every workgroup takes a ticket; the round's last ticket is a multiple of gridDim.x,
// so a launch waits until the counter reaches the end of its own round (co-resident grid: 64 workgroups).
// The spin is bounded so the grid always drains.
__device__ void grid_barrier(uint32_t* cnt) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);
        const uint32_t t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t end = (t / gridDim.x + 1) * gridDim.x;
        for (uint32_t it = 0; it < (1u << 24); ++it) {
            const uint32_t v = __hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if ((int32_t)(v - end) >= 0) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

__global__ void kf(uint32_t* p, uint32_t* cnt) {
    if (threadIdx.x == 0) p[2 + blockIdx.x] = blockIdx.x;   // phase 1 store
    grid_barrier(cnt);
    if (blockIdx.x >= 8) return;
    if (threadIdx.x == 0) p[1] += p[2 + 63 - blockIdx.x];   // phase 2 reads another workgroup's store
}

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
    CK(hipMalloc(&p, 4096));
    CK(hipMemset(p, 0, 4096));
    uint32_t* cnt = p + 512;
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
    hipGraph_t gf;
    hipGraphExec_t ef;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kf, dim3(64), dim3(1024), 0, s, p, cnt);
    CK(hipStreamEndCapture(s, &gf));
    CK(hipGraphInstantiate(&ef, gf, nullptr, nullptr, 0));
    timeit("eager", eager, s);
    timeit("graph", [&] { CK(hipGraphLaunch(e2, s)); }, s);
    timeit("eager1", [&] { hipLaunchKernelGGL(k1, dim3(64), dim3(64), 0, s, p); }, s);
    timeit("graph1", [&] { CK(hipGraphLaunch(e1, s)); }, s);
    timeit("fusedE", [&] { hipLaunchKernelGGL(kf, dim3(64), dim3(1024), 0, s, p, cnt); }, s);
    timeit("fusedG", [&] { CK(hipGraphLaunch(ef, s)); }, s);
    CK(hipGraphExecDestroy(ef));
    CK(hipGraphDestroy(gf));
    CK(hipGraphExecDestroy(e2));
    CK(hipGraphExecDestroy(e1));
    CK(hipGraphDestroy(g2));
    CK(hipGraphDestroy(g1));
    CK(hipFree(p));
    CK(hipStreamDestroy(s));
    return 0;
}
