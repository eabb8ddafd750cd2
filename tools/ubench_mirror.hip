// ubench_mirror.hip -- what a compact probe table would buy k_route: 16M lookups of 1M grains
// (uniform), the 24-B key stream beside them, real linear-probe chains in aligned slot groups.
//   slot32 g2  the directory as built (32-B slots, 2-slot groups = one 64-B read a round, load 0.5)
//   slot16 g4  a 16-B-slot mirror {N1, act, meta} (4-slot groups = one 64-B read a round) at
//              several capacities (load 0.5 .. 0.8; home = multiply-shift, any capacity)
// Each lookup hashes its key, walks groups from the home group until the key or an empty slot,
// and writes act (4 B).  Tables are built on the host (same probe rule).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mirror.hip -o /tmp/umir && /tmp/umir
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__host__ __device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
__host__ __device__ __forceinline__ uint32_t khash(uint64_t n1) { return mix((uint32_t)n1 * 0x9E3779B1u ^ (uint32_t)(n1 >> 32)); }
__host__ __device__ __forceinline__ uint64_t home(uint32_t h, uint64_t cap, uint32_t grp) {
    return (((uint64_t)mix(h ^ 0x5bd1e995u) * cap) >> 32) & ~(uint64_t)(grp - 1);
}

// 32-B slots: {n0, n1, tcd, act, meta}; meta != 0 = live.
template <int G>
__global__ void __launch_bounds__(256) k_probe32(const uint4* __restrict__ tab, uint64_t cap,
                                                 const uint64_t* __restrict__ keys, uint32_t n,
                                                 uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[3ull * i], n1 = keys[3ull * i + 1], tcd = keys[3ull * i + 2];
    uint64_t s = home(khash(n1), cap, G);
    uint32_t act = 0xFFFFFFFFu;
    for (uint32_t r = 0; r < 64; ++r) {
        uint4 q[2 * G];
#pragma unroll
        for (int g = 0; g < 2 * G; ++g) q[g] = tab[2 * s + g];
        bool done = false;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint4 a = q[2 * g], b = q[2 * g + 1];
            if (!done) {
                if (b.w == 0) { done = true; }
                else if ((((uint64_t)a.y << 32) | a.x) == n0 && (((uint64_t)a.w << 32) | a.z) == n1 &&
                         (((uint64_t)b.y << 32) | b.x) == tcd) { act = b.z; done = true; }
            }
        }
        if (done) break;
        s += G;
        if (s >= cap) s = 0;
    }
    out[i] = act;
}

// 16-B slots: {n1, act, meta}; meta != 0 = live (type index / silo in meta).
template <int G>
__global__ void __launch_bounds__(256) k_probe16(const uint4* __restrict__ tab, uint64_t cap,
                                                 const uint64_t* __restrict__ keys, uint32_t n,
                                                 uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[3ull * i], n1 = keys[3ull * i + 1], tcd = keys[3ull * i + 2];
    uint64_t s = home(khash(n1), cap, G);
    uint32_t act = 0xFFFFFFFFu;
    const uint32_t want_meta = 1u | ((uint32_t)(tcd & 0xFF) << 8);
    for (uint32_t r = 0; r < 64; ++r) {
        uint4 q[G];
#pragma unroll
        for (int g = 0; g < G; ++g) q[g] = tab[s + g];
        bool done = false;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (!done) {
                if (q[g].w == 0) { done = true; }
                else if ((((uint64_t)q[g].y << 32) | q[g].x) == n1 && q[g].w == want_meta && n0 == 0) {
                    act = q[g].z;
                    done = true;
                }
            }
        }
        if (done) break;
        s += G;
        if (s >= cap) s = 0;
    }
    out[i] = act;
}

int main() {
    const uint32_t G = 1u << 20, n = 1u << 24;
    const uint64_t tcd = (3ull << 56) | 0x1234;
    std::vector<uint64_t> hk(3ull * n);
    srand(7);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t g = (uint32_t)(((uint64_t)rand() << 16 ^ rand()) % G);
        hk[3ull * i] = 0;
        hk[3ull * i + 1] = g;
        hk[3ull * i + 2] = tcd;
    }
    uint64_t* keys;
    uint32_t* out;
    CK(hipMalloc(&keys, 24ull * n));
    CK(hipMalloc(&out, 4ull * n));
    CK(hipMemcpy(keys, hk.data(), 24ull * n, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> ho(n);
    auto timeit = [&](const char* name, double mb, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipEventRecord(e0));
        for (int r = 0; r < 20; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(ho.data(), out, 4ull * n, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint32_t i = 0; i < n; ++i) bad += ho[i] != (uint32_t)hk[3ull * i + 1] + 7;
        std::printf("%-12s %6.1f MB  %8.4f ms  (%llu wrong)\n", name, mb, ms / 20, (unsigned long long)bad);
    };
    const dim3 grid(n / 256), blk(256);
    {   // 32-B slots, groups of 2, cap 2^21
        const uint64_t cap = 1ull << 21;
        std::vector<uint32_t> t(cap * 8, 0);
        for (uint32_t g = 0; g < G; ++g) {
            uint64_t s = home(khash(g), cap, 2);
            while (t[s * 8 + 7]) s = (s + 1) % cap;
            uint64_t* w = reinterpret_cast<uint64_t*>(&t[s * 8]);
            w[0] = 0; w[1] = g; w[2] = tcd;
            t[s * 8 + 6] = g + 7;
            t[s * 8 + 7] = 1;
        }
        uint4* d;
        CK(hipMalloc(&d, cap * 32));
        CK(hipMemcpy(d, t.data(), cap * 32, hipMemcpyHostToDevice));
        timeit("slot32 g2", cap * 32 / 1048576.0, [&] { hipLaunchKernelGGL((k_probe32<2>), grid, blk, 0, 0, d, cap, keys, n, out); });
        CK(hipFree(d));
    }
    for (double load : {0.5, 0.6, 0.67, 0.75, 0.8}) {
        const uint64_t cap = ((uint64_t)(G / load) + 3) & ~3ull;
        std::vector<uint32_t> t(cap * 4, 0);
        for (uint32_t g = 0; g < G; ++g) {
            uint64_t s = home(khash(g), cap, 4);
            while (t[s * 4 + 3]) s = (s + 1) % cap;
            t[s * 4 + 0] = g;
            t[s * 4 + 1] = 0;
            t[s * 4 + 2] = g + 7;
            t[s * 4 + 3] = 1u | ((uint32_t)(tcd & 0xFF) << 8);
        }
        uint4* d;
        CK(hipMalloc(&d, cap * 16));
        CK(hipMemcpy(d, t.data(), cap * 16, hipMemcpyHostToDevice));
        char name[32];
        std::snprintf(name, sizeof name, "slot16 g4 %.2f", load);
        timeit(name, cap * 16 / 1048576.0, [&] { hipLaunchKernelGGL((k_probe16<4>), grid, blk, 0, 0, d, cap, keys, n, out); });
        CK(hipFree(d));
    }
    return 0;
}
