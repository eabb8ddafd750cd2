// ubench_probe_forms.hip -- forms of the directory probe's table read, alone (no hash, no ring,
// no compare): 16M messages with the 24-B key stream, one random slot group each, 64-MB table.
//   slot32     one 32-B slot per lane (2 x 16-B loads)                  -- route_m_core, group 1
//   grp64      the aligned 64-B pair per lane (4 x 16-B loads)            -- group 2
//   grp128     the aligned 128-B group per lane (8 x 16-B loads)          -- group 4
//   coop128    8-lane groups read each of their 8 messages' 128-B groups (one 16-B load a lane per
//              message, 8 loads a lane, all in flight)                     -- route_coop_core
// each also XCD-regioned (workgroup b probes region b % 8 of the table).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_probe_forms.hip -o /tmp/upf && /tmp/upf
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

__device__ __forceinline__ unsigned long long slot_of(uint32_t h, unsigned long long slots, bool region, uint32_t grp) {
    unsigned long long s;
    if (region) {
        const unsigned long long rs = slots / 8;
        s = (unsigned long long)(blockIdx.x & 7u) * rs + (mix(h) & (rs - 1));
    } else {
        s = mix(h) & (slots - 1);
    }
    return s & ~(unsigned long long)(grp - 1);
}

template <int G, bool REGION>
__global__ void __launch_bounds__(256) k_lane(const uint4* __restrict__ table, unsigned long long slots,
                                              const uint64_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t* kp = keys + 3ull * i;
    const uint32_t h = mix(i * 2654435761u) ^ (uint32_t)(kp[0] ^ kp[1] ^ kp[2]);
    const unsigned long long s = slot_of(h, slots, REGION, G);
    uint32_t acc = 0;
#pragma unroll
    for (int g = 0; g < 2 * G; ++g) {
        const uint4 v = table[2 * s + g];
        acc ^= v.x ^ v.w;
    }
    out[i] = acc;
}

template <bool REGION>
__global__ void __launch_bounds__(256) k_coop(const uint4* __restrict__ table, unsigned long long slots,
                                              const uint64_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, gb = lane & ~7u, t = lane & 7u;
    uint32_t h = 0;
    if (i < n) {
        const uint64_t* kp = keys + 3ull * i;
        h = mix(i * 2654435761u) ^ (uint32_t)(kp[0] ^ kp[1] ^ kp[2]);
    }
    const uint32_t s = (uint32_t)slot_of(h, slots, REGION, 4);
    uint4 q[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint32_t sr = __shfl(s, (int)(gb + r));
        q[r] = table[2ull * sr + t];
    }
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) acc ^= q[r].x ^ q[r].w;
    if (i < n) out[i] = acc;
}

int main() {
    const uint32_t n = 1u << 24;
    uint64_t* keys;
    uint32_t* out;
    CK(hipMalloc(&keys, 24ull * n));
    CK(hipMalloc(&out, 4ull * n));
    CK(hipMemset(keys, 1, 24ull * n));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (size_t mb : {16, 64, 256}) {
        const size_t bytes = mb << 20;
        uint4* table;
        CK(hipMalloc(&table, bytes));
        CK(hipMemset(table, 3, bytes));
        const unsigned long long slots = bytes / 32;
        auto run = [&](const char* name, auto launch) {
            for (int w = 0; w < 3; ++w) launch();
            CK(hipEventRecord(e0));
            for (int r = 0; r < 20; ++r) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("%5zu MB  %-16s %8.4f ms\n", mb, name, ms / 20);
        };
        const dim3 g(n / 256), b(256);
        run("slot32", [&] { hipLaunchKernelGGL((k_lane<1, false>), g, b, 0, 0, table, slots, keys, n, out); });
        run("grp64", [&] { hipLaunchKernelGGL((k_lane<2, false>), g, b, 0, 0, table, slots, keys, n, out); });
        run("grp128", [&] { hipLaunchKernelGGL((k_lane<4, false>), g, b, 0, 0, table, slots, keys, n, out); });
        run("coop128", [&] { hipLaunchKernelGGL((k_coop<false>), g, b, 0, 0, table, slots, keys, n, out); });
        run("slot32 region", [&] { hipLaunchKernelGGL((k_lane<1, true>), g, b, 0, 0, table, slots, keys, n, out); });
        run("grp64 region", [&] { hipLaunchKernelGGL((k_lane<2, true>), g, b, 0, 0, table, slots, keys, n, out); });
        run("grp128 region", [&] { hipLaunchKernelGGL((k_lane<4, true>), g, b, 0, 0, table, slots, keys, n, out); });
        run("coop128 region", [&] { hipLaunchKernelGGL((k_coop<true>), g, b, 0, 0, table, slots, keys, n, out); });
        CK(hipFree(table));
    }
    return 0;
}
