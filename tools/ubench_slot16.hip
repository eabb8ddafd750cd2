// ubench_slot16.hip -- does a 16-B slot directory probe faster than the 32-B one?  One random
// probe per message into a table of T bytes (slot index by multiply-high range reduction, so
// T need not be a power of two), 32-B slots (2 x 16-B loads) vs 16-B slots (1 load), with the
// 24-B key stream beside it.  1M grains at load 0.5 = 64 MB (32 B) / 32 MB (16 B); at load
// 0.7 = 46 MB / 23 MB.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_slot16.hip -o /tmp/ub16 && /tmp/ub16
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

template <int SLOT>
__global__ void __launch_bounds__(256) k_probe(const uint4* __restrict__ table, uint32_t slots,
                                               const uint64_t* __restrict__ keys, uint32_t n,
                                               uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t* kp = keys + 3ull * i;
    const uint32_t h = mix(mix(i * 2654435761u) ^ (uint32_t)(kp[0] ^ kp[1] ^ kp[2]));
    const uint32_t s = (uint32_t)(((uint64_t)h * slots) >> 32);
    uint32_t r;
    if constexpr (SLOT == 32) {
        const uint4 a = table[2ull * s];
        const uint4 b = table[2ull * s + 1];
        r = a.x ^ a.y ^ b.z ^ b.w;
    } else {
        const uint4 a = table[s];
        r = a.x ^ a.y ^ a.z ^ a.w;
    }
    out[i] = r;
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
    const size_t sizes_mb[] = {16, 23, 32, 46, 64};
    uint4* table;
    CK(hipMalloc(&table, 64ull << 20));
    CK(hipMemset(table, 3, 64ull << 20));
    std::printf("table_MB  slot_B  ms/launch  Gprobe/s\n");
    for (size_t mb : sizes_mb) {
        for (int slot : {32, 16}) {
            const uint32_t slots = (uint32_t)((mb << 20) / slot);
            auto launch = [&] {
                if (slot == 32) hipLaunchKernelGGL(k_probe<32>, dim3(n / 256), dim3(256), 0, 0, table, slots, keys, n, out);
                else hipLaunchKernelGGL(k_probe<16>, dim3(n / 256), dim3(256), 0, 0, table, slots, keys, n, out);
            };
            for (int w = 0; w < 3; ++w) launch();
            CK(hipEventRecord(e0));
            const int reps = 20;
            for (int r = 0; r < reps; ++r) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            std::printf("%8zu  %6d  %9.4f  %8.1f\n", mb, slot, ms, n / ms / 1e6);
        }
    }
    return 0;
}
