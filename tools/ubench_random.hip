// ubench_random.hip -- the random-access ceiling k_route runs against.
// Reads one random 32-B slot (2 x 16-B loads) per lane from a table of T bytes,
// with and without a 24-B/lane key stream beside it, and a pure streaming copy
// for reference.  Prints GB/s of requested bytes and G requests/s.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_random.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// one random slot per message; optional 24-B key stream read (KEYS) and 9-B result write
template <bool KEYS>
__global__ void __launch_bounds__(256) k_probe(const uint4* __restrict__ table, unsigned long long slot_mask,
                                               const uint64_t* __restrict__ keys, uint32_t n,
                                               uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t h = mix(i * 2654435761u);
    if constexpr (KEYS) {
        const uint64_t* kp = keys + 3ull * i;
        h ^= (uint32_t)(kp[0] ^ kp[1] ^ kp[2]);
    }
    const unsigned long long s = mix(h) & slot_mask;
    const uint4 a = table[2 * s];
    const uint4 b = table[2 * s + 1];
    out[i] = a.x ^ a.y ^ b.z ^ b.w;
}

// XCD-regioned: workgroup b probes only region b % 8 of the table (one eighth, contiguous).  With
// workgroups dispatched round-robin over the 8 XCDs, each XCD's L2 then serves one region.
template <bool KEYS>
__global__ void __launch_bounds__(256) k_probe_region(const uint4* __restrict__ table, unsigned long long region_mask,
                                                      unsigned long long region_slots,
                                                      const uint64_t* __restrict__ keys, uint32_t n,
                                                      uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t h = mix(i * 2654435761u);
    if constexpr (KEYS) {
        const uint64_t* kp = keys + 3ull * i;
        h ^= (uint32_t)(kp[0] ^ kp[1] ^ kp[2]);
    }
    const unsigned long long s = (unsigned long long)(blockIdx.x & 7u) * region_slots + (mix(h) & region_mask);
    const uint4 a = table[2 * s];
    const uint4 b = table[2 * s + 1];
    out[i] = a.x ^ a.y ^ b.z ^ b.w;
}

__global__ void __launch_bounds__(256) k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n16) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) out[i] = in[i];
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
    const size_t sizes_mb[] = {4, 16, 64, 128, 512, 2048, 8192};
    std::printf("table_MB  keys  ms/launch  probe_GBps(32B)  atoms_GBps(64B)  Greq/s\n");
    for (size_t mb : sizes_mb) {
        const size_t bytes = mb << 20;
        uint4* table;
        CK(hipMalloc(&table, bytes));
        CK(hipMemset(table, 3, bytes));
        const unsigned long long slots = bytes / 32;
        for (int withKeys = 0; withKeys < 2; ++withKeys) {
            auto launch = [&] {
                if (withKeys) hipLaunchKernelGGL(k_probe<true>, dim3(n / 256), dim3(256), 0, 0, table, slots - 1, keys, n, out);
                else hipLaunchKernelGGL(k_probe<false>, dim3(n / 256), dim3(256), 0, 0, table, slots - 1, keys, n, out);
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
            std::printf("%8zu  %4d  %9.4f  %15.1f  %15.1f  %6.1f\n", mb, withKeys, ms, n * 32.0 / ms / 1e6,
                        n * 64.0 / ms / 1e6, n / ms / 1e6);
        }
        for (int withKeys = 0; withKeys < 2; ++withKeys) {       // XCD-regioned probes
            const unsigned long long rs = slots / 8;
            auto launch = [&] {
                if (withKeys)
                    hipLaunchKernelGGL(k_probe_region<true>, dim3(n / 256), dim3(256), 0, 0, table, rs - 1, rs, keys, n, out);
                else
                    hipLaunchKernelGGL(k_probe_region<false>, dim3(n / 256), dim3(256), 0, 0, table, rs - 1, rs, keys, n, out);
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
            std::printf("%8zu  %4d  %9.4f  %15.1f  %15.1f  %6.1f  xcd-regioned\n", mb, withKeys, ms,
                        n * 32.0 / ms / 1e6, n * 64.0 / ms / 1e6, n / ms / 1e6);
        }
        CK(hipFree(table));
    }
    // streaming copy reference (1 GiB in, 1 GiB out)
    const size_t cb = 1ull << 30;
    uint4 *a, *b;
    CK(hipMalloc(&a, cb));
    CK(hipMalloc(&b, cb));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, a, b, cb / 16);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, a, b, cb / 16);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    std::printf("stream copy 1 GiB: %.4f ms = %.1f GB/s (read+write)\n", ms, 2.0 * cb / ms / 1e6);
    return 0;
}
