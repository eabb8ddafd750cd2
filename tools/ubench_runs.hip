// ubench_runs.hip -- what a radix scatter's run length costs on MI355X, apart from its ranking.
// A tile of T consecutive 4-B elements (NT threads x IT items, read coalesced) is written as R
// digit runs of L = T / R elements, digit-major over the whole array (the layout of a uniform
// radix pass: digit d's runs of all tiles are contiguous, tile t's run of digit d at
// d * (n / R) + t * L).  Tiles go to XCD-contiguous ranges (workgroup b -> XCD b % 8), as the
// library's scatter maps them.  Prints us per 16M elements and GB/s (read + write) for each (T, R).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_runs.hip -o /tmp/ubench_runs && /tmp/ubench_runs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
    const uint32_t per = nb / 8u;
    return (nb % 8u == 0) ? (b % 8u) * per + b / 8u : b;
}

// Element p of the tile (in LDS order) belongs to digit p / L at offset p % L.  Each thread writes
// IT elements at p = j * NT + tid (consecutive lanes -> consecutive positions, as the library's
// staged write-out does).
template <int NT, int IT>
__global__ void __launch_bounds__(NT) k_runs(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t n,
                                             uint32_t R, uint32_t L) {
    constexpr uint32_t T = NT * IT;
    const uint32_t t = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t base = t * T;
    const uint32_t per_digit = n / R;
    uint32_t v[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) v[j] = __builtin_nontemporal_load(in + base + j * NT + threadIdx.x);
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t p = j * NT + threadIdx.x;
        const uint32_t d = p / L, o = p - d * L;
        out[(size_t)d * per_digit + (size_t)t * L + o] = v[j];
    }
}

template <int NT, int IT>
void run(const uint32_t* in, uint32_t* out, uint32_t n) {
    constexpr uint32_t T = NT * IT;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (uint32_t R = 64; R <= 4096 && T / R >= 1; R *= 2) {
        const uint32_t L = T / R;
        const uint32_t tiles = n / T;
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_runs<NT, IT>), dim3(tiles), dim3(NT), 0, 0, in, out, n, R, L);
        CK(hipEventRecord(a));
        const int reps = 20;
        for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((k_runs<NT, IT>), dim3(tiles), dim3(NT), 0, 0, in, out, n, R, L);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / reps;
        std::printf("tile %5u (%4d x %2d)  R %4u  run %5u el = %6u B   %7.1f us   %6.0f GB/s\n", T, NT, IT, R, L, L * 4,
                    us, 8.0 * n / (us * 1e-6) / 1e9);
    }
}

int main() {
    const uint32_t n = 1u << 24;
    uint32_t *in = nullptr, *out = nullptr;
    CK(hipMalloc(&in, (size_t)n * 4));
    CK(hipMalloc(&out, (size_t)n * 4));
    CK(hipMemset(in, 1, (size_t)n * 4));
    CK(hipMemset(out, 0, (size_t)n * 4));
    run<512, 8>(in, out, n);
    run<512, 16>(in, out, n);
    run<1024, 16>(in, out, n);
    run<1024, 32>(in, out, n);
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
