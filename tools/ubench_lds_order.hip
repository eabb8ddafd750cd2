// Does one ds_add_rtn_u32 wave instruction serve lanes that hit the same LDS address in
// ascending lane order?  If so, `old = atomicAdd(&cnt[digit], 1)` is a stable in-wave rank
// (what k_radix_scatter computes with ballots today).  Checks TRIALS random digit patterns per
// wave for several digit widths, 8 waves per block, and counts mismatches against the stable
// rank (number of lower lanes with the same digit, plus the counter's prior value).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lds_order tools/ubench_lds_order.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int TRIALS = 64;

__global__ void __launch_bounds__(512) k_check(uint32_t seed, uint32_t bits, unsigned long long* bad,
                                               unsigned long long* checked) {
    __shared__ uint32_t cnt[8][256];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t mask = (1u << bits) - 1;
    uint32_t x = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu);
    unsigned long long nbad = 0, nchk = 0;
    for (uint32_t d = lane; d < 256; d += 64) cnt[w][d] = 0;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    for (int t = 0; t < TRIALS; ++t) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        // a mix of uniform digits and hot digits (many lanes on one address)
        const uint32_t dig = ((x >> 8) & 3) == 0 ? (x & 1) : (x & mask);
        const uint32_t before = cnt[w][dig];       // value before this instruction (no writes pending)
        __builtin_amdgcn_wave_barrier();
        const uint32_t old = atomicAdd(&cnt[w][dig], 1u);
        // stable rank: lower lanes with the same digit
        uint32_t lower = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t dl = __shfl(dig, l, 64);
            if ((uint32_t)l < lane && dl == dig) ++lower;
        }
        nbad += (old != before + lower);
        ++nchk;
        __builtin_amdgcn_wave_barrier();
    }
    atomicAdd(bad, nbad);
    atomicAdd(checked, nchk);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;
    unsigned long long *d_bad, *d_chk, h_bad = 0, h_chk = 0;
    (void)hipMalloc(&d_bad, 8);
    (void)hipMalloc(&d_chk, 8);
    int fail = 0;
    for (uint32_t bits : {1u, 3u, 5u, 7u, 8u}) {
        (void)hipMemset(d_bad, 0, 8);
        (void)hipMemset(d_chk, 0, 8);
        hipLaunchKernelGGL(k_check, dim3(blocks), dim3(512), 0, 0, 0x1234567u + bits, bits, d_bad, d_chk);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel failed\n");
            return 2;
        }
        (void)hipMemcpy(&h_bad, d_bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&h_chk, d_chk, 8, hipMemcpyDeviceToHost);
        printf("bits=%u lane-checks=%llu mismatches=%llu\n", bits, h_chk, h_bad);
        fail |= h_bad != 0;
    }
    printf(fail ? "ORDER NOT LANE-ASCENDING\n" : "ds_add_rtn same-address lanes served in ascending lane order\n");
    return fail;
}
