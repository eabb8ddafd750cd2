// Micro-benchmark of the 8-B probe index's read forms (gd_kernels.h Cx8Args) at BASELINE cfg 4's and
// cfg 2's shapes: N random probes of present keys into an index of C 8-B slots {key, value}, linear
// probing in aligned 8-slot (64-B) groups, with a 4-B/probe key stream in and 8 B/probe out (the
// fan-out's dst read and silo/act write).  Forms:
//   g4    one 64-B group a round as 4 x 16-B loads (the library's k_fan_route / k_route_m CX8)
//   g2    the first 32 B (2 x 16-B loads), the second half only when the first holds no hit or empty
//   g1    16 B (2 slots) a round
//   coop  4 lanes a probe, each one 16-B piece of the group (ballots pick the first hit / empty)
//   g4io  g4 with k_route's streams: 24-B keys {0, key, tcd} in (3 x 8-B loads), silo / act / status out
//         (4 + 4 + 1 B) -- the probe ceiling the route kernel can reach with its own I/O
// Each form runs `reps` times between HIP events; rocprofv3 --pmc on this binary gives its EA requests.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_fanprobe tools/ubench_fanprobe.hip
//   tools/ubench_fanprobe [slots_log2 = 25] [n_probes = 43000000] [load = 0.3]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint64_t home(uint32_t key, uint64_t cap) {
    return (((uint64_t)fmix32(key * 0x9E3779B1u + 7u) * cap) >> 32) & ~7ull;
}

__global__ void k_build(uint64_t* slots, uint64_t cap, const uint32_t* keys, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    const unsigned long long v = (unsigned long long)k | ((unsigned long long)(i + 1) << 32);
    uint64_t s = home(k, cap);
    for (uint64_t d = 0; d < cap; ++d) {
        if (atomicCAS((unsigned long long*)(slots + s), 0ull, v) == 0ull) return;
        s = s + 1 == cap ? 0 : s + 1;
    }
}

__global__ void __launch_bounds__(256) k_probe_io(const uint4* __restrict__ slots, uint64_t cap,
                                                   const unsigned long long* __restrict__ keys24, uint32_t n,
                                                   uint32_t* __restrict__ silo, uint32_t* __restrict__ act,
                                                   uint8_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const unsigned long long n0 = keys24[3 * (size_t)i], n1 = keys24[3 * (size_t)i + 1],
                             tcd = keys24[3 * (size_t)i + 2];
    const uint32_t key = (uint32_t)n1 ^ (uint32_t)n0 ^ (uint32_t)(tcd >> 32) ^ (uint32_t)tcd;
    uint64_t s = home(key, cap);
    uint32_t val = 0;
    for (int round = 0; round < 64; ++round) {
        uint4 q[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) q[g] = slots[(s >> 1) + g];
        bool done = false;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            if (done) continue;
            const uint32_t x = (g & 1) ? q[g / 2].z : q[g / 2].x, y = (g & 1) ? q[g / 2].w : q[g / 2].y;
            if (y == 0) done = true;
            else if (x == key) { val = y; done = true; }
        }
        if (done) break;
        s += 8;
        if (s >= cap) s = 0;
    }
    __builtin_nontemporal_store(val & 7u, silo + i);
    act[i] = val;
    __builtin_nontemporal_store((uint8_t)(val != 0), status + i);
}

template <int FORM>
__global__ void __launch_bounds__(256) k_probe(const uint4* __restrict__ slots, uint64_t cap,
                                                const uint32_t* __restrict__ keys, uint32_t n,
                                                uint2* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if constexpr (FORM == 3) {
        // 4 lanes a probe: lane group g = lane / 4 takes probe base + g, piece lane % 4
        const uint32_t lane = threadIdx.x & 63, piece = lane & 3;
        const uint32_t wbase = (blockIdx.x * 256 + (threadIdx.x & ~63u));
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t pi = wbase + r * 16 + lane / 4;
            const bool live = pi < n;
            const uint32_t key = live ? keys[pi] : 0u;
            uint64_t s = home(key, cap);
            uint32_t val = 0;
            bool done = !live;
            for (int round = 0; round < 64; ++round) {
                uint4 q = make_uint4(0, 0, 0, 0);
                if (!done) q = slots[(s >> 1) + piece];
                // slot order in the group: piece 0 slots 0,1; piece 1 slots 2,3; ...
                const bool h0 = !done && q.y != 0 && q.x == key, h1 = !done && q.w != 0 && q.z == key;
                const bool e0 = !done && q.y == 0, e1 = !done && q.w == 0;
                const unsigned long long t0 = __ballot(h0 || e0), t1 = __ballot(h1 || e1);
                const unsigned long long m0 = __ballot(h0), m1 = __ballot(h1);
                // this lane group's 8-bit terminal / hit masks in slot order
                const uint32_t gs = (lane & ~3u);
                uint32_t term = 0, hit = 0;
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    term |= (uint32_t)((t0 >> (gs + p)) & 1) << (2 * p);
                    term |= (uint32_t)((t1 >> (gs + p)) & 1) << (2 * p + 1);
                    hit |= (uint32_t)((m0 >> (gs + p)) & 1) << (2 * p);
                    hit |= (uint32_t)((m1 >> (gs + p)) & 1) << (2 * p + 1);
                }
                // every lane shuffles (no divergent ds_bpermute): the value sits in lane gs + first / 2,
                // component first & 1
                const uint32_t first = term ? __builtin_ctz(term) : 0u;
                const uint32_t src = gs + first / 2;
                const uint32_t vy = __shfl((int)q.y, (int)src, 64), vw = __shfl((int)q.w, (int)src, 64);
                if (!done && term) {
                    if ((hit >> first) & 1) val = (first & 1) ? vw : vy;
                    done = true;
                }
                if (__ballot(!done) == 0) break;
                if (!done) {
                    s += 8;
                    if (s >= cap) s = 0;
                }
            }
            if (live && piece == 0) out[pi] = make_uint2(val, key);
        }
        return;
    } else {
        if (i >= n) return;
        const uint32_t key = keys[i];
        uint64_t s = home(key, cap);
        uint32_t val = 0;
        for (int round = 0; round < 64; ++round) {
            bool done = false;
            if constexpr (FORM == 0) {
                uint4 q[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) q[g] = slots[(s >> 1) + g];
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    if (done) continue;
                    const uint32_t x = (g & 1) ? q[g / 2].z : q[g / 2].x, y = (g & 1) ? q[g / 2].w : q[g / 2].y;
                    if (y == 0) done = true;
                    else if (x == key) { val = y; done = true; }
                }
                if (done) break;
                s += 8;
            } else if constexpr (FORM == 1) {
                uint4 q[2];
#pragma unroll
                for (int g = 0; g < 2; ++g) q[g] = slots[(s >> 1) + g];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (done) continue;
                    const uint32_t x = (g & 1) ? q[g / 2].z : q[g / 2].x, y = (g & 1) ? q[g / 2].w : q[g / 2].y;
                    if (y == 0) done = true;
                    else if (x == key) { val = y; done = true; }
                }
                if (done) break;
                s += 4;
            } else {
                const uint4 q = slots[s >> 1];
                if (q.y == 0) break;
                if (q.x == key) { val = q.y; break; }
                if (q.w == 0) break;
                if (q.z == key) { val = q.w; break; }
                s += 2;
            }
            if (s >= cap) s = 0;
        }
        out[i] = make_uint2(val, key);
    }
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 25;
    const uint32_t n = argc > 2 ? (uint32_t)atol(argv[2]) : 43000000u;
    const double load = argc > 3 ? atof(argv[3]) : 0.3;
    const uint64_t cap = 1ull << lg;
    const uint32_t m = (uint32_t)(cap * load);
    std::vector<uint32_t> hk(m), hp(n);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (uint32_t i = 0; i < m; ++i) hk[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;   // distinct
    for (uint32_t i = 0; i < n; ++i) hp[i] = hk[rnd() % m];
    uint64_t* d_slots;
    uint32_t *d_keys, *d_probe;
    uint2* d_out;
    CK(hipMalloc(&d_slots, cap * 8));
    CK(hipMalloc(&d_keys, (size_t)m * 4));
    CK(hipMalloc(&d_probe, (size_t)n * 4));
    CK(hipMalloc(&d_out, (size_t)n * 8));
    CK(hipMemset(d_slots, 0, cap * 8));
    CK(hipMemcpy(d_keys, hk.data(), (size_t)m * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_probe, hp.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_build, dim3((m + 255) / 256), dim3(256), 0, 0, d_slots, cap, d_keys, m);
    CK(hipDeviceSynchronize());
    // the route's 24-B keys {0, key, 0}: key ^ 0 ^ 0 = key
    std::vector<unsigned long long> hk24((size_t)n * 3, 0ull);
    for (uint32_t i = 0; i < n; ++i) hk24[3 * (size_t)i + 1] = hp[i];
    unsigned long long* d_k24;
    uint32_t *d_silo, *d_act;
    uint8_t* d_st;
    CK(hipMalloc(&d_k24, (size_t)n * 24));
    CK(hipMalloc(&d_silo, (size_t)n * 4));
    CK(hipMalloc(&d_act, (size_t)n * 4));
    CK(hipMalloc(&d_st, (size_t)n));
    CK(hipMemcpy(d_k24, hk24.data(), (size_t)n * 24, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[4] = {"g4", "g2", "g1", "coop"};
    std::vector<uint2> ref(n), got(n);
    for (int form = 0; form < 4; ++form) {
        const dim3 grid((n + 255) / 256);
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(a));
            switch (form) {
                case 0: hipLaunchKernelGGL(k_probe<0>, grid, dim3(256), 0, 0, (const uint4*)d_slots, cap, d_probe, n, d_out); break;
                case 1: hipLaunchKernelGGL(k_probe<1>, grid, dim3(256), 0, 0, (const uint4*)d_slots, cap, d_probe, n, d_out); break;
                case 2: hipLaunchKernelGGL(k_probe<2>, grid, dim3(256), 0, 0, (const uint4*)d_slots, cap, d_probe, n, d_out); break;
                default: hipLaunchKernelGGL(k_probe<3>, grid, dim3(256), 0, 0, (const uint4*)d_slots, cap, d_probe, n, d_out); break;
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep >= 2) printf("%s slots 2^%d load %.2f probes %u: %.4f ms (%.1f G probes/s)\n", names[form], lg, load, n, ms,
                                 n / ms / 1e6);
        }
        CK(hipMemcpy(form == 0 ? ref.data() : got.data(), d_out, (size_t)n * 8, hipMemcpyDeviceToHost));
        if (form > 0) {
            size_t bad = 0;
            for (uint32_t i = 0; i < n; ++i) bad += ref[i].x != got[i].x;
            printf("%s mismatches vs g4: %zu\n", names[form], bad);
        } else {
            size_t miss = 0;
            for (uint32_t i = 0; i < n; ++i) miss += ref[i].x == 0;
            printf("g4 misses: %zu\n", miss);
        }
    }
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_probe_io, dim3((n + 255) / 256), dim3(256), 0, 0, (const uint4*)d_slots, cap, d_k24, n, d_silo,
                           d_act, d_st);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) printf("g4io slots 2^%d load %.2f probes %u: %.4f ms (%.1f G probes/s)\n", lg, load, n, ms, n / ms / 1e6);
    }
    {
        std::vector<uint32_t> ga(n);
        CK(hipMemcpy(ga.data(), d_act, (size_t)n * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (uint32_t i = 0; i < n; ++i) bad += ga[i] != ref[i].x;
        printf("g4io mismatches vs g4: %zu\n", bad);
    }
    return 0;
}
