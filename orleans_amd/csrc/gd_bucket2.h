// gd_bucket2.h -- gfx950 device code for the two-pass stable bucketing (the north
// star's bucketing kernel) of keys in [0, n_act] with n_act < B2_RMAX2 * 1024 (BASELINE cfg 2:
// n_act = 2^20, so 21-bit keys with the clamp value): LSD over a 10-bit low digit (1,024 buckets),
// then the high digit key >> 10 (<= 1,056 buckets), instead of three 7-bit passes.
//
// Why wide digits pay here only with wide tiles: a radix pass writes each tile's items as R runs of
// TILE / R items.  tools/ubench_runs.hip measured on MI355X what a run length costs apart from the
// ranking: 4-B items in 64-B runs stream at ~4.5-5 TB/s, in 32-B runs ~3.8, in 16-B runs ~2.5.  At
// R ~ 1,024 that takes 16,384-item tiles (16 items per run, 64 B of indices), and a tile of that
// size is ranked in LDS with two waves' counters packed in one u32 (16-bit halves), so the counters
// stay at R x NW x 2 B.
//
// Per item: pass 1 reads the key (4 B) twice (histogram, scatter) and writes (index, key) 8 B; pass 2
// reads the key (4 B) for its histogram, then (index, key) 8 B and writes the index 4 B -- 32 B an
// item over 7 launches (2 histograms, 2 row scans, 2 scatters, 1 range min-scan), against 40 B over
// 11 launches for three packed 7-bit passes.  Stability: a tile is ranked in index order (wave-
// striped rows, ds_add_rtn serves the lanes of one instruction in lane order), tiles in order by
// the row-scanned counts.  HBM-bound, no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "gd_kernels.h"

namespace gd {

constexpr uint32_t B2_LOW_BITS = 10;                     // pass 1 digit: key & 1023
constexpr uint32_t B2_R1 = 1u << B2_LOW_BITS;
constexpr uint32_t B2_RMAX2 = 1056;                      // pass 2 digits: (n_act >> 10) + 1 <= 1056
constexpr uint32_t B2_TILE = 16384;                      // items per tile, both passes

// Histogram of TPB consecutive tiles per workgroup (NT x IT items a tile: B2_TILE, or 8,192 for the
// MSD pass's A/B form), digit-major counts
// hist[d * tiles + t] for d < R.  FIRST: the digit of min(key, clamp) & 1023, and the grid pre-fills
// the bucket starts (fill); else (pass 2) the digit of the already clamped key, key >> 10.  HI with
// FIRST (the MSD pass of gd_msd.h): the raw keys clamped, their high digit.
template <int NT, int IT, int TPB, int RMAX, bool FIRST, bool HI = !FIRST>
__global__ void __launch_bounds__(NT) k_b2_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t clamp,
                                                uint32_t R, uint32_t tiles, uint32_t* __restrict__ hist, FillArgs fill,
                                                uint32_t xcd_rev) {
    constexpr uint32_t TILE = NT * IT;
    static_assert(TILE <= 65536 && IT % 4 == 0, "16-B loads, u16 tile positions");
    __shared__ uint32_t s_cnt[TPB][RMAX];
    for (uint32_t x = threadIdx.x; x < TPB * RMAX; x += NT) (&s_cnt[0][0])[x] = 0;
    __syncthreads();
    const uint32_t t0 = hist_t0(blockIdx.x, gridDim.x, TPB, tiles, xcd_rev);
    const uint32_t lane = lane_id();
    const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0;
#pragma unroll
    for (int t = 0; t < TPB; ++t) {
        const uint64_t base = (uint64_t)(t0 + t) * TILE;
        uint32_t k[IT];
        if (aligned && base + TILE <= n) {
#pragma unroll
            for (int j = 0; j < IT / 4; ++j) {
                const uint4 v = *reinterpret_cast<const uint4*>(keys + base + 4 * (j * NT + threadIdx.x));
                k[4 * j] = v.x; k[4 * j + 1] = v.y; k[4 * j + 2] = v.z; k[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < IT / 4; ++j) {
                const uint64_t i0 = base + 4 * (j * NT + threadIdx.x);
#pragma unroll
                for (int q = 0; q < 4; ++q) k[4 * j + q] = (i0 + q < n) ? keys[i0 + q] : 0u;
            }
        }
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint64_t i = base + 4 * ((j / 4) * NT + threadIdx.x) + (j % 4);
            const bool valid = i < n;
            const uint32_t kc = FIRST ? min(k[j], clamp) : k[j];
            const uint32_t d = HI ? (kc >> B2_LOW_BITS) : (kc & (B2_R1 - 1));
            const unsigned long long act = __ballot(valid);
            if (act == 0) continue;
            const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1;
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead);
            const unsigned long long hot = __ballot(valid && d == d0);
            if (valid) {
                if (d != d0) atomicAdd(&s_cnt[t][d], 1u);
                else if (lane == lead) atomicAdd(&s_cnt[t][d], (uint32_t)__popcll(hot));
            }
        }
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < TPB * R; x += NT) {
        const uint32_t t = x % TPB, d = x / TPB;
        if (t0 + t < tiles) hist[(size_t)d * tiles + t0 + t] = s_cnt[t][d];
    }
    if constexpr (FIRST) fill_grid(fill, NT);
}

// One radix pass over B2 tiles.  FIRST (pass 1): keys_in = the activations (clamped here), values =
// the item indices; writes (key, index) in digit order of key & 1023.  Else (pass 2, the last):
// (key, index) in, the index out in digit order of key >> 10 -- the permutation -- and the bucket
// starts (the first item of each key in a tile's digit run lowers starts[key] with atomicMin; the
// run is sorted by the whole key because pass 1 ordered it), rank_out[index] = position on request.
// gscan: the row-scanned counts (k_radix_rowscan), totals: the digit totals.  HI with FIRST (the MSD
// pass of gd_msd.h): pass 1's inputs and outputs, ordered by the high digit key >> 10; K16 writes
// only the key's low 10 bits, as u16 (its digit is implied by the range it lands in).
template <int NT, int IT, int RMAX, bool FIRST, bool HI = !FIRST, bool K16 = false>
__global__ void __launch_bounds__(NT) k_b2_scatter(const uint32_t* __restrict__ keys_in,
                                                   const uint32_t* __restrict__ vals_in, uint32_t n, uint32_t clamp,
                                                   uint32_t R, uint32_t tiles, const uint32_t* __restrict__ gscan,
                                                   const uint32_t* __restrict__ totals,
                                                   uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                   uint32_t* __restrict__ starts, uint32_t* __restrict__ rank_out,
                                                   uint32_t xcd) {
    constexpr int NW = NT / WAVE;
    constexpr uint32_t TILE = NT * IT;
    static_assert(TILE <= 65536 && NW % 2 == 0, "u16 tile positions, wave pairs");
    constexpr uint32_t DPT = (RMAX + NT - 1) / NT;
    using Val = typename std::conditional<FIRST, uint16_t, uint32_t>::type;   // pass 1: position in the tile
    __shared__ uint32_t s_cnt[NW / 2][RMAX];             // wave pair (2p, 2p + 1): low / high 16 bits
    __shared__ uint32_t s_lstart[RMAX];
    __shared__ uint32_t s_gbase[RMAX];
    __shared__ uint32_t s_key[TILE];
    __shared__ Val s_val[TILE];
    __shared__ uint32_t s_wsum[2 * NW];

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x, xcd);
    const uint32_t base = tile * TILE;
    const uint32_t cnt_tile = min(TILE, n - base);
    for (uint32_t d = threadIdx.x; d < RMAX; d += NT) {
#pragma unroll
        for (int p = 0; p < NW / 2; ++p) s_cnt[p][d] = 0;
        s_gbase[d] = d < R ? gscan[(size_t)d * tiles + tile] : 0u;
    }
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x / WAVE;
    const uint32_t half = (w & 1u) * 16u;
    const uint32_t one = 1u << half;
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t kk[IT], vv[IT], rk[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t idx = base + (w * IT + r) * WAVE + lane;
        const uint32_t li = min(idx, n - 1);
        kk[r] = __builtin_nontemporal_load(keys_in + li);
        if constexpr (!FIRST) vv[r] = __builtin_nontemporal_load(vals_in + li);
    }
    uint32_t tv[DPT], my_g = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t d = threadIdx.x * DPT + q;
        tv[q] = d < R ? totals[d] : 0u;
        my_g += tv[q];
    }
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t pos = (w * IT + r) * WAVE + lane;
        kk[r] = base + pos < n ? (FIRST ? min(kk[r], clamp) : kk[r]) : 0u;
        if constexpr (FIRST) vv[r] = pos;
    }
    __syncthreads();
    // stable rank within the wave: one ds_add_rtn per row on the wave's half of the pair counter (the
    // lanes sharing the first live lane's digit fold into one update by that lane); 8 rows' updates
    // go out before their hot lanes are resolved
#pragma unroll
    for (int r0 = 0; r0 < IT; r0 += 8) {
        unsigned long long hot[8];
        uint32_t lead[8];
#pragma unroll
        for (int r = r0; r < r0 + 8; ++r) {
            const uint32_t idx = base + (w * IT + r) * WAVE + lane;
            const bool valid = idx < n;
            const uint32_t d = HI ? (kk[r] >> B2_LOW_BITS) : (kk[r] & (B2_R1 - 1));
            const unsigned long long live = __ballot(valid);
            const uint32_t ld = live ? (uint32_t)__ffsll((long long)live) - 1 : 0u;
            const uint32_t hd = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)ld);
            hot[r - r0] = __ballot(valid && d == hd);
            lead[r - r0] = ld;
            rk[r] = 0;
            if (valid && (d != hd || lane == ld))
                rk[r] = atomicAdd(&s_cnt[w >> 1][d], lane == ld ? (uint32_t)__popcll(hot[r - r0]) << half : one);
        }
#pragma unroll
        for (int r = r0; r < r0 + 8; ++r) {
            const uint32_t mine = (rk[r] >> half) & 0xFFFFu;
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)lead[r - r0]);
            rk[r] = ((hot[r - r0] >> lane) & 1ull) ? b0 + (uint32_t)__popcll(hot[r - r0] & lt) : mine;
        }
    }
    __syncthreads();
    // per digit: the waves' exclusive prefix (back into the halves), then tile-local digit starts and,
    // with the digit totals, the digit bases
    uint32_t my_total = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t d = threadIdx.x * DPT + q;
        if (d < RMAX) {
            uint32_t run = 0;
#pragma unroll
            for (int p = 0; p < NW / 2; ++p) {
                const uint32_t c = s_cnt[p][d];
                const uint32_t lo = c & 0xFFFFu, hi = c >> 16;
                s_cnt[p][d] = run | ((run + lo) << 16);
                run += lo + hi;
            }
            s_lstart[d] = run;
            my_total += run;
        }
    }
    uint32_t ex, exg;
    block_excl_scan_add2<NT>(my_total, my_g, s_wsum, ex, exg);
    {
        // the pair prefixes become absolute tile positions (+ the digit's tile start, both halves), and
        // the write-out's base is gbase - lstart: one LDS lookup per item on each side
        uint32_t run = ex, rung = exg;
#pragma unroll
        for (uint32_t q = 0; q < DPT; ++q) {
            const uint32_t d = threadIdx.x * DPT + q;
            if (d < RMAX) {
                const uint32_t t = s_lstart[d];
#pragma unroll
                for (int p = 0; p < NW / 2; ++p) s_cnt[p][d] += run | (run << 16);
                s_gbase[d] = s_gbase[d] + rung - run;
                run += t;
                rung += tv[q];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t pos = (w * IT + r) * WAVE + lane;
        if (base + pos < n) {
            const uint32_t d = HI ? (kk[r] >> B2_LOW_BITS) : (kk[r] & (B2_R1 - 1));
            const uint32_t at = ((s_cnt[w >> 1][d] >> half) & 0xFFFFu) + rk[r];
            s_key[at] = kk[r];
            s_val[at] = (Val)vv[r];
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < IT; ++j) {
        const uint32_t p = j * NT + threadIdx.x;
        if (p < cnt_tile) {
            const uint32_t k = s_key[p];
            const uint32_t d = HI ? (k >> B2_LOW_BITS) : (k & (B2_R1 - 1));
            const uint32_t g = s_gbase[d] + p;
            if (g < n) {                  // always true when the counts are right; never write out of bounds
                if constexpr (FIRST) {
                    if constexpr (K16) reinterpret_cast<uint16_t*>(keys_out)[g] = (uint16_t)(k & (B2_R1 - 1));
                    else keys_out[g] = k;
                    vals_out[g] = base + (uint32_t)s_val[p];
                } else {
                    const uint32_t v = s_val[p];
                    if (p == 0 || s_key[p - 1] != k) atomicMin(&starts[k], g);
                    vals_out[g] = v;
                    if (rank_out) rank_out[v] = g;
                }
            }
        }
    }
}

}  // namespace gd
