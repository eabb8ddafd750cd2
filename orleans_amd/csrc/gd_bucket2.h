// gd_bucket2.h -- gfx950 device code for the wide-digit MSD pass of the two-level bucketing (SURVEY 8
// a16, the north star's bucketing kernel; gd_msd.h): a stable partition of the clamped activations
// min(act, n_act) by their high digit kc >> shift, <= RMAX digits, on 8K-item tiles (512 threads x 16
// items, two workgroups a CU).
//
// Why wide digits pay here only with wide tiles: a radix pass writes each tile's items as R runs of
// TILE / R items.  tools/ubench_runs.hip measured on MI355X what a run length costs apart from the
// ranking: 4-B items in 64-B runs stream at ~4.5-5 TB/s, in 32-B runs ~3.8, in 16-B runs ~2.5.  At R
// ~ 1,024 an 8K tile writes 32-B index runs; its counters stay at R x NW x 2 B by packing two waves'
// counters in one u32 (16-bit halves).
//
// Per item: the histogram reads the activation (4 B), the scatter reads it again and writes the
// message index (u32) plus a key (B2Out): the range-local key (key & 1023, u16: the one-pass form for
// n_act < 1,081,344), or for the first pass of the three-pass form (larger n_act, gd_msd2.h) the key
// bits the second pass needs packed into 6 B, or the whole clamped key (u32).  Stability: a tile is ranked in index order (wave-striped rows, ds_add_rtn
// serves the lanes of one instruction in lane order -- checked on the device at handle creation,
// DESIGN 5), tiles in order by the row-scanned counts.  HBM-bound, no MFMA.
//
// Round 3 also built two full wide passes (key & 1023, then key >> 10, 16K tiles; GD_BUCKET2): bit-exact
// and slower than three 7-bit passes (243 against 215 us at cfg 2, profiles/r03_b2_ab.txt); removed in
// round 4 with the other measured losers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_kernels.h"

namespace gd {

constexpr uint32_t B2_LOW_BITS = 10;                     // the second level's range: 1,024 activations
constexpr uint32_t B2_RMAX2 = 1056;                      // one-pass form: (n_act >> 10) + 1 <= 1056 ranges
constexpr int B2_NT = 512;                               // the MSD pass's tile: 512 threads x 16 items
constexpr int B2_IT = 16;
constexpr uint32_t B2_TILE = B2_NT * B2_IT;

// The clamped key: a key >= c.x (n_act: the unrouted messages) becomes c.y -- n_act itself, or (the
// one-pass form, msd_unrouted_key) the first key of a range past n_act's, so that they form their own.
__device__ __forceinline__ uint32_t b2_clamp(uint32_t k, uint2 c) { return k >= c.x ? c.y : k; }

// Histogram of TPB consecutive tiles per workgroup, digit-major counts hist[d * tiles + t] for d < R:
// the digit of b2_clamp(key, clamp) >> shift.
template <int NT, int IT, int TPB, int RMAX>
static __global__ void __launch_bounds__(NT) k_b2_hist(const uint32_t* __restrict__ keys, uint32_t n, uint2 clamp,
                                                uint32_t R, uint32_t tiles, uint32_t* __restrict__ hist,
                                                uint32_t shift, uint32_t xcd_rev) {
    constexpr uint32_t TILE = NT * IT;
    static_assert(TILE <= 65536 && IT % 4 == 0, "16-B loads, u16 tile positions");
    __shared__ uint32_t s_cnt[TPB][RMAX];
    __shared__ uint32_t s_sink[WAVE];
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
        // the wave's hot digit (wave_hot_digit of its first row) counted in a register, the rest in LDS
        const uint32_t h = wave_hot_digit(b2_clamp(k[0], clamp) >> shift, base + 4 * threadIdx.x < n);
        uint32_t hc = 0;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint64_t i = base + 4 * ((j / 4) * NT + threadIdx.x) + (j % 4);
            const uint32_t d = b2_clamp(k[j], clamp) >> shift;
            hist_add(s_cnt[t], s_sink, d, h, i < n, hc);
        }
        hc = wave_sum(hc);
        if (lane == 0 && hc) atomicAdd(&s_cnt[t][h], hc);
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < TPB * R; x += NT) {
        const uint32_t t = x % TPB, d = x / TPB;
        if (t0 + t < tiles) hist[(size_t)d * tiles + t0 + t] = s_cnt[t][d];
    }
}

// What the MSD scatter writes beside each message index.
enum B2Out : int {
    B2_KEY32 = 0,    // the whole clamped key, u32 (8-B records)
    B2_KEY16 = 1,    // the range-local key key & 1023, u16 (the one-pass form: 6-B records)
    B2_PACK = 2,     // the key's low pbits bits P: P >> hb as u16, P's low hb bits above the index's ib
                     // bits in the u32 (the three-pass form's pass A: 6-B records)
};
struct B2Pack {
    uint32_t pbits, hb, ib;
};

// One record of the MSD scatter's output at position g: the key in its B2Out form and the message index.
template <int KOUT>
__device__ __forceinline__ void b2_put(uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, uint32_t g,
                                       uint32_t k, uint32_t idx, const B2Pack& pk) {
    if constexpr (KOUT == B2_KEY16) {
        reinterpret_cast<uint16_t*>(keys_out)[g] = (uint16_t)(k & ((1u << B2_LOW_BITS) - 1));
        vals_out[g] = idx;
    } else if constexpr (KOUT == B2_PACK) {
        const uint32_t P = k & ((1u << pk.pbits) - 1u);
        reinterpret_cast<uint16_t*>(keys_out)[g] = (uint16_t)(P >> pk.hb);
        vals_out[g] = pk.hb ? idx | ((P & ((1u << pk.hb) - 1u)) << pk.ib) : idx;
    } else {
        keys_out[g] = k;
        vals_out[g] = idx;
    }
}

// The MSD pass's scatter: keys_in = the activations (clamped here), writes the message index and the
// key (B2Out form) in digit order of min(key, clamp) >> shift.  gscan: the row-scanned counts
// (k_radix_rowscan), totals: the digit totals.  PERSIST (with a grid smaller than the tile count): the
// workgroups are persistent -- workgroup b takes virtual tiles b, b + grid, ... (grid a multiple of 8, so
// every tile of a workgroup stays in its XCD's range of xcd_tile), the digit totals load once, and the
// next tile's activations load under this tile's write-out (128 VGPRs: four waves a SIMD, two
// workgroups a CU).  Without PERSIST one workgroup a tile, as compiled before the loop existed.
// The persistent scatter's j-th tile for workgroup b (grid a multiple of 8, workgroup b on XCD b % 8):
// strided (order 0: b + j * grid through xcd_tile), or (order 1) run j of the workgroup's consecutive tiles
// in its XCD's tile range.  NONE32 past its last.
__device__ __forceinline__ uint32_t b2_tile_at(uint32_t b, uint32_t j, uint32_t grid, uint32_t tiles, uint32_t xcd,
                                               uint32_t order) {
    if (!order || !xcd) {
        const uint32_t vb = b + j * grid;
        return vb < tiles ? xcd_tile(vb, tiles, xcd) : NONE32;
    }
    const uint32_t x = b & 7u, k = b >> 3, per = grid >> 3, q = tiles >> 3, rem = tiles & 7u;
    const uint32_t lo = x * q + min(x, rem), len = q + (x < rem ? 1u : 0u);
    const uint32_t J = (len + per - 1) / per, t = k * J + j;
    return j < J && t < len ? lo + t : NONE32;
}

template <int NT, int IT, int RMAX, int KOUT, bool BALLOT = false, bool PERSIST = false>
static __global__ void __launch_bounds__(NT, 4) k_b2_scatter(const uint32_t* __restrict__ keys_in, uint32_t n, uint2 clamp,
                                                   uint32_t R, uint32_t tiles, const uint32_t* __restrict__ gscan,
                                                   const uint32_t* __restrict__ totals,
                                                   uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                   uint32_t shift, uint32_t xcd, B2Pack pk, uint32_t order = 0) {
    constexpr int NW = NT / WAVE;
    constexpr uint32_t TILE = NT * IT;
    static_assert(TILE <= 65536 && NW % 2 == 0, "u16 tile positions, wave pairs");
    constexpr uint32_t DPT = (RMAX + NT - 1) / NT;
    __shared__ uint32_t s_cnt[NW / 2][RMAX];             // wave pair (2p, 2p + 1): low / high 16 bits
    __shared__ uint32_t s_lstart[RMAX];
    __shared__ uint32_t s_gbase[RMAX];
    __shared__ uint32_t s_key[TILE];
    __shared__ uint16_t s_val[TILE];                     // position in the tile
    __shared__ uint32_t s_wsum[2 * NW];

    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x / WAVE;
    const uint32_t half = (w & 1u) * 16u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t kk[IT], rk[IT];
    uint32_t vj = 0;                                     // the workgroup's tile number (persistent form)
    uint32_t tile = PERSIST ? b2_tile_at(blockIdx.x, 0, gridDim.x, tiles, xcd, order) : xcd_tile(blockIdx.x, tiles, xcd);
    if (tile == NONE32) return;                          // (persistent, chunked: no tile for this workgroup)
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t idx = tile * TILE + (w * IT + r) * WAVE + lane;
        kk[r] = __builtin_nontemporal_load(keys_in + min(idx, n - 1));
    }
    uint32_t tv[DPT], my_g = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t d = threadIdx.x * DPT + q;
        tv[q] = d < R ? totals[d] : 0u;
        my_g += tv[q];
    }
    for (;;) {
    const uint32_t base = tile * TILE;
    const uint32_t cnt_tile = min(TILE, n - base);
    // this tile's row-scanned counts: one workgroup a tile keeps the thread's own digits' (the scan below
    // owns d = threadIdx.x * DPT + q) in registers from here to after the ranking (cfg 2 0.0626 -> 0.0607
    // ms); the persistent form, at its register limit, stages them through LDS
    uint32_t gb[DPT];
    if constexpr (!PERSIST) {
#pragma unroll
        for (uint32_t q = 0; q < DPT; ++q) {
            const uint32_t d = threadIdx.x * DPT + q;
            gb[q] = d < R ? gscan[(size_t)d * tiles + tile] : 0u;
        }
    }
    for (uint32_t d = threadIdx.x; d < RMAX; d += NT) {
#pragma unroll
        for (int p = 0; p < NW / 2; ++p) s_cnt[p][d] = 0;
        if constexpr (PERSIST) s_gbase[d] = d < R ? gscan[(size_t)d * tiles + tile] : 0u;
    }
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t pos = (w * IT + r) * WAVE + lane;
        kk[r] = base + pos < n ? b2_clamp(kk[r], clamp) : 0u;
    }
    __syncthreads();
    // stable rank within the wave: the wave's hot digit (wave_hot_digit of its first row) by ballot in
    // registers, every other item by its own update of the wave's half of the pair counter (row_rank16)
    constexpr int DB = RMAX <= 512 ? 9 : 11;             // digit bits (BALLOT's matching)
    const uint32_t h = wave_hot_digit(kk[0] >> shift, base + w * IT * WAVE + lane < n);
    uint32_t hrun = 0;
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const bool valid = base + (w * IT + r) * WAVE + lane < n;
        const uint32_t d = kk[r] >> shift;
        const unsigned long long hm = __ballot(valid && d == h);
        const uint32_t cr = row_rank16<BALLOT, DB>(&s_cnt[w >> 1][d], half, d, valid && d != h);
        rk[r] = d == h ? hrun + (uint32_t)__popcll(hm & lt) : cr;
        hrun += (uint32_t)__popcll(hm);
    }
    if (lane == 0 && hrun) atomicAdd(&s_cnt[w >> 1][h], hrun << half);
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
                s_gbase[d] = (PERSIST ? s_gbase[d] : gb[q]) + rung - run;
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
            const uint32_t at = ((s_cnt[w >> 1][kk[r] >> shift] >> half) & 0xFFFFu) + rk[r];
            s_key[at] = kk[r];
            s_val[at] = (uint16_t)pos;
        }
    }
    __syncthreads();
    // the next tile's activations load under this tile's write-out
    ++vj;
    const uint32_t nt_ = PERSIST ? b2_tile_at(blockIdx.x, vj, gridDim.x, tiles, xcd, order) : NONE32;
    const bool more = PERSIST && nt_ != NONE32;
    const uint32_t ntile = more ? nt_ : tile;
    if (more) {
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            // a 32-bit byte offset from the uniform base (n < 2^30 on this path): one VGPR an address, not two
            const uint32_t off = min(ntile * TILE + (w * IT + r) * WAVE + lane, n - 1) * 4u;
            kk[r] = __builtin_nontemporal_load(
                reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(keys_in) + off));
        }
    }
    // The write-out.  One workgroup a tile reads its LDS in batches of WB items -- every staged key, then
    // every digit base, then the positions, then the stores -- rather than one item's two dependent reads
    // and a wait at a time (branches around each item made the compiler serialise them; positions past
    // the tile read in-bounds LDS and store nothing): cfg 3 pass A 0.168 -> 0.158 ms.  The persistent form
    // (at its register limit) keeps one item at a time: batched it spilled and took 0.060 -> 0.067 ms
    // (profiles/r05_writeout_batch_ab.txt).  A branch-free write-out (full tiles without the tail test,
    // g clamped below n instead of tested) was slower for both (0.0606 -> 0.063, 0.0589 -> 0.067 ms).
    if constexpr (PERSIST) {
#pragma unroll 4
        for (int j = 0; j < IT; ++j) {
            const uint32_t p = j * NT + threadIdx.x;
            if (p < cnt_tile) {
                const uint32_t k = s_key[p];
                const uint32_t g = s_gbase[k >> shift] + p;
                if (g < n) {              // always true when the counts are right; never write out of bounds
                    const uint32_t idx = base + (uint32_t)s_val[p];
                    b2_put<KOUT>(keys_out, vals_out, g, k, idx, pk);
                }
            }
        }
    } else {
        constexpr int WB = 8;
#pragma unroll
        for (int j0 = 0; j0 < IT; j0 += WB) {
            uint32_t kq[WB], gq[WB], vq[WB];
#pragma unroll
            for (int u = 0; u < WB; ++u) kq[u] = s_key[(j0 + u) * NT + threadIdx.x];
#pragma unroll
            for (int u = 0; u < WB; ++u)
                gq[u] = s_gbase[min(kq[u] >> shift, (uint32_t)RMAX - 1u)] + (j0 + u) * NT + threadIdx.x;
#pragma unroll
            for (int u = 0; u < WB; ++u) vq[u] = s_val[(j0 + u) * NT + threadIdx.x];
#pragma unroll
            for (int u = 0; u < WB; ++u)
                if ((j0 + u) * NT + threadIdx.x < cnt_tile && gq[u] < n)   // g < n: as above
                    b2_put<KOUT>(keys_out, vals_out, gq[u], kq[u], base + vq[u], pk);
        }
    }
    if (!more) break;
    tile = ntile;
    __syncthreads();                      // s_key / s_val / s_gbase / s_cnt are the next tile's
    }
}

}  // namespace gd
