// gd_msd2.h -- gfx950 device code for the three-pass form of the two-level bucketing (SURVEY 8 a16,
// the per-activation FIFO): the stable partition of message indices by
// min(act, n_act) when n_act is past the one-pass form's digit (n_act >= 1,081,344: BASELINE cfg 3's
// 100M activations, 12.5M a GPU at W = 8, cfg 4's 10M), up to n_act < 2^28.
//
// Ranges of 1,024 activations, k' = min(act, n_act) >> 10 (17 bits at cfg 3), split k' = (d2, d1):
//   pass A  k_b2_hist / row scan / k_b2_scatter (gd_bucket2.h) on d2 = k' >> a (<= 512 digits):
//           every d2 segment contiguous, in message order; the whole clamped key (u32) and the index
//           (u32) written, 8 B a record;
//   pass B  segmented MSD on d1 = k' & (2^a - 1) (<= 512 digits) inside each d2 segment: tiles never
//           cross a segment (k_seg_table lays them out), counts laid out [segment][digit][tile], and ONE
//           flat exclusive scan of that array gives every (segment, digit, tile) its absolute output
//           position -- so each range's start is a lookup, with no atomics and no min-scan over
//           the activations.  Writes the range-local key (key & 1023, u16) and the index (u32), 6 B;
//   level 2 k_l2_classify sorts the ranges into three work lists by their message count S:
//             S <= t_small      k_l2_small, one wave a range (its 1,024 counters in 4 KB of LDS);
//             S <= t_mid        k_msd_local_list<512, 16> (gd_msd.h), one 512-thread workgroup a
//                               range, staged in LDS, three workgroups a CU (t_mid <= 8,192);
//             S <= t_staged     k_msd_local_list<1024, 24>, one 1,024-thread workgroup a range
//                               (t_staged <= MSD_CAP);
//             S >  t_staged     chunks of CH_CAP messages, several workgroups a range: k_l2_chunk_hist
//                               (per-chunk activation counts) -> k_l2_chunk_scan (exclusive prefix of
//                               each activation's counts over the range's chunks, 16-activation columns
//                               scanned in LDS) -> k_l2_chunk_scatter (ranked and staged in LDS like a
//                               range, written at each activation's base for that chunk).
//           Every level-2 kernel writes the bucket starts of the activations it owns (empty ones
//           included), so offsets is written exactly once.
// A Zipf-hot range (BASELINE cfg 3: acts 0..1,023 take ~60 % of a batch) is spread over as many
// workgroups as it has chunks: no range serialises on one CU.
// Per message: 4 + 12 (pass A: histogram, scatter) + 4 + 14 (pass B) + 6 + 4 (level 2) B, plus 4 B a
// activation for the starts -- 44 B + 4 n_act / n, against 4 x (4 + 16) B + three passes over the
// starts (fill, lowered, min-scanned) for four 7-bit LSD passes at cfg 3.  Stability: every pass ranks
// a tile in index order (ds_add_rtn serves the lanes of one instruction in lane order), the
// level-2 forms rank rows in order, chunks in order.  HBM-bound, no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_bucket2.h"
#include "gd_kernels.h"
#include "gd_msd.h"

namespace gd {

constexpr int SEG_NT = 512;                    // pass B tile: 512 threads x 16 items (as pass A)
constexpr int SEG_IT = 16;
constexpr uint32_t SEG_TILE = SEG_NT * SEG_IT;
constexpr uint32_t SEG_RMAX = 512;             // digits of either pass (a, kb - a <= 9 bits)
constexpr uint32_t L2_SMALL_WAVES = 8;         // k_l2_small: waves a workgroup, one range each
constexpr int CH_NT = 512;                     // chunk workgroups: 8 waves (two workgroups a CU, 72 KB of LDS each)
constexpr int CH_NW = CH_NT / WAVE;
constexpr uint32_t CH_CAP = 8192;              // messages a chunk of a hot range (16 rows x 512 lanes)
constexpr uint32_t CH_RW = CH_CAP / CH_NT;
constexpr uint32_t L2_CTR_WORDS = 8;           // [0] small ranges, [1] staged ranges, [2] chunks, [3] chunked ranges,
                                               // [4] chunk-scan items, [5] mid ranges

// Wave-local LDS hand-off: the wave's earlier LDS writes are complete and visible to its other lanes.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The d2 segments' starts (exclusive prefix of pass A's digit totals) and tile bases
// (exclusive prefix of ceil(size / SEG_TILE)), every pass-B tile's segment (NONE32 past the last), and
// the level-2 counters zeroed.  ra <= SEG_RMAX.
static __global__ void __launch_bounds__(1024) k_seg_table(const uint32_t* __restrict__ totals, uint32_t ra,
                                                    uint32_t tbound, uint32_t* __restrict__ seg_start,
                                                    uint32_t* __restrict__ seg_tb, uint32_t* __restrict__ tile_seg,
                                                    uint32_t* __restrict__ ctr) {
    __shared__ uint32_t s_wsum[2 * 1024 / WAVE];
    __shared__ uint32_t s_tb[SEG_RMAX + 1];
    // every workgroup scans the <= 512 totals itself and fills its 1,024 tiles; workgroup 0 writes the
    // segment tables and zeroes the counters
    const uint32_t t = threadIdx.x;
    const uint32_t v = t < ra ? totals[t] : 0u;
    const uint32_t nt = (v + SEG_TILE - 1) / SEG_TILE;
    uint32_t es, et;
    block_excl_scan_add2<1024>(v, nt, s_wsum, es, et);
    const bool w0 = blockIdx.x == 0;
    if (t < ra) {
        if (w0) {
            seg_start[t] = es;
            seg_tb[t] = et;
        }
        s_tb[t] = et;
    }
    if (t == ra - 1) {
        if (w0) {
            seg_start[ra] = es + v;
            seg_tb[ra] = et + nt;
        }
        s_tb[ra] = et + nt;
    }
    if (w0 && t < L2_CTR_WORDS) ctr[t] = 0;
    __syncthreads();
    const uint32_t total = s_tb[ra];
    for (uint32_t j = blockIdx.x * 1024 + t; j < tbound; j += gridDim.x * 1024) {
        uint32_t s = NONE32;
        if (j < total) {
            uint32_t lo = 0, hi = ra;                // largest s < ra with s_tb[s] <= j
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_tb[mid] <= j) lo = mid;
                else hi = mid;
            }
            s = lo;
        }
        tile_seg[j] = s;
    }
}

// A pass-B tile: its segment s, the tile's index in the segment tl, the segment's tiles ts and tile
// base tb, its first item and item count.
struct SegTile {
    uint32_t s, tl, ts, tb, base, cnt;
};
__device__ __forceinline__ bool seg_tile(uint32_t j, const uint32_t* tile_seg, const uint32_t* seg_start,
                                         const uint32_t* seg_tb, SegTile& st) {
    st.s = tile_seg[j];
    if (st.s == NONE32) return false;
    st.tb = seg_tb[st.s];
    st.ts = seg_tb[st.s + 1] - st.tb;
    st.tl = j - st.tb;
    st.base = seg_start[st.s] + st.tl * SEG_TILE;
    st.cnt = min(SEG_TILE, seg_start[st.s + 1] - st.base);
    return true;
}

// Pass A's records as pass B reads them: PK (the default where the index leaves room): u16 keys16 =
// P >> hb and the u32 index word idx | (P & (2^hb - 1)) << ib, P = key & (2^(a + 10) - 1) (6 B);
// else the whole key (u32 keys32) and the index (8 B).
struct SegIn {
    const uint16_t* keys16;
    const uint32_t* keys32;
    const uint32_t* vals;
    uint32_t hb, ib;
};

// Pass B histogram: tile j's counts of d1 = (key >> 10) & (rb - 1), written at
// hseg[tb * rb + d * ts + tl] (segment-major, then digit-major, then tile).  PK reads the u16 keys
// alone, 16 B a load from the 16-B boundary at or below the tile's first item (items outside the tile
// masked): 2 B a message.
template <bool PK>
static __global__ void __launch_bounds__(SEG_NT) k_seg_hist(SegIn in, const uint32_t* __restrict__ tile_seg,
                                                     const uint32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ seg_tb, uint32_t rb,
                                                     uint32_t* __restrict__ hseg) {
    constexpr uint32_t PER = PK ? 8u : 4u;               // items a 16-B load
    constexpr uint32_t NL = SEG_IT / PER;                // 16-B loads a thread covering the aligned tile
    __shared__ uint32_t s_cnt[SEG_RMAX];
    __shared__ uint32_t s_sink[WAVE];                    // the adds of keys not counted there (hist_add)
    SegTile st;
    // XCD-contiguous tiles (xcd_tile): the digit-major counts of neighbouring tiles share cache lines,
    // which then fill in one L2 instead of going out as partial-line writes from eight
    if (!seg_tile(xcd_tile(blockIdx.x, gridDim.x, 1u), tile_seg, seg_start, seg_tb, st)) return;
    for (uint32_t d = threadIdx.x; d < SEG_RMAX; d += SEG_NT) s_cnt[d] = 0;
    const uint32_t lane = lane_id();
    const uint32_t a0 = st.base & ~(PER - 1);            // aligned start: the loads cover [a0, a0 + TILE + PER)
    const uint32_t dsh = PK ? B2_LOW_BITS - in.hb : B2_LOW_BITS;
    uint4 v[NL + 1];
#pragma unroll
    for (uint32_t j = 0; j < NL; ++j) {                  // no load starts past the tile (the array may end there)
        const uint32_t e = a0 + PER * (j * SEG_NT + threadIdx.x);
        v[j] = make_uint4(0, 0, 0, 0);
        if (e < st.base + st.cnt)
            v[j] = PK ? *reinterpret_cast<const uint4*>(in.keys16 + e) : *reinterpret_cast<const uint4*>(in.keys32 + e);
    }
    const uint32_t et = a0 + PER * (NL * SEG_NT + threadIdx.x);     // the tail past the aligned tile
    v[NL] = make_uint4(0, 0, 0, 0);
    if (threadIdx.x == 0 && et < st.base + st.cnt)
        v[NL] = PK ? *reinterpret_cast<const uint4*>(in.keys16 + et) : *reinterpret_cast<const uint4*>(in.keys32 + et);
    __syncthreads();
    // the wave's hot digit (from its first load's last key: past a misaligned segment start) in a
    // register, every other key one LDS add
    uint32_t h, hc = 0;
    {
        const uint32_t e = a0 + PER * threadIdx.x + PER - 1;
        const uint32_t k = PK ? v[0].w >> 16 : v[0].w;
        h = wave_hot_digit((k >> dsh) & (rb - 1), e >= st.base && e < st.base + st.cnt);
    }
    auto count = [&](const uint4& vj, uint32_t e0) {
        const uint32_t w4[4] = {vj.x, vj.y, vj.z, vj.w};
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) {
            const uint32_t e = e0 + q;
            const uint32_t k = PK ? (w4[q / 2] >> (16 * (q & 1))) & 0xFFFFu : w4[q];
            const uint32_t d = (k >> dsh) & (rb - 1);
            hist_add(s_cnt, s_sink, d, h, e - st.base < st.cnt, hc);
        }
    };
#pragma unroll
    for (uint32_t j = 0; j < NL; ++j) count(v[j], a0 + PER * (j * SEG_NT + threadIdx.x));
    if (threadIdx.x == 0) count(v[NL], et);              // the tail past the aligned tile: one thread
    hc = wave_sum(hc);
    if (lane == 0 && hc) atomicAdd(&s_cnt[h], hc);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < rb; d += SEG_NT) hseg[(size_t)st.tb * rb + (size_t)d * st.ts + st.tl] = s_cnt[d];
}

// Pass B scatter: tile j's records ranked stably by d1 and written at the flat-scanned positions
// hseg[tb * rb + d * ts + tl] + rank: the range-local key (key & 1023) as u16 and the index.
template <bool PK, bool BALLOT = false>
static __global__ void __launch_bounds__(SEG_NT) k_seg_scatter(SegIn in, const uint32_t* __restrict__ tile_seg,
                                                        const uint32_t* __restrict__ seg_start,
                                                        const uint32_t* __restrict__ seg_tb, uint32_t rb,
                                                        const uint32_t* __restrict__ hseg,
                                                        uint16_t* __restrict__ keys_out,
                                                        uint32_t* __restrict__ vals_out, uint32_t xcd) {
    constexpr int NW = SEG_NT / WAVE;
    constexpr int IT = SEG_IT;
    __shared__ uint32_t s_cnt[NW / 2][SEG_RMAX];         // wave pair (2p, 2p + 1): low / high 16 bits
    __shared__ uint32_t s_gbase[SEG_RMAX];
    __shared__ uint32_t s_key[SEG_TILE];                 // the key's low a + 10 bits
    __shared__ uint32_t s_val[SEG_TILE];
    __shared__ uint32_t s_wsum[NW];
    SegTile st;
    if (!seg_tile(xcd_tile(blockIdx.x, gridDim.x, xcd), tile_seg, seg_start, seg_tb, st)) return;
    const uint32_t mask = rb - 1;
    for (uint32_t d = threadIdx.x; d < SEG_RMAX; d += SEG_NT) {
#pragma unroll
        for (int p = 0; p < NW / 2; ++p) s_cnt[p][d] = 0;
        s_gbase[d] = d < rb ? hseg[(size_t)st.tb * rb + (size_t)d * st.ts + st.tl] : 0u;
    }
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x / WAVE;
    const uint32_t half = (w & 1u) * 16u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const uint32_t imask = PK ? (in.ib >= 32 ? 0xFFFFFFFFu : (1u << in.ib) - 1u) : 0xFFFFFFFFu;
    uint32_t kk[IT], vv[IT], rk[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t p = st.base + min((w * IT + r) * WAVE + lane, st.cnt - 1);
        vv[r] = __builtin_nontemporal_load(in.vals + p);
        if constexpr (PK) kk[r] = in.keys16[p];
        else kk[r] = __builtin_nontemporal_load(in.keys32 + p);
    }
    if constexpr (PK) {
#pragma unroll
        for (int r = 0; r < IT; ++r) {                   // P = the u16 << hb | the index word's top hb bits
            kk[r] = (kk[r] << in.hb) | (in.hb ? vv[r] >> in.ib : 0u);
            vv[r] &= imask;
        }
    }
    __syncthreads();
    // stable rank within the wave: the wave's hot digit by ballot in registers, the rest by row_rank16
    const uint32_t h = wave_hot_digit((kk[0] >> B2_LOW_BITS) & mask, w * IT * WAVE + lane < st.cnt);
    uint32_t hrun = 0;
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const bool valid = (w * IT + r) * WAVE + lane < st.cnt;
        const uint32_t d = (kk[r] >> B2_LOW_BITS) & mask;
        const unsigned long long hm = __ballot(valid && d == h);
        const uint32_t cr = row_rank16<BALLOT, 9>(&s_cnt[w >> 1][d], half, d, valid && d != h);
        rk[r] = d == h ? hrun + (uint32_t)__popcll(hm & lt) : cr;
        hrun += (uint32_t)__popcll(hm);
    }
    if (lane == 0 && hrun) atomicAdd(&s_cnt[w >> 1][h], hrun << half);
    __syncthreads();
    // per digit (one a thread): the waves' exclusive prefix into the halves, the tile-local digit start
    uint32_t run = 0;
    {
        const uint32_t d = threadIdx.x;
#pragma unroll
        for (int p = 0; p < NW / 2; ++p) {
            const uint32_t c = s_cnt[p][d];
            const uint32_t lo = c & 0xFFFFu, hi = c >> 16;
            s_cnt[p][d] = run | ((run + lo) << 16);
            run += lo + hi;
        }
    }
    const uint32_t ex = block_excl_scan_add_n<SEG_NT>(run, s_wsum);
    {
        const uint32_t d = threadIdx.x;
#pragma unroll
        for (int p = 0; p < NW / 2; ++p) s_cnt[p][d] += ex | (ex << 16);
        s_gbase[d] -= ex;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        if ((w * IT + r) * WAVE + lane < st.cnt) {
            const uint32_t d = (kk[r] >> B2_LOW_BITS) & mask;
            const uint32_t at = ((s_cnt[w >> 1][d] >> half) & 0xFFFFu) + rk[r];
            s_key[at] = kk[r];
            s_val[at] = vv[r];
        }
    }
    __syncthreads();
    // the write-out reads its LDS in batches of WB items (every key, every digit base, every index, then
    // the stores), not one item's dependent reads and a wait at a time (k_b2_scatter's write-out): cfg 3
    // 0.193 -> 0.185 ms (profiles/r05_writeout_batch_ab.txt)
    constexpr int WB = 8;
#pragma unroll
    for (int j0 = 0; j0 < IT; j0 += WB) {
        uint32_t kq[WB], gq[WB], vq[WB];
#pragma unroll
        for (int u = 0; u < WB; ++u) kq[u] = s_key[(j0 + u) * SEG_NT + threadIdx.x];
#pragma unroll
        for (int u = 0; u < WB; ++u) gq[u] = s_gbase[(kq[u] >> B2_LOW_BITS) & mask] + (j0 + u) * SEG_NT + threadIdx.x;
#pragma unroll
        for (int u = 0; u < WB; ++u) vq[u] = s_val[(j0 + u) * SEG_NT + threadIdx.x];
#pragma unroll
        for (int u = 0; u < WB; ++u)
            if ((j0 + u) * SEG_NT + threadIdx.x < st.cnt) {
                keys_out[gq[u]] = (uint16_t)(kq[u] & ((1u << B2_LOW_BITS) - 1));
                vals_out[gq[u]] = vq[u];
            }
    }
}

// Start of range b in pass B's output: the flat-scanned count of its (segment, digit) row's first
// tile, or the segment start when the segment has no tile.
__device__ __forceinline__ uint32_t range_start(uint32_t b, uint32_t a, const uint32_t* hseg,
                                                const uint32_t* seg_start, const uint32_t* seg_tb) {
    const uint32_t s = b >> a, d = b & ((1u << a) - 1);
    const uint32_t tb = seg_tb[s], ts = seg_tb[s + 1] - tb;
    return ts ? hseg[(size_t)tb * (1u << a) + (size_t)d * ts] : seg_start[s];
}

struct L2Lists {
    uint32_t* rs;          // [R + 1] range starts
    uint32_t* small;       // [R]
    uint32_t* staged;      // [R]
    uint32_t* mid;         // [R]
    uint32_t* cr_b;        // chunked ranges: range, first chunk, chunks
    uint32_t* cr_cb;
    uint32_t* cr_n;
    uint32_t* chunk_r;     // chunk -> chunked range
    uint32_t* cr_ib;       // chunked range -> its first chunk-scan item
    uint32_t* item_r;      // chunk-scan item -> chunked range
    uint32_t* ctr;         // L2_CTR_WORDS
};

constexpr uint32_t CS_COLS = 16;               // k_l2_chunk_scan: activations a slab
constexpr uint32_t CS_ROWS = 1024;             // chunks a piece
constexpr uint32_t CS_DIRECT = 64;             // ranges of at most this many chunks: one item, no slabs
constexpr uint32_t CS_SLABS = MSD_L / CS_COLS;
__host__ __device__ __forceinline__ uint32_t cs_items(uint32_t C) {
    return C <= CS_DIRECT ? 1u : CS_SLABS * ((C + CS_ROWS - 1) / CS_ROWS);
}

// Range b's start and size, and its work list.  Appends are aggregated per workgroup (one atomic a
// workgroup and counter: ~100 workgroups at cfg 3 instead of one atomic a wave and list, which queued
// ~7,000 same-address device atomics); range b + 1's start comes from the next lane.  A chunked range
// reserves its chunks and its entry with one 64-bit atomic (chunks in the low word, ranges in the high
// word), so the chunked ranges' first chunks increase with their entries.
constexpr int CL_NT = 1024;                    // (256: 0.025 -> 0.031 ms at cfg 3, the list order less sequential)
constexpr int CL_NW = CL_NT / WAVE;
static __global__ void __launch_bounds__(CL_NT) k_l2_classify(const uint32_t* __restrict__ hseg,
                                                       const uint32_t* __restrict__ seg_start,
                                                       const uint32_t* __restrict__ seg_tb, uint32_t a, uint32_t R,
                                                       uint32_t n, uint32_t t_small, uint32_t t_mid,
                                                       uint32_t t_staged, L2Lists l) {
    // per wave, then (exclusive-scanned) per workgroup: [0] small, [1] staged, [2] mid, [3] chunked
    // ranges, [4] chunks, [5] chunk-scan items
    __shared__ uint32_t s_c[6][CL_NW];
    __shared__ uint32_t s_base[6];
    const uint32_t b = blockIdx.x * CL_NT + threadIdx.x;
    const uint32_t lane = lane_id(), w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const bool valid = b < R;
    const uint32_t r0 = valid ? range_start(b, a, hseg, seg_start, seg_tb) : n;
    uint32_t r1 = __shfl_down(r0, 1, WAVE);
    if (lane == WAVE - 1) r1 = b + 1 < R ? range_start(b + 1, a, hseg, seg_start, seg_tb) : n;
    uint32_t S = 0, cls = 7;                         // 7: no range (past R)
    if (valid) {
        l.rs[b] = r0;
        if (b + 1 == R) l.rs[R] = n;
        S = r1 - r0;
        cls = S <= t_small ? 0u : (S <= min(t_mid, t_staged) ? 3u : (S <= t_staged ? 1u : 2u));
    }
    const unsigned long long m0 = __ballot(cls == 0), m1 = __ballot(cls == 1), m3 = __ballot(cls == 3);
    const unsigned long long mc = __ballot(cls == 2);
    const uint32_t C = cls == 2 ? (S + CH_CAP - 1) / CH_CAP : 0u;
    const uint32_t ni = cls == 2 ? cs_items(C) : 0u;
    const uint32_t cincl = wave_incl_sum_dpp(C), iincl = wave_incl_sum_dpp(ni);
    if (lane == WAVE - 1) {
        s_c[0][w] = (uint32_t)__popcll(m0);
        s_c[1][w] = (uint32_t)__popcll(m1);
        s_c[2][w] = (uint32_t)__popcll(m3);
        s_c[3][w] = (uint32_t)__popcll(mc);
        s_c[4][w] = cincl;
        s_c[5][w] = iincl;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const uint32_t c = threadIdx.x;
        uint32_t run = 0;
#pragma unroll
        for (int q = 0; q < CL_NW; ++q) {
            const uint32_t v = s_c[c][q];
            s_c[c][q] = run;
            run += v;
        }
        s_base[c] = run;                             // the workgroup's total, for now
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const uint32_t c = threadIdx.x;
        const uint32_t tot = s_base[c];
        uint32_t base = 0;
        if (c == 3) {                                // ranges and chunks together
            const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(l.ctr + 2),
                                                     ((unsigned long long)tot << 32) | s_base[4]);
            base = (uint32_t)(old >> 32);
            s_base[4] = (uint32_t)old;               // c = 4 reads it after the barrier below
        } else if (c != 4 && tot) {
            base = atomicAdd(&l.ctr[c == 0 ? 0u : (c == 1 ? 1u : (c == 2 ? 5u : 4u))], tot);
        }
        if (c != 4) s_base[c] = base;
    }
    __syncthreads();
    if (cls == 0) l.small[s_base[0] + s_c[0][w] + (uint32_t)__popcll(m0 & lt)] = b;
    if (cls == 1) l.staged[s_base[1] + s_c[1][w] + (uint32_t)__popcll(m1 & lt)] = b;
    if (cls == 3) l.mid[s_base[2] + s_c[2][w] + (uint32_t)__popcll(m3 & lt)] = b;
    if (mc == 0) return;
    const uint32_t my_r = s_base[3] + s_c[3][w] + (uint32_t)__popcll(mc & lt);
    const uint32_t my_cb = s_base[4] + s_c[4][w] + cincl - C;
    const uint32_t my_ib = s_base[5] + s_c[5][w] + iincl - ni;
    if (cls == 2) {
        l.cr_b[my_r] = b;
        l.cr_cb[my_r] = my_cb;
        l.cr_n[my_r] = C;
        l.cr_ib[my_r] = my_ib;
    }
    // the chunk -> range map, written by the whole wave one chunked lane at a time
    unsigned long long rem = mc;
    while (rem) {
        const uint32_t src = (uint32_t)__ffsll((long long)rem) - 1;
        rem &= rem - 1;
        const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)my_r, (int)src);
        const uint32_t cb = (uint32_t)__builtin_amdgcn_readlane((int)my_cb, (int)src);
        const uint32_t cn = (uint32_t)__builtin_amdgcn_readlane((int)C, (int)src);
        for (uint32_t c = lane; c < cn; c += WAVE) l.chunk_r[cb + c] = r;
        const uint32_t ib = (uint32_t)__builtin_amdgcn_readlane((int)my_ib, (int)src);
        const uint32_t in_ = (uint32_t)__builtin_amdgcn_readlane((int)ni, (int)src);
        for (uint32_t i = lane; i < in_; i += WAVE) l.item_r[ib + i] = r;
    }
}

// Level 2, thin ranges (S <= t_small): one wave a range, its 1,024 counters in the wave's 4 KB of LDS:
// count, exclusive scan (16 DPP wave scans, written out as the range's bucket starts), then rows in
// order ranked by ds_add_rtn (stable) and stored at their places in the range's slice of perm.
// A wave walks its ranges software-pipelined: the next range's records (when it has at most U rows)
// are loaded while this one is scanned and written, and the range after that one's list entry and
// starts before then -- each range is three dependent HBM round trips (list, starts, records), which
// left the thin ranges of BASELINE cfg 3 (~96K ranges of ~60 messages) latency-bound.
template <bool BALLOT>
static __global__ void __launch_bounds__(L2_SMALL_WAVES * WAVE) k_l2_small(const uint16_t* __restrict__ keys16,
                                                                   const uint32_t* __restrict__ idx, L2Lists l,
                                                                   uint32_t n, uint32_t n_act,
                                                                   uint32_t* __restrict__ perm,
                                                                   uint32_t* __restrict__ offsets,
                                                                   uint32_t* __restrict__ rank_out) {
    __shared__ uint32_t s_cnt[L2_SMALL_WAVES][MSD_L];
    const uint32_t lane = lane_id(), w = threadIdx.x / WAVE;
    uint32_t* cnt = s_cnt[w];
    const uint32_t m = l.ctr[0];
    const uint32_t stride = gridDim.x * L2_SMALL_WAVES;
    constexpr uint32_t U = 4;
    uint32_t i = blockIdx.x * L2_SMALL_WAVES + w;
    if (i >= m) return;
    // the pipeline: this range (b, base, S; its records in ck / cv when S <= U rows), the next (nb, nbase,
    // nS), the one after (bb: its list entry only)
    uint32_t b = l.small[i];
    uint32_t base = l.rs[b], S = l.rs[b + 1] - base;
    uint32_t nb = i + stride < m ? l.small[i + stride] : 0u;
    uint32_t nbase = l.rs[nb], nS = l.rs[nb + 1] - nbase;
    uint32_t ck[U], cv[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const uint32_t j = u * WAVE + lane;
        ck[u] = S <= U * WAVE && j < S ? (uint32_t)keys16[base + j] : NONE32;
        cv[u] = S <= U * WAVE && j < S ? idx[base + j] : 0u;
    }
    for (; i < m; i += stride) {
        const uint32_t k0 = b << MSD_SHIFT;
        const uint32_t L = min(MSD_L, n_act + 1 - k0);
        const uint16_t* rk = keys16 + base;
        const uint32_t* ri = idx + base;
        const bool reg = S <= U * WAVE;
#pragma unroll
        for (uint32_t q = 0; q < MSD_L / (4 * WAVE); ++q) reinterpret_cast<uint4*>(cnt)[q * WAVE + lane] = make_uint4(0, 0, 0, 0);
        wave_lds_sync();
        if (reg) {
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (ck[u] != NONE32) atomicAdd(&cnt[ck[u]], 1u);
        }
        for (uint32_t i0 = 0; !reg && i0 < S; i0 += U * WAVE) {
            uint32_t k[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t j = i0 + u * WAVE + lane;
                k[u] = j < S ? (uint32_t)rk[j] : NONE32;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (k[u] != NONE32) atomicAdd(&cnt[k[u]], 1u);
        }
        // in flight during the scan and the ranking: the next range's records, the list entry after it
        const bool has_next = i + stride < m;
        const bool nreg = has_next && nS <= U * WAVE;
        uint32_t nk[U], nv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t j = u * WAVE + lane;
            nk[u] = nreg && j < nS ? (uint32_t)keys16[nbase + j] : NONE32;
            nv[u] = nreg && j < nS ? idx[nbase + j] : 0u;
        }
        const uint32_t bb = i + 2 * stride < m ? l.small[i + 2 * stride] : 0u;
        wave_lds_sync();
        uint32_t carry = 0;
#pragma unroll
        for (uint32_t q = 0; q < MSD_L / WAVE; ++q) {
            const uint32_t x = cnt[q * WAVE + lane];
            const uint32_t inc = wave_incl_sum_dpp(x);
            const uint32_t e = carry + inc - x;
            cnt[q * WAVE + lane] = e;
            if (q * WAVE + lane < L) __builtin_nontemporal_store(base + e, offsets + k0 + q * WAVE + lane);
            carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, WAVE - 1);
        }
        if (lane == 0 && b == (n_act >> MSD_SHIFT)) offsets[n_act + 1] = n;
        wave_lds_sync();
        if (reg) {
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const bool valid = ck[u] != NONE32;
                const uint32_t kq = valid ? ck[u] : 0u;
                const uint32_t p = base + row_rank32<BALLOT, 10>(&cnt[kq], kq, valid);
                if (!valid) continue;
                perm[p] = cv[u];
                if (rank_out) rank_out[cv[u]] = p;
            }
        }
        for (uint32_t i0 = 0; !reg && i0 < S; i0 += U * WAVE) {
            uint32_t k[U], v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t j = i0 + u * WAVE + lane;
                k[u] = j < S ? (uint32_t)rk[j] : NONE32;
                v[u] = j < S ? ri[j] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const bool valid = k[u] != NONE32;
                const uint32_t kq = valid ? k[u] : 0u;
                const uint32_t p = base + row_rank32<BALLOT, 10>(&cnt[kq], kq, valid);
                if (!valid) continue;
                perm[p] = v[u];
                if (rank_out) rank_out[v[u]] = p;
            }
        }
        wave_lds_sync();
        // rotate: next -> this, the one after -> next (its starts loaded now)
        b = nb;
        base = nbase;
        S = nS;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            ck[u] = nk[u];
            cv[u] = nv[u];
        }
        nb = bb;
        nbase = l.rs[nb];
        nS = l.rs[nb + 1] - nbase;
    }
}

// Chunk order of the persistent level-2 grids: workgroup b runs on XCD b % 8 (round-robin dispatch),
// and the workgroups of one XCD walk one contiguous eighth of the chunks together, so the neighbouring
// chunks of a hot range -- whose runs of one activation lie side by side in perm -- meet in one L2.
struct ChunkWalk {
    uint32_t j, end, step;
};
__device__ __forceinline__ ChunkWalk chunk_walk(uint32_t m) {
    const uint32_t g = gridDim.x;
    if (g % 8u) return ChunkWalk{blockIdx.x, m, g};
    const uint32_t x = blockIdx.x & 7u, k = blockIdx.x >> 3, per = g >> 3;
    const uint32_t q = m >> 3, rem = m & 7u;
    const uint32_t lo = x * q + min(x, rem), hi = lo + q + (x < rem ? 1u : 0u);
    return ChunkWalk{lo + k, hi, per};
}

// Level 2, hot ranges: chunk j's activation counts, hh[j * 1,024 + a].
static __global__ void __launch_bounds__(CH_NT) k_l2_chunk_hist(const uint16_t* __restrict__ keys16, L2Lists l,
                                                         uint32_t* __restrict__ hh) {
    __shared__ uint32_t s_cnt[MSD_L];
    __shared__ uint32_t s_sink[WAVE];
    const uint32_t tid = threadIdx.x, lane = lane_id();
    const ChunkWalk cw = chunk_walk(l.ctr[2]);
    for (uint32_t j = cw.j; j < cw.end; j += cw.step) {
        const uint32_t r = l.chunk_r[j], b = l.cr_b[r];
        const uint32_t rsb = l.rs[b], c = j - l.cr_cb[r];
        const uint32_t start = rsb + c * CH_CAP, cs = min(CH_CAP, l.rs[b + 1] - start);
        for (uint32_t x = tid; x < MSD_L; x += CH_NT) s_cnt[x] = 0;
        // 16-B loads of 8 keys from the 16-B boundary at or below the chunk's first key (keys outside the
        // chunk masked), 2 a thread, and one more for the tail past the aligned span
        const uint32_t a0 = start & ~7u;
        uint4 v[CH_RW / 8 + 1];
#pragma unroll
        for (uint32_t q = 0; q < CH_RW / 8; ++q) {
            const uint32_t e = a0 + 8 * (q * CH_NT + tid);
            v[q] = e < start + cs ? *reinterpret_cast<const uint4*>(keys16 + e) : make_uint4(0, 0, 0, 0);
        }
        const uint32_t et = a0 + CH_CAP;
        v[CH_RW / 8] = tid == 0 && et < start + cs ? *reinterpret_cast<const uint4*>(keys16 + et) : make_uint4(0, 0, 0, 0);
        __syncthreads();
        // the wave's hot activation (its first load's last key) in a register, every other key one LDS add
        const uint32_t h = wave_hot_digit(v[0].w >> 16, a0 + 8 * tid + 7 >= start && a0 + 8 * tid + 7 < start + cs);
        uint32_t hc = 0;
        auto count = [&](const uint4& vq, uint32_t e0) {
            const uint32_t w4[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
            for (uint32_t x = 0; x < 8; ++x) {
                const uint32_t e = e0 + x;
                const uint32_t k = (w4[x / 2] >> (16 * (x & 1))) & 0xFFFFu;
                hist_add(s_cnt, s_sink, k, h, e - start < cs, hc);
            }
        };
#pragma unroll
        for (uint32_t q = 0; q < CH_RW / 8; ++q) count(v[q], a0 + 8 * (q * CH_NT + tid));
        if (tid == 0) count(v[CH_RW / 8], et);           // the tail past the aligned chunk: one thread
        hc = wave_sum(hc);
        if (lane == 0 && hc) atomicAdd(&s_cnt[h], hc);
        __syncthreads();
        for (uint32_t x = tid; x < MSD_L; x += CH_NT) hh[(size_t)j * MSD_L + x] = s_cnt[x];
        __syncthreads();
    }
}

// Level 2, hot ranges: the exclusive prefix of each activation's chunk counts over its range's chunks,
// in place (hh), and each activation's total (tot).  A range of at most CS_DIRECT chunks is one work
// item: thread a walks column a down the range's chunks (coalesced 4-KB rows, 8 loads in flight).  A
// longer one (BASELINE cfg 3's hottest range: ~4,900 chunks) is cut into 64 slabs of 16 activations
// (one 64-B line a chunk) x pieces of CS_ROWS chunks, every (slab, piece) an item of its own, in two
// launches: k_l2_chunk_ptot sums each piece's columns, k_l2_chunk_scan scans each piece in LDS (rows
// padded to 17 words: conflict-free column scans; one wave a column, DPP scans of 64 rows) starting
// from the sum of the pieces before it.  (One item walking all of a slab's pieces left the hottest
// range's ~5 pieces in series: 0.064 ms at cfg 3.)
struct CsItem {
    uint32_t r, g, p, cb, C, pieces;
};
// Item it (k_l2_classify laid the items out: cs_items a chunked range): its range, slab and piece.
__device__ __forceinline__ void cs_item(const L2Lists& l, uint32_t it, CsItem& x) {
    x.r = l.item_r[it];
    x.cb = l.cr_cb[x.r];
    x.C = l.cr_n[x.r];
    x.pieces = x.C <= CS_DIRECT ? 1u : (x.C + CS_ROWS - 1) / CS_ROWS;
    const uint32_t li = it - l.cr_ib[x.r];
    x.g = li / x.pieces;
    x.p = li % x.pieces;
}

// One piece of one slab into LDS (rows past the piece zero up to the next 64).  Returns the rows.
__device__ __forceinline__ uint32_t cs_load(const uint32_t* hh, const CsItem& x, uint32_t* s_m) {
    const uint32_t tid = threadIdx.x;
    const uint32_t c0 = x.p * CS_ROWS, rows = min(CS_ROWS, x.C - c0);
    const uint32_t rows64 = (rows + WAVE - 1) & ~(WAVE - 1);
    uint32_t* d = s_m + tid * (CS_COLS + 1);             // CS_ROWS == MSD_NT: one row a thread
    if (tid < rows) {
        const uint4* src = reinterpret_cast<const uint4*>(hh + (size_t)(x.cb + c0 + tid) * MSD_L + x.g * CS_COLS);
#pragma unroll
        for (uint32_t q = 0; q < CS_COLS / 4; ++q) {
            const uint4 v = src[q];
            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
        }
    } else if (tid < rows64) {
#pragma unroll
        for (uint32_t q = 0; q < CS_COLS; ++q) d[q] = 0;
    }
    return rows;
}

// ptot: one CS_COLS-word row a chunk-scan item (its piece's column sums), at the item's index.
static __global__ void __launch_bounds__(MSD_NT) k_l2_chunk_ptot(L2Lists l, const uint32_t* __restrict__ hh,
                                                          uint32_t* __restrict__ ptot) {
    __shared__ uint32_t s_m[CS_ROWS * (CS_COLS + 1)];
    const uint32_t lane = lane_id(), w = threadIdx.x / WAVE;
    const uint32_t items = l.ctr[4];
    for (uint32_t it = blockIdx.x; it < items; it += gridDim.x) {
        CsItem x;
        cs_item(l, it, x);
        if (x.C <= CS_DIRECT) continue;                  // uniform over the workgroup
        const uint32_t rows = cs_load(hh, x, s_m);
        __syncthreads();
        uint32_t sum = 0;                                // wave w: column w
        for (uint32_t q = 0; q < (rows + WAVE - 1) / WAVE; ++q) sum += s_m[(q * WAVE + lane) * (CS_COLS + 1) + w];
        sum = wave_incl_sum_dpp(sum);
        if (lane == WAVE - 1) ptot[(size_t)it * CS_COLS + w] = sum;
        __syncthreads();
    }
}

static __global__ void __launch_bounds__(MSD_NT) k_l2_chunk_scan(L2Lists l, uint32_t* __restrict__ hh,
                                                          const uint32_t* __restrict__ ptot,
                                                          uint32_t* __restrict__ tot) {
    __shared__ uint32_t s_m[CS_ROWS * (CS_COLS + 1)];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
    const uint32_t items = l.ctr[4];
    for (uint32_t it = blockIdx.x; it < items; it += gridDim.x) {
        CsItem x;
        cs_item(l, it, x);
        if (x.C <= CS_DIRECT) {
            uint32_t* col = hh + (size_t)x.cb * MSD_L + tid;
            uint32_t run = 0;
            for (uint32_t c0 = 0; c0 < x.C; c0 += 8) {
                uint32_t v[8];
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q) v[q] = c0 + q < x.C ? col[(size_t)(c0 + q) * MSD_L] : 0u;
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q) {
                    if (c0 + q < x.C) col[(size_t)(c0 + q) * MSD_L] = run;
                    run += v[q];
                }
            }
            tot[(size_t)x.r * MSD_L + tid] = run;
            continue;
        }
        // wave w: column w, carried in from the pieces before this one
        uint32_t carry = 0;
        const uint32_t* pt = ptot + ((size_t)l.cr_ib[x.r] + (size_t)x.g * x.pieces) * CS_COLS + w;
        for (uint32_t p = 0; p < x.p; ++p) carry += pt[(size_t)p * CS_COLS];
        const uint32_t rows = cs_load(hh, x, s_m);
        __syncthreads();
        for (uint32_t q = 0; q < (rows + WAVE - 1) / WAVE; ++q) {
            uint32_t* pp = s_m + (q * WAVE + lane) * (CS_COLS + 1) + w;
            const uint32_t v = *pp;
            const uint32_t inc = wave_incl_sum_dpp(v);
            *pp = carry + inc - v;
            carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, WAVE - 1);
        }
        __syncthreads();
        if (tid < rows) {
            const uint32_t* d = s_m + tid * (CS_COLS + 1);
            uint4* dst = reinterpret_cast<uint4*>(hh + (size_t)(x.cb + x.p * CS_ROWS + tid) * MSD_L + x.g * CS_COLS);
#pragma unroll
            for (uint32_t q = 0; q < CS_COLS / 4; ++q) dst[q] = make_uint4(d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]);
        }
        if (lane == 0 && x.p + 1 == x.pieces) tot[(size_t)x.r * MSD_L + x.g * CS_COLS + w] = carry;
        __syncthreads();
    }
}

// Level 2, hot ranges: chunk j = chunk c of range b, ranked and staged in LDS like a range
// (msd_range), each activation's items written at its start in the range + its count in the earlier
// chunks.  Chunk 0 writes the range's bucket starts.  512 threads, 8K messages: 72 KB of LDS, so two
// workgroups share a CU and one's memory phases run under the other's LDS phases (16K chunks on
// 1,024 threads took 136 KB: one a CU, 0.24 ms at cfg 3).  Thread t owns activations 2t, 2t + 1.
struct ChunkShared {
    uint32_t out[CH_CAP];
    uint16_t key[CH_CAP];
    uint32_t wc[CH_NW][MSD_LW];
    uint32_t delta[MSD_L];
    uint32_t red[CH_NW];
};
template <bool BALLOT>
static __global__ void __launch_bounds__(CH_NT, 2) k_l2_chunk_scatter(const uint16_t* __restrict__ keys16,
                                                               const uint32_t* __restrict__ idx, L2Lists l,
                                                               const uint32_t* __restrict__ hh,
                                                               const uint32_t* __restrict__ tot, uint32_t n,
                                                               uint32_t n_act, uint32_t* __restrict__ perm,
                                                               uint32_t* __restrict__ offsets,
                                                               uint32_t* __restrict__ rank_out) {
    static_assert(CH_NT == (int)MSD_LW, "one thread per u16-pair counter word");
    __shared__ ChunkShared sh;
    const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    const ChunkWalk cw = chunk_walk(l.ctr[2]);
    for (uint32_t j = cw.j; j < cw.end; j += cw.step) {
        const uint32_t r = l.chunk_r[j], b = l.cr_b[r];
        const uint32_t rsb = l.rs[b], c = j - l.cr_cb[r];
        const uint32_t start = rsb + c * CH_CAP, cs = min(CH_CAP, l.rs[b + 1] - start);
        const uint32_t k0 = b << MSD_SHIFT;
        const uint32_t L = min(MSD_L, n_act + 1 - k0);
        // activations 2t, 2t + 1: their starts in the range (scan of the totals), their bases for this chunk
        const uint2 t2 = reinterpret_cast<const uint2*>(tot + (size_t)r * MSD_L)[tid];
        const uint2 h2 = reinterpret_cast<const uint2*>(hh + (size_t)j * MSD_L)[tid];
        const uint32_t as0 = block_excl_scan_add_n<CH_NT>(t2.x + t2.y, sh.red), as1 = as0 + t2.x;
        const uint32_t gb0 = rsb + as0 + h2.x, gb1 = rsb + as1 + h2.y;
        if (c == 0) {
            if (2 * tid < L) offsets[k0 + 2 * tid] = rsb + as0;
            if (2 * tid + 1 < L) offsets[k0 + 2 * tid + 1] = rsb + as1;
            if (tid == 0 && b == (n_act >> MSD_SHIFT)) offsets[n_act + 1] = n;
        }
#pragma unroll
        for (int ww = 0; ww < CH_NW; ++ww) sh.wc[ww][tid] = 0;
        const uint32_t seg = (cs + CH_NW - 1) / CH_NW;
        const uint32_t s0 = min(w * seg, cs), s1 = min((w + 1) * seg, cs);
        const uint16_t* rk = keys16 + start;
        const uint32_t* ri = idx + start;
        uint32_t kp[CH_RW / 2];
        {
            const uint32_t last = cs - 1;
#pragma unroll
            for (uint32_t q = 0; q < CH_RW; q += 2) {
                const uint32_t i = s0 + q * WAVE + lane;
                const uint32_t x = rk[min(i, last)], y = rk[min(i + WAVE, last)];
                kp[q / 2] = (i < s1 ? x : 0xFFFFu) | ((i + WAVE < s1 ? y : 0xFFFFu) << 16);
            }
        }
        __syncthreads();
        // the wave's hot activation (of its first row; Zipf-hot ranges) counted and ranked in registers
        const uint32_t hk = wave_hot_digit(kp[0] & 0xFFFFu, (kp[0] & 0xFFFFu) != 0xFFFFu);
        {
            uint32_t hc = 0;
#pragma unroll
            for (uint32_t q = 0; q < CH_RW; ++q) {
                const uint32_t k = (kp[q / 2] >> (16 * (q & 1))) & 0xFFFFu;
                if (k == hk) ++hc;
                else if (k != 0xFFFFu) atomicAdd(&sh.wc[w][k >> 1], 1u << (16 * (k & 1)));
            }
            hc = wave_sum(hc);
            if (lane == 0 && hc) atomicAdd(&sh.wc[w][hk >> 1], hc << (16 * (hk & 1)));
        }
#pragma unroll
        for (uint32_t q = 0; q < CH_RW / 2; ++q) asm volatile("" : "+v"(kp[q]));
        __syncthreads();
        // each wave's first chunk position per activation (the activation's chunk start + the exclusive
        // prefix over the waves), so a rank is a chunk position; the totals
        uint32_t wv[CH_NW], tlo = 0, thi = 0;
#pragma unroll
        for (int ww = 0; ww < CH_NW; ++ww) {
            wv[ww] = sh.wc[ww][tid];
            tlo += wv[ww] & 0xFFFFu;
            thi += wv[ww] >> 16;
        }
        const uint32_t ex = block_excl_scan_add_n<CH_NT>(tlo + thi, sh.red);
        {
            uint32_t plo = ex, phi = ex + tlo;
#pragma unroll
            for (int ww = 0; ww < CH_NW; ++ww) {
                sh.wc[ww][tid] = plo | (phi << 16);
                plo += wv[ww] & 0xFFFFu;
                phi += wv[ww] >> 16;
            }
        }
        sh.delta[2 * tid] = gb0 - ex;                    // chunk position -> global position
        sh.delta[2 * tid + 1] = gb1 - ex - tlo;
        __syncthreads();
        // the hot activation's ranks: this wave's first chunk position among its items, then ballots
        const uint32_t hk_s = hk == NONE32 ? 0u : hk;
        uint32_t hrun = (sh.wc[w][hk_s >> 1] >> (16 * (hk_s & 1))) & 0xFFFFu;
        const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
        for (uint32_t g = 0; g < CH_RW; g += MSD_G) {
            // unconditional loads, clamped into the chunk (msd_range_kp: no vmcnt(0) at mask joins)
            uint32_t mm[MSD_G];
#pragma unroll
            for (uint32_t q = 0; q < (uint32_t)MSD_G; ++q) mm[q] = ri[min(s0 + (g + q) * WAVE + lane, cs - 1)];
#pragma unroll
            for (uint32_t q = 0; q < (uint32_t)MSD_G; ++q) {
                const uint32_t k = (kp[(g + q) / 2] >> (16 * ((g + q) & 1))) & 0xFFFFu;
                const unsigned long long hm = __ballot(k == hk);
                const bool cold = k != 0xFFFFu && k != hk;
                const uint32_t rr = row_rank16<BALLOT, 10>(&sh.wc[w][k >> 1], 16 * (k & 1), k, cold);
                const uint32_t at = k == hk ? hrun + (uint32_t)__popcll(hm & lt) : rr;
                hrun += (uint32_t)__popcll(hm);
                if (k == 0xFFFFu) continue;
                sh.out[at] = mm[q];
                sh.key[at] = (uint16_t)k;
            }
        }
        __syncthreads();
        // (the write-out's LDS reads batched as in k_b2_scatter / k_seg_scatter measured no faster here:
        // 0.197 -> 0.197 ms at cfg 3, profiles/r05_writeout_batch_ab.txt)
#pragma unroll
        for (uint32_t q = 0; q < CH_RW; ++q) {
            const uint32_t i = q * CH_NT + tid;
            if (i < cs) {
                const uint32_t v = sh.out[i];
                const uint32_t p = sh.delta[sh.key[i]] + i;
                perm[p] = v;
                if (rank_out) rank_out[v] = p;
            }
        }
        __syncthreads();
    }
}

}  // namespace gd
