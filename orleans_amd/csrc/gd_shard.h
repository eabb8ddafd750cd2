// gd_shard.h -- gfx950 device code for the exchange partition (SURVEY 8 a14 / e): a stable
// partition of message records by destination rank (owner silo % n_shards), the per-target-silo
// outbound queues of OutboundMessageQueue.SendMessage (OutboundMessageQueue.cs:54-131) laid out
// as the contiguous per-destination chunks an all-to-all-v sends.
//
// Two kernels per batch (plus one scan):
//   k_shard_hist    ring owner of every record -> dest byte, per-tile destination counts
//   scan            digit-major exclusive scan: (dest, tile) -> global base
//   k_shard_scatter stable rank in the tile by ballot matching, the records (24-B keys or 4-B
//                   node ids) and a 4-B payload staged in LDS in destination order, then written
//                   run by run (coalesced)
// The records move once (read 24 B, write 24 B + 4 B); the earlier form (radix pass over a dest
// array, then a gather of the keys through the permutation) read each key twice, the second
// time at 1/n_shards density.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"
#include "gd_keyext.h"

namespace gd {

constexpr int SH_NT = 256;
constexpr int SH_IT = 8;
constexpr uint32_t SH_TILE = SH_NT * SH_IT;   // 2048 records per tile

// Owner rank of message i.  KeyExt grains go to the owner of their KeyExt hash when the batch's
// strings are given (ext.len != nullptr, gd_route_multi_ext), else they stay here (KEYEXT).
// region (optional): the grain's table region on its owner (grain_region of its uniform hash) for a
// grain the owner probes in its directory table, 0 for everything else.
// EXT = false: the batch carries no KeyExt strings (ext.len == nullptr); the string-hash path is
// compiled out (k_shard_hist unrolls 8 records a thread: with it inlined the kernel was 14K
// instructions, past the instruction cache).
template <int MODE, bool EXT = true>
__device__ __forceinline__ uint32_t key_dest(uint64_t n0, uint64_t n1, uint64_t tcd, const uint32_t* s_pts,
                                             const uint32_t* s_own, const RingArgs& ring, uint32_t n_shards,
                                             const ExtArgs& ext, uint32_t i, uint32_t* region = nullptr) {
    const uint32_t cat = (uint32_t)(tcd >> 56);
    uint32_t silo;
    if (region) *region = 0;
    const uint8_t* s;
    int32_t len;
    if (EXT && (cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT) && ext.len && ext_of(ext, i, s, len)) {
        uint32_t uh;
        if (len < 0) {
            uh = uniform_hash(n0, n1, tcd);
        } else if (len <= KX_FAST_BYTES) {
            uint32_t w[KX_FAST_WORDS];
            load_str_fast(s, len, w);
            uh = jenkins_keyext_fast(n0, n1, tcd, len, w);
        } else {
            uh = jenkins_keyext(n0, n1, tcd, s, len);
        }
        silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, uh)];
    } else if (cat == CAT_SYSTEM_TARGET || cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT) silo = ring.my_silo;
    else if (is_membership(n0, n1, tcd)) silo = ring.seed_silo;
    else {
        const uint32_t uh = uniform_hash(n0, n1, tcd);
        silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, uh)];
        if (region) *region = grain_region(uh);
    }
    return (silo == NONE32 ? ring.my_silo : silo) % n_shards;
}

// Item (w, r, lane) of a tile <-> record base + (w * SH_IT + r) * 64 + lane, as in k_radix_scatter.
// Counts per wave by ballot matching (the lowest lane of each destination group adds the group's
// size), not per-lane LDS atomics: with few destinations every lane of a wave would hit one
// counter.  `bits` = destination bits (n_shards <= 1 << bits).
// regions (keys only; 1 or N_REGIONS): destination = owner rank * regions + the grain's table region,
// so each rank's chunk arrives grouped by region (gd_route_multi's region-mapped probe).
template <int MODE, bool NODES, bool EXT = true>
static __global__ void __launch_bounds__(SH_NT) k_shard_hist(const void* __restrict__ recs, uint32_t n, uint64_t tcd,
                                                      RingArgs ring, uint32_t n_shards, uint32_t bits,
                                                      uint32_t tiles, uint8_t* __restrict__ dest,
                                                      uint32_t* __restrict__ hist, ExtArgs ext,
                                                      uint32_t* __restrict__ kdesc, uint32_t* __restrict__ n1lo,
                                                      uint32_t regions) {
    constexpr int NW = SH_NT / WAVE;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    __shared__ uint32_t s_wc[NW][256];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    for (uint32_t d = threadIdx.x; d < 256; d += SH_NT)
#pragma unroll
        for (int w = 0; w < NW; ++w) s_wc[w][d] = 0;
    stage_ring(ring, s_pts, s_own);
    const uint32_t base = blockIdx.x * SH_TILE;
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    // header compaction (kdesc != nullptr): does every key have N0 == 0 and the first key's TCD?
    uint64_t ref_tcd = 0;
    if constexpr (!NODES)
        if (kdesc && n) ref_tcd = reinterpret_cast<const uint64_t*>(recs)[2];
    bool wide = false, big = false;
    // every record of the thread is loaded before the first hash (one wait, not one per record)
    constexpr int RW = NODES ? 1 : 3;
    uint64_t kv[SH_IT][RW];
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t li = min(base + (w * SH_IT + r) * WAVE + lane, n - 1);
        if constexpr (NODES) {
            kv[r][0] = reinterpret_cast<const uint32_t*>(recs)[li];
        } else {
            const uint64_t* kp = reinterpret_cast<const uint64_t*>(recs) + 3ull * li;
            kv[r][0] = kp[0];
            kv[r][1] = kp[1];
            kv[r][2] = kp[2];
        }
    }
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t i = base + (w * SH_IT + r) * WAVE + lane;
        const bool valid = i < n;
        uint32_t d = 0;
        if (valid) {
            if constexpr (NODES) {
                const uint32_t node = (uint32_t)kv[r][0];
                d = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, uniform_hash(0, node, tcd))] % n_shards;
            } else {
                uint32_t reg = 0;
                d = key_dest<MODE, EXT>(kv[r][0], kv[r][1], kv[r][2], s_pts, s_own, ring, n_shards, ext, i,
                                   regions > 1 ? &reg : nullptr) * regions + reg;
                wide |= kv[r][0] != 0 || kv[r][2] != ref_tcd;
                big |= (kv[r][1] >> 32) != 0;
                if (n1lo) n1lo[i] = (uint32_t)kv[r][1];   // the gather's 4-B header source (mode 2)
            }
            dest[i] = (uint8_t)d;
        }
        unsigned long long peers = __ballot(valid);
        for (uint32_t b = 0; b < bits; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        if (valid && (peers & lt) == 0) s_wc[w][d] += (uint32_t)__popcll(peers);
    }
    if constexpr (!NODES)
        if (kdesc) {
            const bool any_wide = __ballot(wide) != 0, any_big = __ballot(big) != 0;
            if (lane == 0 && (any_wide || any_big)) atomicOr(&kdesc[1], (any_wide ? 1u : 0u) | (any_big ? 2u : 0u));
        }
    __syncthreads();
    const uint32_t n_dest = NODES ? n_shards : n_shards * regions;
    for (uint32_t d = threadIdx.x; d < n_dest; d += SH_NT) {
        uint32_t t = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) t += s_wc[ww][d];
        hist[d * tiles + blockIdx.x] = t;
    }
}

// Header compaction for the exchange (gd_route_multi*): a batch whose keys all have N0 == 0 and one
// TypeCodeData -- long-keyed grains of one type (GrainId.GetGrainId(typeCode, long), GrainId.cs:
// 72-77), the common case -- sends N1 alone per header instead of 24 B: 4 B when every N1 is below
// 2^32 (narrow_ok), else 8 B.  kdesc = {mode (0 full, 1 u64 N1, 2 u32 N1), flags from k_shard_hist
// (bit 0 wide, bit 1 some N1 >= 2^32), TCD lo, TCD hi}: the descriptor every peer receives with the
// counts.
static __global__ void k_key_desc(const gd_key* __restrict__ keys, uint32_t n, uint32_t* __restrict__ kdesc,
                           uint32_t narrow_ok) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t tcd = n ? reinterpret_cast<const uint64_t*>(keys)[2] : 0ull;
    const uint32_t f = kdesc[1];
    kdesc[0] = (f & 1u) ? 0u : ((narrow_ok && !(f & 2u)) ? 2u : 1u);
    kdesc[2] = (uint32_t)tcd;
    kdesc[3] = (uint32_t)(tcd >> 32);
}

// Descriptor flag (kdesc[1]): every chunk of the sender is ordered by region (k_shard_hist with regions).
constexpr uint32_t KD_REGIONS = 4u;
// Descriptor flag: the sender's origin indices travel as their low 16 bits (2 B a message), with,
// per receiving rank, the chunk position where each 65,536-index block of the sender's batch starts
// (k_block_prefix); k_recv_idx16 rebuilds them.  Origin indices increase along a chunk (the
// partition is stable), so block b's messages are a contiguous run of it.
constexpr uint32_t KD_IDX16 = 8u;
constexpr uint32_t IDX16_BLOCK_TILES = 65536u / SH_TILE;

// Sender, after the partition's scan (gscan: exclusive over (dest, tile), rank-major): for rank r
// and block b (tiles 32b .. 32b + 31), the position in r's chunk where block b starts.  Thread 0
// also flags the descriptor and stores this sender's block count (the counts round sends it).
static __global__ void k_block_prefix(const uint32_t* __restrict__ gscan, uint32_t tiles, uint32_t n_shards,
                               uint32_t nblk, uint32_t* __restrict__ out, uint32_t* __restrict__ kdesc,
                               uint32_t* __restrict__ nblk_out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        kdesc[1] |= KD_IDX16;
        *nblk_out = nblk;
    }
    if (t >= n_shards * nblk) return;
    const uint32_t r = t / nblk, b = t % nblk;
    out[t] = gscan[(size_t)r * tiles + (size_t)b * IDX16_BLOCK_TILES] - gscan[(size_t)r * tiles];
}

// Receiver of a header round with 2-B origin indices from some peers: raw = the peers' index chunks
// back to back (2 or 4 B a message by the sender's descriptor, each chunk padded to 4 B), pcol =
// the 2-B senders' block starts back to back (rnblk[q] each).  Writes the 4-B origin index and the
// sender rank of every received message (k_recv_src's job).
static __global__ void __launch_bounds__(BLOCK) k_recv_idx16(const uint8_t* __restrict__ raw,
                                                      const uint32_t* __restrict__ rcount,
                                                      const uint32_t* __restrict__ rdesc,
                                                      const uint32_t* __restrict__ pcol,
                                                      const uint32_t* __restrict__ rnblk, uint32_t world, uint32_t m,
                                                      uint32_t* __restrict__ idx, uint32_t* __restrict__ src) {
    constexpr uint32_t LDS_COL = 4096;   // block starts staged in LDS when they fit (16M-message batches at W <= 16)
    __shared__ uint32_t s_off[257], s_boff[256], s_coff[256], s_nb[256], s_col[LDS_COL];
    __shared__ uint32_t s_ncol;
    if (threadIdx.x == 0) {
        uint32_t run = 0, brun = 0, crun = 0;
        for (uint32_t q = 0; q < world; ++q) {
            // the host's rule (route_multi): a sender that sent this rank nothing sent no block starts
            // either, whatever its descriptor says (one descriptor goes to every peer)
            const bool w16 = rcount[q] != 0 && (rdesc[4 * q + 1] & KD_IDX16) != 0;
            s_off[q] = run;
            s_boff[q] = brun;
            s_coff[q] = crun;
            s_nb[q] = w16 ? rnblk[q] : 0u;
            run += rcount[q];
            brun += w16 ? (2u * rcount[q] + 3u) & ~3u : 4u * rcount[q];
            crun += w16 ? rnblk[q] : 0u;
        }
        s_off[world] = run;
        s_ncol = crun;
    }
    __syncthreads();
    const bool in_lds = s_ncol <= LDS_COL;
    if (in_lds)
        for (uint32_t k = threadIdx.x; k < s_ncol; k += BLOCK) s_col[k] = pcol[k];
    __syncthreads();
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m) return;
    uint32_t lo = 0, hi = world;          // largest q with s_off[q] <= j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= j) lo = mid;
        else hi = mid;
    }
    const uint32_t q = lo, jj = j - s_off[q], nb = s_nb[q];
    uint32_t v;
    if (nb) {
        const uint32_t low = reinterpret_cast<const uint16_t*>(raw + s_boff[q])[jj];
        const uint32_t* col = (in_lds ? s_col : pcol) + s_coff[q];
        uint32_t b = 0, e = nb;           // largest b with col[b] <= jj (col[0] = 0)
        while (e - b > 1) {
            const uint32_t mid = (b + e) >> 1;
            if (col[mid] <= jj) b = mid;
            else e = mid;
        }
        v = (b << 16) | low;
    } else {
        v = reinterpret_cast<const uint32_t*>(raw + s_boff[q])[jj];
    }
    idx[j] = v;
    src[j] = q;
}

// Header bytes of a chunk by its sender's descriptor mode.
__host__ __device__ __forceinline__ uint32_t header_bytes(uint32_t mode) { return mode == 2 ? 4u : mode ? 8u : 24u; }

// Receiver of a header round where some peer sent compact headers: raw = the peers' chunks back to
// back (8 B or 24 B per header by each peer's descriptor); rebuild the 24-B keys and the sender
// rank of every received message (k_recv_src's job otherwise).
static __global__ void __launch_bounds__(BLOCK) k_recv_expand(const uint8_t* __restrict__ raw,
                                                       const uint32_t* __restrict__ rcount,
                                                       const uint32_t* __restrict__ rdesc, uint32_t world,
                                                       uint32_t m, gd_key* __restrict__ keys,
                                                       uint32_t* __restrict__ src) {
    __shared__ uint32_t s_off[257];
    __shared__ uint64_t s_boff[256];
    __shared__ uint64_t s_tcd[256];
    __shared__ uint32_t s_compact[256];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        uint64_t brun = 0;
        for (uint32_t r = 0; r < world; ++r) {
            const uint32_t c = rdesc[4 * r];
            s_off[r] = run;
            s_boff[r] = brun;
            s_compact[r] = c;
            s_tcd[r] = (uint64_t)rdesc[4 * r + 2] | ((uint64_t)rdesc[4 * r + 3] << 32);
            run += rcount[r];
            brun += (uint64_t)rcount[r] * header_bytes(c);
        }
        s_off[world] = run;
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    uint32_t lo = 0, hi = world;          // largest r with s_off[r] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= i) lo = mid;
        else hi = mid;
    }
    const uint64_t j = i - s_off[lo];
    uint64_t* out = reinterpret_cast<uint64_t*>(keys + i);
    // a chunk starts 4-B aligned only (a u32 chunk of odd length before it): read in u32 words
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(raw + s_boff[lo]);
    auto u64_at = [&](uint64_t w) { return (uint64_t)cw[w] | ((uint64_t)cw[w + 1] << 32); };
    if (s_compact[lo]) {
        const uint64_t n1 = s_compact[lo] == 2 ? (uint64_t)cw[j] : u64_at(2 * j);
        out[0] = 0;
        out[1] = n1;
        out[2] = s_tcd[lo];
    } else {
        out[0] = u64_at(6 * j);
        out[1] = u64_at(6 * j + 2);
        out[2] = u64_at(6 * j + 4);
    }
    if (src) src[i] = lo;
}

// Forward partition (SURVEY 8 e, the owner != activation silo case): after the probe on the owner,
// a message whose route is a directory hit goes on to the rank hosting its activation (silo %
// n_shards: the send to ActivationAddress.Silo after the remote lookup, LocalGrainDirectory.cs:920,
// OutboundMessageQueue.cs:125); every other status stays on this rank.  Same counting as
// k_shard_hist; k_shard_scatter then moves the keys with payload = position in the input.
static __global__ void __launch_bounds__(SH_NT) k_fwd_hist(const uint8_t* __restrict__ st, const uint32_t* __restrict__ silo,
                                                    uint32_t n, uint32_t n_shards, uint32_t my_rank, uint32_t bits,
                                                    uint32_t tiles, uint8_t* __restrict__ dest,
                                                    uint32_t* __restrict__ hist) {
    constexpr int NW = SH_NT / WAVE;
    __shared__ uint32_t s_wc[NW][256];
    for (uint32_t d = threadIdx.x; d < 256; d += SH_NT)
#pragma unroll
        for (int w = 0; w < NW; ++w) s_wc[w][d] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * SH_TILE;
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t i = base + (w * SH_IT + r) * WAVE + lane;
        const bool valid = i < n;
        uint32_t d = 0;
        if (valid) {
            d = st[i] == GD_ROUTE_OK ? silo[i] % n_shards : my_rank;
            dest[i] = (uint8_t)d;
        }
        unsigned long long peers = __ballot(valid);
        for (uint32_t b = 0; b < bits; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        if (valid && (peers & lt) == 0) s_wc[w][d] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < n_shards; d += SH_NT) {
        uint32_t t = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) t += s_wc[ww][d];
        hist[d * tiles + blockIdx.x] = t;
    }
}

// The forwarded messages' other fields in send order (pos = k_shard_scatter's payload).
static __global__ void __launch_bounds__(BLOCK) k_fwd_gather(const uint32_t* __restrict__ pos, uint32_t n,
                                                      const uint32_t* __restrict__ idx_in,
                                                      const uint32_t* __restrict__ src_in,
                                                      const uint32_t* __restrict__ silo_in,
                                                      const uint32_t* __restrict__ act_in,
                                                      const uint8_t* __restrict__ st_in, uint32_t* __restrict__ idx,
                                                      uint32_t* __restrict__ src, uint32_t* __restrict__ silo,
                                                      uint32_t* __restrict__ act, uint8_t* __restrict__ st) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = pos[j];
    if (i >= n) return;
    idx[j] = idx_in[i];
    src[j] = src_in[i];
    silo[j] = silo_in[i];
    act[j] = act_in[i];
    st[j] = st_in[i];
}

// payload_in == nullptr: the payload is the record's batch index (the origin index).  PT = uint16_t:
// the payload is written as its low 16 bits (origin indices for the exchange, KD_IDX16).
template <int BITS, bool NODES, bool SKIP_COMPACT = false, typename PT = uint32_t>
static __global__ void __launch_bounds__(SH_NT) k_shard_scatter(const void* __restrict__ recs,
                                                         const uint32_t* __restrict__ payload_in,
                                                         const uint8_t* __restrict__ dest, uint32_t n,
                                                         uint32_t n_shards, uint32_t tiles,
                                                         const uint32_t* __restrict__ gscan,
                                                         void* __restrict__ out_recs,
                                                         PT* __restrict__ out_payload,
                                                         const uint32_t* __restrict__ kdesc) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int NW = SH_NT / WAVE;
    constexpr int RW = NODES ? 1 : 3;           // 8-B words per record (keys) / one u32 (nodes)
    if constexpr (SKIP_COMPACT)
        if (kdesc[0]) return;                   // compact: k_shard_gather's case
    __shared__ uint32_t s_wcnt[NW][R];
    __shared__ uint32_t s_lstart[R];
    __shared__ uint32_t s_gbase[R];
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint64_t s_key[NODES ? 1 : 3][NODES ? 1 : SH_TILE];
    __shared__ uint32_t s_node[NODES ? SH_TILE : 1];
    __shared__ uint32_t s_pay[SH_TILE];
    __shared__ uint8_t s_dig[SH_TILE];

    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * SH_TILE;
    const uint32_t cnt_tile = min(SH_TILE, n - base);
    for (uint32_t d = threadIdx.x; d < R; d += SH_NT) {
#pragma unroll
        for (int w = 0; w < NW; ++w) s_wcnt[w][d] = 0;
        s_gbase[d] = d < n_shards ? gscan[d * tiles + tile] : 0u;   // no record has a digit >= n_shards
    }
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t dd[SH_IT], rk[SH_IT], pay[SH_IT];
    uint64_t kv[SH_IT][RW];
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t idx = base + (w * SH_IT + r) * WAVE + lane;
        const uint32_t li = min(idx, n - 1);
        dd[r] = dest[li];
        if constexpr (NODES) {
            kv[r][0] = reinterpret_cast<const uint32_t*>(recs)[li];
        } else {
            const uint64_t* kp = reinterpret_cast<const uint64_t*>(recs) + 3ull * li;
            kv[r][0] = kp[0];
            kv[r][1] = kp[1];
            kv[r][2] = kp[2];
        }
        pay[r] = payload_in ? payload_in[li] : idx;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t idx = base + (w * SH_IT + r) * WAVE + lane;
        const bool valid = idx < n;
        const uint32_t d = dd[r] & (R - 1);
        const unsigned long long peers = match_digit<BITS>(d, valid);
        uint32_t c = 0;
        if (valid) c = s_wcnt[w][d];
        rk[r] = c + (uint32_t)__popcll(peers & lt);
        if (valid && (peers & lt) == 0) s_wcnt[w][d] = c + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // cross-wave exclusive prefix per digit, then tile-local digit starts
    constexpr uint32_t DPT = (R + SH_NT - 1) / SH_NT;
    uint32_t my_total = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t d = threadIdx.x * DPT + q;
        if (d < R) {
            uint32_t run = 0;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) {
                const uint32_t t = s_wcnt[ww][d];
                s_wcnt[ww][d] = run;
                run += t;
            }
            s_lstart[d] = run;
            my_total += run;
        }
    }
    const uint32_t ex = block_excl_scan_add_n<SH_NT>(my_total, s_wsum);
    {
        uint32_t run = ex;
#pragma unroll
        for (uint32_t q = 0; q < DPT; ++q) {
            const uint32_t d = threadIdx.x * DPT + q;
            if (d < R) {
                const uint32_t t = s_lstart[d];
                s_lstart[d] = run;
                run += t;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t idx = base + (w * SH_IT + r) * WAVE + lane;
        if (idx < n) {
            const uint32_t d = dd[r] & (R - 1);
            const uint32_t p = s_lstart[d] + s_wcnt[w][d] + rk[r];
            if constexpr (NODES) {
                s_node[p] = (uint32_t)kv[r][0];
            } else {
                s_key[0][p] = kv[r][0];
                s_key[1][p] = kv[r][1];
                s_key[2][p] = kv[r][2];
            }
            s_pay[p] = pay[r];
            s_dig[p] = (uint8_t)d;
        }
    }
    __syncthreads();
    const uint32_t compact = !NODES && kdesc ? kdesc[0] : 0u;   // headers as N1 only (k_key_desc)
#pragma unroll
    for (int j = 0; j < SH_IT; ++j) {
        const uint32_t p = j * SH_NT + threadIdx.x;
        if (p < cnt_tile) {
            const uint32_t d = s_dig[p];
            const uint32_t g = s_gbase[d] + (p - s_lstart[d]);
            if (g < n) {            // always true when the scan is right; never write out of bounds
                if constexpr (NODES) {
                    reinterpret_cast<uint32_t*>(out_recs)[g] = s_node[p];
                } else if (compact == 2) {
                    reinterpret_cast<uint32_t*>(out_recs)[g] = (uint32_t)s_key[1][p];
                } else if (compact) {
                    reinterpret_cast<uint64_t*>(out_recs)[g] = s_key[1][p];
                } else {
                    uint64_t* o = reinterpret_cast<uint64_t*>(out_recs) + 3ull * g;
                    o[0] = s_key[0][p];
                    o[1] = s_key[1][p];
                    o[2] = s_key[2][p];
                }
                out_payload[g] = (PT)s_pay[p];
            }
        }
    }
}

// A compact batch (k_key_desc: every key N0 == 0 with one TypeCodeData, sent as N1 alone) without
// staging the keys in LDS: the tile is ranked from its destination bytes alone, LDS keeps each
// output slot's source record (u16) and destination, and the write phase reads each N1 straight
// from the batch and writes the runs coalesced.  6 KB of LDS per workgroup instead of the 58 KB
// of k_shard_scatter's staged 24-B keys: several times the waves per CU.  Returns at once for a
// batch that is not compact (k_shard_scatter<.., SKIP_COMPACT> runs beside it and takes that
// case; gathering whole 24-B records measured slower than staging them: 0.18-0.24 vs 0.16 ms per
// 16M keys at 1-8 destinations).  Same output as k_shard_scatter<BITS, false>.
template <int BITS, typename PT = uint32_t>
static __global__ void __launch_bounds__(SH_NT) k_shard_gather(const gd_key* __restrict__ recs,
                                                        const uint32_t* __restrict__ payload_in,
                                                        const uint8_t* __restrict__ dest, uint32_t n,
                                                        uint32_t n_shards, uint32_t tiles,
                                                        const uint32_t* __restrict__ gscan,
                                                        void* __restrict__ out_recs,
                                                        PT* __restrict__ out_payload,
                                                        const uint32_t* __restrict__ kdesc,
                                                        const uint32_t* __restrict__ n1lo) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int NW = SH_NT / WAVE;
    if (!kdesc[0]) return;                      // not compact: k_shard_scatter's case
    __shared__ uint32_t s_wcnt[NW][R];
    __shared__ uint32_t s_lstart[R];
    __shared__ uint32_t s_gbase[R];
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint16_t s_src[SH_TILE];
    __shared__ uint8_t s_dig[SH_TILE];
    static_assert(SH_TILE <= 65536, "u16 source slots");

    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * SH_TILE;
    const uint32_t cnt_tile = min(SH_TILE, n - base);
    for (uint32_t d = threadIdx.x; d < R; d += SH_NT) {
#pragma unroll
        for (int w = 0; w < NW; ++w) s_wcnt[w][d] = 0;
        s_gbase[d] = d < n_shards ? gscan[d * tiles + tile] : 0u;
    }
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t dd[SH_IT], rk[SH_IT];
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) dd[r] = dest[min(base + (w * SH_IT + r) * WAVE + lane, n - 1)];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t idx = base + (w * SH_IT + r) * WAVE + lane;
        const bool valid = idx < n;
        const uint32_t d = dd[r] & (R - 1);
        const unsigned long long peers = match_digit<BITS>(d, valid);
        uint32_t c = 0;
        if (valid) c = s_wcnt[w][d];
        rk[r] = c + (uint32_t)__popcll(peers & lt);
        if (valid && (peers & lt) == 0) s_wcnt[w][d] = c + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    constexpr uint32_t DPT = (R + SH_NT - 1) / SH_NT;
    uint32_t my_total = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t d = threadIdx.x * DPT + q;
        if (d < R) {
            uint32_t run = 0;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) {
                const uint32_t t = s_wcnt[ww][d];
                s_wcnt[ww][d] = run;
                run += t;
            }
            s_lstart[d] = run;
            my_total += run;
        }
    }
    const uint32_t ex = block_excl_scan_add_n<SH_NT>(my_total, s_wsum);
    {
        uint32_t run = ex;
#pragma unroll
        for (uint32_t q = 0; q < DPT; ++q) {
            const uint32_t d = threadIdx.x * DPT + q;
            if (d < R) {
                const uint32_t t = s_lstart[d];
                s_lstart[d] = run;
                run += t;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SH_IT; ++r) {
        const uint32_t loc = (w * SH_IT + r) * WAVE + lane;
        if (base + loc < n) {
            const uint32_t d = dd[r] & (R - 1);
            const uint32_t p = s_lstart[d] + s_wcnt[w][d] + rk[r];
            s_src[p] = (uint16_t)loc;
            s_dig[p] = (uint8_t)d;
        }
    }
    __syncthreads();
    const uint64_t* k64 = reinterpret_cast<const uint64_t*>(recs);
    uint64_t* o64 = reinterpret_cast<uint64_t*>(out_recs);
    uint32_t* o32 = reinterpret_cast<uint32_t*>(out_recs);
    const bool narrow = kdesc[0] == 2;          // every N1 below 2^32: 4 B a header
    // one N1 (8 or 4 B) and the payload per output slot; every gather of the thread before the stores
    uint64_t kv[SH_IT];
    uint32_t pay[SH_IT], gg[SH_IT];
#pragma unroll
    for (int j = 0; j < SH_IT; ++j) {
        const uint32_t p = j * SH_NT + threadIdx.x;
        gg[j] = 0xFFFFFFFFu;
        if (p < cnt_tile) {
            const uint32_t i = base + s_src[p];
            const uint32_t d = s_dig[p];
            gg[j] = s_gbase[d] + (p - s_lstart[d]);
            kv[j] = narrow && n1lo ? (uint64_t)n1lo[i] : k64[3ull * i + 1];   // 4 B (k_shard_hist's copy) or the key's N1
            pay[j] = payload_in ? payload_in[i] : i;
        }
    }
#pragma unroll
    for (int j = 0; j < SH_IT; ++j)
        if (gg[j] < n) {            // ~0: no record here; else always in bounds when the scan is right
            if (narrow) o32[gg[j]] = (uint32_t)kv[j];
            else o64[gg[j]] = kv[j];
            out_payload[gg[j]] = (PT)pay[j];
        }
}

// counts[d] = records for destination d, from the scanned (dest, tile) bases.
// kdesc != nullptr: thread 0 also completes the header-compaction descriptor (k_key_desc's work;
// k_shard_hist's flags are final by now), one launch fewer on the partition stream.
// counts[d] for the n_shards ranks; with regions, rank d's destinations are d * group .. (d + 1) * group
// - 1 (its region chunks, contiguous in the send buffer).
static __global__ void k_shard_counts(const uint32_t* __restrict__ gscan, uint32_t tiles, uint32_t n_shards, uint32_t n,
                               uint32_t* __restrict__ counts, const gd_key* __restrict__ keys,
                               uint32_t* __restrict__ kdesc, uint32_t narrow_ok, uint32_t group) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (kdesc && d == 0) {
        const uint64_t tcd = n ? reinterpret_cast<const uint64_t*>(keys)[2] : 0ull;
        const uint32_t f = kdesc[1];
        kdesc[0] = (f & 1u) ? 0u : ((narrow_ok && !(f & 2u)) ? 2u : 1u);
        kdesc[2] = (uint32_t)tcd;
        kdesc[3] = (uint32_t)(tcd >> 32);
    }
    if (kdesc && d == 0 && group > 1) kdesc[1] |= KD_REGIONS;
    if (d >= n_shards) return;
    const uint32_t start = gscan[(size_t)d * group * tiles];
    const uint32_t end = d + 1 < n_shards ? gscan[(size_t)(d + 1) * group * tiles] : n;
    counts[d] = end - start;
}

// Region segments of the received chunks (gd_route_multi with regions): every sender's chunk arrives
// sorted by region (k_shard_hist with regions), so thread (q, g) binary-searches chunk q for the first
// message of region >= g.  seg[q * (N_REGIONS + 1) + g] = that position in the receive order
// (seg[.. + N_REGIONS] = the chunk's end).  Keys: 24-B (N1W = 0) or N1s (N1W = 4 / 8, N0 = 0, tcd).
template <int N1W>
static __global__ void k_region_segments(const void* __restrict__ keys, const uint32_t* __restrict__ rcount,
                                  uint32_t world, uint64_t tcd, uint32_t* __restrict__ seg) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= world * (N_REGIONS + 1)) return;
    const uint32_t q = t / (N_REGIONS + 1), g = t % (N_REGIONS + 1);
    uint32_t lo = 0;
    for (uint32_t r = 0; r < q; ++r) lo += rcount[r];
    uint32_t hi = lo + rcount[q];
    if (g == N_REGIONS) {
        seg[t] = hi;
        return;
    }
    auto region_at = [&](uint32_t i) -> uint32_t {
        uint64_t n0 = 0, n1, c = tcd;
        if constexpr (N1W == 8) n1 = reinterpret_cast<const uint64_t*>(keys)[i];
        else if constexpr (N1W == 4) n1 = reinterpret_cast<const uint32_t*>(keys)[i];
        else {
            const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys) + 3ull * i;
            n0 = kp[0];
            n1 = kp[1];
            c = kp[2];
        }
        const uint32_t cat = (uint32_t)(c >> 56);
        if (cat == CAT_SYSTEM_TARGET || cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT || is_membership(n0, n1, c))
            return 0u;
        return grain_region(uniform_hash(n0, n1, c));
    };
    while (lo < hi) {                                  // first i in [lo, hi) with region_at(i) >= g
        const uint32_t mid = lo + (hi - lo) / 2;
        if (region_at(mid) < g) lo = mid + 1;
        else hi = mid;
    }
    seg[t] = lo;
}

// recv_src[i] = the rank chunk i of the receive buffer came from: off[r] <= i < off[r + 1], off =
// exclusive scan of the per-rank receive counts (world <= 256, scanned in LDS by every block).
static __global__ void __launch_bounds__(BLOCK) k_recv_src(const uint32_t* __restrict__ rcount, uint32_t world, uint32_t m,
                                                    uint32_t* __restrict__ src) {
    __shared__ uint32_t s_off[257];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t r = 0; r < world; ++r) {
            s_off[r] = run;
            run += rcount[r];
        }
        s_off[world] = run;
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    uint32_t lo = 0, hi = world;          // largest r with s_off[r] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= i) lo = mid;
        else hi = mid;
    }
    src[i] = lo;
}

// Routes returned to the sender in shard order -> the sender's batch order (send_idx is the
// partition's origin index): Dispatcher.AddressMessage's TargetSilo / TargetActivation per message.
static __global__ void __launch_bounds__(BLOCK) k_unpartition(const uint32_t* __restrict__ send_idx, uint32_t n,
                                                       const uint32_t* __restrict__ silo_in,
                                                       const uint32_t* __restrict__ act_in,
                                                       const uint8_t* __restrict__ st_in, uint32_t* __restrict__ silo,
                                                       uint32_t* __restrict__ act, uint8_t* __restrict__ st) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = send_idx[j];
    if (i >= n) return;
    silo[i] = silo_in[j];
    act[i] = act_in[j];
    st[i] = st_in[j];
}

// CalculateTargetSilo for a batch with KeyExt strings: the owner silo key_dest uses (no modulo).
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_owner_ext(const gd_key* __restrict__ keys, uint32_t n, RingArgs ring,
                                                     ExtArgs ext, uint32_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
    out[i] = key_dest<MODE>(kp[0], kp[1], kp[2], s_pts, s_own, ring, 0xFFFFFFFFu, ext, i);
}

// ---- KeyExt strings through the exchange (gd_route_multi_ext) -----------------------------------
// Payload bytes of message i's KeyExt (0 for null / host-kept / other categories).
__device__ __forceinline__ uint32_t ext_bytes(const ExtArgs& e, uint32_t i) {
    const int32_t l = e.len[i];
    return l > 0 ? (uint32_t)l : 0u;
}

// Per destination rank: bytes of KeyExt payload (LDS per block, one atomic per destination per
// block).  group: destinations per rank in dest (N_REGIONS with a region-ordered partition).
static __global__ void __launch_bounds__(BLOCK) k_dest_bytes(const uint8_t* __restrict__ dest, uint32_t n, ExtArgs ext,
                                                      uint32_t n_shards, uint32_t* __restrict__ out, uint32_t group) {
    __shared__ uint32_t s_b[256];
    for (uint32_t d = threadIdx.x; d < 256; d += BLOCK) s_b[d] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) {
        const uint32_t b = ext_bytes(ext, i);
        if (b) atomicAdd(&s_b[dest[i] / group], b);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < n_shards; d += BLOCK)
        if (s_b[d]) atomicAdd(&out[d], s_b[d]);
}

// Lengths in send order (the partition's origin index picks them); payload sizes for the scan.
static __global__ void __launch_bounds__(BLOCK) k_send_lengths(const uint32_t* __restrict__ send_idx, uint32_t n,
                                                        ExtArgs ext, int32_t* __restrict__ send_len,
                                                        uint32_t* __restrict__ send_bytes) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = send_idx[j];
    send_len[j] = ext.len[i];
    send_bytes[j] = ext_bytes(ext, i);
}

// Copy each message's KeyExt bytes to its place in the send blob (boff = exclusive scan).
static __global__ void __launch_bounds__(BLOCK) k_gather_ext(const uint32_t* __restrict__ send_idx, uint32_t n, ExtArgs ext,
                                                      const uint32_t* __restrict__ boff, uint8_t* __restrict__ blob) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = send_idx[j];
    const uint32_t b = ext_bytes(ext, i);
    if (!b) return;
    const uint64_t off = ext.off[i];
    if (off > ext.bytes_len || b > ext.bytes_len - off) return;   // k_route_keyext keeps such items KEYEXT
    const uint8_t* src = ext.bytes + off;
    uint8_t* dst = blob + boff[j];
    for (uint32_t k = 0; k < b; ++k) dst[k] = src[k];
}

// Receiver: payload sizes of the received lengths (for the scan), then 64-bit offsets.
static __global__ void __launch_bounds__(BLOCK) k_len_bytes(const int32_t* __restrict__ len, uint32_t m,
                                                     uint32_t* __restrict__ bytes) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j < m) bytes[j] = len[j] > 0 ? (uint32_t)len[j] : 0u;
}
static __global__ void __launch_bounds__(BLOCK) k_u32_to_u64(const uint32_t* __restrict__ a, uint32_t m,
                                                      uint64_t* __restrict__ b) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j < m) b[j] = a[j];
}

}  // namespace gd
