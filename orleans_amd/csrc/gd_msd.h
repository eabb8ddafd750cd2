// gd_msd.h -- gfx950 device code for the second level of the two-level bucketing (the
// per-activation FIFO): one workgroup sorts a range of MSD_L = 1,024 activations
// stably inside LDS and writes the range's bucket starts itself.
//
//   one-pass form (n_act < 1,081,344, BASELINE cfg 2): k_b2_hist / row scan / k_b2_scatter
//           (gd_bucket2.h, 8K-item tiles) with the high digit min(act, n_act) >> 10 (<= B2_RMAX2
//           ranges): every range's messages contiguous, in message order, message indices and
//           range-local keys (key & 1023, u16) 6 B a record; then k_msd_local, one workgroup a range;
//   three-pass form (larger n_act, gd_msd2.h): two MSD passes group the messages by range, and the
//           ranges holding T_SMALL < S <= MSD_CAP messages come here through a work list
//           (k_msd_local_list); thinner ones are sorted one wave a range, hotter ones in chunks by
//           several workgroups.
//
// The range sort (msd_range), 1,024 threads.  A range of <= MSD_CAP messages (the uniform case: 16 K
// for BASELINE cfg 2) is held in registers, 24 rows a lane:
//   count     per-wave counts (u16 pairs packed in u32 words: 16 x 512 words, 32 KB);
//   prefix    per activation over the 16 waves (the owner thread of a word does both halves), so a
//             wave's counter holds its first position; the activations' totals are scanned into the
//             bucket starts, written to offsets (every activation of the range once, empty ones
//             included: no min-scan);
//   rank      ds_add_rtn on the wave's counter returns the stable rank (a wave's lanes are served in
//             lane order, its rows in program order); the message index goes to its sorted place in
//             an LDS copy of the range (96 KB);
//   write     the range's permutation slice leaves LDS in order: coalesced 4-B stores.
// In the one-pass form a larger range (a Zipf-hot one) is histogrammed first and ranked in chunks of
// MSD_CAP with the index stored straight to its global position (one workgroup: correct, slow; the
// library then keeps the LSD path for such batches by measurement).
// Why the range is staged: the first form of this pass (ranges of 4,096 activations, 64 K messages,
// too many for LDS) stored each index straight to global memory, and those 16 M scattered 4-B stores
// cost 0.18 ms of its 0.25 ms (measured with the stores removed: profiles/r03_msd4k_nostore_exp.txt);
// staged, the pass takes 0.054 ms at cfg 2 (profiles/r03_msd_ab.txt), the whole stage 0.148 ms.
// Per message (one-pass form): the MSD pass reads 4 B twice (histogram, scatter) and writes 6 B; the
// range sort reads 6 B and writes 4 B in order -- 24 B over 4 launches, against 40 B over 11 for three
// packed 7-bit LSD passes.  Output identical to the LSD path (both are the stable partition by
// min(act, n_act)).
// Round 3 also measured, and round 4 removed: u16 positions staged instead of indices (two workgroups
// a CU, 0.088 against 0.054 ms), the indices loaded with the keys (0.058), u32 range-local keys (8-B
// records) and 16K-item MSD tiles (profiles/r03_msd_ab.txt, r03_msd_early_ab.txt, r03_msd_tile_ab.txt).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_bucket2.h"
#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

constexpr int MSD_NT = 1024;
constexpr int MSD_NW = MSD_NT / WAVE;              // 16 waves
constexpr uint32_t MSD_SHIFT = B2_LOW_BITS;        // range b: keys with key >> 10 == b
constexpr uint32_t MSD_L = 1u << MSD_SHIFT;        // activations per range
constexpr uint32_t MSD_LW = MSD_L / 2;             // u16-pair words per wave
constexpr int MSD_G = 8;                           // rows whose message indices are loaded together
constexpr uint32_t MSD_MAX_RANGES = B2_RMAX2;      // the high digit of the one-pass form
constexpr int MSD_RW = 24;                         // rows of 64 messages a wave holds
constexpr uint32_t MSD_CAP = MSD_RW * MSD_NT;      // messages a workgroup stages (24,576)
constexpr int MSD_MID_NT = 512;                    // the three-pass form's mid-size ranges: 512 threads,
constexpr int MSD_MID_RW = 16;                     // 16 rows a wave: 8,192 messages, 52 KB of LDS (3 a CU)
constexpr uint32_t MSD_MID_CAP = MSD_MID_NT * MSD_MID_RW;
// One-pass form: the key the unrouted messages (act >= n_act) are clamped to -- the first key of a range
// past the one holding n_act (n_act itself when it starts a range), so they form a range of their own.
__host__ __device__ __forceinline__ uint32_t msd_unrouted_key(uint32_t n_act) {
    return (uint32_t)(((uint64_t)n_act + MSD_L - 1) & ~(uint64_t)(MSD_L - 1));
}

template <int NT, int RW>
struct MsdShared {
    static constexpr int NW = NT / WAVE;
    uint32_t run[MSD_L];
    uint32_t wc[NW][MSD_LW];
    uint32_t out[NT * RW];
    uint32_t red[NW];
    uint32_t base;
};

// The per-wave counts (u16 pairs, wc[wave * MSD_LW + word]) become each wave's first position per
// activation (an exclusive prefix over the NW waves); thread t < MSD_LW owns word t (activations 2t,
// 2t + 1) and returns the two totals.
template <int NW = MSD_NW>
__device__ __forceinline__ void msd_wave_prefix(uint32_t* wc, uint32_t tid, uint32_t& tlo, uint32_t& thi) {
    tlo = 0;
    thi = 0;
    if (tid >= MSD_LW) return;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
        const uint32_t v = wc[ww * MSD_LW + tid];
        wc[ww * MSD_LW + tid] = tlo | (thi << 16);
        tlo += v & 0xFFFFu;
        thi += v >> 16;
    }
}

// Range b = activations [b << 10, (b << 10) + L) holding the S messages at [base, base + S) of the
// MSD output (rk: range-local keys, u16; ri: message indices).  Writes perm[base, base + S), the
// range's bucket starts offsets[b << 10, ... + L) and, for the range holding n_act, offsets[n_act + 1]
// = n.  Called by all MSD_NT threads; LDS is free on entry and on return.
// The staged path's keys of a range of S <= NT x RW messages at rk: wave w takes the contiguous segment
// [s0, s1) of the range, the range-local keys (< 1,024; 0xFFFF past the segment) two to a register,
// every load in flight at once (unconditional loads, clamped; selects after).
template <int NT, int RW>
__device__ __forceinline__ void msd_load_keys(const uint16_t* __restrict__ rk, uint32_t S, uint32_t (&kp)[RW / 2]) {
    constexpr int NW = NT / WAVE;
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const uint32_t seg = (S + NW - 1) / NW;
    const uint32_t s0 = min(w * seg, S), s1 = min((w + 1) * seg, S);
#pragma unroll
    for (int j = 0; j < RW / 2; ++j) kp[j] = 0xFFFFFFFFu;   // an empty range: no keys
    if (S == 0 || S > (uint32_t)(NT * RW)) return;
    const uint32_t last = S - 1;
#pragma unroll
    for (int r = 0; r < RW; r += 2) {
        const uint32_t i = s0 + r * WAVE + lane;
        const uint32_t a = rk[min(i, last)], c = rk[min(i + WAVE, last)];
        kp[r / 2] = (i < s1 ? a : 0xFFFFu) | ((i + WAVE < s1 ? c : 0xFFFFu) << 16);
    }
}

struct MsdNoPrefetch {
    __device__ __forceinline__ void operator()() const {}
};

// msd_range with the staged path's keys already in kp (msd_load_keys); after() runs once the count
// sweep is done with them -- the persistent form issues the next range's key loads there, so they
// fly under this range's scan, ranking and write-out.
template <bool BALLOT, int NT, int RW, class After>
__device__ __forceinline__ void msd_range_kp(MsdShared<NT, RW>& sh, uint32_t b, uint32_t base, uint32_t S,
                                             const uint16_t* __restrict__ keys16, const uint32_t* __restrict__ idx,
                                             uint32_t n, uint32_t n_act, uint32_t* __restrict__ perm,
                                             uint32_t* __restrict__ offsets, uint32_t* __restrict__ rank_out,
                                             uint32_t (&kp)[RW / 2], After after) {
    constexpr int NW = NT / WAVE;
    constexpr uint32_t CAP = NT * RW;
    static_assert(NT >= (int)MSD_LW, "a thread for every u16-pair counter word");
    const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    const uint32_t k0 = b << MSD_SHIFT;
    const uint32_t L = k0 > n_act ? 0u : min(MSD_L, n_act + 1 - k0);   // activations of this range
    const uint16_t* rk = keys16 + base;
    const uint32_t* ri = idx + base;
    if (tid == 0 && b == (n_act >> MSD_SHIFT)) offsets[n_act + 1] = n;   // the range holding n_act: the end
    if (L <= 1) {
        // one activation -- or, in the one-pass form, the unrouted messages, which msd_bucket keys at the
        // first key past n_act's range (their own range, L = 0; the range before writes offsets[n_act]):
        // the MSD pass left them in message order, which is their bucket order.  Any size, no LDS.
        if (tid == 0 && L == 1) offsets[k0] = base;
        after();
        constexpr int U = 4;
        for (uint32_t i0 = 0; i0 < S; i0 += U * NT) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * NT + tid;
                v[u] = i < S ? ri[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * NT + tid;
                if (i < S) {
                    __builtin_nontemporal_store(v[u], perm + base + i);
                    if (rank_out) rank_out[v[u]] = base + i;
                }
            }
        }
        __syncthreads();
        return;
    }
    for (uint32_t x = tid; x < MSD_L; x += NT) sh.run[x] = 0;
    for (uint32_t x = tid; x < NW * MSD_LW; x += NT) (&sh.wc[0][0])[x] = 0;
    if (S <= CAP) {
        const uint32_t seg = (S + NW - 1) / NW;
        const uint32_t s0 = min(w * seg, S);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const uint32_t k = (kp[r / 2] >> (16 * (r & 1))) & 0xFFFFu;
            if (k != 0xFFFFu) atomicAdd(&sh.wc[w][k >> 1], 1u << (16 * (k & 1)));
        }
        // the rank sweep decodes the keys again rather than keeping the count sweep's addresses live
        // across the barriers (that spilled)
#pragma unroll
        for (int j = 0; j < RW / 2; ++j) asm volatile("" : "+v"(kp[j]));
        after();
        __syncthreads();
        uint32_t tlo, thi;
        msd_wave_prefix<NW>(&sh.wc[0][0], tid, tlo, thi);
        const uint32_t ex = block_excl_scan_add_n<NT>(tlo + thi, sh.red);
        if (tid < MSD_LW) {
            sh.run[2 * tid] = ex;
            sh.run[2 * tid + 1] = ex + tlo;
            if (2 * tid < L) offsets[k0 + 2 * tid] = base + ex;
            if (2 * tid + 1 < L) offsets[k0 + 2 * tid + 1] = base + ex + tlo;
        }
        __syncthreads();
        // rows in order: the ranks stay stable; the message indices are loaded MSD_G rows at a time,
        // unconditionally (clamped into the range; a row past the wave's segment has key 0xFFFF and stores
        // nothing): a load under a lane mask put the compiler's wait for every outstanding load (vmcnt 0)
        // at each mask's join, so a group's loads and the next group's never overlapped
        const uint32_t* rsrc = S ? ri : idx;             // an empty range: any valid address
        const uint32_t rlast = S ? S - 1 : 0;
#pragma unroll
        for (int g = 0; g < RW; g += MSD_G) {
            uint32_t mm[MSD_G];
#pragma unroll
            for (int r = 0; r < MSD_G && g + r < RW; ++r) mm[r] = rsrc[min(s0 + (g + r) * WAVE + lane, rlast)];
#pragma unroll
            for (int r = 0; r < MSD_G && g + r < RW; ++r) {
                const uint32_t k = (kp[(g + r) / 2] >> (16 * ((g + r) & 1))) & 0xFFFFu;
                const uint32_t at = row_rank16<BALLOT, 10>(&sh.wc[w][k >> 1], 16 * (k & 1), k, k != 0xFFFFu);
                if (k != 0xFFFFu) sh.out[sh.run[k] + at] = mm[r];
            }
        }
        __syncthreads();
        constexpr int U = 4;                             // gathers in flight a lane
        for (uint32_t i0 = 0; i0 < S; i0 += U * NT) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * NT + tid;
                v[u] = i < S ? sh.out[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * NT + tid;
                if (i < S) {
                    __builtin_nontemporal_store(v[u], perm + base + i);
                    if (rank_out) rank_out[v[u]] = base + i;
                }
            }
        }
        __syncthreads();
        return;
    }
    // a hot range (a Zipf-hot activation; one-pass form only): its whole histogram first, so every
    // chunk knows each activation's start, then chunks of MSD_CAP ranked the same way with the
    // indices stored straight to their global places (rolled loops reading the keys again: this form
    // is not the common one)
    if constexpr (NT != MSD_NT) return;                  // the list forms never pass a range over CAP
    __syncthreads();
    for (uint32_t i = tid; i < S; i += MSD_NT) atomicAdd(&sh.run[rk[i]], 1u);
    __syncthreads();
    {
        const uint32_t ex = block_excl_scan_add_n<MSD_NT>(sh.run[tid], sh.red);
        sh.run[tid] = ex;
        if (tid < L) offsets[k0 + tid] = base + ex;
    }
    for (uint32_t c0 = 0; c0 < S; c0 += MSD_CAP) {
        const uint32_t cs = min(MSD_CAP, S - c0);
        const uint32_t seg = (cs + MSD_NW - 1) / MSD_NW;
        const uint32_t s0 = c0 + min(w * seg, cs), s1 = c0 + min((w + 1) * seg, cs);
        __syncthreads();
#pragma unroll 1
        for (uint32_t i = s0 + lane; i < s1; i += WAVE) {
            const uint32_t k = rk[i];
            atomicAdd(&sh.wc[w][k >> 1], 1u << (16 * (k & 1)));
        }
        __syncthreads();
        uint32_t tlo, thi;
        msd_wave_prefix(&sh.wc[0][0], tid, tlo, thi);
        __syncthreads();
#pragma unroll 1
        for (uint32_t r0 = s0; r0 < s1; r0 += WAVE) {     // whole rows, so every lane keeps row order
            const uint32_t i = r0 + lane;
            const bool valid = i < s1;
            const uint32_t k = valid ? rk[i] : 0u, m = valid ? ri[i] : 0u;
            const uint32_t at = row_rank16<BALLOT, 10>(&sh.wc[w][k >> 1], 16 * (k & 1), k, valid);
            if (valid) {
                const uint32_t pos = base + sh.run[k] + at;
                perm[pos] = m;
                if (rank_out) rank_out[m] = pos;
            }
        }
        __syncthreads();
        if (tid < MSD_LW) {
            sh.run[2 * tid] += tlo;
            sh.run[2 * tid + 1] += thi;
        }
        for (uint32_t x = tid; x < MSD_NW * MSD_LW; x += MSD_NT) (&sh.wc[0][0])[x] = 0;
    }
    __syncthreads();
}

template <bool BALLOT, int NT = MSD_NT, int RW = MSD_RW>
__device__ __forceinline__ void msd_range(MsdShared<NT, RW>& sh, uint32_t b, uint32_t base, uint32_t S,
                                          const uint16_t* __restrict__ keys16, const uint32_t* __restrict__ idx,
                                          uint32_t n, uint32_t n_act, uint32_t* __restrict__ perm,
                                          uint32_t* __restrict__ offsets, uint32_t* __restrict__ rank_out) {
    uint32_t kp[RW / 2];
    msd_load_keys<NT, RW>(keys16 + base, S, kp);
    msd_range_kp<BALLOT, NT, RW>(sh, b, base, S, keys16, idx, n, n_act, perm, offsets, rank_out, kp, MsdNoPrefetch{});
}

// The hardware property every stable rank of this library rests on (the LSD and MSD scatters, the
// range sorts, the level-2 and micro-batch ranks): the lanes of one wave's LDS ds_add_rtn to one
// address are served in ascending lane order, so each lane's returned value is the sum of the
// increments of the lower active lanes with the same address.  The ISA does not document the order;
// tools/ubench_lds_order.hip observed it on gfx950 and gd_create checks it here on the device it runs on
// (patterns: one address, u16-pair increments, pseudo-random colliding addresses, partial EXEC),
// refusing the handle when it fails.  One workgroup of 256 threads, 64 rounds; out[t] = thread t's
// mismatches (vector stores, summed by the host).
static __global__ void __launch_bounds__(256) k_lane_order_check(uint32_t* __restrict__ out) {
    __shared__ uint32_t s_w[4][16];
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    uint32_t bad = 0;
    for (uint32_t round = 0; round < 64; ++round) {
        if (lane < 16) s_w[w][lane] = 0;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        uint32_t x = (lane + 1) * 0x9E3779B1u ^ (round * 0x85EBCA6Bu) ^ (w * 0xC2B2AE35u);
        x ^= x >> 15;
        x *= 0x2C1B3C6Du;
        x ^= x >> 12;
        const uint32_t mode = round & 3u;
        const uint32_t addr = mode == 0 ? 0u : (mode == 1 ? (lane % 3u) : (x & (mode == 2 ? 7u : 15u)));
        const uint32_t inc = mode == 1 ? (1u << (16 * (lane & 1))) : (mode == 3 ? (x >> 28) + 1u : 1u);
        const bool active = mode != 3 || ((x >> 8) & 3u) != 0;      // partial EXEC in mode 3
        uint32_t got = 0;
        if (active) got = atomicAdd(&s_w[w][addr], inc);
        // expected: the increments of the lower active lanes on the same address
        uint32_t want = 0;
        for (uint32_t j = 0; j < WAVE; ++j) {
            const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)addr, (int)j);
            const uint32_t ij = (uint32_t)__builtin_amdgcn_readlane((int)inc, (int)j);
            const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)(active ? 1u : 0u), (int)j);
            if (j < lane && vj && aj == addr) want += ij;
        }
        if (active && got != want) ++bad;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    out[threadIdx.x] = bad;
}

// One-pass form, persistent: gridDim.x <= R workgroups (one a CU) walk the ranges b = blockIdx.x +
// k x gridDim.x, every range's first position from one scan of the totals at the start, and each
// range's key loads issued under the previous range's scan, ranking and write-out (msd_range_kp).
// Against one workgroup a range (round 3): 0.0523 -> 0.0495 ms at cfg 2, stage 0.148 -> 0.146 ms
// (3 interleaved rounds each).
template <bool BALLOT>
static __global__ void __launch_bounds__(MSD_NT, 1) k_msd_local(const uint16_t* __restrict__ keys16,
                                                            const uint32_t* __restrict__ idx,
                                                            const uint32_t* __restrict__ totals, uint32_t R,
                                                            uint32_t n, uint32_t n_act, uint32_t* __restrict__ perm,
                                                            uint32_t* __restrict__ offsets,
                                                            uint32_t* __restrict__ rank_out) {
    __shared__ MsdShared<MSD_NT, MSD_RW> sh;
    __shared__ uint32_t s_base[2 * MSD_NT];
    const uint32_t tid = threadIdx.x;
    {
        const uint32_t t0 = 2 * tid < R ? totals[2 * tid] : 0u, t1 = 2 * tid + 1 < R ? totals[2 * tid + 1] : 0u;
        const uint32_t ex = block_excl_scan_add_n<MSD_NT>(t0 + t1, sh.red);
        s_base[2 * tid] = ex;
        s_base[2 * tid + 1] = ex + t0;
    }
    __syncthreads();
    // The last range holds one key (msd_bucket clamps the unrouted messages to it: L <= 1), so its bucket
    // order is the MSD pass's order: every workgroup copies a slice of it (a 1 % miss rate puts 168K
    // messages there at cfg 2 -- one workgroup copying them was the stage's tail).
    {
        const uint32_t bl = R - 1, Sl = totals[bl], basel = s_base[bl];
        if (blockIdx.x == 0 && tid == 0 && bl == (n_act >> MSD_SHIFT)) {
            offsets[n_act] = basel;                      // n_act starts the last range: its one activation
            offsets[n_act + 1] = n;
        }
        const uint32_t per = (Sl + gridDim.x - 1) / gridDim.x;
        const uint32_t c0 = min(Sl, blockIdx.x * per), c1 = min(Sl, c0 + per);
        for (uint32_t i = c0 + tid; i < c1; i += MSD_NT) {
            const uint32_t v = idx[basel + i];
            __builtin_nontemporal_store(v, perm + basel + i);
            if (rank_out) rank_out[v] = basel + i;
        }
    }
    const uint32_t RL = R - 1;                           // the ranges sorted in LDS
    uint32_t b = blockIdx.x;
    if (b >= RL) return;                                 // uniform over the workgroup
    uint32_t kp[MSD_RW / 2], kn[MSD_RW / 2];
    uint32_t S = totals[b];
    msd_load_keys<MSD_NT, MSD_RW>(keys16 + s_base[b], S, kp);
    for (; b < RL; b += gridDim.x) {
        const uint32_t nb = b + gridDim.x;
        const uint32_t nS = nb < RL ? totals[nb] : 0u;
        const uint32_t nbase = nb < RL ? s_base[nb] : 0u;
        auto next = [&] { msd_load_keys<MSD_NT, MSD_RW>(keys16 + nbase, nS, kn); };
        msd_range_kp<BALLOT, MSD_NT, MSD_RW>(sh, b, s_base[b], S, keys16, idx, n, n_act, perm, offsets, rank_out, kp,
                                            next);
        // a hot range of several activations takes the chunked path: no after()
        if (S > MSD_CAP && min(MSD_L, n_act + 1 - min(b << MSD_SHIFT, n_act + 1)) > 1) next();
#pragma unroll
        for (int j = 0; j < MSD_RW / 2; ++j) kp[j] = kn[j];
        S = nS;
    }
}

// Three-pass form: the ranges of list[0, *count) (each <= NT x RW messages), range b at rs[b] .. rs[b + 1]
// of the grouped output, a grid-stride loop (every workgroup exits when the list is done).  <1024, 24>:
// up to 24,576 messages, 135 KB of LDS (one a CU); <512, 16>: up to 8,192, 52 KB (three a CU) -- the
// ranges of a few thousand messages of BASELINE cfg 4 (~4,400 a range) and cfg 3's mid ranks.  (Hot-key
// folding measured slower here: 0.077 against 0.059 ms at cfg 3.)
template <int NT, int RW, bool BALLOT>
static __global__ void __launch_bounds__(NT, (NT == MSD_NT ? 4 : 6)) k_msd_local_list(const uint16_t* __restrict__ keys16,
                                                                              const uint32_t* __restrict__ idx,
                                                                              const uint32_t* __restrict__ rs,
                                                                              const uint32_t* __restrict__ list,
                                                                              const uint32_t* __restrict__ count,
                                                                              uint32_t n, uint32_t n_act,
                                                                              uint32_t* __restrict__ perm,
                                                                              uint32_t* __restrict__ offsets,
                                                                              uint32_t* __restrict__ rank_out) {
    __shared__ MsdShared<NT, RW> sh;
    const uint32_t m = *count;
    for (uint32_t i = blockIdx.x; i < m; i += gridDim.x) {
        const uint32_t b = list[i];
        const uint32_t base = rs[b];
        msd_range<BALLOT, NT, RW>(sh, b, base, rs[b + 1] - base, keys16, idx, n, n_act, perm, offsets, rank_out);
    }
}

}  // namespace gd
