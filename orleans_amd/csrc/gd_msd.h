// gd_msd.h -- gfx950 device code for the two-level bucketing (the per-activation FIFO;
// VERDICT r02 item 3): an MSD radix pass into ranges of MSD_L = 1,024 activations, then one
// workgroup per range sorts it stably inside LDS and writes the range's bucket starts itself.
//
//   pass 1  k_b2_hist / row scan / k_b2_scatter (gd_bucket2.h, 8K-item tiles) with the high digit
//           min(act, n_act) >> 10 (<= B2_RMAX2 ranges): every range's messages contiguous, in message
//           order, message indices and range-local keys (key & 1023, u16) 6 B a record;
//   pass 2  k_msd_local, one 1,024-thread workgroup per range.  A range of <= MSD_CAP messages (the
//           uniform case: 16 K for BASELINE cfg 2) is held in registers, 24 rows a lane:
//             count     per-wave counts (u16 pairs packed in u32 words: 16 x 512 words, 32 KB);
//             prefix    per activation over the 16 waves (the owner thread of a word does both halves),
//                       so a wave's counter holds its first position; the activations' totals are
//                       scanned into the bucket starts, written to offsets (every activation of the
//                       range once, empty ones included: no min-scan);
//             rank      ds_add_rtn on the wave's counter returns the stable rank (a wave's lanes are
//                       served in lane order, its rows in program order); the message index goes to
//                       its sorted place in an LDS copy of the range (96 KB);
//             write     the range's permutation slice leaves LDS in order: coalesced 4-B stores.
//           A larger range (a Zipf-hot one) is histogrammed first and ranked in chunks of MSD_CAP with
//           the index stored straight to its global position.
// Why the range is staged: the first form of this pass (ranges of 4,096 activations, 64 K messages,
// too many for LDS) stored each index straight to global memory, and those 16 M scattered 4-B stores
// cost 0.18 ms of its 0.25 ms (measured with the stores removed: profiles/r03_msd4k_nostore_exp.txt);
// staged, the pass takes 0.054 ms at cfg 2 (profiles/r03_msd_ab.txt), the whole stage 0.148 ms.
// Per message: pass 1 reads 4 B twice (histogram, scatter) and writes 6 B; pass 2 reads 6 B and
// writes 4 B in order -- 24 B over 4 launches, against 40 B over 11 for three packed 7-bit LSD passes.  Output identical to the LSD path (both are the stable
// partition by min(act, n_act)); the library times both per batch size and keeps the faster.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

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
constexpr uint32_t MSD_MAX_RANGES = B2_RMAX2;      // the high digit of pass 1

// G16 = false (the default): the staging copy holds the message indices (4 bytes a message, 24 rows
// a lane, one workgroup a CU).  G16: u16 positions in the range (2 bytes, 20 rows a lane, two
// workgroups a CU at <= 64 VGPRs) and the write-out gathers the indices from the range's slice --
// measured slower at cfg 2 (0.088 against 0.054 ms, profiles/r03_msd_ab.txt), kept for A/B.
template <bool G16>
struct MsdCfg {
    static constexpr int RW = G16 ? 20 : 24;                      // rows of 64 messages a wave holds
    static constexpr uint32_t CAP = RW * MSD_NT;                  // messages per chunk (<= 1,536 a wave)
    static constexpr int WPE = G16 ? 8 : 4;                       // waves per SIMD: 2 or 1 workgroups a CU
    using Out = typename std::conditional<G16, uint16_t, uint32_t>::type;
};

// The per-wave counts (u16 pairs, wc[wave * MSD_LW + word]) become each wave's first position per
// activation (an exclusive prefix over the waves); thread t < MSD_LW owns word t (activations 2t,
// 2t + 1) and returns the two totals.
__device__ __forceinline__ void msd_wave_prefix(uint32_t* wc, uint32_t tid, uint32_t& tlo, uint32_t& thi) {
    tlo = 0;
    thi = 0;
    if (tid >= MSD_LW) return;
#pragma unroll
    for (int ww = 0; ww < MSD_NW; ++ww) {
        const uint32_t v = wc[ww * MSD_LW + tid];
        wc[ww * MSD_LW + tid] = tlo | (thi << 16);
        tlo += v & 0xFFFFu;
        thi += v >> 16;
    }
}

template <bool G16, bool EARLY = false, bool K16 = false>
__global__ void __launch_bounds__(MSD_NT, MsdCfg<G16>::WPE) k_msd_local(const uint32_t* __restrict__ keys,
                                                                      const uint32_t* __restrict__ idx,
                                                                      const uint32_t* __restrict__ totals,
                                                                      uint32_t n, uint32_t n_act,
                                                                      uint32_t* __restrict__ perm,
                                                                      uint32_t* __restrict__ offsets,
                                                                      uint32_t* __restrict__ rank_out) {
    static_assert(!(G16 && EARLY), "G16 stages positions: no indices to load early");
    static_assert(MSD_NT == (int)MSD_L && MSD_LW <= (uint32_t)MSD_NT, "one thread per activation of a range");
    constexpr int MSD_RW = MsdCfg<G16>::RW;
    constexpr uint32_t MSD_CAP = MsdCfg<G16>::CAP;
    __shared__ uint32_t s_run[MSD_L];
    __shared__ uint32_t s_wc[MSD_NW][MSD_LW];
    __shared__ typename MsdCfg<G16>::Out s_out[MSD_CAP];
    __shared__ uint32_t s_red[MSD_NW];
    __shared__ uint32_t s_base;
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    // the range's first output position: the digit totals before it
    uint32_t part = 0;
    for (uint32_t d = tid; d < b; d += MSD_NT) part += totals[d];
    for (int off = WAVE / 2; off > 0; off >>= 1) part += __shfl_xor(part, off, WAVE);
    if (lane == 0) s_red[w] = part;
    s_run[tid] = 0;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (int q = 0; q < MSD_NW; ++q) t += s_red[q];
        s_base = t;
    }
    __syncthreads();
    const uint32_t base = s_base;
    const uint32_t S = totals[b];
    const uint32_t k0 = b << MSD_SHIFT;
    const uint32_t L = min(MSD_L, n_act + 1 - k0);       // activations of this range
    // K16: pass 1 wrote the range-local keys (key & 1023) as u16, 6 B a record instead of 8
    using KT = typename std::conditional<K16, uint16_t, uint32_t>::type;
    const KT* rk = reinterpret_cast<const KT*>(keys) + base;
    const uint32_t koff = K16 ? 0u : k0;                 // what turns a stored key into a range-local one
    const uint32_t* ri = idx + base;
    if (tid == 0 && b == (n_act >> MSD_SHIFT)) offsets[n_act + 1] = n;   // the range holding n_act: the end
    for (uint32_t x = tid; x < MSD_NW * MSD_LW; x += MSD_NT) (&s_wc[0][0])[x] = 0;
    if (S <= MSD_CAP) {
        // staged: wave w takes the contiguous segment [s0, s1) of the range, the range-local keys
        // (< 1,024; 0xFFFF past the segment) two to a register, every load in flight at once
        const uint32_t seg = (S + MSD_NW - 1) / MSD_NW;
        const uint32_t s0 = min(w * seg, S), s1 = min((w + 1) * seg, S);
        uint32_t kp[MSD_RW / 2];
#pragma unroll
        for (int j = 0; j < MSD_RW / 2; ++j) kp[j] = 0xFFFFFFFFu;   // an empty range: no keys
        // EARLY: the message indices are loaded right behind the keys and stay in registers (122 VGPRs),
        // their latency under the count, prefix and scan phases -- measured slower at cfg 2 (0.058
        // against 0.054 ms, profiles/r03_msd_early_ab.txt): the key and index streams then compete
        // for the CU's share of HBM in the same phase; kept for A/B
        uint32_t mi[EARLY ? MSD_RW : 1] = {};
        if (S) {                                         // unconditional loads (clamped), selects after
            const uint32_t last = S - 1;
#pragma unroll
            for (int r = 0; r < MSD_RW; r += 2) {
                const uint32_t i = s0 + r * WAVE + lane;
                const uint32_t a = rk[min(i, last)], c = rk[min(i + WAVE, last)];
                kp[r / 2] = (i < s1 ? a - koff : 0xFFFFu) | ((i + WAVE < s1 ? c - koff : 0xFFFFu) << 16);
            }
            if constexpr (EARLY) {
#pragma unroll
                for (int r = 0; r < MSD_RW; ++r) mi[r] = ri[min(s0 + r * WAVE + lane, last)];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < MSD_RW; ++r) {
            const uint32_t k = (kp[r / 2] >> (16 * (r & 1))) & 0xFFFFu;
            if (k != 0xFFFFu) atomicAdd(&s_wc[w][k >> 1], 1u << (16 * (k & 1)));
        }
        // the rank sweep decodes the keys again rather than keeping the count sweep's addresses live
        // across the barriers (that spilled)
#pragma unroll
        for (int j = 0; j < MSD_RW / 2; ++j) asm volatile("" : "+v"(kp[j]));
        __syncthreads();
        uint32_t tlo, thi;
        msd_wave_prefix(&s_wc[0][0], tid, tlo, thi);
        const uint32_t ex = block_excl_scan_add_n<MSD_NT>(tlo + thi, s_red);
        if (tid < MSD_LW) {
            s_run[2 * tid] = ex;
            s_run[2 * tid + 1] = ex + tlo;
            if (2 * tid < L) offsets[k0 + 2 * tid] = base + ex;
            if (2 * tid + 1 < L) offsets[k0 + 2 * tid + 1] = base + ex + tlo;
        }
        __syncthreads();
        // rows in order: the ranks stay stable.  G16 stages the message's place in the range, else the
        // message index (loaded MSD_G rows at a time)
#pragma unroll
        for (int g = 0; g < MSD_RW; g += MSD_G) {
            uint32_t mm[MSD_G];
#pragma unroll
            for (int r = 0; r < MSD_G && g + r < MSD_RW; ++r) {
                const uint32_t i = s0 + (g + r) * WAVE + lane;
                if constexpr (EARLY) mm[r] = mi[g + r];
                else mm[r] = G16 ? i : (i < s1 ? ri[i] : 0u);
            }
#pragma unroll
            for (int r = 0; r < MSD_G && g + r < MSD_RW; ++r) {
                const uint32_t k = (kp[(g + r) / 2] >> (16 * ((g + r) & 1))) & 0xFFFFu;
                if (k == 0xFFFFu) continue;
                const uint32_t old = atomicAdd(&s_wc[w][k >> 1], 1u << (16 * (k & 1)));
                s_out[s_run[k] + ((old >> (16 * (k & 1))) & 0xFFFFu)] = (typename MsdCfg<G16>::Out)mm[r];
            }
        }
        __syncthreads();
        constexpr int U = 4;                             // gathers in flight a lane
        for (uint32_t i0 = 0; i0 < S; i0 += U * MSD_NT) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * MSD_NT + tid;
                v[u] = i < S ? (G16 ? ri[s_out[i]] : (uint32_t)s_out[i]) : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * MSD_NT + tid;
                if (i < S) {
                    perm[base + i] = v[u];
                    if (rank_out) rank_out[v[u]] = base + i;
                }
            }
        }
        return;
    }
    // a hot range (a Zipf-hot activation): its whole histogram first, so every chunk knows each
    // activation's start, then chunks of MSD_CAP ranked the same way with the indices stored straight
    // to their global places (rolled loops reading the keys again: this form is not the common one)
    for (uint32_t i = tid; i < S; i += MSD_NT) atomicAdd(&s_run[rk[i] - koff], 1u);
    __syncthreads();
    {
        const uint32_t ex = block_excl_scan_add_n<MSD_NT>(s_run[tid], s_red);
        s_run[tid] = ex;
        if (tid < L) offsets[k0 + tid] = base + ex;
    }
    for (uint32_t c0 = 0; c0 < S; c0 += MSD_CAP) {
        const uint32_t cs = min(MSD_CAP, S - c0);
        const uint32_t seg = (cs + MSD_NW - 1) / MSD_NW;
        const uint32_t s0 = c0 + min(w * seg, cs), s1 = c0 + min((w + 1) * seg, cs);
        __syncthreads();
#pragma unroll 1
        for (uint32_t i = s0 + lane; i < s1; i += WAVE) {
            const uint32_t k = rk[i] - koff;
            atomicAdd(&s_wc[w][k >> 1], 1u << (16 * (k & 1)));
        }
        __syncthreads();
        uint32_t tlo, thi;
        msd_wave_prefix(&s_wc[0][0], tid, tlo, thi);
        __syncthreads();
#pragma unroll 1
        for (uint32_t r0 = s0; r0 < s1; r0 += WAVE) {     // whole rows, so every lane keeps row order
            const uint32_t i = r0 + lane;
            if (i < s1) {
                const uint32_t k = rk[i] - koff, m = ri[i];
                const uint32_t old = atomicAdd(&s_wc[w][k >> 1], 1u << (16 * (k & 1)));
                const uint32_t pos = base + s_run[k] + ((old >> (16 * (k & 1))) & 0xFFFFu);
                perm[pos] = m;
                if (rank_out) rank_out[m] = pos;
            }
        }
        __syncthreads();
        if (tid < MSD_LW) {
            s_run[2 * tid] += tlo;
            s_run[2 * tid + 1] += thi;
        }
        for (uint32_t x = tid; x < MSD_NW * MSD_LW; x += MSD_NT) (&s_wc[0][0])[x] = 0;
    }
}

}  // namespace gd
