// gd_msd.h -- gfx950 device code for the two-level bucketing (the per-activation FIFO;
// VERDICT r02 item 3): an MSD radix pass into ranges of MSD_L = 4,096 activations, then one
// workgroup per range sorts it stably inside LDS and writes the range's bucket starts itself.
//
//   pass 1  k_radix_hist / row scan / k_radix_scatter with 9-bit digits = min(act, n_act) >> 12
//           (the LSD kernels of gd_kernels.h, used as a stable MSD partition): every range's messages
//           contiguous, in message order, keys and message indices 8 B a record;
//   pass 2  k_msd_local, one 1,024-thread workgroup per range (<= 512 ranges: n_act < 2^21):
//             sweep 1   the range's histogram over its <= 4,096 activations in LDS (32-bit counters),
//                       exclusive scan -> the activations' bucket starts, written to offsets
//                       (every activation of the range once, empty ones included: no min-scan);
//             then in chunks of <= 16 x 4,095 messages, each wave taking a contiguous 1/16 of it:
//             sweep 2a  per-wave counts (u16 pairs packed in u32 words: 16 x 2,048 words, 128 KB);
//             prefix    per activation over the 16 waves (the owner thread of a word does both
//                       halves), so a wave's counter now holds its first position in the chunk;
//             sweep 2b  the same items again in the same order: ds_add_rtn on the wave's counter
//                       returns the stable rank (a wave's lanes are served in lane order, its rows in
//                       program order), perm[range base + start + rank] = message index.
// Per message: pass 1 reads 4 + 4 B and writes 8 B; pass 2 reads the key 3 x 4 B (mostly from the
// MALL) and the index 4 B and writes 4 B -- against 3 LSD passes, 3 histograms and a min-scan.
// Output identical to the LSD path (both are the stable partition by min(act, n_act)).  A range's
// workgroup processes all of its messages, so a Zipf-hot range is one workgroup's work: the library
// times both paths per batch size and keeps the faster (bucket_device).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

constexpr int MSD_NT = 1024;
constexpr int MSD_NW = MSD_NT / WAVE;              // 16 waves
constexpr uint32_t MSD_SHIFT = 12;
constexpr uint32_t MSD_L = 1u << MSD_SHIFT;        // activations per range (range b: keys with b = key >> 12)
constexpr uint32_t MSD_LW = MSD_L / 2;             // u16-pair words per wave
constexpr uint32_t MSD_SEG = 4095;                 // messages per wave per chunk: u16 counts never carry
constexpr uint32_t MSD_CHUNK = MSD_NW * MSD_SEG;
constexpr uint32_t MSD_MAX_RANGES = 512;           // the 9-bit MSD digit

__global__ void __launch_bounds__(MSD_NT) k_msd_local(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ idx,
                                                      const uint32_t* __restrict__ totals, uint32_t n,
                                                      uint32_t n_act, uint32_t* __restrict__ perm,
                                                      uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ rank_out) {
    __shared__ uint32_t s_run[MSD_L];
    __shared__ uint32_t s_wc[MSD_NW][MSD_LW];
    __shared__ uint32_t s_red[MSD_NW];
    __shared__ uint32_t s_base;
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    // the range's first output position: the digit totals before it
    uint32_t part = 0;
    for (uint32_t d = tid; d < b; d += MSD_NT) part += totals[d];
    for (int off = WAVE / 2; off > 0; off >>= 1) part += __shfl_xor(part, off, WAVE);
    if (lane == 0) s_red[w] = part;
    for (uint32_t k = tid; k < MSD_L; k += MSD_NT) s_run[k] = 0;
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
    const uint32_t* rk = keys + base;
    const uint32_t* ri = idx + base;
    // sweep 1: counts, then starts (each thread 4 consecutive activations)
    for (uint32_t i = tid; i < S; i += MSD_NT) atomicAdd(&s_run[rk[i] - k0], 1u);
    __syncthreads();
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        c[q] = s_run[4 * tid + q];
        sum += c[q];
    }
    const uint32_t ex = block_excl_scan_add_n<MSD_NT>(sum, s_red);
    {
        uint32_t run = ex;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t k = 4 * tid + q;
            s_run[k] = run;
            if (k < L) offsets[k0 + k] = base + run;
            run += c[q];
        }
    }
    if (tid == 0 && b == (n_act >> MSD_SHIFT)) offsets[n_act + 1] = n;   // the range holding n_act: the end
    __syncthreads();
    // sweeps 2a / 2b over chunks of <= MSD_CHUNK messages
    for (uint32_t c0 = 0; c0 < S; c0 += MSD_CHUNK) {
        const uint32_t cs = min(MSD_CHUNK, S - c0);
        const uint32_t seg = (cs + MSD_NW - 1) / MSD_NW;
        const uint32_t s0 = c0 + min(w * seg, cs), s1 = c0 + min((w + 1) * seg, cs);
        for (uint32_t x = tid; x < MSD_NW * MSD_LW; x += MSD_NT) (&s_wc[0][0])[x] = 0;
        __syncthreads();
        for (uint32_t i = s0 + lane; i < s1; i += WAVE) {
            const uint32_t k = rk[i] - k0;
            atomicAdd(&s_wc[w][k >> 1], 1u << (16 * (k & 1)));
        }
        __syncthreads();
        // prefix over the waves: thread t owns words 2t, 2t + 1 (activations 4t .. 4t + 3)
        uint32_t tot[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t word = 2 * tid + j;
            uint32_t plo = 0, phi = 0;
#pragma unroll
            for (int ww = 0; ww < MSD_NW; ++ww) {
                const uint32_t v = s_wc[ww][word];
                s_wc[ww][word] = plo | (phi << 16);
                plo += v & 0xFFFFu;
                phi += v >> 16;
            }
            tot[j][0] = plo;
            tot[j][1] = phi;
        }
        __syncthreads();
        for (uint32_t i = s0 + lane; i < s1; i += WAVE) {
            const uint32_t k = rk[i] - k0;
            const uint32_t old = atomicAdd(&s_wc[w][k >> 1], 1u << (16 * (k & 1)));
            const uint32_t r = (old >> (16 * (k & 1))) & 0xFFFFu;
            const uint32_t pos = base + s_run[k] + r;
            const uint32_t m = ri[i];
            perm[pos] = m;
            if (rank_out) rank_out[m] = pos;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t word = 2 * tid + j;
            s_run[2 * word] += tot[j][0];
            s_run[2 * word + 1] += tot[j][1];
        }
        __syncthreads();
    }
}

}  // namespace gd
