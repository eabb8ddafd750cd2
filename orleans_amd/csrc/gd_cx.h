// gd_cx.h -- builds the compact probe index (gd_kernels.h, CxArgs) from the directory table.
//
// The index is derived state: the library rebuilds it on the first route after any change of the
// directory table (a launch that takes the table as a writable Slot*, a clear, a rehash), so every
// directory operation keeps its semantics on the authoritative 32-B-slot table and the probe reads
// the copy.  Two passes over the table:
//   k_cx_types  eligibility (every live entry has N0 = 0) and the set of distinct TypeCodeData
//               (at most CX_TYPES, open addressing, CAS-inserted);
//   k_cx_build  each live entry into the index at cx_home(uniform hash), first free slot in probe
//               order (CAS on the meta word), and the largest group distance any entry sits at.
// A directory with N0 != 0 keys or more than CX_TYPES types is left to the directory probe.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

struct CxCounters {
    uint32_t flag;         // bit 0: an entry with N0 != 0; bit 1: more than CX_TYPES types
    uint32_t max_rounds;   // CxArgs::max_rounds
    uint32_t full;         // the index ran out of slots (cannot happen at cap >= live)
    uint32_t flag8;        // the 8-B index: bit 0 an N1 >= 2^32 (one type more: the host counts them)
    uint32_t max_rounds8;  // Cx8Args::max_rounds
    uint32_t full8;
    uint32_t act_max;      // the largest activation (GD_ACT_MULTI aside) and silo: the host's bit split
    uint32_t silo_max;
};

static __global__ void __launch_bounds__(BLOCK) k_cx_types(const Slot* __restrict__ slots, unsigned long long cap,
                                                    unsigned long long* types, CxCounters* ctr) {
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= cap) return;
    const uint4* q = reinterpret_cast<const uint4*>(slots + j);
    const uint4 a = q[0], b = q[1];
    if (slot_state(b.w) != SLOT_LIVE) return;
    if ((a.x | a.y) != 0) {
        atomicOr(&ctr->flag, 1u);
        return;
    }
    if (a.w != 0) atomicOr(&ctr->flag8, 1u);
    if (b.z != GD_ACT_MULTI) atomicMax(&ctr->act_max, b.z);
    atomicMax(&ctr->silo_max, slot_silo(b.w));
    const unsigned long long tcd = (unsigned long long)b.x | ((unsigned long long)b.y << 32);
    // one insert per distinct type in the wave: lanes holding the first lane's type stand down
    const unsigned long long lead = __shfl(tcd, __ffsll((long long)__ballot(1)) - 1);
    const bool is_lead = (threadIdx.x & (WAVE - 1)) == (uint32_t)(__ffsll((long long)__ballot(1)) - 1);
    if (tcd == lead && !is_lead) return;
    uint32_t t = cx_type_home(tcd);
    for (uint32_t k = 0; k < CX_TYPES; ++k) {
        unsigned long long cur = __hip_atomic_load(types + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == tcd) return;
        if (cur == CX_NO_TYPE) {
            cur = atomicCAS(types + t, CX_NO_TYPE, tcd);
            if (cur == CX_NO_TYPE || cur == tcd) return;
        }
        t = (t + 1) & (CX_TYPES - 1);
    }
    atomicOr(&ctr->flag, 2u);
}

static __global__ void __launch_bounds__(BLOCK) k_cx_build(const Slot* __restrict__ slots, unsigned long long cap,
                                                    const unsigned long long* __restrict__ types, uint4* cx,
                                                    unsigned long long cx_cap, CxCounters* ctr) {
    if (ctr->flag) return;                             // not eligible (uniform): nothing to build
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t rounds = 0;
    bool placed = false, live = false;
    if (j < cap) {
        const uint4* q = reinterpret_cast<const uint4*>(slots + j);
        const uint4 a = q[0], b = q[1];
        live = slot_state(b.w) == SLOT_LIVE;
        if (live) {
            const uint64_t n1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
            const uint64_t tcd = (uint64_t)b.x | ((uint64_t)b.y << 32);
            uint32_t t = cx_type_home(tcd);
            while (types[t] != tcd) t = (t + 1) & (CX_TYPES - 1);     // present: k_cx_types put it there
            const uint32_t meta = CX_LIVE | (t << 16) | slot_silo(b.w);
            const unsigned long long home = cx_home(uniform_hash(0, n1, tcd), cx_cap);
            unsigned long long s = home;
            for (unsigned long long d = 0; d < cx_cap; ++d) {
                if (atomicCAS(&cx[s].w, 0u, meta) == 0u) {
                    cx[s].x = (uint32_t)n1;
                    cx[s].y = (uint32_t)(n1 >> 32);
                    cx[s].z = b.z;
                    rounds = (uint32_t)((s >= home ? s - home : s + cx_cap - home) / CX_GROUP);
                    placed = true;
                    break;
                }
                s = s + 1 == cx_cap ? 0 : s + 1;
            }
            if (!placed) atomicOr(&ctr->full, 1u);
        }
    }
    // one atomicMax per wave on the shared counter (one per entry serialises a million of them);
    // every lane of the wave takes part in the reduction
    for (int off = WAVE / 2; off > 0; off >>= 1) rounds = max(rounds, (uint32_t)__shfl_xor(rounds, off, WAVE));
    if (lane_id() == 0 && rounds) atomicMax(&ctr->max_rounds, rounds);
}

// The 8-B index (Cx8Args), built after the 16-B one when the host found it eligible (flag8 == 0, one
// type, activations and silos fitting a u32 together): slot = (silo + 1) << ab | act (all ab bits set
// for a multi-activation grain) above the N1 low word, placed by a 64-bit CAS in probe order from
// cx8_home.
static __global__ void __launch_bounds__(BLOCK) k_cx8_build(const Slot* __restrict__ slots, unsigned long long cap,
                                                     unsigned long long* cx8, unsigned long long cx8_cap,
                                                     uint32_t ab, CxCounters* ctr) {
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t rounds = 0;
    if (j < cap) {
        const uint4* q = reinterpret_cast<const uint4*>(slots + j);
        const uint4 a = q[0], b = q[1];
        if (slot_state(b.w) == SLOT_LIVE) {
            const uint64_t n1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
            const uint64_t tcd = (uint64_t)b.x | ((uint64_t)b.y << 32);
            const uint32_t am = (1u << ab) - 1u;
            const uint32_t y = ((slot_silo(b.w) + 1u) << ab) | (b.z == GD_ACT_MULTI ? am : b.z);
            const unsigned long long v = ((unsigned long long)y << 32) | (uint32_t)n1;
            const unsigned long long home = cx8_home(uniform_hash(0, n1, tcd), cx8_cap);
            unsigned long long s = home;
            bool placed = false;
            for (unsigned long long d = 0; d < cx8_cap; ++d) {
                if (atomicCAS(cx8 + s, 0ull, v) == 0ull) {
                    rounds = (uint32_t)((s >= home ? s - home : s + cx8_cap - home) / CX8_GROUP);
                    placed = true;
                    break;
                }
                s = s + 1 == cx8_cap ? 0 : s + 1;
            }
            if (!placed) atomicOr(&ctr->full8, 1u);
        }
    }
    for (int off = WAVE / 2; off > 0; off >>= 1) rounds = max(rounds, (uint32_t)__shfl_xor(rounds, off, WAVE));
    if (lane_id() == 0 && rounds) atomicMax(&ctr->max_rounds8, rounds);
}

}  // namespace gd
