// gd_cx.h -- builds and maintains the compact probe indexes (gd_kernels.h CxArgs, Cx8Args).
//
// The indexes are derived state: index slot j is a narrow projection of directory table slot j
// (round 6), so every directory operation keeps its semantics on the authoritative 32-B-slot table
// and the probe reads the copy.
//   k_cx_types    one pass over the table: the set of distinct TypeCodeData of N0 = 0 entries with a
//                 count each (per-workgroup LDS sets, one global insert per type and workgroup), the
//                 largest activation and silo, the entries no index can hold (N0 != 0) and those the
//                 8-B index cannot (N1 >= 2^32).  The host picks the 8-B layout from them.
//   k_cx_project  one streaming pass: every table slot -> its 16-B and 8-B index slots (the full build).
//   k_cx_sync     the slots one directory batch touched (register, upsert, unregister) re-projected
//                 in place: the directory change costs a pass over the batch, not over the table
//                 (GrainDirectoryPartition.AddSingleActivation / RemoveActivation are O(1) dictionary
//                 operations, GrainDirectoryPartition.cs:304-363, and activations register all the
//                 time, Catalog.cs:540-552).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

// An 8-B slot that matches no key but keeps probe chains going: y = 1 (u = 0), x = 0.
constexpr unsigned long long CX8_HOLE = 1ull << 32;

struct CxCounters {
    uint32_t n0_live;      // live entries with N0 != 0 (directory probe only)
    uint32_t big_n1;       // live N0 = 0 entries with N1 >= 2^32 (not in the 8-B index)
    uint32_t types_full;   // a type did not fit the 256-slot set (its entries: directory probe)
    uint32_t act_max;      // the largest activation (GD_ACT_MULTI aside) and silo: the host's bit split
    uint32_t silo_max;
    uint32_t out8;         // projections (build and sync) the 8-B index does not hold or redirects
    uint32_t pad[2];
};

// ---- type sets ------------------------------------------------------------------
// Global type set (CX_TYPES u64 slots, CX_NO_TYPE empty) with a count per slot: insert tcd, add c.
__device__ __forceinline__ int cx_type_add(unsigned long long* types, uint32_t* count, uint64_t tcd, uint32_t c,
                                           CxCounters* ctr) {
    uint32_t t = cx_type_home(tcd);
    for (uint32_t k = 0; k < CX_TYPES; ++k) {
        unsigned long long cur = __hip_atomic_load(types + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == CX_NO_TYPE) cur = atomicCAS(types + t, CX_NO_TYPE, (unsigned long long)tcd);
        if (cur == CX_NO_TYPE || cur == tcd) {
            if (count && c) atomicAdd(count + t, c);
            return (int)t;
        }
        t = (t + 1) & (CX_TYPES - 1);
    }
    if (ctr) atomicOr(&ctr->types_full, 1u);
    return -1;
}

// Workgroup type set in LDS (CXT_LDS slots): a run of c entries of type tcd; a full set spills to the
// global one.
constexpr uint32_t CXT_LDS = 64;
__device__ __forceinline__ void cx_type_note(unsigned long long* s_t, uint32_t* s_c, uint64_t tcd, uint32_t c,
                                             unsigned long long* types, uint32_t* count, CxCounters* ctr) {
    uint32_t t = cx_type_home(tcd) & (CXT_LDS - 1);
    for (uint32_t k = 0; k < CXT_LDS; ++k) {
        unsigned long long cur = __hip_atomic_load(s_t + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == CX_NO_TYPE) cur = atomicCAS(s_t + t, CX_NO_TYPE, (unsigned long long)tcd);
        if (cur == CX_NO_TYPE || cur == tcd) {
            atomicAdd(s_c + t, c);
            return;
        }
        t = (t + 1) & (CXT_LDS - 1);
    }
    (void)cx_type_add(types, count, tcd, c, ctr);
}

constexpr int CXT_IT = 4;   // table slots a thread reads per round (all in flight)

// Grid-stride over the table, CXT_IT coalesced slots a thread a round.  Per workgroup: the types in LDS
// (a thread folds runs of one type before touching LDS), counters reduced, then one global update each.
static __global__ void __launch_bounds__(BLOCK) k_cx_types(const Slot* __restrict__ slots, unsigned long long cap,
                                                    unsigned long long* types, uint32_t* count, CxCounters* ctr) {
    __shared__ unsigned long long s_t[CXT_LDS];
    __shared__ uint32_t s_c[CXT_LDS];
    __shared__ uint32_t s_red[4][BLOCK / WAVE];
    for (uint32_t k = threadIdx.x; k < CXT_LDS; k += BLOCK) {
        s_t[k] = CX_NO_TYPE;
        s_c[k] = 0;
    }
    __syncthreads();
    uint32_t n0c = 0, bigc = 0, amax = 0, smax = 0, run_c = 0;
    unsigned long long run_t = CX_NO_TYPE;
    const unsigned long long stride = (unsigned long long)gridDim.x * BLOCK * CXT_IT;
    for (unsigned long long base = (unsigned long long)blockIdx.x * BLOCK * CXT_IT + threadIdx.x; base < cap;
         base += stride) {
        uint4 a[CXT_IT], b[CXT_IT];
#pragma unroll
        for (int r = 0; r < CXT_IT; ++r) {
            const unsigned long long j = base + (unsigned long long)r * BLOCK;
            b[r] = make_uint4(0, 0, 0, 0);
            if (j < cap) {
                const uint4* q = reinterpret_cast<const uint4*>(slots + j);
                a[r] = q[0];
                b[r] = q[1];
            }
        }
#pragma unroll
        for (int r = 0; r < CXT_IT; ++r) {
            if (slot_state(b[r].w) != SLOT_LIVE) continue;
            if ((a[r].x | a[r].y) != 0) {
                ++n0c;
                continue;
            }
            if (a[r].w != 0) ++bigc;
            if (b[r].z != GD_ACT_MULTI) amax = max(amax, b[r].z);
            smax = max(smax, slot_silo(b[r].w));
            const unsigned long long tcd = (unsigned long long)b[r].x | ((unsigned long long)b[r].y << 32);
            if (tcd != run_t) {
                if (run_c) cx_type_note(s_t, s_c, run_t, run_c, types, count, ctr);
                run_t = tcd;
                run_c = 0;
            }
            ++run_c;
        }
    }
    if (run_c) cx_type_note(s_t, s_c, run_t, run_c, types, count, ctr);
    // workgroup reductions: wave shuffles, then LDS
    for (int off = WAVE / 2; off > 0; off >>= 1) {
        n0c += __shfl_xor(n0c, off, WAVE);
        bigc += __shfl_xor(bigc, off, WAVE);
        amax = max(amax, (uint32_t)__shfl_xor(amax, off, WAVE));
        smax = max(smax, (uint32_t)__shfl_xor(smax, off, WAVE));
    }
    const uint32_t w = threadIdx.x / WAVE;
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        s_red[0][w] = n0c;
        s_red[1][w] = bigc;
        s_red[2][w] = amax;
        s_red[3][w] = smax;
    }
    __syncthreads();                                   // also: every cx_type_note of the workgroup is done
    if (threadIdx.x == 0) {
        for (int k = 1; k < BLOCK / WAVE; ++k) {
            n0c += s_red[0][k];
            bigc += s_red[1][k];
            amax = max(amax, s_red[2][k]);
            smax = max(smax, s_red[3][k]);
        }
        if (n0c) atomicAdd(&ctr->n0_live, n0c);
        if (bigc) atomicAdd(&ctr->big_n1, bigc);
        if (amax) atomicMax(&ctr->act_max, amax);
        if (smax) atomicMax(&ctr->silo_max, smax);
    }
    for (uint32_t k = threadIdx.x; k < CXT_LDS; k += BLOCK)
        if (s_t[k] != CX_NO_TYPE) (void)cx_type_add(types, count, s_t[k], s_c[k], ctr);
}

// ---- projection -------------------------------------------------------------------
struct CxBuild {
    uint4* cx16;                   // the 16-B index (null: not kept)
    unsigned long long* types;     // its global type set (staged in LDS by the kernels below)
    unsigned long long* cx8;       // the 8-B index (null: not kept)
    Cx8Args p8;                    // its layout (types, ab, sb)
};

__device__ __forceinline__ void cx_stage_types(const unsigned long long* types, unsigned long long* s_types) {
    for (uint32_t t = threadIdx.x; t < CX_TYPES; t += blockDim.x) s_types[t] = types[t];
    __syncthreads();
}

// Table slot j (a, b: its two halves) -> index slot j.  add_types (k_cx_sync): a type the staged set
// lacks is looked up / inserted in the global set (a batch may register a new grain class).
// Returns whether the 8-B index holds the entry (false for a live entry it does not hold or redirects).
__device__ __forceinline__ bool cx_project(const uint4 a, const uint4 b, unsigned long long j, const CxBuild& B,
                                           const unsigned long long* s_types, bool add_types) {
    const uint32_t st = slot_state(b.w);
    uint4 v16 = make_uint4(0, 0, 0, 0);
    unsigned long long v8 = 0;
    bool held8 = true;
    if (st == SLOT_LIVE) {
        const uint64_t n0 = (uint64_t)a.x | ((uint64_t)a.y << 32);
        const uint64_t n1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
        const uint64_t tcd = (uint64_t)b.x | ((uint64_t)b.y << 32);
        const uint32_t act = b.z, silo = slot_silo(b.w);
        if (B.cx16) {
            int t = n0 == 0 ? cx_type_index(s_types, tcd) : -1;
            if (t < 0 && n0 == 0 && add_types) t = cx_type_add(B.types, nullptr, tcd, 0, nullptr);
            v16 = t >= 0 ? make_uint4(a.z, a.w, act, CX_LIVE | ((uint32_t)t << 16) | silo) : make_uint4(0, 0, 0, CX_TOMB);
        }
        if (B.cx8) {
            const int t8 = cx8_type(B.p8, n0, n1, tcd);
            if (t8 < 0) {
                v8 = CX8_HOLE;                                     // not held: its key probes the directory
                held8 = false;
            } else {
                const uint32_t ab = B.p8.ab, sb = B.p8.sb;
                const uint32_t am = (1u << ab) - 1u, umax = ~0u >> ab;
                uint32_t u = ((uint32_t)t8 << sb) | (silo + 1u);
                if (((silo + 1u) >> sb) != 0 || u >= umax) u = umax;   // redirect: silo / type too wide
                uint32_t av = act == GD_ACT_MULTI ? am : act;
                if (act != GD_ACT_MULTI && act >= am - 1u) av = am - 1u;   // redirect: activation too wide
                held8 = u != umax && av != am - 1u;
                v8 = ((unsigned long long)((u << ab) | av) << 32) | a.z;
            }
        }
    } else if (st != SLOT_EMPTY) {
        v16 = make_uint4(0, 0, 0, CX_TOMB);
        v8 = CX8_HOLE;
    }
    if (B.cx16) B.cx16[j] = v16;
    if (B.cx8) B.cx8[j] = v8;
    return held8;
}

// The full build: every table slot, grid-stride, CXT_IT slots a thread a round.
static __global__ void __launch_bounds__(BLOCK) k_cx_project(const Slot* __restrict__ slots, unsigned long long cap,
                                                      CxBuild B, CxCounters* ctr) {
    __shared__ unsigned long long s_types[CX_TYPES];
    cx_stage_types(B.types, s_types);
    uint32_t out8 = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * BLOCK * CXT_IT;
    for (unsigned long long base = (unsigned long long)blockIdx.x * BLOCK * CXT_IT + threadIdx.x; base < cap;
         base += stride) {
        uint4 a[CXT_IT], b[CXT_IT];
#pragma unroll
        for (int r = 0; r < CXT_IT; ++r) {
            const unsigned long long j = base + (unsigned long long)r * BLOCK;
            if (j < cap) {
                const uint4* q = reinterpret_cast<const uint4*>(slots + j);
                a[r] = q[0];
                b[r] = q[1];
            }
        }
#pragma unroll
        for (int r = 0; r < CXT_IT; ++r) {
            const unsigned long long j = base + (unsigned long long)r * BLOCK;
            if (j < cap && !cx_project(a[r], b[r], j, B, s_types, false)) ++out8;
        }
    }
    for (int off = WAVE / 2; off > 0; off >>= 1) out8 += __shfl_xor(out8, off, WAVE);
    if ((threadIdx.x & (WAVE - 1)) == 0 && out8) atomicAdd(&ctr->out8, out8);
}

// Incremental: the table slots a directory batch touched (slot_of[i]; NONE32 / SLOT_RETRY: none),
// re-projected after the batch's last table write.  Duplicates are harmless (a projection is a function
// of the table slot).
static __global__ void __launch_bounds__(BLOCK) k_cx_sync(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                   const Slot* __restrict__ slots, CxBuild B, CxCounters* ctr) {
    __shared__ unsigned long long s_types[CX_TYPES];
    cx_stage_types(B.types, s_types);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool out = false;
    if (i < n) {
        const uint32_t s = slot_of[i];
        if (s < SLOT_RETRY) {
            const uint4* q = reinterpret_cast<const uint4*>(slots + s);
            out = !cx_project(q[0], q[1], s, B, s_types, true);
        }
    }
    const unsigned long long m = __ballot(out);
    if (lane_id() == 0 && m) atomicAdd(&ctr->out8, (uint32_t)__popcll(m));
}

// A directory batch's commits with the committed slots projected at once (the indexes current before
// the batch): AddSingleActivation's winner (k_reg_commit) and RemoveActivation's remover
// (k_unreg_commit) re-project their slot; no k_cx_sync launch.
static __global__ void __launch_bounds__(BLOCK) k_reg_commit_cx(const uint32_t* __restrict__ slot_of,
                                                         const uint32_t* __restrict__ win,
                                                         const gd_val* __restrict__ vals, uint32_t n, Slot* slots,
                                                         DevCounters* ctr, uint32_t* __restrict__ vtag, uint32_t op,
                                                         CxBuild B, CxCounters* cctr) {
    __shared__ unsigned long long s_types[CX_TYPES];
    cx_stage_types(B.types, s_types);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool out = false;
    const bool w = i < n && win[i] == i;
    live_delta(ctr, w, false);
    if (w) {
        reg_commit_item(i, slot_of, vals, slots, ctr, vtag, op);
        const uint32_t s = slot_of[i];
        const uint4* q = reinterpret_cast<const uint4*>(slots + s);
        out = !cx_project(q[0], q[1], s, B, s_types, true);
    }
    const unsigned long long m = __ballot(out);
    if (lane_id() == 0 && m) atomicAdd(&cctr->out8, (uint32_t)__popcll(m));
}

static __global__ void __launch_bounds__(BLOCK) k_reg_commit_elect_cx(const uint32_t* __restrict__ slot_of,
                                                               const uint8_t* __restrict__ is_new,
                                                               const gd_val* __restrict__ vals, uint32_t n,
                                                               Slot* slots, DevCounters* ctr,
                                                               uint32_t* __restrict__ vtag, uint32_t op,
                                                               uint32_t* __restrict__ last,
                                                               uint32_t* __restrict__ win,
                                                               const uint32_t* __restrict__ unsettled,
                                                               uint32_t* __restrict__ retry0, CxBuild B,
                                                               CxCounters* cctr) {
    __shared__ unsigned long long s_types[CX_TYPES];
    cx_stage_types(B.types, s_types);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i == 0 && unsettled) {
        if (*unsettled) atomicOr(&ctr->err, ERR_UNSETTLED);
        *retry0 = 0;
    }
    const bool w = reg_elected(i, n, slot_of, is_new, last, win);
    live_delta(ctr, w, false);
    bool out = false;
    if (w) {
        reg_commit_item(i, slot_of, vals, slots, ctr, vtag, op);
        const uint32_t s = slot_of[i];
        const uint4* q = reinterpret_cast<const uint4*>(slots + s);
        out = !cx_project(q[0], q[1], s, B, s_types, true);
    }
    const unsigned long long m = __ballot(out);
    if (lane_id() == 0 && m) atomicAdd(&cctr->out8, (uint32_t)__popcll(m));
}

static __global__ void __launch_bounds__(BLOCK) k_unreg_commit_elect_cx(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                                 Slot* slots, DevCounters* ctr,
                                                                 uint32_t* __restrict__ last,
                                                                 uint8_t* __restrict__ out_removed, CxBuild B) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool rm = unreg_elected_commit(i, n, slot_of, slots, last, out_removed);
    live_delta(ctr, rm, true);
    if (!rm) return;
    const uint32_t s = slot_of[i];
    if (B.cx16) B.cx16[s] = make_uint4(0, 0, 0, CX_TOMB);
    if (B.cx8) B.cx8[s] = CX8_HOLE;
}

// RemoveActivation as one launch, for a batch whose caller does not ask which item removed (round 6,
// gd_dir_unregister_device with no out_removed): the table's end state does not depend on which of a
// key's matching items removes it -- every one writes the same tombstone -- so the item whose CAS turns
// the slot's LIVE meta (as its walk read it) into TOMB removes, and projects the tombstone into the
// indexes (B.cx16 / B.cx8; null: not current).  No election word, no slot_of, no second launch.  A walk
// never stops at a tombstone, so an item meeting another item's fresh tombstone walks on as it would
// have past the live entry; a duplicate's CAS fails on the changed meta.
static __global__ void __launch_bounds__(BLOCK) k_unreg_cas(const gd_key* __restrict__ keys,
                                                     const uint32_t* __restrict__ acts, uint32_t n, Slot* slots,
                                                     unsigned long long mask, DevCounters* ctr, CxBuild B) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool rm = false;
    unsigned long long s = 0;
    if (i < n) {
        const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
        const uint32_t act = acts[i], maxp = ctr->max_probe;
        s = home_slot(uniform_hash(n0, n1, tcd), mask);
        for (uint32_t p = 0; p <= maxp; ++p) {
            const uint4* q = reinterpret_cast<const uint4*>(slots + s);
            const uint4 a = q[0], b = q[1];
            const uint32_t st = slot_state(b.w);
            if (st == SLOT_EMPTY) break;
            if (st == SLOT_LIVE && ((uint64_t)a.x | ((uint64_t)a.y << 32)) == n0 &&
                ((uint64_t)a.z | ((uint64_t)a.w << 32)) == n1 && ((uint64_t)b.x | ((uint64_t)b.y << 32)) == tcd) {
                if (b.z == act) {
                    uint32_t expected = b.w;
                    rm = __hip_atomic_compare_exchange_strong(&slots[s].meta, &expected, make_meta(SLOT_TOMB, 0),
                                                              __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
                }
                break;
            }
            s = (s + 1) & mask;
        }
    }
    live_delta(ctr, rm, true);
    if (!rm) return;
    if (B.cx16) B.cx16[s] = make_uint4(0, 0, 0, CX_TOMB);
    if (B.cx8) B.cx8[s] = CX8_HOLE;
}

static __global__ void __launch_bounds__(BLOCK) k_unreg_commit_cx(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                           Slot* slots, DevCounters* ctr,
                                                           uint8_t* __restrict__ out_removed, CxBuild B) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool rm = i < n && unreg_commit_item(i, slot_of, slots, ctr, out_removed);
    live_delta(ctr, rm, true);
    if (!rm) return;
    const uint32_t s = slot_of[i];
    if (B.cx16) B.cx16[s] = make_uint4(0, 0, 0, CX_TOMB);       // the tombstone (cx_project of a non-live slot)
    if (B.cx8) B.cx8[s] = CX8_HOLE;
}

}  // namespace gd
