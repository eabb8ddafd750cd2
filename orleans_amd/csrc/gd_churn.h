// gd_churn.h -- gfx950 device code for SURVEY 8 f4: directory split on a membership change.
//
// GrainDirectoryPartition.Split(predicate, modifyOrigin) (GrainDirectoryPartition.cs:532-570)
// with the predicate GrainDirectoryHandoffManager.ProcessSiloAddEvent uses
// (GrainDirectoryHandoffManager.cs:212-218): "CalculateTargetSilo(grain) is not me", where "me"
// is the set of silos whose partitions this handle holds.  The owner is computed under the
// installed ring exactly as k_route computes it (LocalGrainDirectory.cs:477-545).  Entries are
// emitted in slot order (a scan of per-slot flags), so the output is deterministic.  The receiving
// side of a join is what ProcessSiloAddEvent sends the successor: RegisterMany(split,
// singleActivation: true) (GrainDirectoryHandoffManager.cs:229 -> RemoteGrainDirectory.cs:31-43 ->
// RegisterAsync -> AddSingleActivation), i.e. a batched gd_dir_register where the first
// registration wins and the existing address is reported.  GrainDirectoryPartition.Merge
// (:497-522, the lowest-ActivationId rule of GrainInfo.Merge :139-179) is the silo-REMOVAL path
// (ProcessSiloRemoveEvent, GrainDirectoryHandoffManager.cs:125-158): gd_dir_merge, gd_dirops.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

// CalculateTargetSilo for a stored key; NONE32 when the owner needs the KeyExt string.
template <int MODE>
__device__ __forceinline__ uint32_t key_owner(uint64_t n0, uint64_t n1, uint64_t tcd, const uint32_t* s_pts,
                                              const uint32_t* s_own, const RingArgs& ring) {
    const uint32_t cat = (uint32_t)(tcd >> 56);
    if (cat == CAT_SYSTEM_TARGET) return ring.my_silo;
    if (is_membership(n0, n1, tcd)) return ring.seed_silo;
    if (cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT) return NONE32;
    return s_own[ring_position<MODE>(s_pts, ring.n, ring.top, uniform_hash(n0, n1, tcd))];
}

// flag[s] = 1 for a live slot whose owner is known and not kept here (keep[owner] == 0 or owner
// outside keep[]).
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_split_mark(const Slot* __restrict__ slots, unsigned long long cap,
                                                      RingArgs ring, const uint8_t* __restrict__ keep,
                                                      uint32_t n_keep, uint32_t* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const unsigned long long i = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= cap) return;
    const Slot sl = slots[i];
    uint32_t f = 0;
    if (slot_state(sl.meta) == SLOT_LIVE) {
        const uint32_t o = key_owner<MODE>(sl.n0, sl.n1, sl.tcd, s_pts, s_own, ring);
        f = o != NONE32 && (o >= n_keep || keep[o] == 0);
    }
    flag[i] = f;
}

// Emit flagged slots at their scanned positions; with `move`, tombstone them (the reference's
// RemoveGrain after RegisterMany, GrainDirectoryHandoffManager.cs:228-232).
static __global__ void __launch_bounds__(BLOCK) k_split_emit(Slot* __restrict__ slots, unsigned long long cap,
                                                      const uint32_t* __restrict__ flag,
                                                      const uint32_t* __restrict__ pos, int move,
                                                      gd_key* __restrict__ out_keys, gd_val* __restrict__ out_vals,
                                                      DevCounters* ctr) {
    const unsigned long long i = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= cap || !flag[i]) return;
    const Slot sl = slots[i];
    const uint32_t p = pos[i];
    out_keys[p] = gd_key{sl.n0, sl.n1, sl.tcd};
    out_vals[p] = gd_val{sl.act, slot_silo(sl.meta)};
    if (move) {
        slots[i].meta = make_meta(SLOT_TOMB, 0);
        atomicAdd(&ctr->live, ~0ull);
        atomicAdd(&ctr->tomb, 1ull);
    }
}

}  // namespace gd
