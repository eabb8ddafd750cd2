// gd_dirops.h -- gfx950 device code for the directory operations around a membership change
// (SURVEY 8 f4): IsValidSilo, VersionTag, silo removal and the handoff merge.
//
//   k_dir_lookup_tagged   LookUpActivations with its VersionTag and the IsValidSilo filter
//                         (GrainDirectoryPartition.cs:385-441)
//   k_dir_remove_silos    LocalGrainDirectory.AdjustLocalDirectory (LocalGrainDirectory.cs:351-361):
//                         drop every entry whose activation lives on a removed silo
//   k_cache_adjust        LocalGrainDirectory.AdjustLocalCache (:371-385): drop cached entries that
//                         point at a removed silo or whose grain this handle now owns
//   k_merge_apply         GrainDirectoryPartition.Merge (:497-522) with GrainInfo.Merge's
//                         single-instance rule (:139-179): the lowest ActivationId stays, the others
//                         are reported for Catalog.DeleteActivations
// Integer table walks and random slot updates: HBM-bound, no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_cache.h"
#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

// found: 0 = no entry (AddressesAndTag default: no list, VersionTag 0), 1 = entry with a valid
// address, 2 = entry whose activation's silo is not valid (the filtered list is empty, the tag
// is still returned: GrainDirectoryPartition.cs:401,425-431).
static __global__ void __launch_bounds__(BLOCK) k_dir_lookup_tagged(const gd_key* __restrict__ keys, uint32_t n,
                                                             TableArgs tab, const uint32_t* __restrict__ vtag,
                                                             gd_val* __restrict__ out_vals,
                                                             int32_t* __restrict__ out_tags,
                                                             uint8_t* __restrict__ out_found) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    const uint32_t h = uniform_hash(n0, n1, tcd);
    unsigned long long s = home_slot(h, tab.mask);
    const uint32_t max_probe = tab.ctr->max_probe;
    gd_val v{NONE32, NONE32};
    int32_t tag = 0;
    uint8_t f = 0;
    for (uint32_t p = 0; p <= max_probe; ++p) {
        const Slot sl = tab.slots[s];
        const uint32_t st = slot_state(sl.meta);
        if (st == SLOT_EMPTY) break;
        if (st == SLOT_LIVE && sl.n0 == n0 && sl.n1 == n1 && sl.tcd == tcd) {
            tag = (int32_t)(vtag[s] & 0x7FFFFFFFu);
            if (sl.act == GD_ACT_MULTI || tab_silo_valid(tab, slot_silo(sl.meta))) {
                v = gd_val{sl.act, slot_silo(sl.meta)};
                f = 1;
            } else {
                f = 2;
            }
            break;
        }
        s = (s + 1) & tab.mask;
    }
    out_vals[i] = v;
    out_tags[i] = tag;
    out_found[i] = f;
}

// Silo-set membership as a bitset over silo indices (65,536 bits max).
__device__ __forceinline__ bool in_set(const uint32_t* set, uint32_t silo) {
    return (set[silo >> 5] >> (silo & 31u)) & 1u;
}

// AdjustLocalDirectory: RemoveActivation(grain, act, Force) for every instance on a removed
// silo; a single-activation grain loses its only instance and so the grain.  Multi-activation
// entries (GD_ACT_MULTI) keep no per-instance silos here: they are counted, left to the host.
static __global__ void __launch_bounds__(BLOCK) k_dir_remove_silos(Slot* slots, unsigned long long cap,
                                                            const uint32_t* __restrict__ set, DevCounters* ctr,
                                                            unsigned long long* __restrict__ counts) {
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    bool rm = false, multi = false;
    if (j < cap) {
        const uint32_t meta = slots[j].meta;
        if (slot_state(meta) == SLOT_LIVE && in_set(set, slot_silo(meta))) {
            if (slots[j].act == GD_ACT_MULTI) {
                multi = true;
            } else {
                slots[j].meta = make_meta(SLOT_TOMB, 0);
                rm = true;
            }
        }
    }
    const unsigned long long b_rm = __ballot(rm), b_mu = __ballot(multi);
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        if (b_rm) {
            const unsigned long long c = (unsigned long long)__popcll(b_rm);
            atomicAdd(&ctr->live, 0ull - c);
            atomicAdd(&ctr->tomb, c);
            atomicAdd(&counts[0], c);
        }
        if (b_mu) atomicAdd(&counts[1], (unsigned long long)__popcll(b_mu));
    }
}

// AdjustLocalCache over the cache table, under the ring installed after the removal: an entry
// goes if its grain is now owned by a local silo (CalculateTargetSilo == MyAddress) or its
// activation lives on a removed silo (RemoveActivations with t.Item1 == removedSilo).  Removal is
// LRU.RemoveKey: no generation moves.
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_cache_adjust(CacheSlot* slots, unsigned long long cap, RingArgs ring,
                                                        const uint8_t* __restrict__ local, uint32_t n_local,
                                                        const uint32_t* __restrict__ set, CacheCounters* ctr,
                                                        unsigned long long* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    bool rm = false;
    if (j < cap) {
        const uint32_t meta = slots[j].meta;
        if (slot_state(meta) == SLOT_LIVE) {
            const CacheSlot& c = slots[j];
            const uint32_t owner = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, cache_slot_hash(c))];
            rm = (owner < n_local && local[owner]) || in_set(set, slot_silo(meta));
            if (rm) slots[j].meta = make_meta(SLOT_TOMB, 0);
        }
    }
    const unsigned long long b = __ballot(rm);
    if ((threadIdx.x & (WAVE - 1)) == 0 && b) {
        const unsigned long long c = (unsigned long long)__popcll(b);
        atomicAdd(&ctr->live, 0ull - c);
        atomicAdd(&ctr->tomb, c);
        atomicAdd(&counts[2], c);
    }
}

// A merge batch is a partition (a Dictionary): one item per grain.  Items sharing a slot are
// flagged (err bit 8).
static __global__ void __launch_bounds__(BLOCK) k_dup_mark(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                    uint32_t* __restrict__ last, DevCounters* ctr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || slot_of[i] >= SLOT_RETRY) return;
    if (atomicAdd(&last[slot_of[i]], 1u) != 0) atomicOr(&ctr->err, 8u);
}

// A rejected merge batch leaves no half-made entry: its new claims become tombstones (probe chains
// through them stay intact).
static __global__ void __launch_bounds__(BLOCK) k_reg_abort(const uint32_t* __restrict__ slot_of,
                                                     const uint8_t* __restrict__ is_new, uint32_t n, Slot* slots,
                                                     DevCounters* ctr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || !is_new[i] || slot_of[i] >= SLOT_RETRY) return;
    // PENDING carries its claim launch's tag (claim_tag) in the silo field
    uint32_t* mp = &slots[slot_of[i]].meta;
    uint32_t expected = __hip_atomic_load(mp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (slot_state(expected) == SLOT_PENDING &&
        __hip_atomic_compare_exchange_strong(mp, &expected, make_meta(SLOT_TOMB, 0), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicAdd(&ctr->tomb, 1ull);
}

// gd_activation_ids_set: ids[acts[i]] = the i-th ActivationId (batch order; the last of a repeated
// index wins only if the host repeats it -- it should not).
static __global__ void __launch_bounds__(BLOCK) k_scatter_ids(const uint32_t* __restrict__ acts,
                                                       const gd_key* __restrict__ in, uint32_t n,
                                                       gd_key* __restrict__ ids) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) ids[acts[i]] = in[i];
}

// UniqueKey.CompareTo (UniqueKey.cs:255-265): TypeCodeData, then N0, then N1 (ActivationIds carry
// no KeyExt).  < 0 when a sorts first.
__device__ __forceinline__ int key_cmp(const gd_key& a, const gd_key& b) {
    if (a.type_code_data != b.type_code_data) return a.type_code_data < b.type_code_data ? -1 : 1;
    if (a.n0 != b.n0) return a.n0 < b.n0 ? -1 : 1;
    if (a.n1 != b.n1) return a.n1 < b.n1 ? -1 : 1;
    return 0;
}

// GD_MERGE_* statuses (include/graindispatch.h)
constexpr uint8_t MERGE_INSERTED = 0, MERGE_KEPT = 1, MERGE_SAME = 2, MERGE_DROPPED = 3, MERGE_HOST = 4,
                  MERGE_UNION = 5;
constexpr uint32_t MERGE_TAG_MULTI = 0x80000000u;   // GD_MERGE_TAG_MULTI_INSTANCE

// One item per grain (k_dup_mark); slot_of / is_new from k_reg_claim.  out_dropped[i] = the
// activation Catalog.DeleteActivations gets (KEPT: the displaced entry, DROPPED: the incoming
// one), else none.  ids[act] = the
// ActivationId of host activation index act (gd_activation_ids_set); an index without one sets
// err bit 16.  in_tags: the incoming entries' VersionTags (NULL: a new tag); bit 31 (MERGE_TAG_MULTI)
// marks an incoming GrainInfo whose SingleInstance is false (an AddActivation grain with one
// instance), which partitionData.Add keeps as it is (:517-520).
static __global__ void __launch_bounds__(BLOCK) k_merge_apply(const gd_key* __restrict__ keys,
                                                       const gd_val* __restrict__ vals,
                                                       const int32_t* __restrict__ in_tags, uint32_t n,
                                                       const uint32_t* __restrict__ slot_of,
                                                       const uint8_t* __restrict__ is_new, Slot* slots,
                                                       uint32_t* __restrict__ vtag, DevCounters* ctr,
                                                       const gd_key* __restrict__ ids, unsigned long long n_ids,
                                                       uint32_t op, uint8_t* __restrict__ out_status,
                                                       gd_val* __restrict__ out_dropped) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    const gd_val in = vals[i];
    gd_val dropped{NONE32, NONE32};
    uint8_t st = MERGE_HOST;
    if (s < SLOT_RETRY) {
        Slot& sl = slots[s];
        const uint32_t h = uniform_hash(keys[i].n0, keys[i].n1, keys[i].type_code_data);
        if (is_new[i]) {                              // partitionData.Add(pair.Key, pair.Value) (:509-512)
            sl.act = in.act;
            sl.meta = make_meta(SLOT_LIVE, in.silo);
            const bool in_multi = in_tags && ((uint32_t)in_tags[i] & MERGE_TAG_MULTI);
            const uint32_t single = (in.act == GD_ACT_MULTI || in_multi) ? 0u : VTAG_SINGLE;
            vtag[s] = single | (in_tags ? ((uint32_t)in_tags[i] & 0x7FFFFFFFu) : version_tag(op, h));
            atomicAdd(&ctr->live, 1ull);
            st = MERGE_INSERTED;
        } else {
            const uint32_t cur = sl.act;
            if (cur == GD_ACT_MULTI || in.act == GD_ACT_MULTI) {
                st = MERGE_HOST;                      // instance lists are unioned by C# (GrainInfo.Merge :141-152)
            } else if (!(vtag[s] & VTAG_SINGLE)) {
                // a multi-instance grain (AddActivation) holding one instance: Merge unions the lists
                // (:141-152) and keeps both -- no lowest-id rule, SingleInstance is false (:159)
                if (cur == in.act || (cur < n_ids && in.act < n_ids && key_cmp(ids[in.act], ids[cur]) == 0)) {
                    st = MERGE_SAME;                  // Instances.ContainsKey -> not modified
                } else {
                    sl.act = GD_ACT_MULTI;            // two instances now: routes answer MULTI_ACT
                    vtag[s] = version_tag(op, h);     // modified -> VersionTag = rand.Next() (:154-157)
                    st = MERGE_UNION;
                }
            } else if (cur == in.act) {
                st = MERGE_SAME;                      // Instances.ContainsKey -> continue; not modified (:146)
            } else if (cur >= n_ids || in.act >= n_ids) {
                atomicOr(&ctr->err, 16u);
                st = MERGE_HOST;
            } else if (key_cmp(ids[in.act], ids[cur]) == 0) {
                st = MERGE_SAME;                      // the same ActivationId under another host index
            } else {
                // modified: VersionTag = rand.Next() (:154-157), then keep the lowest ActivationId (:159-176)
                const bool in_wins = key_cmp(ids[in.act], ids[cur]) < 0;
                if (in_wins) {
                    dropped = gd_val{cur, slot_silo(sl.meta)};
                    sl.act = in.act;
                    sl.meta = make_meta(SLOT_LIVE, in.silo);
                    st = MERGE_KEPT;
                } else {
                    dropped = in;
                    st = MERGE_DROPPED;
                }
                vtag[s] = VTAG_SINGLE | version_tag(op, h);
            }
        }
    }
    out_status[i] = st;
    if (out_dropped) out_dropped[i] = dropped;
}

// ---- the multi-rank handoff (gd_dir_handoff_multi) -----------------------------------------------
// Split entries with what travels: the ActivationId of their activation index (ids[act]; none for a
// multi-activation entry) and their VersionTag in the public merge form (bit 31 = not SingleInstance).
// `flag` / `pos` from k_split_mark + scan, as k_split_emit; move = tombstone the slot.
static __global__ void __launch_bounds__(BLOCK) k_split_emit_tagged(Slot* __restrict__ slots, unsigned long long cap,
                                                             const uint32_t* __restrict__ flag,
                                                             const uint32_t* __restrict__ pos, int move,
                                                             const uint32_t* __restrict__ vtag,
                                                             const gd_key* __restrict__ ids, unsigned long long n_ids,
                                                             gd_key* __restrict__ out_keys, gd_key* __restrict__ out_ids,
                                                             uint32_t* __restrict__ out_silo,
                                                             uint32_t* __restrict__ out_tag, DevCounters* ctr) {
    const unsigned long long i = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= cap || !flag[i]) return;
    const Slot sl = slots[i];
    const uint32_t p = pos[i];
    out_keys[p] = gd_key{sl.n0, sl.n1, sl.tcd};
    gd_key id{0, 0, 0};
    if (sl.act != GD_ACT_MULTI) {
        if (sl.act < n_ids) id = ids[sl.act];
        else atomicOr(&ctr->err, 16u);
    }
    out_ids[p] = id;
    out_silo[p] = sl.act == GD_ACT_MULTI ? (slot_silo(sl.meta) | 0x80000000u) : slot_silo(sl.meta);
    const uint32_t t = vtag[i];
    out_tag[p] = (t & 0x7FFFFFFFu) | ((t & VTAG_SINGLE) ? 0u : MERGE_TAG_MULTI);
    if (move) {
        slots[i].meta = make_meta(SLOT_TOMB, 0);
        atomicAdd(&ctr->live, ~0ull);
        atomicAdd(&ctr->tomb, 1ull);
    }
}

// Partition order: the split's fields by the positions k_shard_scatter left (send_idx).
static __global__ void __launch_bounds__(BLOCK) k_gather_handoff(const uint32_t* __restrict__ idx, uint32_t n,
                                                          const gd_key* __restrict__ ids,
                                                          const uint32_t* __restrict__ silo,
                                                          const uint32_t* __restrict__ tag,
                                                          gd_key* __restrict__ o_ids, uint32_t* __restrict__ o_silo,
                                                          uint32_t* __restrict__ o_tag) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = idx[i];
    o_ids[i] = ids[j];
    o_silo[i] = silo[j];
    o_tag[i] = tag[j];
}

// Received entries take the receiver's activation indices act_base + j (their ActivationIds are
// appended to its index -> ActivationId map); multi-activation entries stay GD_ACT_MULTI.
static __global__ void __launch_bounds__(BLOCK) k_handoff_vals(const gd_key* __restrict__ rids,
                                                        const uint32_t* __restrict__ rsilo, uint32_t m,
                                                        uint32_t act_base, gd_key* __restrict__ ids,
                                                        gd_val* __restrict__ vals, uint32_t* __restrict__ acts) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m) return;
    const uint32_t s = rsilo[j];
    const bool multi = s & 0x80000000u;
    const uint32_t a = multi ? GD_ACT_MULTI : act_base + j;
    vals[j] = gd_val{a, s & 0xFFFFu};
    acts[j] = a;
    if (!multi) ids[act_base + j] = rids[j];
}

// ProcessSiloAddEvent's RegisterMany(singleActivation: true) on the receiver (first registration
// wins, AddSingleActivation :304-326): INSERTED, SAME (the same ActivationId was there), DROPPED
// (another activation holds the grain: the incoming one is not registered; dropped = the holder),
// HOST (a multi-activation entry: C# unions its instances).
static __global__ void __launch_bounds__(BLOCK) k_handoff_add_status(const gd_val* __restrict__ in,
                                                              const gd_val* __restrict__ got,
                                                              const uint8_t* __restrict__ ins, uint32_t m,
                                                              const gd_key* __restrict__ ids,
                                                              unsigned long long n_ids, uint8_t* __restrict__ status,
                                                              gd_val* __restrict__ dropped) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m) return;
    const uint32_t v_act = in[j].act, g_act = got[j].act, g_silo = got[j].silo;
    uint8_t st;
    uint32_t d_act = NONE32, d_silo = NONE32;
    // (written as a select: an if / else-if chain assigning the struct in two branches lost the silo
    // half of `got` on this compiler -- the ISA reused its register for the id comparison)
    if (v_act == GD_ACT_MULTI || g_act == GD_ACT_MULTI) {
        st = MERGE_HOST;
    } else if (ins[j]) {
        st = MERGE_INSERTED;
    } else if (g_act == NONE32) {
        st = MERGE_DROPPED;                          // refused: the silo is not valid (IsValidSilo)
    } else {
        bool same = false;
        if (g_act < n_ids && v_act < n_ids) same = key_cmp(ids[g_act], ids[v_act]) == 0;
        st = same ? MERGE_SAME : MERGE_DROPPED;
        d_act = same ? NONE32 : g_act;
        d_silo = same ? NONE32 : g_silo;
    }
    status[j] = st;
    dropped[j] = gd_val{d_act, d_silo};
}

}  // namespace gd
