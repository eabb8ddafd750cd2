// gd_cache.h -- gfx950 device code for the non-owner directory cache:
// AdaptiveGrainDirectoryCache over LRU<GrainId, entry>
// (src/Orleans.Runtime/GrainDirectory/AdaptiveGrainDirectoryCache.cs, src/Orleans.Core/Utils/LRU.cs)
// consulted by LocalGrainDirectory.LocalLookup for grains this silo does not own
// (LocalGrainDirectory.cs:797-850).
//
// The LRU is exact.  Every entry carries the reference's Generation: a hit sets it to
// ++nextGeneration (LRU.cs:119-146), an add gives it ++nextGeneration after AdjustSize
// (:71-76), and AdjustSize evicts the entry of the lowest live generation (its generationToFree
// sweep, :165-182, always lands on the minimum: every live generation is above it).  A batch of
// lookups hands out generations in batch order: an inclusive scan of the hit flags gives hit k
// generation next_gen + k, applied with atomicMax so the last hit of a key wins, then next_gen
// advances by the hit count -- all on the stream, no host round trip.  Adds are the slow path
// (they follow a remote lookup, LocalGrainDirectory.cs:920): the host simulates AdjustSize
// over the batch against the device's lowest generations and applies the outcome with the
// kernels below.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"
#include "gd_keyext.h"

namespace gd {

// 64-B slot: one DRAM atom per probe (the 32-B directory slot costs the same 64 B).
struct alignas(64) CacheSlot {
    uint64_t n0, n1, tcd;        // GrainId key
    uint32_t act;                // activation index
    uint32_t meta;               // (state << 16) | silo
    unsigned long long gen;      // LRU generation
    int32_t version;             // ETag (AdaptiveGrainDirectoryCache.cs:20)
    uint32_t xuh;                // KeyExt entry: uniform hash of ToByteArray() (the home slot's hash)
    uint32_t xlen1;              // 0 = a three-word key (KeyExt null included); else KeyExt length + 1
    uint32_t xoff;               // KeyExt entry: byte offset of the string in the cache heap (16-B aligned)
    uint32_t pad[2];
};
static_assert(sizeof(CacheSlot) == 64, "cache slot must be 64 bytes");

struct CacheCounters {
    unsigned long long next_gen;   // LRU.nextGeneration
    unsigned long long accesses;   // AdaptiveGrainDirectoryCache.NumAccesses
    unsigned long long hits;       // NumHits
    unsigned long long live;
    unsigned long long tomb;
    uint32_t max_probe;
    uint32_t err;                  // bit 1: table full
};

struct CacheArgs {
    const CacheSlot* slots;
    unsigned long long mask;
    const CacheCounters* ctr;
    const uint8_t* local;          // local[silo] != 0: this handle owns that silo's partition
    const uint8_t* valid;          // valid[silo] != 0: IsValidSilo
    uint32_t n_silos;              // entries of local / valid
    const uint8_t* heap;           // KeyExt strings of the cache's KeyExt entries
};

// The hash an entry is homed by: the three-word uniform hash, or the KeyExt one.
__device__ __forceinline__ uint32_t cache_slot_hash(const CacheSlot& c) {
    return c.xlen1 ? c.xuh : uniform_hash(c.n0, c.n1, c.tcd);
}

__device__ __forceinline__ bool cache_probe(const CacheSlot* slots, unsigned long long mask, uint32_t max_probe,
                                            uint32_t h, uint64_t n0, uint64_t n1, uint64_t tcd, uint32_t& slot,
                                            uint32_t& act, uint32_t& meta) {
    unsigned long long s = fmix32(h) & mask;
    for (uint32_t p = 0; p <= max_probe; ++p) {
        const uint4* q = reinterpret_cast<const uint4*>(slots + s);
        const uint4 a = q[0];
        const uint4 b = q[1];
        const uint32_t st = slot_state(b.w);
        if (st == SLOT_EMPTY) return false;
        const uint64_t k0 = (uint64_t)a.x | ((uint64_t)a.y << 32);
        const uint64_t k1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
        const uint64_t k2 = (uint64_t)b.x | ((uint64_t)b.y << 32);
        // a KeyExt-category key without a string (KeyExt null) never equals a KeyExt entry
        if (st == SLOT_LIVE && k0 == n0 && k1 == n1 && k2 == tcd &&
            (!is_keyext_tcd(tcd) || slots[s].xlen1 == 0)) {
            slot = (uint32_t)s;
            act = b.z;
            meta = b.w;
            return true;
        }
        s = (s + 1) & mask;
    }
    return false;
}

// The cache's KeyExt entry equal to (n0, n1, tcd, s[0..len)), len >= 0 (UniqueKey.Equals,
// UniqueKey.cs:245-251); FAST: the string is in w[] (len <= KX_FAST_BYTES).
template <bool FAST>
__device__ __forceinline__ bool cache_probe_ext(const CacheSlot* slots, unsigned long long mask, uint32_t max_probe,
                                                const uint8_t* heap, uint32_t uh, uint64_t n0, uint64_t n1,
                                                uint64_t tcd, const uint8_t* s, int32_t len,
                                                const uint32_t (&w)[KX_FAST_WORDS], uint32_t& slot, uint32_t& act,
                                                uint32_t& meta) {
    unsigned long long i = fmix32(uh) & mask;
    for (uint32_t p = 0; p <= max_probe; ++p) {
        const uint4* q = reinterpret_cast<const uint4*>(slots + i);
        const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
        const uint32_t st = slot_state(b.w);
        if (st == SLOT_EMPTY) return false;
        if (st == SLOT_LIVE && d.x == (uint32_t)len + 1u && c.w == uh &&
            ((uint64_t)a.x | ((uint64_t)a.y << 32)) == n0 && ((uint64_t)a.z | ((uint64_t)a.w << 32)) == n1 &&
            ((uint64_t)b.x | ((uint64_t)b.y << 32)) == tcd) {
            bool eq = true;
            if (len > 0) {
                if constexpr (FAST) eq = heap_equal_fast(heap, d.y, len, w);
                else eq = bytes_equal(heap + d.y, s, len);
            }
            if (eq) {
                slot = (uint32_t)i;
                act = b.z;
                meta = b.w;
                return true;
            }
        }
        i = (i + 1) & mask;
    }
    return false;
}

// KeyExt uniform hash of message i's key (JenkinsHash over ToByteArray(), UniqueKey.cs:272-336),
// the string left in w[] when it fits the registers; len = GD_KEYEXT_NULL: the three-word hash.
__device__ __forceinline__ uint32_t keyext_hash(uint64_t n0, uint64_t n1, uint64_t tcd, const uint8_t* s,
                                                int32_t len, uint32_t (&w)[KX_FAST_WORDS]) {
    if (len >= 0 && len <= KX_FAST_BYTES) {
        load_str_fast(s, len, w);
        return jenkins_keyext_fast(n0, n1, tcd, len, w);
    }
#pragma unroll
    for (int q = 0; q < KX_FAST_WORDS; ++q) w[q] = 0;
    return len < 0 ? uniform_hash(n0, n1, tcd) : jenkins_keyext(n0, n1, tcd, s, len);
}

// A KeyExt key in the cache: its KeyExt entry, or (KeyExt null) the three-word entry.
__device__ __forceinline__ bool cache_find_any(const CacheArgs& c, uint32_t max_probe, uint32_t uh, uint64_t n0,
                                               uint64_t n1, uint64_t tcd, const uint8_t* s, int32_t len,
                                               const uint32_t (&w)[KX_FAST_WORDS], uint32_t& slot, uint32_t& act,
                                               uint32_t& meta) {
    if (len < 0) return cache_probe(c.slots, c.mask, max_probe, uh, n0, n1, tcd, slot, act, meta);
    if (len <= KX_FAST_BYTES)
        return cache_probe_ext<true>(c.slots, c.mask, max_probe, c.heap, uh, n0, n1, tcd, s, len, w, slot, act, meta);
    return cache_probe_ext<false>(c.slots, c.mask, max_probe, c.heap, uh, n0, n1, tcd, s, len, w, slot, act, meta);
}

__device__ __forceinline__ bool silo_flag(const uint8_t* m, uint32_t n, uint32_t silo) {
    return silo < n && m[silo] != 0;
}

// LocalLookup over a batch: the owner's partition when this handle holds it, the cache
// otherwise.  hit[i] = 1 for a cache hit (generation update follows), cslot[i] its slot.
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_route_cached(const gd_key* __restrict__ keys, uint32_t n, RingArgs ring,
                                                        TableArgs tab, CacheArgs cache,
                                                        uint32_t* __restrict__ out_silo,
                                                        uint32_t* __restrict__ out_act,
                                                        uint8_t* __restrict__ out_status,
                                                        uint32_t* __restrict__ hit, uint32_t* __restrict__ cslot,
                                                        CacheCounters* cctr) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    __shared__ uint32_t s_acc;
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    if (threadIdx.x == 0) s_acc = 0;
    stage_ring(ring, s_pts, s_own);
    const uint32_t max_probe = tab.ctr->max_probe;
    const uint32_t cmax_probe = cache.ctr->max_probe;
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t silo = NONE32, act = NONE32, h_flag = 0, slot = NONE32;
    uint8_t status = GD_ROUTE_MISS;
    bool access = false;
    if (i < n) {
        const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
        const uint64_t n0 = kp[0], n1 = kp[1], tcd = kp[2];
        const uint32_t cat = (uint32_t)(tcd >> 56);
        if (cat == CAT_SYSTEM_TARGET) {                        // LocalGrainDirectory.cs:480-485
            silo = ring.my_silo;
            status = GD_ROUTE_SYSTEM_TARGET;
        } else if (is_membership(n0, n1, tcd)) {               // :487-503
            silo = ring.seed_silo;
            status = GD_ROUTE_MEMBERSHIP;
        } else if (cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT) {
            status = GD_ROUTE_KEYEXT;
        } else {
            const uint32_t h = uniform_hash(n0, n1, tcd);
            const uint32_t owner = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h)];
            silo = owner;
            uint32_t a, meta;
            if (silo_flag(cache.local, cache.n_silos, owner)) {     // we own the grain (:806-821)
                if (probe(tab.slots, tab.mask, max_probe, h, n0, n1, tcd, a, meta)) {
                    if (a == GD_ACT_MULTI) {
                        status = GD_ROUTE_MULTI_ACT;          // RandomPlacementDirector.cs:33-53, in C#
                    } else if (tab_silo_valid(tab, slot_silo(meta))) {   // LookUpActivations' filter (:431)
                        act = a;
                        silo = slot_silo(meta);
                        status = GD_ROUTE_OK;
                    }
                }
            } else {                                              // cache (:823-836)
                access = true;
                if (cache_probe(cache.slots, cache.mask, cmax_probe, h, n0, n1, tcd, slot, a, meta)) {
                    h_flag = 1;
                    if (silo_flag(cache.valid, cache.n_silos, slot_silo(meta))) {   // IsValidSilo (:848)
                        act = a;
                        silo = slot_silo(meta);
                        status = GD_ROUTE_OK;
                    }
                }
            }
        }
        out_silo[i] = silo;
        out_act[i] = act;
        out_status[i] = status;
        hit[i] = h_flag;
        cslot[i] = slot;
    }
    const unsigned long long acc = __ballot(access);
    if ((threadIdx.x & (WAVE - 1)) == 0 && acc) atomicAdd(&s_acc, (uint32_t)__popcll(acc));
    __syncthreads();
    if (threadIdx.x == 0 && s_acc) atomicAdd(&cctr->accesses, (unsigned long long)s_acc);
}

// LocalLookup for the messages k_route_cached left at GD_ROUTE_KEYEXT (string-keyed grains): owner
// by the KeyExt hash (CalculateTargetSilo, LocalGrainDirectory.cs:477-545); a local owner probes
// this handle's KeyExt partition (as k_route_keyext), any other owner the cache's KeyExt entries
// (AdaptiveGrainDirectoryCache.cs:93-110 with UniqueKey KeyExt equality, UniqueKey.cs:245-251).
// Writes the hit flags / slots the batch's generation scan reads, so plain and KeyExt hits take
// their generations in one batch order.
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_route_cached_keyext(const gd_key* __restrict__ keys, uint32_t n,
                                                               ExtArgs ext, RingArgs ring, KxArgs kx, CacheArgs cache,
                                                               uint32_t* __restrict__ out_silo,
                                                               uint32_t* __restrict__ out_act,
                                                               uint8_t* __restrict__ out_status,
                                                               uint32_t* __restrict__ hit,
                                                               uint32_t* __restrict__ cslot, CacheCounters* cctr) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    __shared__ uint32_t s_acc;
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    if (threadIdx.x == 0) s_acc = 0;
    stage_ring(ring, s_pts, s_own);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool access = false;
    const uint8_t* s = nullptr;
    int32_t len = 0;
    if (i < n && out_status[i] == GD_ROUTE_KEYEXT && ext_of(ext, i, s, len)) {
        const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
        const uint64_t n0 = kp[0], n1 = kp[1], tcd = kp[2];
        uint32_t w[KX_FAST_WORDS];
        const uint32_t uh = keyext_hash(n0, n1, tcd, s, len, w);
        const uint32_t owner = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, uh)];
        // (select form: the branch form lost the partition hit's activation in this compiler's
        // codegen -- status OK with act unset; cf. k_handoff_add_status)
        const bool local = silo_flag(cache.local, cache.n_silos, owner);
        uint32_t ka = NONE32, km = 0, ca = NONE32, cm = 0, slot = NONE32;
        bool kfound = false, cfound = false;
        if (local && kx.slots) {                                        // we own the grain (:806-821)
            if (len <= KX_FAST_BYTES) kfound = kx_find<true>(kx, n0, n1, tcd, s, len, uh, w, ka, km);
            else kfound = kx_find<false>(kx, n0, n1, tcd, s, len, uh, w, ka, km);
        }
        if (!local) {                                                   // cache (:823-836)
            access = true;
            cfound = cache_find_any(cache, cache.ctr->max_probe, uh, n0, n1, tcd, s, len, w, slot, ca, cm);
        }
        const bool kok = kfound && valid_silo(kx.valid, kx.n_valid, slot_silo(km));   // IsValidSilo (:431)
        const bool cok = cfound && silo_flag(cache.valid, cache.n_silos, slot_silo(cm));   // (:848)
        const uint32_t a = local ? ka : ca, m = local ? km : cm;
        const bool ok = local ? kok : cok;
        if (cfound) {
            hit[i] = 1;
            cslot[i] = slot;
        }
        const uint32_t silo = ok ? slot_silo(m) : owner, act = ok ? a : NONE32;
        const uint8_t status = ok ? (uint8_t)GD_ROUTE_OK : (uint8_t)GD_ROUTE_MISS;
        out_silo[i] = silo;
        out_act[i] = act;
        out_status[i] = status;
    }
    const unsigned long long acc = __ballot(access);
    if ((threadIdx.x & (WAVE - 1)) == 0 && acc) atomicAdd(&s_acc, (uint32_t)__popcll(acc));
    __syncthreads();
    if (threadIdx.x == 0 && s_acc) atomicAdd(&cctr->accesses, (unsigned long long)s_acc);
}

// Message i's cache entry: KeyExt keys by their string when the batch has one (ext.len != NULL),
// else by the three words.  false when the message names no entry the device can match
// (GD_KEYEXT_HOST or a range outside the bytes).
__device__ __forceinline__ bool cache_find_msg(const CacheArgs& c, const gd_key* keys, const ExtArgs& ext,
                                               uint32_t i, uint32_t& slot, uint32_t& act, uint32_t& meta) {
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    const uint32_t mp = c.ctr->max_probe;
    if (ext.len && is_keyext_tcd(tcd)) {
        const uint8_t* s;
        int32_t len;
        if (!ext_of(ext, i, s, len)) return false;
        uint32_t w[KX_FAST_WORDS];
        const uint32_t uh = keyext_hash(n0, n1, tcd, s, len, w);
        return cache_find_any(c, mp, uh, n0, n1, tcd, s, len, w, slot, act, meta);
    }
    return cache_probe(c.slots, c.mask, mp, uniform_hash(n0, n1, tcd), n0, n1, tcd, slot, act, meta);
}

// AdaptiveGrainDirectoryCache.LookUp over a batch (explicit form, no routing).
static __global__ void __launch_bounds__(BLOCK) k_cache_lookup(const gd_key* __restrict__ keys, uint32_t n, ExtArgs ext,
                                                        CacheArgs cache, gd_val* __restrict__ out_vals,
                                                        int32_t* __restrict__ out_ver, uint32_t* __restrict__ hit,
                                                        uint32_t* __restrict__ cslot) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t slot = NONE32, act, meta;
    const bool h = cache_find_msg(cache, keys, ext, i, slot, act, meta);
    out_vals[i] = h ? gd_val{act, slot_silo(meta)} : gd_val{NONE32, NONE32};
    out_ver[i] = h ? cache.slots[slot].version : 0;
    hit[i] = h ? 1u : 0u;
    cslot[i] = h ? slot : NONE32;
}

// pos = inclusive scan of the hit flags: hit k of the batch gets generation next_gen + k
// (TryGetValue's Interlocked.Increment in batch order); the last hit of a key wins.
static __global__ void __launch_bounds__(BLOCK) k_cache_touch(const uint32_t* __restrict__ cslot,
                                                       const uint32_t* __restrict__ pos, uint32_t n, CacheSlot* slots,
                                                       const CacheCounters* ctr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || cslot[i] == NONE32) return;
    atomicMax(&slots[cslot[i]].gen, ctr->next_gen + pos[i]);
}

static __global__ void k_cache_advance(const uint32_t* __restrict__ pos, uint32_t n, CacheCounters* ctr) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n) {
        ctr->next_gen += pos[n - 1];
        ctr->hits += pos[n - 1];
    }
}

static __global__ void k_cache_count_access(uint32_t n, CacheCounters* ctr) {
    if (threadIdx.x == 0 && blockIdx.x == 0) ctr->accesses += n;
}

// Slot and generation of each key (NONE32 / 0 when absent).
static __global__ void __launch_bounds__(BLOCK) k_cache_find(const gd_key* __restrict__ keys, uint32_t n, ExtArgs ext,
                                                      CacheArgs cache, uint32_t* __restrict__ slot_of,
                                                      unsigned long long* __restrict__ gen_of) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t slot = NONE32, act, meta;
    const bool h = cache_find_msg(cache, keys, ext, i, slot, act, meta);
    slot_of[i] = h ? slot : NONE32;
    gen_of[i] = h ? cache.slots[slot].gen : 0ull;
}

// Live entries with generation <= t: count, then collect (gen, slot) in any order.
static __global__ void __launch_bounds__(BLOCK) k_cache_count_le(const CacheSlot* __restrict__ slots,
                                                          unsigned long long cap, unsigned long long t,
                                                          unsigned long long* __restrict__ out) {
    __shared__ uint32_t s_c;
    if (threadIdx.x == 0) s_c = 0;
    __syncthreads();
    uint32_t c = 0;
    for (unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x; j < cap;
         j += (unsigned long long)gridDim.x * BLOCK)
        c += (slot_state(slots[j].meta) == SLOT_LIVE && slots[j].gen <= t) ? 1u : 0u;
    for (int off = WAVE / 2; off > 0; off >>= 1) c += __shfl_xor(c, off, WAVE);
    if ((threadIdx.x & (WAVE - 1)) == 0 && c) atomicAdd(&s_c, c);
    __syncthreads();
    if (threadIdx.x == 0 && s_c) atomicAdd(out, (unsigned long long)s_c);
}

static __global__ void __launch_bounds__(BLOCK) k_cache_collect_le(const CacheSlot* __restrict__ slots,
                                                            unsigned long long cap, unsigned long long t,
                                                            uint32_t* __restrict__ cursor,
                                                            unsigned long long* __restrict__ out_gen,
                                                            uint32_t* __restrict__ out_slot, uint32_t max_out) {
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= cap) return;
    if (slot_state(slots[j].meta) != SLOT_LIVE || slots[j].gen > t) return;
    const uint32_t k = atomicAdd(cursor, 1u);
    if (k < max_out) {
        out_gen[k] = slots[j].gen;
        out_slot[k] = (uint32_t)j;
    }
}

// Outcome of an add batch on existing slots: kind 0 = evict (tombstone), 1 = update in place.
struct CacheOp {
    uint32_t slot;
    uint32_t kind;
    uint32_t act;
    uint32_t silo;
    unsigned long long gen;
    int32_t version;
    uint32_t pad;
};

static __global__ void __launch_bounds__(BLOCK) k_cache_apply(const CacheOp* __restrict__ ops, uint32_t n, CacheSlot* slots,
                                                       CacheCounters* ctr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const CacheOp op = ops[i];
    CacheSlot& s = slots[op.slot];
    if (op.kind == 0) {
        s.meta = make_meta(SLOT_TOMB, 0);
        atomicAdd(&ctr->live, ~0ull);
        atomicAdd(&ctr->tomb, 1ull);
    } else {
        s.act = op.act;
        s.gen = op.gen;
        s.version = op.version;
        s.meta = make_meta(SLOT_LIVE, op.silo);
    }
}

// New entries (distinct keys, known absent): claim the first empty or tombstoned slot.  xm (may be
// NULL): per entry {KeyExt uniform hash, KeyExt length + 1 (0: three-word key), heap offset}.
static __global__ void __launch_bounds__(BLOCK) k_cache_insert(const gd_key* __restrict__ keys,
                                                        const CacheOp* __restrict__ vals,
                                                        const uint32_t* __restrict__ xm, uint32_t n, CacheSlot* slots,
                                                        unsigned long long mask, CacheCounters* ctr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    const uint32_t xuh = xm ? xm[3 * i] : 0u, xlen1 = xm ? xm[3 * i + 1] : 0u, xoff = xm ? xm[3 * i + 2] : 0u;
    unsigned long long s = fmix32(xlen1 ? xuh : uniform_hash(n0, n1, tcd)) & mask;
    for (uint32_t dist = 0; dist <= mask; ++dist) {
        uint32_t* mp = &slots[s].meta;
        uint32_t cur = __hip_atomic_load(mp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t st = slot_state(cur);
        if ((st == SLOT_EMPTY || st == SLOT_TOMB) &&
            __hip_atomic_compare_exchange_strong(mp, &cur, make_meta(SLOT_CLAIMED, 0), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            CacheSlot& d = slots[s];
            d.n0 = n0;
            d.n1 = n1;
            d.tcd = tcd;
            d.act = vals[i].act;
            d.gen = vals[i].gen;
            d.version = vals[i].version;
            d.xuh = xuh;
            d.xlen1 = xlen1;
            d.xoff = xoff;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_store(mp, make_meta(SLOT_LIVE, vals[i].silo), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicMax(&ctr->max_probe, dist);
            atomicAdd(&ctr->live, 1ull);
            if (st == SLOT_TOMB) atomicAdd(&ctr->tomb, ~0ull);
            return;
        }
        if (st == SLOT_EMPTY || st == SLOT_TOMB) continue;      // lost the race for this slot: re-read it
        s = (s + 1) & mask;
    }
    atomicOr(&ctr->err, 2u);
}

// Live entries into a fresh table (tombstone compaction / growth).
static __global__ void __launch_bounds__(BLOCK) k_cache_rehash(const CacheSlot* __restrict__ old_slots,
                                                        unsigned long long old_cap, CacheSlot* slots,
                                                        unsigned long long mask, CacheCounters* ctr) {
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (j >= old_cap) return;
    const CacheSlot sl = old_slots[j];
    if (slot_state(sl.meta) != SLOT_LIVE) return;
    unsigned long long s = fmix32(cache_slot_hash(sl)) & mask;
    for (uint32_t dist = 0; dist <= mask; ++dist) {
        uint32_t expected = make_meta(SLOT_EMPTY, 0);
        if (__hip_atomic_compare_exchange_strong(&slots[s].meta, &expected, make_meta(SLOT_CLAIMED, 0),
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            CacheSlot d = sl;
            d.meta = make_meta(SLOT_CLAIMED, 0);
            slots[s] = d;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_store(&slots[s].meta, sl.meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicMax(&ctr->max_probe, dist);
            atomicAdd(&ctr->live, 1ull);
            return;
        }
        s = (s + 1) & mask;
    }
    atomicOr(&ctr->err, 2u);
}

// Live-slot flags for the KeyValues dump (slot order).
static __global__ void __launch_bounds__(BLOCK) k_cache_live_flag(const CacheSlot* __restrict__ slots, uint32_t cap,
                                                           uint32_t* __restrict__ flag) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j < cap) flag[j] = slot_state(slots[j].meta) == SLOT_LIVE ? 1u : 0u;
}

static __global__ void __launch_bounds__(BLOCK) k_cache_dump(const CacheSlot* __restrict__ slots, uint32_t cap,
                                                      const uint32_t* __restrict__ flag,
                                                      const uint32_t* __restrict__ pos, gd_key* __restrict__ keys,
                                                      gd_val* __restrict__ vals, int32_t* __restrict__ vers,
                                                      unsigned long long* __restrict__ gens,
                                                      uint32_t* __restrict__ xlen1, uint32_t* __restrict__ xoff) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= cap || !flag[j]) return;
    const uint32_t k = pos[j] - 1;
    const CacheSlot s = slots[j];
    keys[k] = gd_key{s.n0, s.n1, s.tcd};
    vals[k] = gd_val{s.act, slot_silo(s.meta)};
    vers[k] = s.version;
    gens[k] = s.gen;
    if (xlen1) {
        xlen1[k] = s.xlen1;
        xoff[k] = s.xoff;
    }
}

// Heap compaction: each live KeyExt entry's string size rounded to 16 B, then (after an
// inclusive scan of the sizes) its string moved to the new heap and its offset rewritten.
static __global__ void __launch_bounds__(BLOCK) k_cx_sizes(const CacheSlot* __restrict__ slots, uint32_t cap,
                                                    uint32_t* __restrict__ size) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= cap) return;
    const CacheSlot& s = slots[j];
    size[j] = (slot_state(s.meta) == SLOT_LIVE && s.xlen1 > 1) ? ((s.xlen1 - 1u + 15u) & ~15u) : 0u;
}

static __global__ void __launch_bounds__(BLOCK) k_cx_move(CacheSlot* slots, uint32_t cap, const uint32_t* __restrict__ size,
                                                   const uint32_t* __restrict__ pos, const uint8_t* __restrict__ old_heap,
                                                   uint8_t* __restrict__ new_heap) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= cap || size[j] == 0) return;
    const uint32_t to = pos[j] - size[j];
    const uint4* src = reinterpret_cast<const uint4*>(old_heap + slots[j].xoff);
    uint4* dst = reinterpret_cast<uint4*>(new_heap + to);
    for (uint32_t q = 0; q < size[j] / 16; ++q) dst[q] = src[q];
    slots[j].xoff = to;
}

}  // namespace gd
