// gd_kernels.h -- gfx950 device code of libgraindispatch.
//
// Hot path (per message, all integer, HBM-bound, no MFMA):
//   K0+K1+K2  k_route        Jenkins hash of the 24-B GrainId (JenkinsHash.cs:85-105),
//                            ring search over an LDS-staged snapshot
//                            (LocalGrainDirectory.cs:477-545 / ConsistentRingProvider.cs:322-372 /
//                            VirtualBucketsRingProvider.cs:257-293), linear-probe of the
//                            open-addressing directory (GrainDirectoryPartition.cs:385-441).
//   K3        k_radix_*      stable LSD partition of message indices by activation
//                            (ActivationData.cs:566-606 per-activation FIFO), reduce-then-scan.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"

namespace gd {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;               // 4 waves
constexpr int RADIX_ITEMS = 16;          // items per thread in a radix tile
constexpr int RADIX_TILE = BLOCK * RADIX_ITEMS;   // 4096 messages per tile
constexpr int SCAN_ITEMS = 4;     // 1024-entry scan tiles: enough blocks to fill the chip
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;

struct DevCounters {
    uint32_t max_probe;     // largest probe distance of any entry placed so far
    uint32_t err;           // bit 1: table full
    uint32_t retry;         // items k_reg_claim deferred to a relaunch
    uint32_t pad;
    unsigned long long live;
    unsigned long long tomb;
};
// Striped deltas of live / tomb behind the counters (one allocation of CTR_BYTES): the directory batches'
// kernels add a wave's (or workgroup's) count into stripe blockIdx % CTR_STRIPES, 256 B apart, instead of
// into DevCounters itself -- device-scope atomics on one address from every XCD serialise (cfg 3's 1M-item
// batches: 1.6 of their 2.0 ms a churn step).  k_ctr_fold adds the stripes into live / tomb (and zeroes
// them) before every read-back (pull_counters).
constexpr uint32_t CTR_STRIPES = 64;
constexpr uint32_t CTR_STRIPE_U64 = 32;       // 256 B a stripe: {live delta, tomb delta, unused}
constexpr size_t CTR_HDR = 256;
constexpr size_t CTR_BYTES = CTR_HDR + (size_t)CTR_STRIPES * CTR_STRIPE_U64 * 8;
static_assert(sizeof(DevCounters) <= CTR_HDR, "counters header");
__device__ __forceinline__ unsigned long long* ctr_stripe(DevCounters* ctr) {
    return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ctr) + CTR_HDR) +
           (size_t)(blockIdx.x % CTR_STRIPES) * CTR_STRIPE_U64;
}
static __global__ void __launch_bounds__(64) k_ctr_fold(DevCounters* ctr) {
    unsigned long long* s = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ctr) + CTR_HDR) +
                            (size_t)threadIdx.x * CTR_STRIPE_U64;
    unsigned long long l = 0, t = 0;
    if (threadIdx.x < CTR_STRIPES) {
        l = s[0];
        t = s[1];
        s[0] = 0;
        s[1] = 0;
    }
    for (int off = 32; off > 0; off >>= 1) {
        l += __shfl_xor(l, off, 64);
        t += __shfl_xor(t, off, 64);
    }
    if (threadIdx.x == 0) {
        ctr->live += l;
        ctr->tomb += t;
    }
}

// ------------------------------------------------------------------ identity
__device__ __forceinline__ void jmix(uint32_t& a, uint32_t& b, uint32_t& c) {
    a -= b; a -= c; a ^= (c >> 13);
    b -= c; b -= a; b ^= (a << 8);
    c -= a; c -= b; c ^= (b >> 13);
    a -= b; a -= c; a ^= (c >> 12);
    b -= c; b -= a; b ^= (a << 16);
    c -= a; c -= b; c ^= (b >> 5);
    a -= b; a -= c; a ^= (c >> 3);
    b -= c; b -= a; b ^= (a << 10);
    c -= a; c -= b; c ^= (b >> 15);
}

// UniqueKey.GetUniformHashCode = JenkinsHash.ComputeHash(TypeCodeData, N0, N1)
// (UniqueKey.cs:285; JenkinsHash.cs:85-105).
__device__ __forceinline__ uint32_t uniform_hash(uint64_t n0, uint64_t n1, uint64_t tcd) {
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    a += (uint32_t)tcd;
    b += (uint32_t)(tcd >> 32);
    c += (uint32_t)n0;
    jmix(a, b, c);
    a += (uint32_t)(n0 >> 32);
    b += (uint32_t)n1;
    c += (uint32_t)(n1 >> 32);
    jmix(a, b, c);
    c += 24;
    jmix(a, b, c);
    return c;
}

// ------------------------------------------------------------------ ring
// Count of the prefix of the ring satisfying the mode's monotone predicate,
// by a branch-free power-of-two search over the LDS copy.
template <int MODE>
__device__ __forceinline__ bool ring_pred(uint32_t p, uint32_t h) {
    if constexpr (MODE == GD_RING_DIRECTORY) {
        // IsSiloNextInTheRing: siloHash <= (int)grainHash (LocalGrainDirectory.cs:1141-1144)
        return (int32_t)p <= (int32_t)h;
    } else if constexpr (MODE == GD_RING_CONSISTENT) {
        // complement of (long)siloHash >= (long)key (ConsistentRingProvider.cs:369-372)
        return (int32_t)p < 0 || p < h;
    } else {
        // complement of point >= key, uint (VirtualBucketsRingProvider.cs:276)
        return p < h;
    }
}

template <int MODE>
__device__ __forceinline__ uint32_t ring_position(const uint32_t* pts, uint32_t n, uint32_t top, uint32_t h) {
    uint32_t cnt = 0;
    for (uint32_t step = top; step > 0; step >>= 1) {
        const uint32_t c = cnt + step;
        if (c <= n && ring_pred<MODE>(pts[c - 1], h)) cnt = c;
    }
    if constexpr (MODE == GD_RING_DIRECTORY) {
        // scan from the end for the first match; none -> last silo (:521-538)
        return cnt == 0 ? n - 1 : cnt - 1;
    } else {
        // scan from the start for the first match; none -> first (:341-352 / :279-289)
        return cnt == n ? 0 : cnt;
    }
}

struct RingArgs {
    const uint32_t* pts;
    const uint32_t* own;
    uint32_t n;
    uint32_t top;       // highest power of two <= n
    uint32_t my_silo;
    uint32_t seed_silo;
};

struct TableArgs {
    const Slot* slots;
    unsigned long long mask;
    const DevCounters* ctr;
    const uint32_t* valid;     // IsValidSilo bitset over silo indices [0, n_valid) (gd_dir_set_valid_silos)
    uint32_t n_valid;          // 0: every silo valid
};

// GrainDirectoryPartition.IsValidSilo (GrainDirectoryPartition.cs:242-245): silos outside the
// configured range count as valid.
__device__ __forceinline__ bool valid_silo(const uint32_t* valid, uint32_t n_valid, uint32_t silo) {
    return n_valid == 0 || silo >= n_valid || ((valid[silo >> 5] >> (silo & 31u)) & 1u);
}
__device__ __forceinline__ bool tab_silo_valid(const TableArgs& t, uint32_t silo) {
    return valid_silo(t.valid, t.n_valid, silo);
}

// VersionTag side array (one u32 per table slot): bits 0..30 the tag (the reference draws
// rand.Next() on every change, GrainDirectoryPartition.cs:106,120,135,154; here a deterministic
// function of the change's sequence number and the grain), bit 31 = GrainInfo.SingleInstance.
constexpr uint32_t VTAG_SINGLE = 0x80000000u;
__device__ __host__ __forceinline__ uint32_t version_tag(uint32_t op, uint32_t h) {
    return fmix32(h ^ (op * 0x9E3779B9u)) & 0x7FFFFFFFu;
}

__device__ __forceinline__ void stage_ring(const RingArgs& r, uint32_t* s_pts, uint32_t* s_own) {
    for (uint32_t i = threadIdx.x; i < r.n; i += blockDim.x) {
        s_pts[i] = r.pts[i];
        s_own[i] = r.own[i];
    }
    __syncthreads();
}

__device__ __forceinline__ bool is_membership(uint64_t n0, uint64_t n1, uint64_t tcd) {
    return n0 == MEMBERSHIP_N0 && n1 == MEMBERSHIP_N1 && tcd == MEMBERSHIP_TCD;
}

// ---- compact probe indexes (gd_cx.h builds and maintains them) -------------------------------
// Narrow copies of the directory table for the probe, slot for slot: index slot j mirrors table slot
// j (round 6), so a key's entry sits at the same probe distance from the same home (home_slot) as in
// the table, the table's max_probe bounds the index walk too, the build is one streaming pass
// (k_cx_project), and a directory change re-projects only the slots it touched (k_cx_sync) instead
// of rebuilding.  A read covers the aligned 64-B group holding the home slot; the walk starts at the
// home's offset in it and stops at the first empty slot (the table's own rule).
// An index covers a subset of the keys; every other key is probed in the directory itself, per
// message (route_m_core's fallback lanes), so a Guid key or an extra grain class no longer turns the
// index off table-wide.
//   16-B index: keys with N0 = 0 (GrainId.GetGrainId(typeCode, long), GrainId.cs:72-77) whose
//   TypeCodeData is in a 256-slot type set (open addressing, CX_NO_TYPE empty; staged in LDS by the
//   route kernel).  Slot {N1, act, meta = silo | type slot << 16 | CX_LIVE}; meta 0 = empty table
//   slot, CX_TOMB = a tombstone, or a live entry the index does not hold (matches no key).
constexpr uint32_t CX_GROUP = 4;
constexpr uint32_t CX_LIVE = 1u << 24;
constexpr uint32_t CX_TOMB = 1u << 25;
constexpr uint32_t CX_TYPES = 256;
constexpr unsigned long long CX_NO_TYPE = ~0ull;
struct CxArgs {
    const uint4* slots;
    unsigned long long cap;        // = the table's capacity
    const unsigned long long* types;
};
__host__ __device__ __forceinline__ uint32_t cx_type_home(uint64_t tcd) {
    return fmix32((uint32_t)tcd ^ fmix32((uint32_t)(tcd >> 32))) & (CX_TYPES - 1);
}
//   8-B index: keys with N0 = 0, N1 < 2^32 and one of up to CX8_TYPES TypeCodeData (the most
//   populous at the build, passed in the kernel arguments).  Slot {N1 low word, y}: y = u << ab | a,
//   a = the activation (all ab bits set: GD_ACT_MULTI; all but the lowest: an activation too wide
//   for ab bits -- probe the directory), u = type index << sb | (silo + 1) (all 32 - ab bits set: a
//   silo or type too wide -- probe the directory).  y = 0: empty; u = 0 (y = 1): a tombstone or a
//   live entry the index does not hold.
constexpr uint32_t CX8_GROUP = 8;
constexpr uint32_t CX8_TYPES = 8;
struct Cx8Args {
    const uint4* slots;            // two 8-B slots an uint4
    unsigned long long cap;        // = the table's capacity
    uint64_t tcd[CX8_TYPES];       // the types it holds, index order
    uint32_t ntypes;
    uint32_t ab;                   // activation bits
    uint32_t sb;                   // silo + 1 bits
    uint32_t pad;
};
// Type index of tcd in the staged type set, or -1.
__device__ __forceinline__ int cx_type_index(const unsigned long long* s_types, uint64_t tcd) {
    uint32_t t = cx_type_home(tcd);
    for (uint32_t k = 0; k < CX_TYPES; ++k) {
        const unsigned long long v = s_types[t];
        if (v == tcd) return (int)t;
        if (v == CX_NO_TYPE) return -1;
        t = (t + 1) & (CX_TYPES - 1);
    }
    return -1;
}
// The 8-B index's type index of a key, or -1 when the index does not hold it.
__device__ __forceinline__ int cx8_type(const Cx8Args& c, uint64_t n0, uint64_t n1, uint64_t tcd) {
    if (n0 != 0 || (n1 >> 32) != 0) return -1;
    if (c.ntypes <= 1) return c.ntypes && tcd == c.tcd[0] ? 0 : -1;   // one grain class (a uniform branch)
    int t = -1;
#pragma unroll
    for (int k = (int)CX8_TYPES - 1; k >= 0; --k)
        if ((uint32_t)k < c.ntypes && c.tcd[k] == tcd) t = k;
    return t;
}

// Directory entry -> route result (LookUpActivations + IsValidSilo + the single-activation choice).
__device__ __forceinline__ void entry_result(const TableArgs& tab, uint32_t a, uint32_t silo_of, uint32_t& silo,
                                             uint32_t& act, uint8_t& status) {
    if (a == GD_ACT_MULTI) {                       // several activations: the C# random choice
        status = GD_ROUTE_MULTI_ACT;               // (RandomPlacementDirector.cs:33-53)
    } else if (tab_silo_valid(tab, silo_of)) {
        act = a;
        silo = silo_of;                            // ActivationAddress.Silo (Message.cs:629-639)
        status = GD_ROUTE_OK;
    } else {
        status = GD_ROUTE_MISS;                    // IsValidSilo filtered it (GrainDirectoryPartition.cs:431)
    }
}

// The table's max_probe, read when a walk first leaves its home group (rare): kernels on the index do not
// load it at their start, where the scalar load would share lgkmcnt with the LDS ring staging.
__device__ __forceinline__ uint32_t lazy_max_probe(const TableArgs& tab) {
    return __hip_atomic_load(&tab.ctr->max_probe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The 16-B index's walk from the home's group q (RG slots, already read): the entry of (want = 0x100 |
// type slot, n1) or a miss (status left as is).  A key's entry lies within max_probe slots of its home;
// homes are HOME_ALIGN-aligned, so a walk starts at its group's first slot.
static_assert(HOME_ALIGN % CX_GROUP == 0 && HOME_ALIGN % CX8_GROUP == 0, "index groups start at homes");
template <int RG>
__device__ __forceinline__ void cx16_walk(const CxArgs& c, const TableArgs& tab, uint32_t want, uint64_t n1,
                                          unsigned long long home, uint4 (&q)[RG], uint32_t& silo, uint32_t& act,
                                          uint8_t& status) {
    unsigned long long g = home;
    uint32_t last = 0;
    bool done = false;
    for (uint32_t base = 0;; base += RG) {
#pragma unroll
        for (int k = 0; k < RG; ++k) {
            if (done) continue;
            const uint4 v = q[k];
            if (v.w == 0) {
                done = true;                                            // miss
            } else if ((v.w >> 16) == want && ((uint64_t)v.x | ((uint64_t)v.y << 32)) == n1) {
                entry_result(tab, v.z, slot_silo(v.w), silo, act, status);
                done = true;
            }
        }
        if (done) return;
        if (base == 0) last = lazy_max_probe(tab);
        if (base + RG > last) return;                                   // past every entry's reach: miss
        g += RG;
        if (g >= c.cap) g = 0;
#pragma unroll
        for (int k = 0; k < RG; ++k) q[k] = c.slots[g + k];
    }
}

// The 8-B index's walk from the home's group q (8 slots as 4 uint4, already read), for the key's low
// N1 word and type index qt.  Returns true when a redirect entry matched: the directory must answer.
// Per slot only the tests (empty; key; live with this type or a redirect); the hit is decoded once.
__device__ __forceinline__ bool cx8_walk(const Cx8Args& c, const TableArgs& tab, uint32_t key, uint32_t qt,
                                         unsigned long long home, uint4 (&q)[CX8_GROUP / 2], uint32_t& silo,
                                         uint32_t& act, uint8_t& status) {
    const uint32_t umax = ~0u >> c.ab;
    unsigned long long g = home;
    uint32_t last = 0;
    bool done = false;
    uint32_t hit = 0;
    for (uint32_t base = 0;; base += CX8_GROUP) {
#pragma unroll
        for (int k = 0; k < (int)CX8_GROUP; ++k) {
            if (done) continue;
            const uint4 v = q[k / 2];
            const uint32_t x = (k & 1) ? v.z : v.x, y = (k & 1) ? v.w : v.y;
            const uint32_t u = y >> c.ab;
            if (y == 0) {
                done = true;                                            // miss
            } else if (x == key && u != 0 && (u == umax || (u >> c.sb) == qt)) {
                done = true;
                hit = y;
            }
        }
        if (done) break;
        if (base == 0) last = lazy_max_probe(tab);
        if (base + CX8_GROUP > last) return false;                      // past every entry's reach: miss
        g += CX8_GROUP;
        if (g >= c.cap) g = 0;
        const uint4* qp = c.slots + (g >> 1);
#pragma unroll
        for (int k = 0; k < (int)CX8_GROUP / 2; ++k) q[k] = qp[k];
    }
    if (hit == 0) return false;
    const uint32_t am = (1u << c.ab) - 1u, u = hit >> c.ab, a = hit & am;
    if (u == umax || a == am - 1u) return true;                         // redirect: the directory answers
    entry_result(tab, a == am ? GD_ACT_MULTI : a, (u & ((1u << c.sb) - 1u)) - 1u, silo, act, status);
    return false;
}

// cx8_walk over a pure index (PURE route_m_core: one class, every live entry held, none redirected): a
// slot matches on its key word (a hole, y = 1, never -- live slots have y >= 2), no redirect is decoded,
// and the bound is the workgroup's staged max_probe.  With the fallback probe compiled out of the kernel
// and no max_probe load in the walk, k_route at cfg 2 runs 0.287 against 0.292 ms.
__device__ __forceinline__ void cx8_walk_pure(const Cx8Args& c, const TableArgs& tab, uint32_t key,
                                              unsigned long long home, uint4 (&q)[CX8_GROUP / 2], uint32_t mp,
                                              uint32_t& silo, uint32_t& act, uint8_t& status) {
    unsigned long long g = home;
    bool done = false;
    uint32_t hit = 0;
    for (uint32_t base = 0;; base += CX8_GROUP) {
#pragma unroll
        for (int k = 0; k < (int)CX8_GROUP; ++k) {
            if (done) continue;
            const uint4 v = q[k / 2];
            const uint32_t x = (k & 1) ? v.z : v.x, y = (k & 1) ? v.w : v.y;
            if (y == 0) {
                done = true;                                            // miss
            } else if (x == key && y > 1u) {
                done = true;
                hit = y;
            }
        }
        if (done || base + CX8_GROUP > mp) break;                       // found, empty, or past every entry
        g += CX8_GROUP;
        if (g >= c.cap) g = 0;
        const uint4* qp = c.slots + (g >> 1);
#pragma unroll
        for (int k = 0; k < (int)CX8_GROUP / 2; ++k) q[k] = qp[k];
    }
    if (hit == 0) return;
    const uint32_t am = (1u << c.ab) - 1u, u = hit >> c.ab, a = hit & am;
    entry_result(tab, a == am ? GD_ACT_MULTI : a, (u & ((1u << c.sb) - 1u)) - 1u, silo, act, status);
}

// Linear probe of the open-addressing directory for a live entry with this key.
__device__ __forceinline__ bool probe(const Slot* slots, unsigned long long mask, uint32_t max_probe,
                                      uint32_t h, uint64_t n0, uint64_t n1, uint64_t tcd,
                                      uint32_t& act, uint32_t& meta) {
    unsigned long long s = home_slot(h, mask);
    for (uint32_t p = 0; p <= max_probe; ++p) {
        const uint4* q = reinterpret_cast<const uint4*>(slots + s);
        const uint4 a = q[0];
        const uint4 b = q[1];
        const uint32_t st = slot_state(b.w);
        if (st == SLOT_EMPTY) return false;
        const uint64_t k0 = (uint64_t)a.x | ((uint64_t)a.y << 32);
        const uint64_t k1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
        const uint64_t k2 = (uint64_t)b.x | ((uint64_t)b.y << 32);
        if (st == SLOT_LIVE && k0 == n0 && k1 == n1 && k2 == tcd) {
            act = b.z;
            meta = b.w;
            return true;
        }
        s = (s + 1) & mask;
    }
    return false;
}

// ------------------------------------------------------------------ K0+K1+K2: route
// One message: ring owner (ring staged in LDS) and, PROBE, the directory entry.
template <int MODE, bool PROBE>
__device__ __forceinline__ void route_one(uint64_t n0, uint64_t n1, uint64_t tcd, const RingArgs& ring,
                                          const uint32_t* s_pts, const uint32_t* s_own, const TableArgs& tab,
                                          uint32_t max_probe, uint32_t& silo, uint32_t& act, uint8_t& status) {
    const uint32_t cat = (uint32_t)(tcd >> 56);
    act = NONE32;
    if (cat == CAT_SYSTEM_TARGET) {                        // LocalGrainDirectory.cs:480-485
        silo = ring.my_silo;
        status = GD_ROUTE_SYSTEM_TARGET;
    } else if (is_membership(n0, n1, tcd)) {               // :487-503
        silo = ring.seed_silo;
        status = GD_ROUTE_MEMBERSHIP;
    } else if (cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT) {  // UniqueKey.cs:279-281
        silo = NONE32;
        status = GD_ROUTE_KEYEXT;
    } else {
        const uint32_t h = uniform_hash(n0, n1, tcd);
        silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h)];
        status = GD_ROUTE_OK;
        if constexpr (PROBE) {
            uint32_t a, meta;
            if (probe(tab.slots, tab.mask, max_probe, h, n0, n1, tcd, a, meta)) {
                if (a == GD_ACT_MULTI) {
                    status = GD_ROUTE_MULTI_ACT;           // RandomPlacementDirector.cs:33-53, in C#
                } else if (!tab_silo_valid(tab, slot_silo(meta))) {
                    status = GD_ROUTE_MISS;                // LookUpActivations filters it (:431): no address
                } else {
                    act = a;
                    silo = slot_silo(meta);                // ActivationAddress.Silo (Message.cs:629-639)
                }
            } else {
                status = GD_ROUTE_MISS;                    // Dispatcher.cs:742 slow path
            }
        }
    }
}

// One message per thread.  PROBE=false gives CalculateTargetSilo only.
template <int MODE, bool PROBE>
static __global__ void __launch_bounds__(BLOCK) k_route(const gd_key* __restrict__ keys, uint32_t n, RingArgs ring,
                                                 TableArgs tab, uint32_t* __restrict__ out_silo,
                                                 uint32_t* __restrict__ out_act,
                                                 uint8_t* __restrict__ out_status) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const uint32_t max_probe = PROBE ? tab.ctr->max_probe : 0;

    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
    uint32_t silo, act;
    uint8_t status;
    route_one<MODE, PROBE>(kp[0], kp[1], kp[2], ring, s_pts, s_own, tab, max_probe, silo, act, status);
    out_silo[i] = silo;
    if constexpr (PROBE) {
        out_act[i] = act;
        out_status[i] = status;
    }
}

template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// The route kernel proper: M messages per thread (coalesced: message
// base + j*BLOCK + tid), all M first probes issued before any is inspected so
// that each lane keeps M random 32-B slot reads in flight.  NT streams the key
// reads (and with NT_SIDE the silo / status writes) non-temporally so they do not
// push the table out of the caches it shares with them.
// N1W: 0 = 24-B keys; 8 / 4 = the keys arrive as N1 alone (u64 / u32 each; N0 = 0, TypeCodeData =
// tcd_u for all), the forms a compact exchange header round delivers (k_key_desc, gd_shard.h).
// The per-thread part: messages base + j * STRIDE, j < M; lds_act (optional) gets act too.
// CX: probe the compact index (cx, its type set staged in s_types) instead of the directory, RG slots
// (16 B each) a read: CX_GROUP (one 64-B atom, the layout's group) or 1 (16 B, for hot key sets).
// CX8: probe the 8-B index (cx8) instead, one 64-B group (8 slots) a read.
// PURE (with CX8, k_route_m): the index is pure (gd_engine.h cx8_pure) -- a key it does not hold is in no
// entry, so there is no directory fallback at all; mp = the table's max_probe, staged by the caller.
template <int MODE, int M, int STRIDE, bool NT, int N1W, bool NT_SIDE = false, bool CX = false,
          int RG_CX = (int)CX_GROUP, bool CX8 = false, bool PURE = false>
__device__ __forceinline__ void route_m_core(const gd_key* __restrict__ keys, uint32_t n, uint32_t base,
                                             const RingArgs& ring, const uint32_t* s_pts, const uint32_t* s_own,
                                             const TableArgs& tab, uint32_t max_probe,
                                             uint32_t* __restrict__ out_silo, uint32_t* __restrict__ out_act,
                                             uint8_t* __restrict__ out_status, uint64_t tcd_u,
                                             uint32_t* lds_act, uint32_t lds_stride, const CxArgs* cx = nullptr,
                                             const unsigned long long* s_types = nullptr,
                                             const Cx8Args* cx8 = nullptr, uint32_t mp = 0) {

    uint64_t n0[M], n1[M], tcd[M];
    uint32_t h[M], silo[M], act[M];
    uint8_t status[M];
    bool need[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t i = base + j * STRIDE;
        n0[j] = n1[j] = tcd[j] = 0;
        if (i < n) {
            if constexpr (N1W == 8) {
                n1[j] = ld<NT>(reinterpret_cast<const uint64_t*>(keys) + i);
                tcd[j] = tcd_u;
            } else if constexpr (N1W == 4) {
                n1[j] = ld<NT>(reinterpret_cast<const uint32_t*>(keys) + i);
                tcd[j] = tcd_u;
            } else {
                const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
                n0[j] = ld<NT>(kp);
                n1[j] = ld<NT>(kp + 1);
                tcd[j] = ld<NT>(kp + 2);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t cat = (uint32_t)(tcd[j] >> 56);
        act[j] = NONE32;
        need[j] = false;
        h[j] = 0;
        if (cat == CAT_SYSTEM_TARGET) {                        // LocalGrainDirectory.cs:480-485
            silo[j] = ring.my_silo;
            status[j] = GD_ROUTE_SYSTEM_TARGET;
        } else if (is_membership(n0[j], n1[j], tcd[j])) {     // :487-503
            silo[j] = ring.seed_silo;
            status[j] = GD_ROUTE_MEMBERSHIP;
        } else if (cat == CAT_KEYEXT_GRAIN || cat == CAT_GEO_CLIENT) {  // UniqueKey.cs:279-281
            silo[j] = NONE32;
            status[j] = GD_ROUTE_KEYEXT;
        } else {
            h[j] = uniform_hash(n0[j], n1[j], tcd[j]);
            status[j] = GD_ROUTE_MISS;
            need[j] = true;
        }
    }
    if constexpr (CX || CX8) {
        static_assert(!(CX && CX8), "one index form a launch");
        static_assert(RG_CX == 1 || RG_CX == (int)CX_GROUP, "16-B index reads: one slot or one group");
        // Lanes whose key the index holds walk the index from the home's group; the others (fb: an N0 !=
        // 0 key, a type or N1 the index does not hold, or a redirect entry) probe the directory itself.
        constexpr int QW = CX ? RG_CX : (int)CX8_GROUP / 2;
        uint32_t want[M];
        bool fb[M];
        unsigned long long s[M];
        uint4 q[M][QW];
#pragma unroll
        for (int j = 0; j < M; ++j) {
            want[j] = 0;
            fb[j] = false;
            s[j] = home_slot(h[j], tab.mask);
            if (need[j]) {
                if constexpr (CX) {
                    const int t = n0[j] == 0 ? cx_type_index(s_types, tcd[j]) : -1;
                    want[j] = t < 0 ? 0u : (0x100u | (uint32_t)t);
                } else {
                    const int t = cx8_type(*cx8, n0[j], n1[j], tcd[j]);
                    want[j] = t < 0 ? 0u : 1u + (uint32_t)t;
                }
                fb[j] = !PURE && want[j] == 0;
            }
            if (want[j]) {
                if constexpr (CX) {
                    const uint4* qp = cx->slots + (s[j] & ~(unsigned long long)(RG_CX - 1));
#pragma unroll
                    for (int g = 0; g < QW; ++g) q[j][g] = qp[g];
                } else {
                    const uint4* qp = cx8->slots + ((s[j] & ~(unsigned long long)(CX8_GROUP - 1)) >> 1);
#pragma unroll
                    for (int g = 0; g < QW; ++g) q[j][g] = qp[g];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < M; ++j)
            if (need[j]) silo[j] = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h[j])];
#pragma unroll
        for (int j = 0; j < M; ++j) {
            if (!want[j]) continue;
            if constexpr (CX) cx16_walk<RG_CX>(*cx, tab, want[j], n1[j], s[j], q[j], silo[j], act[j], status[j]);
            else if constexpr (PURE) cx8_walk_pure(*cx8, tab, (uint32_t)n1[j], s[j], q[j], mp, silo[j], act[j], status[j]);
            else fb[j] = cx8_walk(*cx8, tab, (uint32_t)n1[j], want[j] - 1u, s[j], q[j], silo[j], act[j], status[j]);
        }
        if constexpr (!PURE) {
#pragma unroll
            for (int j = 0; j < M; ++j) {
                if (!fb[j]) continue;
                uint32_t a, meta;
                if (probe(tab.slots, tab.mask, lazy_max_probe(tab), h[j], n0[j], n1[j], tcd[j], a, meta))
                    entry_result(tab, a, slot_silo(meta), silo[j], act[j], status[j]);   // else MISS (Dispatcher.cs:742)
            }
        }
    } else {
    // first probe of every message, all in flight together; the ring search (LDS) runs under them.
    // A round reads the whole aligned group of SLOT_GROUP slots (home_slot) and walks it in order.
    constexpr int RG = (int)SLOT_GROUP;
    unsigned long long s[M];
    uint4 q[M][2 * RG];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        s[j] = home_slot(h[j], tab.mask);
        if (need[j]) {
            const uint4* qp = reinterpret_cast<const uint4*>(tab.slots + s[j]);
#pragma unroll
            for (int g = 0; g < 2 * RG; ++g) q[j][g] = qp[g];
        }
    }
#pragma unroll
    for (int j = 0; j < M; ++j)
        if (need[j]) silo[j] = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h[j])];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        if (!need[j]) continue;
        bool done = false;
        for (uint32_t p = 0;;) {
#pragma unroll
            for (int g = 0; g < RG; ++g) {
                if (done) continue;
                const uint4 a = q[j][2 * g], b = q[j][2 * g + 1];
                const uint32_t stt = slot_state(b.w);
                const uint64_t k0 = (uint64_t)a.x | ((uint64_t)a.y << 32);
                const uint64_t k1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
                const uint64_t k2 = (uint64_t)b.x | ((uint64_t)b.y << 32);
                if (stt == SLOT_EMPTY) {
                    done = true;                                  // miss
                } else if (stt == SLOT_LIVE && k0 == n0[j] && k1 == n1[j] && k2 == tcd[j]) {
                    if (b.z == GD_ACT_MULTI) {                    // several activations: the C# random
                        status[j] = GD_ROUTE_MULTI_ACT;           // choice (RandomPlacementDirector.cs:33-53)
                    } else if (tab_silo_valid(tab, slot_silo(b.w))) {
                        act[j] = b.z;
                        silo[j] = slot_silo(b.w);                 // ActivationAddress.Silo (Message.cs:629-639)
                        status[j] = GD_ROUTE_OK;
                    }                                             // else: IsValidSilo filtered it (:431) -> MISS
                    done = true;
                } else if (++p > max_probe) {
                    done = true;                                  // miss: Dispatcher.cs:742 slow path
                }
            }
            if (done) break;
            s[j] = (s[j] + RG) & tab.mask;
            const uint4* qp = reinterpret_cast<const uint4*>(tab.slots + s[j]);
#pragma unroll
            for (int g = 0; g < 2 * RG; ++g) q[j][g] = qp[g];
        }
    }
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t i = base + j * STRIDE;
        if (i < n) {
            st<NT || NT_SIDE>(out_silo + i, silo[j]);      // silo / status: not read again on the device
            out_act[i] = act[j];                            // act: the bucketing's input, next (temporal)
            st<NT || NT_SIDE>(out_status + i, status[j]);
            if (lds_act) lds_act[(size_t)i * lds_stride] = act[j];
        }
    }
}

// Micro-batch route over keys in pinned host memory: one-wave workgroups, so the host reads (and
// the host stores of silo / status) of a 4,096-message batch spread over 64 CUs.
constexpr int MB_ROUTE_BLOCK = 64;

// GD_MB_TRACE: workgroup 0, thread 0 adds phase durations (100-MHz wall clock ticks) into ts[]
__device__ __forceinline__ void mb_mark(unsigned long long* ts, int k, unsigned long long& t) {
    if (ts && blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long now = wall_clock64();
        if (k > 0) atomicAdd(ts + k, now - t);
        t = now;
    }
}

// CX8: through the 8-B index (when it is current: gd_microbatch_run re-captures its graphs when the
// index is rebuilt or goes stale), the directory otherwise.
template <int MODE, bool CX8 = false>
static __global__ void __launch_bounds__(MB_ROUTE_BLOCK) k_mb_route(const gd_key* __restrict__ keys, uint32_t n,
                                                            RingArgs ring, TableArgs tab,
                                                            uint32_t* __restrict__ out_silo,
                                                            uint32_t* __restrict__ out_act,
                                                            uint8_t* __restrict__ out_status,
                                                            uint32_t* __restrict__ act_host,
                                                            unsigned long long* ts, Cx8Args cx8 = Cx8Args{}) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    unsigned long long t = 0;
    mb_mark(ts, 0, t);
    stage_ring(ring, s_pts, s_own);
    mb_mark(ts, 1, t);
    // act goes to HBM for the sort and, from these 64 workgroups, to the host block as well
    route_m_core<MODE, 1, MB_ROUTE_BLOCK, false, 0, false, false, (int)CX_GROUP, CX8>(
        keys, n, blockIdx.x * MB_ROUTE_BLOCK + threadIdx.x, ring, s_pts, s_own, tab,
        CX8 ? 0u : tab.ctr->max_probe, out_silo, out_act, out_status, 0, act_host, act_host ? 1u : 0u, nullptr,
        nullptr, &cx8);
    mb_mark(ts, 2, t);
    if (ts) {
        __threadfence_system();
        mb_mark(ts, 3, t);
    }
}

// Workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each with its own
// L2.  With xcd != 0 block b processes tile start(b % 8) + b / 8, so every XCD owns a contiguous
// tile range: the digit-run fragments that consecutive tiles write next to each other in the
// output meet in one L2 instead of being written back as partial lines by two.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb, uint32_t xcd) {
    if (!xcd) return b;
    const uint32_t x = b & 7u, k = b >> 3, q = nb >> 3, rem = nb & 7u;
    return x * q + min(x, rem) + k;
}

// src_out (optional, the exchange's receive side): message i's sender rank, from the per-sender
// receive counts rcnt[world] (k_recv_src's job, done here beside the probe's own writes).
template <int MODE, int M, bool NT, int N1W = 0, bool CX = false, int RG_CX = (int)CX_GROUP, bool CX8 = false,
          bool PURE = false>
static __global__ void __launch_bounds__(BLOCK) k_route_m(const gd_key* __restrict__ keys, uint32_t n, RingArgs ring,
                                                   TableArgs tab, uint32_t* __restrict__ out_silo,
                                                   uint32_t* __restrict__ out_act,
                                                   uint8_t* __restrict__ out_status, uint64_t tcd_u, uint32_t xcd,
                                                   const uint32_t* __restrict__ rcnt = nullptr, uint32_t world = 0,
                                                   uint32_t* __restrict__ src_out = nullptr, CxArgs cx = CxArgs{},
                                                   Cx8Args cx8 = Cx8Args{}) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    __shared__ uint32_t s_soff[257];
    __shared__ unsigned long long s_types[CX ? CX_TYPES : 1];
    __shared__ uint32_t s_mp;
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    if constexpr (CX)
        for (uint32_t t = threadIdx.x; t < CX_TYPES; t += BLOCK) s_types[t] = cx.types[t];
    if (PURE && threadIdx.x == 0) s_mp = lazy_max_probe(tab);   // the walks' bound, one load beside the ring
    if (src_out && threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t q = 0; q < world; ++q) {
            s_soff[q] = run;
            run += rcnt[q];
        }
        s_soff[world] = run;
    }
    stage_ring(ring, s_pts, s_own);                    // its barrier publishes s_soff (and s_types) too
    // xcd: each XCD routes a contiguous message range (xcd_tile), so the act it writes is the act the
    // same XCD's histogram and scatter workgroups read next (their XCD tile ranges match)
    const uint32_t blk = xcd_tile(blockIdx.x, gridDim.x, xcd);
    route_m_core<MODE, M, BLOCK, NT, N1W, true, CX, RG_CX, CX8, PURE>(
        keys, n, blk * (BLOCK * M) + threadIdx.x, ring, s_pts, s_own, tab, (CX || CX8) ? 0u : tab.ctr->max_probe,
        out_silo, out_act, out_status, tcd_u, nullptr, 0, &cx, s_types, &cx8, PURE ? s_mp : 0u);
    if (src_out) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const uint32_t i = blk * (BLOCK * M) + j * BLOCK + threadIdx.x;
            if (i >= n) continue;
            uint32_t lo = 0, hi = world;               // largest q with s_soff[q] <= i
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_soff[mid] <= i) lo = mid;
                else hi = mid;
            }
            st<true>(src_out + i, lo);
        }
    }
}

// The route's memory bound (gd_route_bound_device, a diagnostic, not a route): k_route_m<…, CX8>'s XCD
// mapping, ring-sized LDS, key reads, home hash, one 64-B group read of the 8-B index per message and
// silo / act / status writes -- without the ring search, the class checks, the walk past the home group,
// the redirect decode and the directory fallback; M messages a thread (2: the fastest measured).  On the
// route's own index and key stream it is the time k_route cannot go under without reading or writing less.
template <int M, bool NT>
static __global__ void __launch_bounds__(BLOCK) k_route_bound(const gd_key* __restrict__ keys, uint32_t n,
                                                       unsigned long long mask, Cx8Args cx8,
                                                       uint32_t* __restrict__ out_silo,
                                                       uint32_t* __restrict__ out_act,
                                                       uint8_t* __restrict__ out_status, uint32_t xcd) {
    const uint32_t base = xcd_tile(blockIdx.x, gridDim.x, xcd) * (BLOCK * M) + threadIdx.x;
    uint64_t n1[M];
    uint4 q[M][CX8_GROUP / 2];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t i = base + j * BLOCK;
        uint64_t n0 = 0, tcd = 0;
        n1[j] = 0;
        if (i < n) {
            const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
            n0 = ld<NT>(kp);
            n1[j] = ld<NT>(kp + 1);
            tcd = ld<NT>(kp + 2);
        }
        const unsigned long long s = home_slot(uniform_hash(n0, n1[j], tcd), mask);
        const uint4* qp = cx8.slots + ((s & ~(unsigned long long)(CX8_GROUP - 1)) >> 1);
#pragma unroll
        for (int g = 0; g < (int)CX8_GROUP / 2; ++g) q[j][g] = qp[g];
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const uint32_t i = base + j * BLOCK;
        uint32_t hit = 0;
#pragma unroll
        for (int k = 0; k < (int)CX8_GROUP; ++k) {
            const uint4 v = q[j][k / 2];
            const uint32_t x = (k & 1) ? v.z : v.x, y = (k & 1) ? v.w : v.y;
            if (hit == 0 && y != 0 && x == (uint32_t)n1[j]) hit = y;
        }
        if (i < n) {
            st<true>(out_silo + i, (hit >> cx8.ab) - 1u);
            out_act[i] = hit & ((1u << cx8.ab) - 1u);
            st<true>(out_status + i, (uint8_t)(hit == 0));
        }
    }
}

// The owner's probe over received chunks grouped by region (gd_route_multi with regions, SURVEY 8 e):
// workgroup b takes region g = b % 8.  Workgroups are dispatched round-robin over the 8 XCDs (b -> XCD
// b % 8), so all of one XCD's workgroups probe one eighth of the table (home_slot's top bits) and its
// 4-MB L2 serves that eighth alone (tools/ubench_random.hip: 16M probes of a 64-MB table 0.344 ->
// 0.224 ms).  The region's messages are W segments, one per sender (seg: k_region_segments); the
// G = gridDim.x / 8 workgroups of a region take its blocks of BLOCK messages grid-stride.
template <int MODE, int N1W>
static __global__ void __launch_bounds__(BLOCK) k_route_region(const gd_key* __restrict__ keys, uint32_t n, RingArgs ring,
                                                        TableArgs tab, uint32_t* __restrict__ out_silo,
                                                        uint32_t* __restrict__ out_act,
                                                        uint8_t* __restrict__ out_status, uint64_t tcd_u,
                                                        const uint32_t* __restrict__ seg, uint32_t world) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    __shared__ uint32_t s_beg[257], s_pre[257];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    const uint32_t g = blockIdx.x % N_REGIONS, G = gridDim.x / N_REGIONS;
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t q = 0; q < world; ++q) {
            const uint32_t b = seg[q * (N_REGIONS + 1) + g], e = seg[q * (N_REGIONS + 1) + g + 1];
            s_beg[q] = b;
            s_pre[q] = run;
            run += e - b;
        }
        s_pre[world] = run;
    }
    stage_ring(ring, s_pts, s_own);                   // its barrier publishes s_beg / s_pre too
    const uint32_t total = s_pre[world];
    const uint32_t max_probe = tab.ctr->max_probe;
    for (uint32_t k = blockIdx.x / N_REGIONS; k * BLOCK < total; k += G) {
        const uint32_t e = k * BLOCK + threadIdx.x;
        uint32_t i = n;                                // past the region: route_m_core skips it
        if (e < total) {
            uint32_t lo = 0, hi = world;               // largest q with s_pre[q] <= e
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_pre[mid] <= e) lo = mid;
                else hi = mid;
            }
            i = s_beg[lo] + (e - s_pre[lo]);
        }
        route_m_core<MODE, 1, BLOCK, false, N1W, true>(keys, n, i, ring, s_pts, s_own, tab, max_probe, out_silo,
                                                      out_act, out_status, tcd_u, nullptr, 0);
    }
}

// GetPrimaryTargetSilo(uint key) over raw ring keys.
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_ring_hashes(const uint32_t* __restrict__ hashes, uint32_t n,
                                                       RingArgs ring, uint32_t* __restrict__ out_silo) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    out_silo[i] = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, hashes[i])];
}

// ------------------------------------------------------------------ directory maintenance
// AddSingleActivation (GrainDirectoryPartition.cs:304-326, GrainInfo :110-124) for a batch.
// Phase 1: find the key's slot or claim an empty one.  A lane that meets a slot
// another lane has claimed but not yet published does NOT wait (a divergent
// wait can starve the claimer of the same wave once the compiler sinks its
// publish to the loop exit): it is marked RETRY and the host relaunches the
// kernel for the retried items, after the kernel boundary has published every
// claim.  "Not yet published" is read off the meta alone (round 6): CLAIMED, or
// PENDING with this launch's tag in the silo field (claim_tag) -- a PENDING slot of
// an earlier launch has its key published by that launch's end.  So a claim needs no
// release fence (an agent-scope release writes the XCD's L2 back, per wave) and a
// walk no acquire loads (an agent-scope acquire invalidates it): the metas are read
// and swapped with relaxed device-coherent atomics, the keys with plain loads.
constexpr uint32_t SLOT_RETRY = 0xFFFFFFFEu;
// PENDING's tag of claim launch `pass` (k_reg_take's claims carry 0)
__device__ __forceinline__ uint32_t claim_tag(uint32_t pass) { return (pass + 1u) & 0xFFFFu; }

// vals / valid (nullable): an item whose silo is not valid is skipped (slot_of = NONE32): the
// IsValidSilo check of AddSingleActivation / AddActivation (GrainDirectoryPartition.cs:279,310).
__device__ __forceinline__ void reg_claim_item(uint32_t i, const gd_key* __restrict__ keys, Slot* slots,
                                               unsigned long long mask, DevCounters* ctr,
                                               uint32_t* __restrict__ slot_of, uint8_t* __restrict__ is_new,
                                               const gd_val* __restrict__ vals, const TableArgs& vt, uint32_t* retry,
                                               uint32_t& pdist, bool& reused, uint32_t tag,
                                               uint32_t* __restrict__ last = nullptr);
// The claims' counter updates, one atomic a wave (one per item queued ~10^4 same-address atomics behind a
// 1 % registration batch: 0.12 ms of it at cfg 2).  Every lane of the wave calls it.
__device__ __forceinline__ void claim_counters(DevCounters* ctr, uint32_t pdist, bool reused) {
    for (int off = WAVE / 2; off > 0; off >>= 1) pdist = max(pdist, (uint32_t)__shfl_xor(pdist, off, WAVE));
    const unsigned long long m = __ballot(reused);
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        // max_probe only grows: a wave whose distance is not past it (nearly all) skips the atomic
        if (pdist && pdist > __hip_atomic_load(&ctr->max_probe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMax(&ctr->max_probe, pdist);
        if (m) atomicAdd(ctr_stripe(ctr) + 1, ~(unsigned long long)__popcll(m) + 1ull);   // tomb - reused
    }
}

// last (optional): one word per table slot, zero between batches -- an item that ends with a new entry
// (claimed it, or found it PENDING) elects itself: atomicMax(~i), so the lowest batch index wins
// (k_reg_commit_elect); null: the k_reg_minwin / k_reg_resolve election on the slot's act word.
static __global__ void __launch_bounds__(BLOCK) k_reg_claim(const gd_key* __restrict__ keys, uint32_t n, Slot* slots,
                                                     unsigned long long mask, DevCounters* ctr,
                                                     uint32_t* __restrict__ slot_of,
                                                     uint8_t* __restrict__ is_new, uint32_t pass,
                                                     const gd_val* __restrict__ vals, TableArgs vt,
                                                     uint32_t* __restrict__ last = nullptr) {
    // pass 0: every item; later passes: the items the previous one deferred
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t pd = 0;
    bool reused = false;
    if (i < n && (pass == 0 || slot_of[i] == SLOT_RETRY)) {
        reg_claim_item(i, keys, slots, mask, ctr, slot_of, is_new, vals, vt, &ctr->retry, pd, reused,
                       claim_tag(pass), last);
        if (last && is_new[i]) atomicMax(&last[slot_of[i]], ~i);
    }
    claim_counters(ctr, pd, reused);
}

// k_reg_take + the gated claim passes of an asynchronous batch: a pass settles one new grain of each group
// of new grains colliding on their first free slots (a claim hides its key from its own pass), so a
// large batch needs several (300,000 new grains in a 2M-slot table: more than 3)
constexpr uint32_t REG_PASSES = 12;
constexpr uint32_t REG_PASSES_SMALL = 4;    // ... for a batch of at most 2^16 items
// The claim pass of an asynchronous batch (gd_dir_register_device_async): pass p > 0 runs only when
// pass p - 1 deferred items (gate = its retry count; all lanes read the same word), so the host enqueues
// REG_PASSES passes without reading a count back; k_reg_settled flags a batch still unsettled after them.
static __global__ void __launch_bounds__(BLOCK) k_reg_claim_gated(const gd_key* __restrict__ keys, uint32_t n,
                                                           Slot* slots, unsigned long long mask, DevCounters* ctr,
                                                           uint32_t* __restrict__ slot_of,
                                                           uint8_t* __restrict__ is_new,
                                                           const gd_val* __restrict__ vals, TableArgs vt,
                                                           const uint32_t* __restrict__ gate, uint32_t* retry,
                                                           uint32_t* __restrict__ last, uint32_t pass) {
    if (gate && *gate == 0) return;
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    // pass 0 zeroes the later passes' counters (its own, retry[0], was zeroed by the previous batch's
    // k_reg_minwin_gated, or at allocation)
    if (!gate && i < REG_PASSES - 1) retry[1 + i] = 0;
    uint32_t pd = 0;
    bool reused = false;
    if (i < n && (!gate || slot_of[i] == SLOT_RETRY)) {
        reg_claim_item(i, keys, slots, mask, ctr, slot_of, is_new, vals, vt, retry, pd, reused, claim_tag(pass),
                       last);
        if (is_new[i]) atomicMax(&last[slot_of[i]], ~i);    // the election (k_reg_commit_elect)
    }
    claim_counters(ctr, pd, reused);
}
// The claim as two kernels (round 6; the single claim kernel walked each chain with agent-scope atomic
// loads, two dependent L2 round trips a slot, 0.08 ms for a 10^4-item batch at cfg 2):
//   k_reg_find  read-only (nothing writes the table during it): each item's existing entry, or the first
//               free slot of its chain (its first tombstone, else the empty slot ending it) and that
//               slot's meta, with plain loads;
//   k_reg_take  one CAS on that slot from the meta seen; an item that loses it (another item of the
//               batch took the slot: the same key or a colliding one) is deferred to the gated claim
//               passes (k_reg_claim_gated, the full protocol).
constexpr uint8_t REG_CANDIDATE = 2;        // is_new: k_reg_find left a free slot to take
// LIVE_CLAIMS (k_reg_find_take): other items of the launch claim slots while this one walks -- a slot
// CLAIMED or PENDING holds a key unpublished to this launch, whose claimer the slot's election word
// names (last): this key's twin -- join it (is_new 1) -- or another key -- walk on; a claim not yet
// recorded defers the item (SLOT_RETRY).  A stale EMPTY or tombstone in a cached line only makes the
// take's CAS fail (the CAS is the arbiter).
template <bool LIVE_CLAIMS = false>
__device__ __forceinline__ void reg_find_item(uint32_t i, const gd_key* __restrict__ keys,
                                              const Slot* __restrict__ slots, unsigned long long mask,
                                              DevCounters* ctr, uint32_t* __restrict__ slot_of,
                                              uint8_t* __restrict__ is_new, uint32_t* __restrict__ seen,
                                              const gd_val* __restrict__ vals, const TableArgs& vt,
                                              uint32_t* __restrict__ last = nullptr) {
    if (vals && !tab_silo_valid(vt, vals[i].silo)) {
        slot_of[i] = NONE32;
        is_new[i] = 0;
        return;
    }
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    unsigned long long s = home_slot(uniform_hash(n0, n1, tcd), mask);
    unsigned long long free_s = ~0ull;
    uint32_t free_meta = 0, res = NONE32;
    uint8_t st_out = 0;
    // four slots (one 128-B line) a step: homes are 8-slot aligned, so a chain is mostly one or two steps
    bool done = false;
    for (unsigned long long dist = 0; !done && dist <= mask; dist += 4) {
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4* p = reinterpret_cast<const uint4*>(slots + ((s + k) & mask));
            q[2 * k] = p[0];
            q[2 * k + 1] = p[1];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (done) continue;
            const uint4 a = q[2 * k], b = q[2 * k + 1];
            const uint32_t st = slot_state(b.w);
            const unsigned long long sk = (s + k) & mask;
            if (st == SLOT_EMPTY) {
                if (free_s == ~0ull) {
                    free_s = sk;
                    free_meta = b.w;
                }
                done = true;
            } else if (LIVE_CLAIMS && (st == SLOT_CLAIMED || st == SLOT_PENDING)) {
                const uint32_t w = __hip_atomic_load(&last[sk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (w == 0) {
                    res = SLOT_RETRY;                    // a claim of this launch not yet recorded
                    done = true;
                } else {
                    const gd_key& c = keys[~w];
                    if (c.n0 == n0 && c.n1 == n1 && c.type_code_data == tcd) {
                        res = (uint32_t)sk;              // the twin's claim: join it
                        st_out = 1;
                        done = true;
                    }                                    // else another key's claim: walk on
                }
            } else {
                if (st == SLOT_TOMB && free_s == ~0ull) {
                    free_s = sk;
                    free_meta = b.w;
                }
                if (st == SLOT_LIVE && ((uint64_t)a.x | ((uint64_t)a.y << 32)) == n0 &&
                    ((uint64_t)a.z | ((uint64_t)a.w << 32)) == n1 && ((uint64_t)b.x | ((uint64_t)b.y << 32)) == tcd) {
                    res = (uint32_t)sk;                  // registered already
                    done = true;
                }
            }
        }
        s = (s + 4) & mask;
    }
    if (res == NONE32 && !(LIVE_CLAIMS && st_out == 1)) {
        if (free_s == ~0ull) {
            atomicOr(&ctr->err, 2u);                     // no free slot: the table is full
        } else {
            res = (uint32_t)free_s;
            seen[i] = free_meta;
            st_out = REG_CANDIDATE;
        }
    }
    slot_of[i] = res;
    is_new[i] = st_out;
}
static __global__ void __launch_bounds__(BLOCK) k_reg_find(const gd_key* __restrict__ keys, uint32_t n,
                                                    const Slot* __restrict__ slots, unsigned long long mask,
                                                    DevCounters* ctr, uint32_t* __restrict__ slot_of,
                                                    uint8_t* __restrict__ is_new, uint32_t* __restrict__ seen,
                                                    const gd_val* __restrict__ vals, TableArgs vt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) reg_find_item(i, keys, slots, mask, ctr, slot_of, is_new, seen, vals, vt);
}

// k_reg_take's item: one CAS on the slot k_reg_find left (pd / reused for claim_counters; deferred: the
// item lost the CAS and goes to the next claim pass).
__device__ __forceinline__ void reg_take_item(uint32_t i, const gd_key* __restrict__ keys, Slot* slots,
                                              unsigned long long mask, uint32_t* __restrict__ slot_of,
                                              uint8_t* __restrict__ is_new, const uint32_t* __restrict__ seen,
                                              uint32_t* __restrict__ last, uint32_t& pd, bool& reused,
                                              bool& deferred) {
    if (is_new[i] == REG_CANDIDATE) {
        const uint32_t t = slot_of[i];
        uint32_t expected = seen[i];
        uint32_t* mp = &slots[t].meta;
        if (__hip_atomic_compare_exchange_strong(mp, &expected, make_meta(SLOT_CLAIMED, 0), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            // No item of this launch reads a slot another item claimed (k_reg_find read the table before it,
            // a CAS loser defers below), so the key needs no release here: the kernel's end publishes it to
            // the passes and commit that read it (an agent-scope release fence writes the XCD's L2 back,
            // per wave: 2.2 ns an item at cfg 3's 100M registrations, 72 ms a 33M batch)
            atomicMax(&last[t], ~i);                     // the election (k_reg_commit_elect), and the claimer
            const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
            Slot& sl = slots[t];
            sl.n0 = n0;
            sl.n1 = n1;
            sl.tcd = tcd;
            sl.act = NONE32;
            __hip_atomic_store(mp, make_meta(SLOT_PENDING, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long home = home_slot(uniform_hash(n0, n1, tcd), mask);
            pd = (uint32_t)((t - home) & mask);
            reused = slot_state(seen[i]) == SLOT_TOMB;
            is_new[i] = 1;
        } else {
            // taken meanwhile (another new grain homed nearby, or this key's twin, whose key this launch
            // has not published): the full protocol in the next claim pass
            slot_of[i] = SLOT_RETRY;
            is_new[i] = 0;
            deferred = true;
        }
    }
}
// The deferred items' count, one atomic a wave (every lane of the wave calls it).
__device__ __forceinline__ void count_deferred(uint32_t* retry, bool deferred) {
    const unsigned long long dm = __ballot(deferred);
    if ((threadIdx.x & (WAVE - 1)) == 0 && dm) atomicAdd(retry, (uint32_t)__popcll(dm));
}
static __global__ void __launch_bounds__(BLOCK) k_reg_take(const gd_key* __restrict__ keys, uint32_t n, Slot* slots,
                                                    unsigned long long mask, DevCounters* ctr,
                                                    const gd_val* __restrict__ vals, TableArgs vt,
                                                    uint32_t* __restrict__ slot_of, uint8_t* __restrict__ is_new,
                                                    const uint32_t* __restrict__ seen, uint32_t* retry,
                                                    uint32_t* zero, uint32_t* __restrict__ last) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (zero && i < REG_PASSES - 1) zero[i] = 0;         // the gated passes' counters (asynchronous batches)
    uint32_t pd = 0;
    bool reused = false, deferred = false;
    if (i < n) reg_take_item(i, keys, slots, mask, slot_of, is_new, seen, last, pd, reused, deferred);
    count_deferred(retry, deferred);
    claim_counters(ctr, pd, reused);
}
// k_reg_find and k_reg_take as one launch (round 6): each item walks with plain loads and takes its free
// slot at once; an item whose walk meets a claim of this launch defers to the claim passes.
static __global__ void __launch_bounds__(BLOCK) k_reg_find_take(const gd_key* __restrict__ keys, uint32_t n,
                                                         Slot* slots, unsigned long long mask, DevCounters* ctr,
                                                         const gd_val* __restrict__ vals, TableArgs vt,
                                                         uint32_t* __restrict__ slot_of, uint8_t* __restrict__ is_new,
                                                         uint32_t* __restrict__ seen, uint32_t* retry, uint32_t* zero,
                                                         uint32_t* __restrict__ last) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (zero && i < REG_PASSES - 1) zero[i] = 0;         // the gated passes' counters (asynchronous batches)
    uint32_t pd = 0;
    bool reused = false, deferred = false;
    if (i < n) {
        reg_find_item<true>(i, keys, slots, mask, ctr, slot_of, is_new, seen, vals, vt, last);
        if (slot_of[i] == SLOT_RETRY) deferred = true;
        else if (is_new[i] == 1) atomicMax(&last[slot_of[i]], ~i);      // joined its twin's claim
        else reg_take_item(i, keys, slots, mask, slot_of, is_new, seen, last, pd, reused, deferred);
    }
    count_deferred(retry, deferred);
    claim_counters(ctr, pd, reused);
}

constexpr uint32_t ERR_UNSETTLED = 64u;     // DevCounters::err: an asynchronous batch's claims did not settle
// k_reg_minwin for an asynchronous batch: also flags claims still deferred after the last gated pass
// (ERR_UNSETTLED) and zeroes pass 0's counter for the next batch.
static __global__ void __launch_bounds__(BLOCK) k_reg_minwin_gated(const uint32_t* __restrict__ slot_of,
                                                            const uint8_t* __restrict__ is_new, uint32_t n, Slot* slots,
                                                            uint32_t* retry, DevCounters* ctr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i == 0) {
        if (retry[REG_PASSES - 1]) atomicOr(&ctr->err, ERR_UNSETTLED);
        retry[0] = 0;
    }
    if (i >= n || !is_new[i]) return;
    atomicMin(&slots[slot_of[i]].act, i);
}

__device__ __forceinline__ void reg_claim_item(uint32_t i, const gd_key* __restrict__ keys, Slot* slots,
                                               unsigned long long mask, DevCounters* ctr,
                                               uint32_t* __restrict__ slot_of, uint8_t* __restrict__ is_new,
                                               const gd_val* __restrict__ vals, const TableArgs& vt, uint32_t* retry,
                                               uint32_t& pdist, bool& reused, uint32_t tag,
                                               uint32_t* __restrict__ last) {
    if (vals && !tab_silo_valid(vt, vals[i].silo)) {
        slot_of[i] = NONE32;
        is_new[i] = 0;
        return;
    }
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    unsigned long long s = home_slot(uniform_hash(n0, n1, tcd), mask);
    unsigned long long dist = 0;
    uint32_t res = NONE32;
    uint8_t fresh = 0;
    // The key's first tombstone, reused when the chain does not hold the key (round 6: a directory under
    // continuous RemoveActivation / AddSingleActivation churn no longer fills with tombstones until a
    // rehash).  Every item of one key meets the same first free slot, and a claim is a CAS, so a key is
    // never placed twice; a tombstone taken meanwhile defers the item to the next pass.
    unsigned long long tomb_s = ~0ull, tomb_dist = 0;
    uint32_t tomb_meta = 0;
    // claim slot t (its meta `expected`) for the key: the key, then PENDING with this launch's tag (read
    // as unpublished by this launch's other items; published to later launches by the kernel boundary)
    auto claim = [&](unsigned long long t, uint32_t expected, unsigned long long d) -> bool {
        uint32_t* mp = &slots[t].meta;
        if (!__hip_atomic_compare_exchange_strong(mp, &expected, make_meta(SLOT_CLAIMED, 0), __ATOMIC_RELAXED,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return false;
        if (last) atomicMax(&last[t], ~i);                   // the claimer, readable by this launch's walks
        Slot& sl = slots[t];
        sl.n0 = n0;
        sl.n1 = n1;
        sl.tcd = tcd;
        sl.act = NONE32;
        __hip_atomic_store(mp, make_meta(SLOT_PENDING, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pdist = (uint32_t)d;                                 // max_probe: claim_counters
        return true;
    };
    // the chain holds no copy of the key: take its first tombstone (or report a full table)
    auto take_tomb = [&]() {
        if (tomb_s == ~0ull) {
            atomicOr(&ctr->err, 2u);
        } else if (claim(tomb_s, tomb_meta, tomb_dist)) {
            reused = true;                                   // tomb - 1: claim_counters
            res = (uint32_t)tomb_s;
            fresh = 1;
        } else {
            res = SLOT_RETRY;
            atomicAdd(retry, 1u);
        }
    };
    for (;;) {
        uint32_t* meta_p = &slots[s].meta;
        const uint32_t meta = __hip_atomic_load(meta_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t st = slot_state(meta);
        if (st == SLOT_EMPTY) {
            if (tomb_s != ~0ull) {
                take_tomb();
                break;
            }
            if (claim(s, meta, dist)) {
                res = (uint32_t)s;
                fresh = 1;
                break;
            }
            continue;   // lost the CAS: re-read the same slot
        }
        if (st == SLOT_CLAIMED || (st == SLOT_PENDING && slot_silo(meta) == tag)) {
            // claimed in this launch: its key is not published to this launch, but its claimer is (the slot's
            // election word, written right after the claim): the key's twin -- join it -- or another key's
            // claim -- walk on.  Only a claim not yet recorded defers.
            const uint32_t w = last ? __hip_atomic_load(&last[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            if (w == 0) {
                res = SLOT_RETRY;
                atomicAdd(retry, 1u);
                break;
            }
            const gd_key& c = keys[~w];
            if (c.n0 == n0 && c.n1 == n1 && c.type_code_data == tcd) {
                res = (uint32_t)s;
                fresh = 1;
                break;
            }
        }
        const bool unpublished = st == SLOT_CLAIMED || (st == SLOT_PENDING && slot_silo(meta) == tag);
        if (st == SLOT_TOMB && tomb_s == ~0ull) {
            tomb_s = s;
            tomb_meta = meta;
            tomb_dist = dist;
        }
        if (!unpublished && (st == SLOT_LIVE || st == SLOT_PENDING)) {   // a key published before this launch
            const uint64_t k0 = slots[s].n0, k1 = slots[s].n1, k2 = slots[s].tcd;
            if (k0 == n0 && k1 == n1 && k2 == tcd) {
                res = (uint32_t)s;
                fresh = (st == SLOT_PENDING) ? 1 : 0;
                break;
            }
        }
        s = (s + 1) & mask;
        if (++dist > mask) {
            take_tomb();
            break;
        }
    }
    slot_of[i] = res;
    is_new[i] = fresh;
}

// Phase 2: the lowest batch index among the items of a new entry wins (sequential
// "first registration wins" order).
static __global__ void __launch_bounds__(BLOCK) k_reg_minwin(const uint32_t* __restrict__ slot_of,
                                                      const uint8_t* __restrict__ is_new, uint32_t n, Slot* slots) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || !is_new[i]) return;
    atomicMin(&slots[slot_of[i]].act, i);   // is_new implies a real slot index
}

static __global__ void __launch_bounds__(BLOCK) k_reg_resolve(const uint32_t* __restrict__ slot_of,
                                                       const uint8_t* __restrict__ is_new, uint32_t n,
                                                       const Slot* slots, uint32_t* __restrict__ win) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    win[i] = is_new[i] ? slots[slot_of[i]].act : NONE32;
}

__device__ __forceinline__ void reg_commit_item(uint32_t i, const uint32_t* __restrict__ slot_of,
                                                const gd_val* __restrict__ vals, Slot* slots, DevCounters* ctr,
                                                uint32_t* __restrict__ vtag, uint32_t op);
// live (+1 an insert, or -1 and tomb +1 a removal) for the wave's flagged lanes, one atomic each a wave.
// Every lane of the wave calls it.
__device__ __forceinline__ void live_delta(DevCounters* ctr, bool flag, bool removal) {
    const unsigned long long m = __ballot(flag);
    if ((threadIdx.x & (WAVE - 1)) != 0 || !m) return;
    const unsigned long long c = (unsigned long long)__popcll(m);
    unsigned long long* st = ctr_stripe(ctr);        // folded into live / tomb by k_ctr_fold
    atomicAdd(st, removal ? ~c + 1ull : c);
    if (removal) atomicAdd(st + 1, c);
}
static __global__ void __launch_bounds__(BLOCK) k_reg_commit(const uint32_t* __restrict__ slot_of,
                                                      const uint32_t* __restrict__ win,
                                                      const gd_val* __restrict__ vals, uint32_t n, Slot* slots,
                                                      DevCounters* ctr, uint32_t* __restrict__ vtag, uint32_t op) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool w = i < n && win[i] == i;
    if (w) reg_commit_item(i, slot_of, vals, slots, ctr, vtag, op);
    live_delta(ctr, w, false);
}
// The commit of a batch elected by `last` (k_reg_take / the claim passes): item i commits when it holds its
// slot's word (~i), clears the word for the next batch, and records win[i] (i or NONE32) for k_reg_report.
// unsettled (optional): the last gated pass's deferred count -- a batch still unsettled flags ERR_UNSETTLED
// -- and retry0, zeroed here for the next batch (k_reg_take counts into it).
__device__ __forceinline__ bool reg_elected(uint32_t i, uint32_t n, const uint32_t* __restrict__ slot_of,
                                            const uint8_t* __restrict__ is_new, uint32_t* __restrict__ last,
                                            uint32_t* __restrict__ win) {
    if (i >= n) return false;
    bool w = false;
    if (is_new[i]) {
        const uint32_t s = slot_of[i];
        w = last[s] == ~i;
        if (w) last[s] = 0;                              // losers read ~winner or 0: never their own
    }
    win[i] = w ? i : NONE32;
    return w;
}
__device__ __forceinline__ void reg_commit_item(uint32_t i, const uint32_t* __restrict__ slot_of,
                                                const gd_val* __restrict__ vals, Slot* slots, DevCounters* ctr,
                                                uint32_t* __restrict__ vtag, uint32_t op) {
    Slot& sl = slots[slot_of[i]];
    if (vals[i].silo > 0xFFFEu) atomicOr(&ctr->err, 4u);   // silo index out of range (device-side values)
    sl.act = vals[i].act;
    sl.meta = make_meta(SLOT_LIVE, vals[i].silo);
    // GrainInfo.AddSingleActivation: SingleInstance = true, VersionTag = rand.Next() (:110-124)
    if (vtag) vtag[slot_of[i]] = VTAG_SINGLE | version_tag(op, uniform_hash(sl.n0, sl.n1, sl.tcd));
}

static __global__ void __launch_bounds__(BLOCK) k_reg_commit_elect(const uint32_t* __restrict__ slot_of,
                                                            const uint8_t* __restrict__ is_new,
                                                            const gd_val* __restrict__ vals, uint32_t n, Slot* slots,
                                                            DevCounters* ctr, uint32_t* __restrict__ vtag, uint32_t op,
                                                            uint32_t* __restrict__ last, uint32_t* __restrict__ win,
                                                            const uint32_t* __restrict__ unsettled,
                                                            uint32_t* __restrict__ retry0) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i == 0 && unsettled) {
        if (*unsettled) atomicOr(&ctr->err, ERR_UNSETTLED);
        *retry0 = 0;                                     // k_reg_take's counter, for the next batch
    }
    const bool w = reg_elected(i, n, slot_of, is_new, last, win);
    if (w) reg_commit_item(i, slot_of, vals, slots, ctr, vtag, op);
    live_delta(ctr, w, false);
}


// gd_dir_upsert: the last batch item of each slot wins (batch order), then writes its value.
// `last` (one u32 per table slot, zero between calls) holds 1 + the winning index.
static __global__ void __launch_bounds__(BLOCK) k_up_last(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                   uint32_t* __restrict__ last) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || slot_of[i] >= SLOT_RETRY) return;
    atomicMax(&last[slot_of[i]], i + 1);
}
static __global__ void __launch_bounds__(BLOCK) k_up_apply(const uint32_t* __restrict__ slot_of,
                                                    const uint8_t* __restrict__ is_new, const gd_val* __restrict__ vals,
                                                    uint32_t n, const uint32_t* __restrict__ last, Slot* slots,
                                                    DevCounters* ctr, uint8_t* __restrict__ out_inserted,
                                                    uint32_t* __restrict__ vtag, uint32_t op) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    uint8_t ins = 0;
    if (s < SLOT_RETRY && last[s] == i + 1) {
        Slot& sl = slots[s];
        // GrainInfo.AddActivation (:89-108): a new tag unless the same activation is refreshed on the
        // same silo; the entry is no longer in single-instance mode
        const bool same = !is_new[i] && sl.act == vals[i].act && slot_silo(sl.meta) == vals[i].silo;
        if (vtag && !same) vtag[s] = version_tag(op, uniform_hash(sl.n0, sl.n1, sl.tcd));
        sl.act = vals[i].act;
        sl.meta = make_meta(SLOT_LIVE, vals[i].silo);
        if (is_new[i]) {
            atomicAdd(&ctr->live, 1ull);
            ins = 1;
        }
    }
    out_inserted[i] = ins;
}
static __global__ void __launch_bounds__(BLOCK) k_up_clear(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                    uint32_t* __restrict__ last) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n && slot_of[i] < SLOT_RETRY) last[slot_of[i]] = 0;
}

static __global__ void __launch_bounds__(BLOCK) k_reg_report(const uint32_t* __restrict__ slot_of,
                                                      const uint32_t* __restrict__ win, uint32_t n,
                                                      const Slot* slots, gd_val* __restrict__ out_vals,
                                                      uint8_t* __restrict__ out_inserted) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    if (s >= SLOT_RETRY) {
        if (out_vals) out_vals[i] = gd_val{NONE32, NONE32};
        if (out_inserted) out_inserted[i] = 0;
        return;
    }
    const Slot sl = slots[s];
    if (out_vals) out_vals[i] = gd_val{sl.act, slot_silo(sl.meta)};
    if (out_inserted) out_inserted[i] = (win[i] == i) ? 1 : 0;
}

// RemoveActivation (GrainDirectoryPartition.cs:335-363, Force): find the live entry
// whose single activation matches; the first matching item of the batch removes it.
static __global__ void __launch_bounds__(BLOCK) k_unreg_find(const gd_key* __restrict__ keys,
                                                      const uint32_t* __restrict__ acts, uint32_t n,
                                                      const Slot* slots, unsigned long long mask,
                                                      const DevCounters* ctr, uint32_t* __restrict__ slot_of) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    const uint32_t h = uniform_hash(n0, n1, tcd);
    unsigned long long s = home_slot(h, mask);
    uint32_t res = NONE32;
    for (uint32_t p = 0; p <= ctr->max_probe; ++p) {
        const Slot sl = slots[s];
        const uint32_t st = slot_state(sl.meta);
        if (st == SLOT_EMPTY) break;
        if (st == SLOT_LIVE && sl.n0 == n0 && sl.n1 == n1 && sl.tcd == tcd) {
            if (sl.act == acts[i]) res = (uint32_t)s;
            break;
        }
        s = (s + 1) & mask;
    }
    slot_of[i] = res;
}

// RemoveActivation with the election in a per-slot word (round 6: 2 launches instead of 4): the find also
// elects the first matching item of the batch (atomicMax(~i)), the commit tombstones the slot for the
// elected item and clears the word.
__device__ __forceinline__ void unreg_find_elect_item(uint32_t i, const gd_key* __restrict__ keys,
                                                      const uint32_t* __restrict__ acts, const Slot* slots,
                                                      unsigned long long mask, const DevCounters* ctr,
                                                      uint32_t* __restrict__ slot_of, uint32_t* __restrict__ last) {
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    unsigned long long s = home_slot(uniform_hash(n0, n1, tcd), mask);
    uint32_t res = NONE32;
    for (uint32_t p = 0; p <= ctr->max_probe; ++p) {
        const uint4* q = reinterpret_cast<const uint4*>(slots + s);
        const uint4 a = q[0], b = q[1];
        const uint32_t st = slot_state(b.w);
        if (st == SLOT_EMPTY) break;
        if (st == SLOT_LIVE && ((uint64_t)a.x | ((uint64_t)a.y << 32)) == n0 &&
            ((uint64_t)a.z | ((uint64_t)a.w << 32)) == n1 && ((uint64_t)b.x | ((uint64_t)b.y << 32)) == tcd) {
            if (b.z == acts[i]) res = (uint32_t)s;
            break;
        }
        s = (s + 1) & mask;
    }
    slot_of[i] = res;
    if (res != NONE32) atomicMax(&last[res], ~i);
}
static __global__ void __launch_bounds__(BLOCK) k_unreg_find_elect(const gd_key* __restrict__ keys,
                                                            const uint32_t* __restrict__ acts, uint32_t n,
                                                            const Slot* slots, unsigned long long mask,
                                                            const DevCounters* ctr, uint32_t* __restrict__ slot_of,
                                                            uint32_t* __restrict__ last) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) unreg_find_elect_item(i, keys, acts, slots, mask, ctr, slot_of, last);
}
__device__ __forceinline__ bool unreg_elected_commit(uint32_t i, uint32_t n, const uint32_t* __restrict__ slot_of,
                                                     Slot* slots, uint32_t* __restrict__ last,
                                                     uint8_t* __restrict__ out_removed) {
    if (i >= n) return false;
    const uint32_t s = slot_of[i];
    const bool rm = s != NONE32 && last[s] == ~i;
    if (rm) {
        slots[s].meta = make_meta(SLOT_TOMB, 0);
        last[s] = 0;
    }
    if (out_removed) out_removed[i] = rm ? 1 : 0;
    return rm;
}
static __global__ void __launch_bounds__(BLOCK) k_unreg_commit_elect(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                              Slot* slots, DevCounters* ctr,
                                                              uint32_t* __restrict__ last,
                                                              uint8_t* __restrict__ out_removed) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    live_delta(ctr, unreg_elected_commit(i, n, slot_of, slots, last, out_removed), true);
}

// The matched entry is being removed, so its n0 word can carry the election.
static __global__ void __launch_bounds__(BLOCK) k_unreg_poison(const uint32_t* __restrict__ slot_of, uint32_t n, Slot* slots) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || slot_of[i] == NONE32) return;
    slots[slot_of[i]].n0 = ~0ull;
}

static __global__ void __launch_bounds__(BLOCK) k_unreg_min(const uint32_t* __restrict__ slot_of, uint32_t n, Slot* slots) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || slot_of[i] == NONE32) return;
    atomicMin(reinterpret_cast<unsigned long long*>(&slots[slot_of[i]].n0), (unsigned long long)i);
}

__device__ __forceinline__ bool unreg_commit_item(uint32_t i, const uint32_t* __restrict__ slot_of, Slot* slots,
                                                  DevCounters* ctr, uint8_t* __restrict__ out_removed) {
    const uint32_t s = slot_of[i];
    uint8_t removed = 0;
    if (s != NONE32 && slots[s].n0 == (uint64_t)i) {
        slots[s].meta = make_meta(SLOT_TOMB, 0);       // live - 1, tomb + 1: the kernel's live_delta
        removed = 1;
    }
    if (out_removed) out_removed[i] = removed;
    return removed != 0;
}
static __global__ void __launch_bounds__(BLOCK) k_unreg_commit(const uint32_t* __restrict__ slot_of, uint32_t n,
                                                        Slot* slots, DevCounters* ctr,
                                                        uint8_t* __restrict__ out_removed) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool rm = i < n && unreg_commit_item(i, slot_of, slots, ctr, out_removed);
    live_delta(ctr, rm, true);
}

static __global__ void __launch_bounds__(BLOCK) k_dir_lookup(const gd_key* __restrict__ keys, uint32_t n, TableArgs tab,
                                                      gd_val* __restrict__ out_vals, uint8_t* __restrict__ found) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    uint32_t act, meta;
    const bool hit = probe(tab.slots, tab.mask, tab.ctr->max_probe, uniform_hash(n0, n1, tcd), n0, n1, tcd, act, meta);
    out_vals[i] = hit ? gd_val{act, slot_silo(meta)} : gd_val{NONE32, NONE32};
    found[i] = hit ? 1 : 0;
}

// Rebuild: every live entry of the old table into the new one (keys are distinct,
// so a claimer never needs to compare keys).
static __global__ void __launch_bounds__(BLOCK) k_rehash(const Slot* __restrict__ old_slots, unsigned long long old_cap,
                                                  Slot* slots, unsigned long long mask, DevCounters* ctr,
                                                  const uint32_t* __restrict__ old_vtag, uint32_t* __restrict__ vtag) {
    const unsigned long long j = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t pd = 0;
    bool placed = false;
    const Slot sl = j < old_cap ? old_slots[j] : Slot{};
    if (j < old_cap && slot_state(sl.meta) == SLOT_LIVE) {
        unsigned long long s = home_slot(uniform_hash(sl.n0, sl.n1, sl.tcd), mask);
        for (uint32_t dist = 0; dist <= mask; ++dist) {
            uint32_t expected = make_meta(SLOT_EMPTY, 0);
            if (__hip_atomic_compare_exchange_strong(&slots[s].meta, &expected, make_meta(SLOT_CLAIMED, 0),
                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                slots[s].n0 = sl.n0;
                slots[s].n1 = sl.n1;
                slots[s].tcd = sl.tcd;
                slots[s].act = sl.act;
                if (vtag) vtag[s] = old_vtag[j];
                __hip_atomic_store(&slots[s].meta, sl.meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                pd = dist;
                placed = true;
                break;
            }
            s = (s + 1) & mask;
        }
        if (!placed) atomicOr(&ctr->err, 2u);
    }
    // one max_probe / live update a wave (one an entry queued 10^6 same-address atomics at cfg 2)
    claim_counters(ctr, pd, false);
    live_delta(ctr, placed, false);
}

// ------------------------------------------------------------------ wave helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Lanes of the wave holding the same BITS-bit digit (match_any by ballots).
template <int BITS>
__device__ __forceinline__ unsigned long long match_digit(uint32_t d, bool valid) {
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

// ------------------------------------------------------------------ K3: stable radix partition
// LSD passes, reduce-then-scan (no in-kernel waiting between workgroups: on
// gfx950 every cross-CU hand-off round-trips through the memory side, which a
// chained look-back pays per step; a kernel boundary costs ~1.5 us once).
// Tile = NT*IT consecutive positions.  Per pass:
//   k_radix_hist    per-tile digit counts, stored digit-major hist[d * tiles + t]
//   scan            one exclusive scan gives every (digit, tile) its global base
//   k_radix_scatter stable rank in the tile (wave-striped order = index order),
//                   stage the tile in LDS in digit order, write each digit run
//                   contiguously.

// Block-wide exclusive add-scan of one value per thread (NTH threads).
template <int NTH>
__device__ __forceinline__ uint32_t block_excl_scan_add_n(uint32_t v, uint32_t* s_wsum) {
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, WAVE);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == WAVE - 1) s_wsum[w] = x;
    __syncthreads();
    uint32_t wbase = 0;
#pragma unroll
    for (int k = 0; k < NTH / WAVE; ++k)
        if ((uint32_t)k < w) wbase += s_wsum[k];
    __syncthreads();
    return wbase + x - v;
}

// Two block-wide exclusive add-scans (one value each per thread) sharing one pair of barriers.
template <int NTH>
__device__ __forceinline__ void block_excl_scan_add2(uint32_t a, uint32_t b, uint32_t* s_wsum2, uint32_t& ea,
                                                     uint32_t& eb) {
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    uint32_t x = a, y = b;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        const uint32_t xa = __shfl_up(x, off, WAVE), yb = __shfl_up(y, off, WAVE);
        if (lane >= (uint32_t)off) {
            x += xa;
            y += yb;
        }
    }
    if (lane == WAVE - 1) {
        s_wsum2[w] = x;
        s_wsum2[NTH / WAVE + w] = y;
    }
    __syncthreads();
    uint32_t wa = 0, wb = 0;
#pragma unroll
    for (int k = 0; k < NTH / WAVE; ++k)
        if ((uint32_t)k < w) {
            wa += s_wsum2[k];
            wb += s_wsum2[NTH / WAVE + k];
        }
    __syncthreads();
    ea = wa + x - a;
    eb = wb + y - b;
}

// p[0..n) = v by the whole grid, at the end of a kernel that has other work: the first pass's
// histogram pre-fills the bucket starts this way (one launch fewer per bucketing).
struct FillArgs {
    uint32_t* p;
    uint32_t n, v;
};
__device__ __forceinline__ void fill_grid(const FillArgs& f, uint32_t nt) {
    if (!f.p) return;
    for (uint32_t i = blockIdx.x * nt + threadIdx.x; i < f.n; i += gridDim.x * nt) f.p[i] = f.v;
}

// Histogram.  Keys are read 16 B per lane (order is irrelevant here).  Equal
// digits within a wave instruction: the lanes sharing the first active lane's
// digit (the hot key under Zipf skew) are folded into one LDS atomic.
template <int BITS, int NT, int IT>
static __global__ void __launch_bounds__(NT) k_radix_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t clamp,
                                                   uint32_t shift, uint32_t tiles, uint32_t* __restrict__ hist,
                                                   FillArgs fill) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int NW = NT / WAVE;
    constexpr uint32_t TILE = NT * IT;
    static_assert(IT % 4 == 0, "16-B loads");
    __shared__ uint32_t s_cnt[NW * R];
    for (uint32_t d = threadIdx.x; d < NW * R; d += NT) s_cnt[d] = 0;
    __syncthreads();
    uint32_t* my_cnt = s_cnt + (threadIdx.x / WAVE) * R;
    const uint32_t base = blockIdx.x * TILE;
    const uint32_t lane = lane_id();
    const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0 && base + TILE <= n;
    uint32_t k[IT];
#pragma unroll
    for (int j = 0; j < IT / 4; ++j) {
        const uint32_t i0 = base + 4 * (j * NT + threadIdx.x);
        if (vec) {
            const uint4 v = *reinterpret_cast<const uint4*>(keys + i0);
            k[4 * j] = v.x; k[4 * j + 1] = v.y; k[4 * j + 2] = v.z; k[4 * j + 3] = v.w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) k[4 * j + q] = (i0 + q < n) ? keys[i0 + q] : NONE32;
        }
    }
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t i = base + 4 * ((j / 4) * NT + threadIdx.x) + (j % 4);
        const bool valid = i < n;
        const uint32_t d = (min(k[j], clamp) >> shift) & (R - 1);
        const unsigned long long act = __ballot(valid);
        if (act == 0) continue;
        const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1;
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead);
        const unsigned long long hot = __ballot(valid && d == d0);
        if (valid) {
            if (d != d0) atomicAdd(&my_cnt[d], 1u);
            else if (lane == lead) atomicAdd(&my_cnt[d], (uint32_t)__popcll(hot));
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += NT) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) c += s_cnt[w * R + d];
        hist[d * tiles + blockIdx.x] = c;
    }
    fill_grid(fill, NT);
}

// First tile of a TPB-tile histogram workgroup.  xcd_rev: workgroup b runs on XCD b % 8 (round-robin
// dispatch) and counts tiles from the XCD's range of the scatter's tile order (xcd_tile) in reverse,
// so the tiles the XCD's scatter workgroups read first are the ones its histogram read last -- still
// in that XCD's L2.  Only when the ranges split evenly (tiles a multiple of 8 * TPB).
__device__ __forceinline__ uint32_t hist_t0(uint32_t b, uint32_t nb, uint32_t tpb, uint32_t tiles, uint32_t xcd_rev) {
    if (!xcd_rev || (tiles % (8u * tpb)) != 0 || (nb & 7u) != 0) return b * tpb;
    const uint32_t per = nb >> 3, x = b & 7u, g = b >> 3;
    return (x * per + (per - 1u - g)) * tpb;
}

// Multi-tile histogram: one workgroup counts TPB consecutive tiles, with every tile's 16-B key
// loads issued before the first count, and one counter set per tile shared by the waves.  The
// digit-major counts it writes for one digit are then TPB consecutive words, instead of one word
// every `tiles` words per workgroup.  Same output as k_radix_hist.
template <int BITS, int NT, int IT, int TPB>
static __global__ void __launch_bounds__(NT) k_radix_hist_multi(const uint32_t* __restrict__ keys, uint32_t n,
                                                         uint32_t clamp, uint32_t shift, uint32_t tiles,
                                                         uint32_t* __restrict__ hist, FillArgs fill,
                                                         uint32_t xcd_rev) {
    constexpr uint32_t R = 1u << BITS;
    constexpr uint32_t TILE = NT * IT;
    static_assert(IT % 4 == 0, "16-B loads");
    __shared__ uint32_t s_cnt[TPB][R];
    for (uint32_t x = threadIdx.x; x < TPB * R; x += NT) (&s_cnt[0][0])[x] = 0;
    __syncthreads();
    const uint32_t t0 = hist_t0(blockIdx.x, gridDim.x, TPB, tiles, xcd_rev);
    const uint32_t lane = lane_id();
    const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0;
    uint32_t k[TPB][IT];
    // One workgroup-uniform branch: in a full, aligned range every 16-B load is unconditional, so
    // all TPB * IT / 4 of them are issued before the first wait (a per-tile branch around them
    // makes the compiler wait at each).
    if (aligned && (uint64_t)(t0 + TPB) * TILE <= n) {
#pragma unroll
        for (int t = 0; t < TPB; ++t)
#pragma unroll
            for (int j = 0; j < IT / 4; ++j) {
                const uint64_t i0 = (uint64_t)(t0 + t) * TILE + 4 * (j * NT + threadIdx.x);
                const uint4 v = *reinterpret_cast<const uint4*>(keys + i0);
                k[t][4 * j] = v.x; k[t][4 * j + 1] = v.y; k[t][4 * j + 2] = v.z; k[t][4 * j + 3] = v.w;
            }
    } else {
#pragma unroll
        for (int t = 0; t < TPB; ++t)
#pragma unroll
            for (int j = 0; j < IT / 4; ++j) {
                const uint64_t i0 = (uint64_t)(t0 + t) * TILE + 4 * (j * NT + threadIdx.x);
#pragma unroll
                for (int q = 0; q < 4; ++q) k[t][4 * j + q] = (i0 + q < n) ? keys[i0 + q] : NONE32;
            }
    }
#pragma unroll
    for (int t = 0; t < TPB; ++t) {
        const uint64_t base = (uint64_t)(t0 + t) * TILE;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint64_t i = base + 4 * ((j / 4) * NT + threadIdx.x) + (j % 4);
            const bool valid = i < n;
            const uint32_t d = (min(k[t][j], clamp) >> shift) & (R - 1);
            const unsigned long long act = __ballot(valid);
            if (act == 0) continue;
            const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1;
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead);
            const unsigned long long hot = __ballot(valid && d == d0);
            if (valid) {
                if (d != d0) atomicAdd(&s_cnt[t][d], 1u);
                else if (lane == lead) atomicAdd(&s_cnt[t][d], (uint32_t)__popcll(hot));
            }
        }
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < TPB * R; x += NT) {
        const uint32_t t = x % TPB, d = x / TPB;
        if (t0 + t < tiles) hist[d * tiles + t0 + t] = s_cnt[t][d];
    }
    fill_grid(fill, NT);
}

// Histogram of a packed pass (k_radix_scatter with Pack::in): the key bits above the first pass's
// digit are a u16 array (8 keys per 16-B load), already clamped by the first pass.  TPB tiles per
// workgroup as k_radix_hist_multi (TPB = 1: k_radix_hist's layout).  Same output as those for the
// full keys.
template <int BITS, int NT, int IT, int TPB>
static __global__ void __launch_bounds__(NT) k_radix_hist16(const uint16_t* __restrict__ keys, uint32_t n, uint32_t shift,
                                                     uint32_t tiles, uint32_t* __restrict__ hist, uint32_t xcd_rev) {
    constexpr uint32_t R = 1u << BITS;
    constexpr uint32_t TILE = NT * IT;
    static_assert(IT % 8 == 0, "16-B loads of 8 keys");
    __shared__ uint32_t s_cnt[TPB][R];
    for (uint32_t x = threadIdx.x; x < TPB * R; x += NT) (&s_cnt[0][0])[x] = 0;
    __syncthreads();
    const uint32_t t0 = hist_t0(blockIdx.x, gridDim.x, TPB, tiles, xcd_rev);
    const uint32_t lane = lane_id();
    const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0;
    uint32_t k[TPB][IT];
    if (aligned && (uint64_t)(t0 + TPB) * TILE <= n) {
#pragma unroll
        for (int t = 0; t < TPB; ++t)
#pragma unroll
            for (int j = 0; j < IT / 8; ++j) {
                const uint64_t i0 = (uint64_t)(t0 + t) * TILE + 8 * (j * NT + threadIdx.x);
                const uint4 v = *reinterpret_cast<const uint4*>(keys + i0);
                const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    k[t][8 * j + 2 * q] = u[q] & 0xFFFFu;
                    k[t][8 * j + 2 * q + 1] = u[q] >> 16;
                }
            }
    } else {
#pragma unroll
        for (int t = 0; t < TPB; ++t)
#pragma unroll
            for (int j = 0; j < IT / 8; ++j) {
                const uint64_t i0 = (uint64_t)(t0 + t) * TILE + 8 * (j * NT + threadIdx.x);
#pragma unroll
                for (int q = 0; q < 8; ++q) k[t][8 * j + q] = (i0 + q < n) ? keys[i0 + q] : 0u;
            }
    }
#pragma unroll
    for (int t = 0; t < TPB; ++t) {
        const uint64_t base = (uint64_t)(t0 + t) * TILE;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint64_t i = base + 8 * ((j / 8) * NT + threadIdx.x) + (j % 8);
            const bool valid = i < n;
            const uint32_t d = (k[t][j] >> shift) & (R - 1);
            const unsigned long long act = __ballot(valid);
            if (act == 0) continue;
            const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1;
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead);
            const unsigned long long hot = __ballot(valid && d == d0);
            if (valid) {
                if (d != d0) atomicAdd(&s_cnt[t][d], 1u);
                else if (lane == lead) atomicAdd(&s_cnt[t][d], (uint32_t)__popcll(hot));
            }
        }
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < TPB * R; x += NT) {
        const uint32_t t = x % TPB, d = x / TPB;
        if (t0 + t < tiles) hist[d * tiles + t0 + t] = s_cnt[t][d];
    }
}


// Packed records between radix passes (bucket_device, when the key bits above the first pass's
// digit fit 16 bits and the message index fits beside that digit in 32): A = (key's low b1 bits)
// << ib | index, in the keys array, and B = key >> b1 as u16, in the values array.  6 B a record
// instead of 8, and the later histograms read B alone (2 B).  in: this pass reads packed records;
// out: it writes them (never the last pass, which writes the permutation and the starts).
struct Pack {
    uint32_t ib, b1;
    bool in, out;
};

// Downsweep.  FIRST: values are the message indices themselves.  The keys are
// clamped to `clamp` (unrouted messages -> trailing bucket).
// starts != nullptr (the last pass): the output is fully sorted, so instead of the keys the
// pass writes bucket starts -- the first item of each key in a tile's digit run (the run is
// sorted by the whole key: the lower passes ordered it) lowers starts[key] to its output
// position with atomicMin; the earliest tile holding the key wins (starts pre-filled with n).
template <int BITS, bool FIRST, int NT, int IT>
static __global__ void __launch_bounds__(NT) k_radix_scatter(const uint32_t* __restrict__ keys_in,
                                                      const uint32_t* __restrict__ vals_in, uint32_t n,
                                                      uint32_t clamp, uint32_t shift, uint32_t tiles,
                                                      const uint32_t* __restrict__ gscan,
                                                      uint32_t* __restrict__ keys_out,
                                                      uint32_t* __restrict__ vals_out, uint32_t rank_atomic,
                                                      uint32_t* __restrict__ starts, uint32_t xcd,
                                                      uint32_t* __restrict__ rank_out,
                                                      const uint32_t* __restrict__ totals, Pack pk) {
    constexpr uint32_t R = 1u << BITS;
    constexpr int NW = NT / WAVE;
    constexpr uint32_t TILE = NT * IT;
    __shared__ uint32_t s_wcnt[NW][R];
    __shared__ uint32_t s_lstart[R];
    __shared__ uint32_t s_gbase[R];
    __shared__ uint2 s_kv[TILE];
    __shared__ uint32_t s_wsum[2 * NW];

    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x, xcd);
    const uint32_t base = tile * TILE;
    const uint32_t cnt_tile = min(TILE, n - base);
    for (uint32_t d = threadIdx.x; d < R; d += NT) {
#pragma unroll
        for (int w = 0; w < NW; ++w) s_wcnt[w][d] = 0;
        s_gbase[d] = gscan[d * tiles + tile];
    }
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    // thread t owns digits [t*DPT, (t+1)*DPT) in the digit-total scans below
    constexpr uint32_t DPT = (R + NT - 1) / NT;
    uint32_t rk[IT], kk[IT], vv[IT];
    // Branch-free loads (clamped index, masked after): a per-item `if (valid)` around
    // each load makes hipcc wait vmcnt(0) after every one of them.
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t idx = base + (w * IT + r) * WAVE + lane;
        const uint32_t li = min(idx, n - 1);
        kk[r] = __builtin_nontemporal_load(keys_in + li);          // read once: stream past the caches
        if constexpr (!FIRST) {
            if (pk.in) vv[r] = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(vals_in) + li);
            else vv[r] = __builtin_nontemporal_load(vals_in + li);
        }
    }
    if constexpr (!FIRST)
        if (pk.in) {                       // (A, B) -> (key, index)
            const uint32_t imask = (1u << pk.ib) - 1u;
#pragma unroll
            for (int r = 0; r < IT; ++r) {
                const uint32_t a = kk[r];
                kk[r] = (vv[r] << pk.b1) | (a >> pk.ib);
                vv[r] = a & imask;
            }
        }
    // totals != nullptr: k_radix_rowscan left gscan per digit row only, and the digit's base (the
    // exclusive prefix of the R row totals) is added below, in the tile-local digit scan; the
    // totals are loaded here, beside the keys
    uint32_t tv[DPT], my_g = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t d = threadIdx.x * DPT + q;
        tv[q] = totals && d < R ? totals[d] : 0u;
        my_g += tv[q];
    }
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t idx = base + (w * IT + r) * WAVE + lane;
        kk[r] = idx < n ? min(kk[r], clamp) : 0u;
        if constexpr (FIRST) vv[r] = idx;
    }
    __syncthreads();
    if (rank_atomic) {
        // One ds_add_rtn per item: lanes of one wave instruction that hit the same counter are
        // served in ascending lane order (checked on gfx950 by tools/ubench_lds_order.hip), and a
        // wave's LDS instructions complete in program order, so the returned count is the stable
        // rank in (row, lane) = index order.
        // The lanes sharing the first valid lane's digit (the hot key under skew) take one
        // counter update by that lane and rank among themselves by ballot; the others use
        // their own ds_add_rtn.  Different digits are different counters, so the two groups
        // do not interact.
        // Issue every row's counter update first (one ds_add_rtn per row: the lead adds the
        // hot group's size, the other non-hot lanes add 1, hot non-lead lanes stay idle), then
        // resolve the hot lanes' ranks: no per-row wait for an LDS result.
        unsigned long long hot[IT];
        uint32_t lead[IT], hd[IT];
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            const uint32_t idx = base + (w * IT + r) * WAVE + lane;
            const bool valid = idx < n;
            const uint32_t d = (kk[r] >> shift) & (R - 1);
            const unsigned long long live = __ballot(valid);
            lead[r] = live ? (uint32_t)__ffsll((long long)live) - 1 : 0u;
            hd[r] = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)lead[r]);
            hot[r] = __ballot(valid && d == hd[r]);
            rk[r] = 0;
            if (valid && (d != hd[r] || lane == lead[r]))
                rk[r] = atomicAdd(&s_wcnt[w][d], lane == lead[r] ? (uint32_t)__popcll(hot[r]) : 1u);
        }
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)rk[r], (int)lead[r]);
            if ((hot[r] >> lane) & 1ull) rk[r] = b0 + (uint32_t)__popcll(hot[r] & lt);
        }
    } else {
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            const uint32_t idx = base + (w * IT + r) * WAVE + lane;
            const bool valid = idx < n;
            const uint32_t d = (kk[r] >> shift) & (R - 1);
            const unsigned long long peers = match_digit<BITS>(d, valid);
            uint32_t c = 0;
            if (valid) c = s_wcnt[w][d];
            rk[r] = c + (uint32_t)__popcll(peers & lt);
            if (valid && (peers & lt) == 0) s_wcnt[w][d] = c + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
    // cross-wave exclusive prefix per digit, then tile-local digit starts
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
            s_lstart[d] = run;          // digit total for now
            my_total += run;
        }
    }
    uint32_t ex, exg;
    block_excl_scan_add2<NT>(my_total, my_g, s_wsum, ex, exg);     // its barrier orders s_gbase's stores
    {
        // one LDS lookup per item on each side below: the waves' prefixes become absolute tile
        // positions (s_wcnt += the digit's tile start), and the write-out's base is gbase - lstart
        uint32_t run = ex, rung = exg;
#pragma unroll
        for (uint32_t q = 0; q < DPT; ++q) {
            const uint32_t d = threadIdx.x * DPT + q;
            if (d < R) {
                const uint32_t t = s_lstart[d];
#pragma unroll
                for (int ww = 0; ww < NW; ++ww) s_wcnt[ww][d] += run;
                s_gbase[d] = s_gbase[d] + (totals ? rung : 0u) - run;
                run += t;
                rung += tv[q];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t idx = base + (w * IT + r) * WAVE + lane;
        if (idx < n) {
            const uint32_t d = (kk[r] >> shift) & (R - 1);
            s_kv[s_wcnt[w][d] + rk[r]] = make_uint2(kk[r], vv[r]);
        }
    }
    __syncthreads();
    // the write-out's LDS reads in batches of WB items (every staged record, then every digit base), not
    // one item's two dependent reads and a wait at a time (as k_b2_scatter / k_seg_scatter; past the tile
    // the records are stale LDS, masked to a digit, and nothing is stored)
    constexpr int WB = IT < 8 ? IT : 8;
#pragma unroll
    for (int j0 = 0; j0 < IT; j0 += WB) {
    uint2 kq[WB];
    uint32_t gq[WB];
#pragma unroll
    for (int u = 0; u < WB; ++u) kq[u] = s_kv[(j0 + u) * NT + threadIdx.x];
#pragma unroll
    for (int u = 0; u < WB; ++u) gq[u] = s_gbase[(kq[u].x >> shift) & (R - 1)] + (j0 + u) * NT + threadIdx.x;
#pragma unroll
    for (int u = 0; u < WB; ++u) {
        const uint32_t p = (j0 + u) * NT + threadIdx.x;
        if (p < cnt_tile) {
            const uint2 kv = kq[u];
            const uint32_t g = gq[u];                // s_gbase holds the digit's global base - its tile start
            if (g < n) {            // always true when the scan is right; never write out of bounds
                if (starts) {
                    // a key's first item in the tile: the item before it holds another key (a digit
                    // boundary is a key boundary too)
                    if (p == 0 || s_kv[p - 1].x != kv.x) atomicMin(&starts[kv.x], g);
                    vals_out[g] = kv.y;
                } else if (pk.out) {
                    keys_out[g] = ((kv.x & ((1u << pk.b1) - 1u)) << pk.ib) | kv.y;
                    reinterpret_cast<uint16_t*>(vals_out)[g] = (uint16_t)(kv.x >> pk.b1);
                } else {
                    keys_out[g] = kv.x;
                    vals_out[g] = kv.y;
                }
                if (rank_out) rank_out[kv.y] = g;     // the inverse permutation (last pass, on request)
            }
        }
    }
    }
}

// offsets[k] = first position of key k in the sorted keys (others stay at the fill
// value and are fixed by a reverse min-scan).
static __global__ void __launch_bounds__(BLOCK) k_bucket_starts(const uint32_t* __restrict__ skeys, uint32_t n,
                                                         uint32_t* __restrict__ offsets) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = skeys[i];
    if (i == 0 || skeys[i - 1] != k) offsets[k] = i;
}

static __global__ void k_fill_u32(uint32_t* __restrict__ p, uint32_t n, uint32_t v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// ------------------------------------------------------------------ device-wide scan
struct OpAdd {
    static constexpr uint32_t identity = 0u;
    __device__ static uint32_t apply(uint32_t a, uint32_t b) { return a + b; }
};
struct OpMin {
    static constexpr uint32_t identity = 0xFFFFFFFFu;
    __device__ static uint32_t apply(uint32_t a, uint32_t b) { return min(a, b); }
};

template <class Op>
__device__ __forceinline__ uint32_t block_reduce(uint32_t v, uint32_t* s_wsum) {
#pragma unroll
    for (int off = WAVE / 2; off > 0; off >>= 1) v = Op::apply(v, __shfl_xor(v, off, WAVE));
    if ((threadIdx.x & (WAVE - 1)) == 0) s_wsum[threadIdx.x / WAVE] = v;
    __syncthreads();
    uint32_t r = Op::identity;
#pragma unroll
    for (int k = 0; k < BLOCK / WAVE; ++k) r = Op::apply(r, s_wsum[k]);
    __syncthreads();
    return r;
}

template <class Op>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wsum) {
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, WAVE);
        if (lane >= (uint32_t)off) x = Op::apply(y, x);
    }
    uint32_t ex = __shfl_up(x, 1, WAVE);
    if (lane == 0) ex = Op::identity;
    if (lane == WAVE - 1) s_wsum[w] = x;
    __syncthreads();
    uint32_t wbase = Op::identity;
#pragma unroll
    for (int k = 0; k < BLOCK / WAVE; ++k)
        if ((uint32_t)k < w) wbase = Op::apply(wbase, s_wsum[k]);
    __syncthreads();
    return Op::apply(wbase, ex);
}

// Tiles are physical: block b scans physical tile T = b (forward) or nb - 1 - b (reverse), and
// thread t the IPT entries at T * IPT * BLOCK + IPT * c with c = t (forward) or BLOCK - 1 - t
// (reverse), taken high to low in a reverse scan.  Every thread's entries are then IPT / 4 aligned
// 16-B loads / stores; a reverse scan meets the entries past n (identity) first, which changes
// nothing.  IPT = 4 (1,024-entry tiles: enough blocks to fill the chip) or 16 (4,096-entry tiles,
// for arrays whose 1,024-entry tiles would be too many aggregates to fold in the down-sweep).
static_assert(SCAN_ITEMS == 4, "scan tiles are read as uint4 per thread");

template <int IPT>
__device__ __forceinline__ uint32_t scan_chunk_base(uint32_t n, bool rev) {
    constexpr uint32_t TILE = BLOCK * IPT;
    const uint32_t nb = (n + TILE - 1) / TILE;
    const uint32_t tile = rev ? nb - 1 - blockIdx.x : blockIdx.x;
    const uint32_t c = rev ? BLOCK - 1 - threadIdx.x : threadIdx.x;
    return tile * TILE + IPT * c;
}

// The thread's IPT entries in scan order (identity past n).
template <class Op, int IPT>
__device__ __forceinline__ void scan_load(const uint32_t* in, uint32_t n, bool rev, uint32_t p0, uint32_t (&v)[IPT]) {
    uint32_t x[IPT];
    if (p0 + IPT - 1 < n && (reinterpret_cast<uintptr_t>(in) & 15) == 0) {
#pragma unroll
        for (int q = 0; q < IPT / 4; ++q) {
            const uint4 u = *reinterpret_cast<const uint4*>(in + p0 + 4 * q);
            x[4 * q] = u.x; x[4 * q + 1] = u.y; x[4 * q + 2] = u.z; x[4 * q + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < IPT; ++k) {                 // clamped loads: no per-item branch
            const uint32_t y = in[min(p0 + k, n - 1)];
            x[k] = p0 + k < n ? y : Op::identity;
        }
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) v[k] = rev ? x[IPT - 1 - k] : x[k];
}

template <class Op, int IPT = SCAN_ITEMS>
static __global__ void __launch_bounds__(BLOCK) k_scan_reduce(const uint32_t* __restrict__ in, uint32_t n, bool rev,
                                                       uint32_t* __restrict__ partials) {
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    uint32_t v[IPT];
    scan_load<Op, IPT>(in, n, rev, scan_chunk_base<IPT>(n, rev), v);
    uint32_t acc = Op::identity;
#pragma unroll
    for (int k = 0; k < IPT; ++k) acc = Op::apply(acc, v[k]);
    acc = block_reduce<Op>(acc, s_wsum);
    if (threadIdx.x == 0) partials[blockIdx.x] = acc;
}

// Exclusive scan of `m` partials in one block (sequential over chunks).
template <class Op>
static __global__ void __launch_bounds__(BLOCK) k_scan_partials(uint32_t* partials, uint32_t m) {
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    __shared__ uint32_t s_carry;
    if (threadIdx.x == 0) s_carry = Op::identity;
    __syncthreads();
    for (uint32_t c = 0; c < m; c += BLOCK) {
        const uint32_t j = c + threadIdx.x;
        const uint32_t v = j < m ? partials[j] : Op::identity;
        const uint32_t ex = block_excl_scan<Op>(v, s_wsum);
        const uint32_t carry = s_carry;
        __syncthreads();
        if (j < m) partials[j] = Op::apply(carry, ex);
        if (threadIdx.x == BLOCK - 1) s_carry = Op::apply(carry, Op::apply(ex, v));
        __syncthreads();
    }
}

template <class Op, int IPT = SCAN_ITEMS>
static __global__ void __launch_bounds__(BLOCK) k_scan_down(const uint32_t* in, uint32_t* out, uint32_t n, bool rev,
                                                     bool inclusive, const uint32_t* __restrict__ partials,
                                                     uint32_t n_partials_raw) {
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    __shared__ uint32_t s_prefix;
    // n_partials_raw > 0: `partials` holds raw block aggregates; fold those of the
    // preceding blocks here instead of a separate single-block scan launch.
    if (n_partials_raw) {
        uint32_t acc = Op::identity;
        for (uint32_t j = threadIdx.x; j < blockIdx.x; j += BLOCK) acc = Op::apply(acc, partials[j]);
        acc = block_reduce<Op>(acc, s_wsum);
        if (threadIdx.x == 0) s_prefix = acc;
    } else if (threadIdx.x == 0) {
        s_prefix = partials[blockIdx.x];
    }
    __syncthreads();
    const uint32_t prefix = s_prefix;
    const uint32_t p0 = scan_chunk_base<IPT>(n, rev);
    uint32_t v[IPT];
    scan_load<Op, IPT>(in, n, rev, p0, v);
    uint32_t acc = Op::identity;
#pragma unroll
    for (int k = 0; k < IPT; ++k) acc = Op::apply(acc, v[k]);
    uint32_t run = Op::apply(prefix, block_excl_scan<Op>(acc, s_wsum));
    uint32_t r[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t next = Op::apply(run, v[k]);
        r[k] = inclusive ? next : run;
        run = next;
    }
    uint32_t x[IPT];                                    // back to physical order
#pragma unroll
    for (int k = 0; k < IPT; ++k) x[k] = rev ? r[IPT - 1 - k] : r[k];
    if (p0 + IPT - 1 < n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
#pragma unroll
        for (int q = 0; q < IPT / 4; ++q)
            *reinterpret_cast<uint4*>(out + p0 + 4 * q) = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < IPT; ++k)
            if (p0 + k < n) out[p0 + k] = x[k];
    }
}

// One workgroup per digit d (the radix pass's counts are digit-major): exclusive add-scan of the
// row hist[d * tiles, (d + 1) * tiles) in place, and the row total into totals[d].  The scatter
// adds the digit's base (the exclusive prefix of the totals) itself, so a pass takes one scan
// launch here instead of a device-wide reduce + down-sweep.
static __global__ void __launch_bounds__(BLOCK) k_radix_rowscan(uint32_t* __restrict__ hist, uint32_t tiles,
                                                         uint32_t* __restrict__ totals) {
    constexpr int IPT = 16;
    constexpr uint32_t CH = BLOCK * IPT;
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    uint32_t* row = hist + (size_t)blockIdx.x * tiles;
    const bool aligned = (reinterpret_cast<uintptr_t>(row) & 15u) == 0;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < tiles; c0 += CH) {
        const uint32_t p0 = c0 + IPT * threadIdx.x;
        const bool vec = aligned && p0 + IPT <= tiles;
        uint32_t v[IPT];
        if (vec) {
#pragma unroll
            for (int q = 0; q < IPT / 4; ++q) {
                const uint4 u = *reinterpret_cast<const uint4*>(row + p0 + 4 * q);
                v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < IPT; ++k) v[k] = p0 + k < tiles ? row[p0 + k] : 0u;
        }
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < IPT; ++k) acc += v[k];
        uint32_t run = carry + block_excl_scan<OpAdd>(acc, s_wsum);
        uint32_t chunk = 0;
#pragma unroll
        for (int k = 0; k < BLOCK / WAVE; ++k) chunk += s_wsum[k];
        uint32_t r[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            r[k] = run;
            run += v[k];
        }
        if (vec) {
#pragma unroll
            for (int q = 0; q < IPT / 4; ++q)
                *reinterpret_cast<uint4*>(row + p0 + 4 * q) = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < IPT; ++k)
                if (p0 + k < tiles) row[p0 + k] = r[k];
        }
        carry += chunk;
        __syncthreads();                    // s_wsum is rewritten by the next chunk's scan
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// The bucket starts' reverse inclusive min-scan in one launch, when the last radix pass's digit
// covers at most RS_RANGE * RS_MAX_SUB activations (1 << shift): workgroup d scans the activations
// [d << shift, (d + 1) << shift) of offsets[0, n_scan) alone, RS_RANGE at a time from the top.  Its
// carry -- the first start past the range -- is the last pass's digit base base(d + 1) = the
// number of messages whose (clamped) key lies below the range's end (n when there is none): the
// starts of non-empty activations increase with the activation, and the empty ones hold n.  Each
// lower sub-range then carries the minimum of the ones above it.
constexpr uint32_t RS_THREADS = 1024;
constexpr uint32_t RS_IPT = 16;
constexpr uint32_t RS_RANGE = RS_THREADS * RS_IPT;      // 16,384 activations per sub-range
constexpr uint32_t RS_MAX_SUB = 16;                      // digit ranges up to 2^18 activations
static __global__ void __launch_bounds__(RS_THREADS) k_starts_rangescan(uint32_t* __restrict__ offsets, uint32_t n_scan,
                                                                 uint32_t shift, const uint32_t* __restrict__ totals,
                                                                 uint32_t n_digits) {
    constexpr uint32_t NW = RS_THREADS / WAVE;
    __shared__ uint32_t s_w[2][NW];
    const uint32_t d = blockIdx.x;
    const uint64_t lo64 = (uint64_t)d << shift;
    if (lo64 >= n_scan) return;                          // workgroup-uniform: an empty top range
    const uint32_t lo = (uint32_t)lo64;
    const uint32_t hi = (uint32_t)min<uint64_t>(lo64 + (1ull << shift), n_scan);
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    // thread t takes chunk c = RS_THREADS - 1 - t of a sub-range, so a forward exclusive scan over
    // the threads is the minimum over the chunks above c.  The next sub-range's loads go out before
    // the current one is scanned (the top one's before the carry is summed).
    const uint32_t c = RS_THREADS - 1 - threadIdx.x;
    const uint32_t n_sub = (hi - lo + RS_RANGE - 1) / RS_RANGE;
    auto load = [&](uint32_t sub, uint32_t (&v)[RS_IPT]) {
        const uint32_t p0 = lo + sub * RS_RANGE + c * RS_IPT;
        if (p0 + RS_IPT <= hi && (reinterpret_cast<uintptr_t>(offsets + p0) & 15u) == 0) {
#pragma unroll
            for (uint32_t q = 0; q < RS_IPT / 4; ++q) {
                const uint4 u = *reinterpret_cast<const uint4*>(offsets + p0 + 4 * q);
                v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < RS_IPT; ++k) v[k] = p0 + k < hi ? offsets[min(p0 + k, n_scan - 1)] : 0xFFFFFFFFu;
        }
    };
    uint32_t v[RS_IPT], nx[RS_IPT];
    load(n_sub - 1, v);
    // base(d + 1), the carry into the range's top
    uint32_t part = 0;
    for (uint32_t j = threadIdx.x; j <= d && j < n_digits; j += RS_THREADS) part += totals[j];
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) part += __shfl_xor(part, off, WAVE);
    if (lane == 0) s_w[1][w] = part;
    __syncthreads();
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t k = 0; k < NW; ++k) carry += s_w[1][k];
    for (uint32_t sub = n_sub; sub-- > 0;) {
        if (sub > 0) load(sub - 1, nx);
        const uint32_t p0 = lo + sub * RS_RANGE + c * RS_IPT;
        const bool vec = p0 + RS_IPT <= hi && (reinterpret_cast<uintptr_t>(offsets + p0) & 15u) == 0;
        uint32_t m = 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t k = 0; k < RS_IPT; ++k) m = min(m, v[k]);
        uint32_t x = m;
#pragma unroll
        for (int off = 1; off < WAVE; off <<= 1) {
            const uint32_t y = __shfl_up(x, off, WAVE);
            if (lane >= (uint32_t)off) x = min(x, y);
        }
        uint32_t ex = __shfl_up(x, 1, WAVE);
        if (lane == 0) ex = 0xFFFFFFFFu;
        if (lane == WAVE - 1) s_w[0][w] = x;
        __syncthreads();
        uint32_t wmin = 0xFFFFFFFFu, bmin = 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t k = 0; k < NW; ++k) {
            const uint32_t t = s_w[0][k];
            if (k < w) wmin = min(wmin, t);
            bmin = min(bmin, t);
        }
        uint32_t run = min(carry, min(wmin, ex));
#pragma unroll
        for (int k = RS_IPT - 1; k >= 0; --k) {
            run = min(run, v[k]);
            v[k] = run;
        }
        if (vec) {
#pragma unroll
            for (uint32_t q = 0; q < RS_IPT / 4; ++q)
                *reinterpret_cast<uint4*>(offsets + p0 + 4 * q) = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        } else {
#pragma unroll
            for (uint32_t k = 0; k < RS_IPT; ++k)
                if (p0 + k < hi) offsets[p0 + k] = v[k];
        }
        carry = min(carry, bmin);
#pragma unroll
        for (uint32_t k = 0; k < RS_IPT; ++k) v[k] = nx[k];
        __syncthreads();                                 // s_w[0] is rewritten by the next sub-range
    }
}

// ------------------------------------------------------------------ micro-batch bucketing (f3)
// One workgroup sorts the whole micro-batch: LSD radix passes of BITS-bit digits (up to 11, so
// 2^20..2^22 activations take 2 passes) of min(act, n_act), each pass ranking stably inside the
// block and exchanging the (key, index) pairs through LDS.  Item (w, r, lane) <-> position
// (w * IT + r) * 64 + lane; IT = 4 for batches up to 4,096 messages (all 16 waves busy), 8 above.
// Ranking: per row, the wave-ballot ranking of k_radix_scatter into per-(digit, wave) counters
// kept as packed u16 pairs in digit-major order, so ONE block-wide exclusive scan of the counters
// gives every (digit, wave) its output base (the digits' starts and the waves' offsets at once).
// Then the runs of equal keys are compacted with ballots.  For micro-batches this replaces the
// multi-launch radix pipeline and the O(n_act) offsets: the host gets perm[n] and, per activation
// present, run_act[r] / run_start[r] (run_start[n_runs] = n), each run in arrival order
// (ActivationData.cs:566-606).
constexpr int MB_THREADS = 1024;
constexpr int MB_NW = MB_THREADS / WAVE;
constexpr uint32_t MB_MAX = MB_THREADS * 8;        // 8192 messages
constexpr int MB_MAX_BITS = 11;

struct MbShared {
    uint32_t cnt[(1u << MB_MAX_BITS) * MB_NW / 2];  // u16 (digit, wave) counters, digit-major, 2 per word
    uint2 kv[MB_MAX];
    uint32_t wsum[MB_NW];
};

// Wave-wide inclusive sum with DPP (row shifts, then the row broadcasts of lanes 15 and 31): no
// LDS round trips, unlike ds_bpermute shuffles.
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}

// Wave-wide sum, uniform.
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(x), WAVE - 1);
}

// ---- row counts and ranks of the bucketing kernels (gd_bucket2.h, gd_msd.h, gd_msd2.h) ----------
// A row is one wave instruction's 64 items, each with a digit d; counters are per wave.
//
// The wave's hot digit: the digit most of a row holds, of four candidate lanes' digits (lanes 0, 16,
// 32, 48), when at least 8 of the row's valid lanes hold it; else NONE32.  Uniform over the wave.
// Under Zipf skew (BASELINE cfg 3: one pass-A digit holds 86 % of the messages, one range 62 %) the
// hot digit's items are then counted and ranked in registers by ballot -- no LDS atomic and none of the
// same-address serialisation a hot counter costs (64 lanes on one LDS address take 64 cycles) -- and
// every other item takes its own counter update.  A wave keeps one hot digit for all its rows of a tile.
// One histogram item without a branch: a live item of the wave's hot digit h counts in the register hc,
// any other live item adds 1 to its counter, and an item that is not live (past the tile) or hot adds 1
// to its lane's own sink word (never read; lane-distinct, so no two lanes of one instruction meet there).
// Replaces two nested lane-masked branches an item (their exec-mask juggling was most of the issued
// instructions of the histogram kernels).
__device__ __forceinline__ void hist_add(uint32_t* s_cnt, uint32_t* s_sink, uint32_t d, uint32_t h, bool live,
                                         uint32_t& hc) {
    const bool hot = d == h;
    hc += live && hot ? 1u : 0u;
    atomicAdd(live && !hot ? &s_cnt[d] : &s_sink[threadIdx.x & (WAVE - 1)], 1u);
}

__device__ __forceinline__ uint32_t wave_hot_digit(uint32_t d, bool valid) {
    uint32_t best = NONE32, bc = 7;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t cd = (uint32_t)__builtin_amdgcn_readlane((int)(valid ? d : NONE32), 16 * q);
        const uint32_t c = (uint32_t)__popcll(__ballot(valid && d == cd));
        if (cd != NONE32 && c > bc) {
            bc = c;
            best = cd;
        }
    }
    return best;
}

// This lane's place among the wave's earlier items with its digit d, from the wave's u16 counter at
// bit sh of *p, which this row's valid items then advance.  BALLOT = false: one ds_add_rtn a lane --
// the lanes of one instruction on one address are served in ascending lane order (gd_create
// checks it on the device).  BALLOT = true: stable by construction -- the lanes sharing d found by
// ballots over its B bits (match_digit), the lowest of them adds the group's size, every lane of the
// group takes the base from that lane (ds_bpermute) plus its count of lower peers (GD_OPT_STABLE_RANK
// 0, and the library's choice when gd_create finds the lane order missing).  Call with every lane.
template <bool BALLOT, int B>
__device__ __forceinline__ uint32_t row_rank16(uint32_t* p, uint32_t sh, uint32_t d, bool valid) {
    if constexpr (!BALLOT) {
        uint32_t old = 0;
        if (valid) old = atomicAdd(p, 1u << sh);
        return (old >> sh) & 0xFFFFu;
    } else {
        const unsigned long long peers = match_digit<B>(d, valid);
        const uint32_t lane = lane_id();
        const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        uint32_t old = 0;
        if (valid && below == 0) old = atomicAdd(p, (uint32_t)__popcll(peers) << sh);
        const int src = peers ? __ffsll((long long)peers) - 1 : (int)lane;
        old = (uint32_t)__shfl((int)old, src, WAVE);
        return ((old >> sh) & 0xFFFFu) + below;
    }
}

// row_rank16 over whole u32 counters.
template <bool BALLOT, int B>
__device__ __forceinline__ uint32_t row_rank32(uint32_t* p, uint32_t d, bool valid) {
    if constexpr (!BALLOT) {
        uint32_t old = 0;
        if (valid) old = atomicAdd(p, 1u);
        return old;
    } else {
        const unsigned long long peers = match_digit<B>(d, valid);
        const uint32_t lane = lane_id();
        const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        uint32_t old = 0;
        if (valid && below == 0) old = atomicAdd(p, (uint32_t)__popcll(peers));
        const int src = peers ? __ffsll((long long)peers) - 1 : (int)lane;
        old = (uint32_t)__shfl((int)old, src, WAVE);
        return old + below;
    }
}

// Block-wide exclusive sum over MB_THREADS threads (two barriers).
__device__ __forceinline__ uint32_t mb_block_excl_sum(uint32_t v, uint32_t* s_wsum) {
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const uint32_t x = wave_incl_sum_dpp(v);
    if (lane == WAVE - 1) s_wsum[w] = x;
    __syncthreads();
    const uint32_t ws = lane < (uint32_t)MB_NW ? s_wsum[lane] : 0u;
    const uint32_t wi = wave_incl_sum_dpp(lane < w ? ws : 0u);   // sum of the waves before w
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readlane((int)wi, WAVE - 1);
    __syncthreads();
    return wbase + x - v;
}

// The sort + runs over keys kk (already clamped to n_act) and indices vv held in registers.
// Outputs are written for positions in [lo, hi) only (the calling workgroup's share; n_runs and
// run_start[n_runs] by the share holding n).
template <int BITS, int IT>
__device__ __forceinline__ void mb_sort_runs_core(MbShared& sh, uint32_t (&kk)[IT], uint32_t (&vv)[IT], uint32_t n,
                                                  uint32_t passes, uint32_t* __restrict__ perm,
                                                  uint32_t* __restrict__ run_act, uint32_t* __restrict__ run_start,
                                                  uint32_t* __restrict__ n_runs, uint32_t lo, uint32_t hi,
                                                  unsigned long long* ts, bool ballot) {
    constexpr uint32_t R = 1u << BITS;
    constexpr uint32_t WORDS = R * MB_NW / 2;
    constexpr uint32_t WPT = WORDS >= MB_THREADS ? WORDS / MB_THREADS : 1;   // counter words per thread
    constexpr uint32_t COLS = WORDS / WPT;
    // scan word q (q = thread * WPT + j) lives at word (q % WPT) * COLS + q / WPT: the scan's reads
    // are unit-stride across lanes, the ranking atomics spread over the banks by digit
    auto cw = [](uint32_t q) { return (q % WPT) * COLS + q / WPT; };
    static_assert(BITS <= MB_MAX_BITS && IT * MB_THREADS <= (int)MB_MAX, "micro-batch shape");
    uint32_t* s_cnt = sh.cnt;
    uint2* s_kv = sh.kv;
    uint32_t* s_wsum = sh.wsum;
    const uint32_t lane = lane_id(), w = threadIdx.x / WAVE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long t = 0;
    mb_mark(ts, 0, t);
    const unsigned long long c0 = ts ? clock64() : 0, r0 = t;
    for (uint32_t e = threadIdx.x * 4; e < WORDS; e += MB_THREADS * 4)
        *reinterpret_cast<uint4*>(s_cnt + e) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (uint32_t pass = 0; pass < passes; ++pass) {
        const uint32_t shift = pass * BITS;
        // Stable in-wave rank: the wave's hot digit by ballot in registers, the others by row_rank16
        // (ds_add_rtn in lane order, or ballots when `ballot`: GD_OPT_STABLE_RANK 0).  Rows past n are
        // skipped wave-uniformly.
        uint32_t rk[IT];
        const uint32_t h = wave_hot_digit(kk[0] >> shift & (R - 1), (uint32_t)(w * IT) * WAVE + lane < n);
        uint32_t hrun = 0;
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            rk[r] = 0;
            if ((uint32_t)(w * IT + r) * WAVE >= n) continue;
            const bool valid = (w * IT + r) * WAVE + lane < n;
            const uint32_t d = (kk[r] >> shift) & (R - 1);
            const uint32_t e = d * MB_NW + w, sh16 = (e & 1u) * 16u;
            const unsigned long long hm = __ballot(valid && d == h);
            const bool cold = valid && d != h;
            const uint32_t cr = ballot ? row_rank16<true, BITS>(&s_cnt[cw(e >> 1)], sh16, d, cold)
                                       : row_rank16<false, BITS>(&s_cnt[cw(e >> 1)], sh16, d, cold);
            rk[r] = d == h ? hrun + (uint32_t)__popcll(hm & lt) : cr;
            hrun += (uint32_t)__popcll(hm);
        }
        if (lane == 0 && hrun) {
            const uint32_t e = h * MB_NW + w;
            atomicAdd(&s_cnt[cw(e >> 1)], hrun << ((e & 1u) * 16u));
        }
        __syncthreads();
        if (pass == 0) mb_mark(ts, 4, t);
        // exclusive scan of the counters in (digit, wave) order: base of every (digit, wave)
        {
            const bool mine = threadIdx.x < COLS;
            uint32_t cv[WPT];
            uint32_t sum = 0;
#pragma unroll
            for (uint32_t j = 0; j < WPT; ++j) {
                cv[j] = mine ? s_cnt[j * COLS + threadIdx.x] : 0u;
                sum += (cv[j] & 0xFFFFu) + (cv[j] >> 16);
            }
            uint32_t run = mb_block_excl_sum(sum, s_wsum);
            if (mine) {
#pragma unroll
                for (uint32_t j = 0; j < WPT; ++j) {
                    const uint32_t a = run;
                    run += cv[j] & 0xFFFFu;
                    s_cnt[j * COLS + threadIdx.x] = a | (run << 16);
                    run += cv[j] >> 16;
                }
            }
        }
        __syncthreads();
        if (pass == 0) mb_mark(ts, 14, t);
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            if ((w * IT + r) * WAVE + lane < n) {
                const uint32_t d = (kk[r] >> shift) & (R - 1);
                const uint32_t e = d * MB_NW + w;
                const uint32_t base = (s_cnt[cw(e >> 1)] >> ((e & 1u) * 16u)) & 0xFFFFu;
                s_kv[base + rk[r]] = make_uint2(kk[r], vv[r]);
            }
        }
        __syncthreads();
        if (pass == 0) mb_mark(ts, 15, t);
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            const uint32_t p = (w * IT + r) * WAVE + lane;
            if (p < n) {
                const uint2 kv = s_kv[p];
                kk[r] = kv.x;
                vv[r] = kv.y;
            }
        }
        if (pass + 1 < passes)       // the counters are free again: clear them for the next pass
            for (uint32_t e = threadIdx.x * 4; e < WORDS; e += MB_THREADS * 4)
                *reinterpret_cast<uint4*>(s_cnt + e) = make_uint4(0, 0, 0, 0);
        __syncthreads();
        mb_mark(ts, 5 + (int)pass, t);
    }
    // runs: a head where the key changes; wave w owns positions [w * IT * 64, (w + 1) * IT * 64)
    // in (r, lane) order, so heads are counted per wave, scanned across waves, ranked in-wave.
    uint32_t prev[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t p = (w * IT + r) * WAVE + lane;
        // key of position p - 1: lane - 1 of the same row, lane 63 of the previous row, or the
        // previous wave's last item (read through LDS, which still holds the sorted pairs)
        const uint32_t up = __shfl_up(kk[r], 1, WAVE);
        uint32_t pk = up;
        if (lane == 0) pk = (p > 0 && p - 1 < n) ? s_kv[p - 1].x : ~0u;
        prev[r] = pk;
    }
    uint32_t heads_w = 0;
    unsigned long long hb[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t p = (w * IT + r) * WAVE + lane;
        hb[r] = __ballot(p < n && (p == 0 || prev[r] != kk[r]));
        heads_w += (uint32_t)__popcll(hb[r]);
    }
    const uint32_t wbase = mb_block_excl_sum(lane == 0 ? heads_w : 0u, s_wsum);
    mb_mark(ts, 9, t);
    const uint32_t base = __shfl(wbase, 0, WAVE);
    uint32_t before = base;
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t p = (w * IT + r) * WAVE + lane;
        if (p < n && p >= lo && p < hi) {
            perm[p] = vv[r];
            if ((hb[r] >> lane) & 1ull) {
                const uint32_t q = before + (uint32_t)__popcll(hb[r] & lt);
                run_act[q] = kk[r];
                run_start[q] = p;
            }
        }
        before += (uint32_t)__popcll(hb[r]);
    }
    if (threadIdx.x == MB_THREADS - 1 && n >= lo && n < hi) {
        const uint32_t tot = base + heads_w;   // last wave's base + its heads = all runs
        n_runs[0] = tot;
        run_start[tot] = n;
    }
    mb_mark(ts, 10, t);
    if (ts) {
        __threadfence_system();
        mb_mark(ts, 11, t);
        if (blockIdx.x == 0 && threadIdx.x == 0) {     // shader clocks vs wall ticks over the kernel
            atomicAdd(ts + 12, clock64() - c0);
            atomicAdd(ts + 13, t - r0);
        }
    }
}

// gridDim.x workgroups sort the same batch redundantly and each writes its 1/gridDim.x share of
// the outputs: zero-copy stores to host memory are spread over as many CUs.  act_copy (optional):
// the activations also go to the host block.  done (optional, pinned host memory): each workgroup adds
// 1 once its share is stored and fenced, so the host sees the batch finished without waiting for the
// dispatch's completion signal (gd_microbatch_run's poll).
template <int BITS, int IT>
static __global__ void __launch_bounds__(MB_THREADS) k_mb_sort_runs(const uint32_t* __restrict__ act, uint32_t n,
                                                              uint32_t passes, uint32_t n_act,
                                                              uint32_t* __restrict__ perm,
                                                              uint32_t* __restrict__ run_act,
                                                              uint32_t* __restrict__ run_start,
                                                              uint32_t* __restrict__ n_runs,
                                                              uint32_t* __restrict__ act_copy,
                                                              unsigned long long* ts, uint32_t ballot,
                                                              uint32_t* done) {
    __shared__ MbShared sh;
    const uint32_t lane = lane_id(), w = threadIdx.x / WAVE;
    const uint32_t lo = (uint32_t)((uint64_t)n * blockIdx.x / gridDim.x);
    const uint32_t hi = blockIdx.x + 1 == gridDim.x ? n + 1 : (uint32_t)((uint64_t)n * (blockIdx.x + 1) / gridDim.x);
    uint32_t kk[IT], vv[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const uint32_t idx = (w * IT + r) * WAVE + lane;
        const uint32_t a = act[idx < n ? idx : (n ? n - 1 : 0)];
        if (act_copy && idx < n && idx >= lo && idx < hi) act_copy[idx] = a;
        kk[r] = a < n_act ? a : n_act;
        vv[r] = idx;
    }
    mb_sort_runs_core<BITS, IT>(sh, kk, vv, n, passes, perm, run_act, run_start, n_runs, lo, hi, ts, ballot != 0);
    if (done) {
        __threadfence_system();                    // this thread's host stores before the count
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace gd
