// gd_fanout.h -- gfx950 device code for SURVEY 8 f2: follower fan-out (Chirper, cfg 4).
//
// ChirperAccount.PublishMessage (Samples/Chirper/ChirperGrains/ChirperAccount.cs:106-147) sends
// one NewChirp per follower, in State.Followers enumeration order (:131-134).  For a frontier of
// publishers F (node ids = long grain keys of one grain type) over a CSR follower graph
// (row_off[u]..row_off[u+1] = u's followers in enumeration order), one hop emits the messages
//     for i in 0..|F|:  for j in row(F[i]):  (target = dst[j], sender = F[i])
// in that order.  The emission is a load-balanced expansion: an inclusive scan of the degrees
// gives ends[i]; output p belongs to item upper_bound(ends, p).  Each block owns FAN_TILE
// consecutive outputs, finds its item range with two global searches, stages the items'
// (end, dst base, sender) in LDS and searches there, so a celebrity row is spread over many
// blocks and a run of zero-follower publishers costs nothing.  Writes are coalesced
// (output p = block base + j * BLOCK + lane).
//
// k_fan_route fuses the expansion with K0+K1+K2: the target's GrainId(typeCode, node) is
// formed in registers (GrainId.cs:72-77, UniqueKey.cs:122-128), hashed, looked up on the
// LDS ring and probed, so the 24-B key never goes to HBM.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

constexpr int FAN_IT = 8;
constexpr uint32_t FAN_TILE = BLOCK * FAN_IT;      // 2048 messages per block
constexpr uint32_t FAN_LDS_ITEMS = FAN_TILE;       // publishers staged per block (24 KB: 6 blocks / CU)

// ends[i] = out-degree of frontier[i] (0 for ids outside the graph: a grain nobody follows);
// the u64 total goes to *total (block reduce + one atomic per block).
static __global__ void __launch_bounds__(BLOCK) k_fan_degree(const uint32_t* __restrict__ row_off, uint32_t n_nodes,
                                                      const uint32_t* __restrict__ frontier, uint32_t n_front,
                                                      uint32_t* __restrict__ ends,
                                                      unsigned long long* __restrict__ total) {
    __shared__ unsigned long long s_sum[BLOCK / WAVE];
    unsigned long long v = 0;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n_front; i += gridDim.x * BLOCK) {  // grid-stride:
        const uint32_t u = frontier[i];                                                           // few atomics
        const uint32_t d = u < n_nodes ? row_off[u + 1] - row_off[u] : 0u;
        ends[i] = d;
        v += d;
    }
#pragma unroll
    for (int off = WAVE / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, WAVE);
    if ((threadIdx.x & (WAVE - 1)) == 0) s_sum[threadIdx.x / WAVE] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
#pragma unroll
        for (int k = 0; k < BLOCK / WAVE; ++k) s += s_sum[k];
        if (s) atomicAdd(total, s);
    }
}

// The same as the first half of a scan: block b covers the scan tile b of k_scan_down<OpAdd, IPT>
// (entries b * IPT * BLOCK ..), writes the degrees (coalesced: entry b * IPT * BLOCK + k * BLOCK + t
// for thread t) and the tile's sum to part[b], so the inclusive scan of ends is the down-sweep
// alone; the host adds the partials up for the u64 total.
template <int IPT>
// d_nf (optional): the frontier's length on the device (<= n_front, the grid's bound), as
// k_frontier_compact left it -- the in-library cascade sizes a hop without reading it back first.
static __global__ void __launch_bounds__(BLOCK) k_fan_degree_tiles(const uint32_t* __restrict__ row_off, uint32_t n_nodes,
                                                            const uint32_t* __restrict__ frontier, uint32_t n_front,
                                                            uint32_t* __restrict__ ends, uint32_t* __restrict__ part,
                                                            const uint32_t* __restrict__ d_nf) {
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    if (d_nf) n_front = min(n_front, *d_nf);
    const uint32_t i0 = blockIdx.x * (BLOCK * IPT) + threadIdx.x;
    uint32_t u[IPT], v = 0;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t i = i0 + k * BLOCK;
        u[k] = i < n_front ? frontier[i] : n_nodes;
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t i = i0 + k * BLOCK;
        const uint32_t d = u[k] < n_nodes ? row_off[u[k] + 1] - row_off[u[k]] : 0u;
        if (i < n_front) ends[i] = d;
        v += d;
    }
    v = block_reduce<OpAdd>(v, s_wsum);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// first i in [lo, hi) with a[i] > p  (hi if none)
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t p) {
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] <= p) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The same by one wave (all 64 lanes call it): each round tests the last entry of 64 equal pieces of
// [lo, hi) and keeps the piece holding the answer -- log64 dependent reads instead of log2 (4 instead
// of 22 over a 5M-publisher frontier, the latency each block of k_fan_route waits before its first probe).
__device__ __forceinline__ uint32_t wave_upper_bound_u32(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t p) {
    const uint32_t lane = threadIdx.x & (WAVE - 1);
    while (hi - lo > (uint32_t)WAVE) {
        const uint32_t step = (hi - lo + WAVE - 1) / WAVE;
        const uint32_t i = lo + (lane + 1) * step - 1;
        const uint32_t k = (uint32_t)__popcll(__ballot(i < hi && a[i] <= p));   // pieces wholly <= p: a prefix
        const uint32_t nlo = lo + k * step;
        hi = min(hi, nlo + step);
        lo = nlo;
    }
    const uint32_t i = lo + lane;
    return lo + (uint32_t)__popcll(__ballot(i < hi && a[i] <= p));
}

// Per-block staging of the publishers covering outputs [p0, p1): items [lo, lo + cnt).  When
// cnt exceeds FAN_LDS_ITEMS (a long run of zero-follower publishers inside the range) nothing
// is staged and fan_item searches global memory instead.
struct FanStage {
    uint32_t end[FAN_LDS_ITEMS];
    uint32_t base[FAN_LDS_ITEMS];   // row_off[u] - (first output of item): dst index = base + p
    uint32_t src[FAN_LDS_ITEMS];    // publisher node id (the NewChirp sender)
    uint32_t lo, cnt;
};

__device__ __forceinline__ void fan_stage(FanStage& s, const uint32_t* __restrict__ row_off,
                                          const uint32_t* __restrict__ frontier, uint32_t n_front,
                                          const uint32_t* __restrict__ ends, uint32_t p0, uint32_t p1) {
    // wave 0 finds the first item, wave 1 the last, in parallel
    if (threadIdx.x < 2 * WAVE) {
        const uint32_t r = wave_upper_bound_u32(ends, 0, n_front, threadIdx.x < WAVE ? p0 : p1 - 1);
        if (threadIdx.x == 0) s.lo = r;
        if (threadIdx.x == WAVE) s.cnt = r;
    }
    __syncthreads();
    if (threadIdx.x == 0) s.cnt = s.cnt - s.lo + 1;
    __syncthreads();
    const uint32_t lo = s.lo, cnt = s.cnt;
    if (cnt <= FAN_LDS_ITEMS) {
        for (uint32_t k = threadIdx.x; k < cnt; k += BLOCK) {
            const uint32_t i = lo + k;
            const uint32_t e = ends[i];
            const uint32_t b = i ? ends[i - 1] : 0u;
            const uint32_t u = frontier[i];
            s.end[k] = e;
            s.base[k] = (e != b ? row_off[u] : 0u) - b;   // zero-degree items are never selected
            s.src[k] = u;
        }
    }
    __syncthreads();
}

// Item of output p: (dst index, sender).
__device__ __forceinline__ void fan_item(const FanStage& s, const uint32_t* __restrict__ row_off,
                                         const uint32_t* __restrict__ frontier, uint32_t n_front,
                                         const uint32_t* __restrict__ ends, uint32_t p, uint32_t& j,
                                         uint32_t& sender) {
    if (s.cnt <= FAN_LDS_ITEMS) {
        const uint32_t k = upper_bound_u32(s.end, 0, s.cnt, p);
        j = s.base[k] + p;
        sender = s.src[k];
    } else {
        const uint32_t i = upper_bound_u32(ends, s.lo, min(s.lo + s.cnt, n_front), p);
        const uint32_t b = i ? ends[i - 1] : 0u;
        sender = frontier[i];
        j = row_off[sender] + (p - b);
    }
}

// Expansion only: (target, sender) per message -- the multi-GPU path ships these 8 B to the
// owner instead of a 28-B header.
// node_of (partitioned graphs, gd_fanout_multi_part_device): the frontier holds this rank's local rows
// (activation indices); the sender written is the row's node.
static __global__ void __launch_bounds__(BLOCK) k_fan_expand(const uint32_t* __restrict__ row_off,
                                                      const uint32_t* __restrict__ dst,
                                                      const uint32_t* __restrict__ frontier, uint32_t n_front,
                                                      const uint32_t* __restrict__ ends, uint32_t total,
                                                      uint32_t* __restrict__ out_target,
                                                      uint32_t* __restrict__ out_sender,
                                                      const uint32_t* __restrict__ node_of) {
    __shared__ FanStage s;
    const uint32_t p0 = blockIdx.x * FAN_TILE;
    const uint32_t p1 = min(p0 + FAN_TILE, total);
    fan_stage(s, row_off, frontier, n_front, ends, p0, p1);
    for (int it = 0; it < FAN_IT; ++it) {
        const uint32_t p = p0 + it * BLOCK + threadIdx.x;
        if (p >= p1) break;
        uint32_t j, sender;
        fan_item(s, row_off, frontier, n_front, ends, p, j, sender);
        out_target[p] = dst[j];
        out_sender[p] = node_of ? node_of[sender] : sender;
    }
}

// Route of GrainId(typeCode, node) (category Grain, N0 = 0, N1 = node): ring owner + probe.
// Returns the status; silo / act as k_route_m writes them.
template <int MODE>
__device__ __forceinline__ uint8_t route_node(uint32_t node, uint64_t tcd, const uint32_t* s_pts,
                                              const uint32_t* s_own, const RingArgs& ring, const TableArgs& tab,
                                              uint32_t max_probe, uint32_t& silo, uint32_t& act) {
    const uint64_t n0 = 0, n1 = node;
    const uint32_t h = uniform_hash(n0, n1, tcd);
    silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h)];
    act = NONE32;
    uint32_t a, meta;
    if (probe(tab.slots, tab.mask, max_probe, h, n0, n1, tcd, a, meta)) {
        if (a == GD_ACT_MULTI) return GD_ROUTE_MULTI_ACT;   // RandomPlacementDirector.cs:33-53, in C#
        if (!tab_silo_valid(tab, slot_silo(meta))) return GD_ROUTE_MISS;   // IsValidSilo (:431)
        act = a;
        silo = slot_silo(meta);                    // ActivationAddress.Silo (Message.cs:629-639)
        return GD_ROUTE_OK;
    }
    return GD_ROUTE_MISS;                          // Dispatcher.cs:742 slow path
}

// The compact probe indexes' walks for GrainId(tcd, node) from the home's group already read
// (gd_kernels.h cx16_walk / cx8_walk); a key the index does not hold (want 0) or a redirect entry
// is probed in the directory (route_node).
template <int MODE, int RG>
__device__ __forceinline__ uint8_t cx_walk_node(const CxArgs& cx, const TableArgs& tab, uint32_t mp, uint32_t want,
                                                uint32_t node, uint64_t tcd, unsigned long long s, uint4 (&q)[RG],
                                                const uint32_t* s_pts, const uint32_t* s_own, const RingArgs& ring,
                                                uint32_t& silo, uint32_t& act) {
    if (!want) return route_node<MODE>(node, tcd, s_pts, s_own, ring, tab, lazy_max_probe(tab), silo, act);
    uint8_t st = GD_ROUTE_MISS;
    cx16_walk<RG>(cx, tab, want, node, s, q, silo, act, st);
    return st;
}

template <int MODE>
__device__ __forceinline__ uint8_t cx8_walk_node(const Cx8Args& cx8, const TableArgs& tab, uint32_t mp, int t8,
                                                 uint32_t node, uint64_t tcd, unsigned long long s,
                                                 uint4 (&q)[CX8_GROUP / 2], const uint32_t* s_pts,
                                                 const uint32_t* s_own, const RingArgs& ring, uint32_t& silo,
                                                 uint32_t& act) {
    uint8_t st = GD_ROUTE_MISS;
    if (t8 < 0 || cx8_walk(cx8, tab, node, (uint32_t)t8, s, q, silo, act, st))
        return route_node<MODE>(node, tcd, s_pts, s_own, ring, tab, lazy_max_probe(tab), silo, act);
    return st;
}

__device__ __forceinline__ uint32_t cx_want(const CxArgs& cx, uint64_t tcd) {
    const int t = cx_type_index(cx.types, tcd);
    return t < 0 ? 0u : (0x100u | (uint32_t)t);
}
// The first read of an index walk: the aligned group holding home slot s.
template <int RG>
__device__ __forceinline__ void cx_first(const CxArgs& cx, unsigned long long s, uint4 (&q)[RG]) {
    const uint4* qp = cx.slots + (s & ~(unsigned long long)(RG - 1));
#pragma unroll
    for (int g = 0; g < RG; ++g) q[g] = qp[g];
}
__device__ __forceinline__ void cx8_first(const Cx8Args& cx8, unsigned long long s, uint4 (&q)[CX8_GROUP / 2]) {
    const uint4* qp = cx8.slots + ((s & ~(unsigned long long)(CX8_GROUP - 1)) >> 1);
#pragma unroll
    for (int g = 0; g < (int)CX8_GROUP / 2; ++g) q[g] = qp[g];
}

// Route a batch of node ids (GrainId(typeCode, node), the owner side of the sharded fan-out).
// CX: through the compact probe index.
template <int MODE, bool CX = false, int RG = (int)CX_GROUP, bool CX8 = false>
static __global__ void __launch_bounds__(BLOCK) k_route_nodes(const uint32_t* __restrict__ nodes, uint32_t n, uint64_t tcd,
                                                       RingArgs ring, TableArgs tab, uint32_t* __restrict__ out_silo,
                                                       uint32_t* __restrict__ out_act,
                                                       uint8_t* __restrict__ out_status, CxArgs cx = CxArgs{},
                                                       Cx8Args cx8 = Cx8Args{}) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const uint32_t max_probe = (CX || CX8) ? 0u : tab.ctr->max_probe;   // the index walks read it lazily
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t silo, act;
    uint8_t st;
    if constexpr (CX8) {                               // the 8-B index (gd_kernels.h Cx8Args)
        const uint32_t node = nodes[i];
        const int t8 = cx8_type(cx8, 0, node, tcd);
        const uint32_t h = uniform_hash(0, node, tcd);
        const unsigned long long s0 = home_slot(h, tab.mask);
        uint4 q[CX8_GROUP / 2];
        if (t8 >= 0) cx8_first(cx8, s0, q);
        silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h)];
        act = NONE32;
        st = cx8_walk_node<MODE>(cx8, tab, max_probe, t8, node, tcd, s0, q, s_pts, s_own, ring, silo, act);
    } else if constexpr (CX) {
        const uint32_t want = cx_want(cx, tcd);
        const uint32_t node = nodes[i];
        const uint32_t h = uniform_hash(0, node, tcd);
        const unsigned long long s0 = home_slot(h, tab.mask);
        uint4 q[RG];
        if (want) cx_first<RG>(cx, s0, q);
        silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h)];
        act = NONE32;
        st = cx_walk_node<MODE, RG>(cx, tab, max_probe, want, node, tcd, s0, q, s_pts, s_own, ring, silo, act);
    } else {
        st = route_node<MODE>(nodes[i], tcd, s_pts, s_own, ring, tab, max_probe, silo, act);
    }
    out_silo[i] = silo;
    out_act[i] = act;
    out_status[i] = st;
}

// Fused expansion + route.  out_target may be null.  ILP items of a thread at a time: their
// follower-list reads, then their first directory probes, are in flight together (one dependent
// chain per item otherwise).
// IT: rounds of BLOCK outputs a block (a tile of BLOCK * IT outputs; 2 for a small hop, whose 2048-output
// tiles would leave most CUs idle).  d_nf / dev_total: the frontier's length on the device, and the
// hop's total read from the inclusive scan (ends[nf - 1]) instead of the host -- `total` is then the
// outputs' capacity and the grid is sized for it; blocks past the device total exit at once.
// BOUND (with CX8; k_fan_bound, round 6): the kernel's memory traffic alone -- the same expansion reads
// (staged publishers, follower lists), home hash, one 64-B index group read a message and the same result
// writes, with no ring search and no walk (silo / act taken from the group read so it is not dead code).
// Launched on the hop's own inputs into scratch outputs beside the real launch (GD_OPT_FAN_BOUND), it is
// the live memory bound bench.py divides k_fan_route's time by.
template <int MODE, int ILP, bool CX = false, int RG = (int)CX_GROUP, bool CX8 = false, int IT = FAN_IT,
          bool BOUND = false>
static __global__ void __launch_bounds__(BLOCK) k_fan_route(const uint32_t* __restrict__ row_off,
                                                     const uint32_t* __restrict__ dst,
                                                     const uint32_t* __restrict__ frontier, uint32_t n_front,
                                                     const uint32_t* __restrict__ ends, uint32_t total, uint64_t tcd,
                                                     RingArgs ring, TableArgs tab,
                                                     uint32_t* __restrict__ out_target,
                                                     uint32_t* __restrict__ out_sender,
                                                     uint32_t* __restrict__ out_silo, uint32_t* __restrict__ out_act,
                                                     uint8_t* __restrict__ out_status, CxArgs cx = CxArgs{},
                                                     Cx8Args cx8 = Cx8Args{}, const uint32_t* __restrict__ d_nf = nullptr,
                                                     uint32_t dev_total = 0) {
    static_assert(IT % ILP == 0 && BLOCK * IT <= FAN_LDS_ITEMS, "whole rounds, staged items");
    constexpr uint32_t TILE = BLOCK * IT;
    if (d_nf) n_front = min(n_front, *d_nf);
    if (dev_total) total = min(total, n_front ? ends[n_front - 1] : 0u);
    const uint32_t p0 = blockIdx.x * TILE;
    if (p0 >= total) return;                              // block-uniform, before any barrier
    __shared__ FanStage s;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const uint32_t max_probe = (CX || CX8) ? 0u : tab.ctr->max_probe;   // the index walks read it lazily
    const uint32_t p1 = min(p0 + TILE, total);
    fan_stage(s, row_off, frontier, n_front, ends, p0, p1);
    for (int it0 = 0; it0 < IT; it0 += ILP) {
        if (p0 + it0 * BLOCK >= p1) break;                 // block-uniform
        uint32_t j[ILP], sender[ILP], target[ILP], h[ILP];
        bool live[ILP];
#pragma unroll
        for (int q = 0; q < ILP; ++q) {
            const uint32_t p = p0 + (it0 + q) * BLOCK + threadIdx.x;
            live[q] = p < p1;
            j[q] = 0;
            sender[q] = 0;
            if (live[q]) fan_item(s, row_off, frontier, n_front, ends, p, j[q], sender[q]);
        }
#pragma unroll
        for (int q = 0; q < ILP; ++q) target[q] = live[q] ? dst[j[q]] : 0u;
        if constexpr (CX8) {                                  // the 8-B index (gd_kernels.h Cx8Args)
            const int t8 = cx8_type(cx8, 0, 0, tcd);          // node grains: N0 = 0, N1 = node < 2^32
            unsigned long long s8[ILP];
            uint4 q8[ILP][CX8_GROUP / 2];
#pragma unroll
            for (int q = 0; q < ILP; ++q) {
                h[q] = uniform_hash(0, target[q], tcd);
                s8[q] = home_slot(h[q], tab.mask);
                if (live[q] && t8 >= 0) cx8_first(cx8, s8[q], q8[q]);
            }
#pragma unroll
            for (int q = 0; q < ILP; ++q) {
                if (!live[q]) continue;
                const uint32_t p = p0 + (it0 + q) * BLOCK + threadIdx.x;
                uint32_t silo, act = NONE32;
                uint8_t st;
                if constexpr (BOUND) {
                    silo = q8[q][0].x & 7u;
                    act = q8[q][CX8_GROUP / 2 - 1].w;
                    st = 0;
                } else {
                    silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h[q])];
                    st = cx8_walk_node<MODE>(cx8, tab, max_probe, t8, target[q], tcd, s8[q], q8[q], s_pts, s_own, ring,
                                             silo, act);
                }
                if (out_target) out_target[p] = target[q];
                out_sender[p] = sender[q];
                out_silo[p] = silo;
                out_act[p] = act;
                out_status[p] = st;
            }
            continue;
        }
        if constexpr (CX) {                                   // the compact probe index (gd_kernels.h)
            const uint32_t want = cx_want(cx, tcd);
            unsigned long long sc[ILP];
            uint4 qc[ILP][RG];
#pragma unroll
            for (int q = 0; q < ILP; ++q) {
                h[q] = uniform_hash(0, target[q], tcd);
                sc[q] = home_slot(h[q], tab.mask);
                if (live[q] && want) cx_first<RG>(cx, sc[q], qc[q]);
            }
#pragma unroll
            for (int q = 0; q < ILP; ++q) {
                if (!live[q]) continue;
                const uint32_t p = p0 + (it0 + q) * BLOCK + threadIdx.x;
                uint32_t silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h[q])], act = NONE32;
                const uint8_t st = cx_walk_node<MODE, RG>(cx, tab, max_probe, want, target[q], tcd, sc[q], qc[q], s_pts,
                                                          s_own, ring, silo, act);
                if (out_target) out_target[p] = target[q];
                out_sender[p] = sender[q];
                out_silo[p] = silo;
                out_act[p] = act;
                out_status[p] = st;
            }
            continue;
        }
        unsigned long long sl[ILP];
        uint4 qa[ILP], qb[ILP];
#pragma unroll
        for (int q = 0; q < ILP; ++q) {
            h[q] = uniform_hash(0, target[q], tcd);
            sl[q] = home_slot(h[q], tab.mask);
            if (live[q]) {
                const uint4* a = reinterpret_cast<const uint4*>(tab.slots + sl[q]);
                qa[q] = a[0];
                qb[q] = a[1];
            }
        }
#pragma unroll
        for (int q = 0; q < ILP; ++q) {
            if (!live[q]) continue;
            const uint32_t p = p0 + (it0 + q) * BLOCK + threadIdx.x;
            uint32_t silo = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, h[q])], act = NONE32;
            uint8_t st = GD_ROUTE_MISS;
            uint4 a = qa[q], b = qb[q];
            for (uint32_t k = 0;;) {                        // the probe of route_node, from the first slot read
                const uint32_t stt = slot_state(b.w);
                if (stt == SLOT_EMPTY) break;
                const uint64_t k0 = (uint64_t)a.x | ((uint64_t)a.y << 32);
                const uint64_t k1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
                const uint64_t k2 = (uint64_t)b.x | ((uint64_t)b.y << 32);
                if (stt == SLOT_LIVE && k0 == 0 && k1 == target[q] && k2 == tcd) {
                    if (b.z == GD_ACT_MULTI) {
                        st = GD_ROUTE_MULTI_ACT;                 // RandomPlacementDirector.cs:33-53, in C#
                    } else if (tab_silo_valid(tab, slot_silo(b.w))) {
                        act = b.z;
                        silo = slot_silo(b.w);                   // ActivationAddress.Silo (Message.cs:629-639)
                        st = GD_ROUTE_OK;
                    }                                            // else IsValidSilo (:431) -> MISS
                    break;
                }
                if (++k > max_probe) break;                      // Dispatcher.cs:742 slow path
                sl[q] = (sl[q] + 1) & tab.mask;
                const uint4* n = reinterpret_cast<const uint4*>(tab.slots + sl[q]);
                a = n[0];
                b = n[1];
            }
            if (out_target) out_target[p] = target[q];
            out_sender[p] = sender[q];
            out_silo[p] = silo;
            out_act[p] = act;
            out_status[p] = st;
        }
    }
}

// The next frontier in two launches (instead of flag + a 4-launch scan + emit over n_act).
// k_frontier_count: thread t of block b looks at activations a0 .. a0 + 15 (a0 = b * FR_TILE +
// 16 t): fresh = got a message this hop (offsets[a + 1] > offsets[a]) and not visited yet; marks
// them visited, keeps the 16 flags as one u16 and the block's count.  k_frontier_compact: every
// block folds the counts of the blocks before it, ranks its flags and writes its fresh activations
// in activation order (the order the oracle's next_frontier gives); the last thread of the last
// block writes the total.
constexpr uint32_t FR_ITEMS = 16;
constexpr uint32_t FR_TILE = BLOCK * FR_ITEMS;

static __global__ void __launch_bounds__(BLOCK) k_frontier_count(const uint32_t* __restrict__ offsets, uint32_t n_act,
                                                          uint8_t* __restrict__ visited, uint16_t* __restrict__ flags,
                                                          uint32_t* __restrict__ counts) {
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    const uint32_t a0 = blockIdx.x * FR_TILE + threadIdx.x * FR_ITEMS;
    uint32_t m = 0;
    if (a0 + FR_ITEMS <= n_act && (reinterpret_cast<uintptr_t>(offsets) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(visited) & 15) == 0) {
        uint32_t o[FR_ITEMS + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 u = *reinterpret_cast<const uint4*>(offsets + a0 + 4 * q);
            o[4 * q] = u.x; o[4 * q + 1] = u.y; o[4 * q + 2] = u.z; o[4 * q + 3] = u.w;
        }
        o[FR_ITEMS] = offsets[a0 + FR_ITEMS];            // offsets has n_act + 2 entries
        uint4 vis = *reinterpret_cast<const uint4*>(visited + a0);
        uint8_t* vb = reinterpret_cast<uint8_t*>(&vis);
#pragma unroll
        for (int k = 0; k < (int)FR_ITEMS; ++k)
            if (o[k + 1] > o[k] && vb[k] == 0) {
                vb[k] = 1;
                m |= 1u << k;
            }
        if (m) *reinterpret_cast<uint4*>(visited + a0) = vis;
    } else {
        for (uint32_t k = 0; k < FR_ITEMS; ++k) {
            const uint32_t a = a0 + k;
            if (a < n_act && offsets[a + 1] > offsets[a] && visited[a] == 0) {
                visited[a] = 1;
                m |= 1u << k;
            }
        }
    }
    flags[blockIdx.x * BLOCK + threadIdx.x] = (uint16_t)m;
    const uint32_t c = block_reduce<OpAdd>((uint32_t)__popc(m), s_wsum);
    if (threadIdx.x == 0) counts[blockIdx.x] = c;
}

static __global__ void __launch_bounds__(BLOCK) k_frontier_compact(const uint16_t* __restrict__ flags,
                                                            const uint32_t* __restrict__ counts, uint32_t nb,
                                                            uint32_t* __restrict__ out, uint32_t* __restrict__ total) {
    __shared__ uint32_t s_wsum[BLOCK / WAVE];
    uint32_t acc = 0;
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += BLOCK) acc += counts[j];
    const uint32_t prefix = block_reduce<OpAdd>(acc, s_wsum);
    const uint32_t m = flags[blockIdx.x * BLOCK + threadIdx.x];
    const uint32_t c = (uint32_t)__popc(m);
    uint32_t pos = prefix + block_excl_scan<OpAdd>(c, s_wsum);
    const uint32_t a0 = blockIdx.x * FR_TILE + threadIdx.x * FR_ITEMS;
    for (uint32_t k = 0; k < FR_ITEMS; ++k)
        if ((m >> k) & 1u) out[pos++] = a0 + k;
    if (blockIdx.x + 1 == nb && threadIdx.x == BLOCK - 1) *total = pos;
}

// Partitioned graphs: this rank's seeds (node ids, routed on their owner) become local rows = their
// activation indices; a seed without a live activation here counts in *bad (the host refuses the call).
static __global__ void __launch_bounds__(BLOCK) k_seed_rows(const uint32_t* __restrict__ act,
                                                     const uint8_t* __restrict__ status, uint32_t n, uint32_t n_act,
                                                     uint32_t* __restrict__ rows, uint32_t* __restrict__ bad) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const bool ok = status[i] == GD_ROUTE_OK && act[i] < n_act;
    rows[i] = ok ? act[i] : 0u;
    if (!ok) atomicAdd(bad, 1u);
}

// out[i] = table[in[i]] (a partitioned cascade's frontier rows -> their nodes).
static __global__ void __launch_bounds__(BLOCK) k_gather_u32(const uint32_t* __restrict__ in, uint32_t n,
                                                      const uint32_t* __restrict__ table, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = table[in[i]];
}

// The seeds of a cascade have published: visited[u] = 1 for u < n_act (gd_fanout_multi_device).
static __global__ void __launch_bounds__(BLOCK) k_mark_visited(const uint32_t* __restrict__ nodes, uint32_t n, uint32_t n_act,
                                                        uint8_t* __restrict__ visited) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n && nodes[i] < n_act) visited[nodes[i]] = 1;
}

}  // namespace gd
