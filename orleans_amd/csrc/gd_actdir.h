// gd_actdir.h -- gfx950 device code for the silo receive path: the
// ActivationDirectory (src/Orleans.Runtime/Catalog/ActivationDirectory.cs) as an open-addressing
// HBM table keyed by ActivationId, and IncomingMessageAgent.ReceiveMessage
// (src/Orleans.Runtime/Messaging/IncomingMessageAgent.cs:92-170) for a batch of arrived messages.
//
// Table: the 32-B directory slot (gd_common.h) with key = ActivationId (UniqueKey N0, N1,
// TypeCodeData), act = the host's scheduling-context index, meta low 16 bits = GD_ACTDIR_* flags.
// The reference's two dictionaries (activations, systemTargets, :15-16) are one table here with a
// kind bit: FindTarget only sees activations, FindSystemTarget only system targets.
//
// k_receive: one lane per message -- category of TargetGrain (8 B), TargetActivation (24 B),
// Direction (1 B), one probe (one 64-B atom) -> (context, status).  The per-context FIFO
// (WorkItemGroup.EnqueueTask, WorkItemGroup.cs:174-201) is the stable bucketing of gd_bucket over
// the context indices.  HBM-bound, no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_frames.h"
#include "gd_kernels.h"

namespace gd {

// GD_ACTDIR_* / GD_RECV_* (include/graindispatch.h)
constexpr uint32_t AD_VALID = 1u, AD_SYSTEM_TARGET = 2u, AD_STATELESS_WORKER = 4u;
constexpr uint8_t RECV_ACTIVATION = 0, RECV_SYSTEM_TARGET = 1, RECV_NULL_CONTEXT = 2, RECV_REJECT_UNKNOWN = 3,
                  RECV_REJECT_OVERLOADED = 4, RECV_DROPPED = 5, RECV_UNDECODED = 6;
constexpr uint8_t RECV_STATELESS_BIT = 0x80;   // transient mark for the overload pass
constexpr uint8_t DIR_RESPONSE = 1;
constexpr uint32_t ERR_CTX_RANGE = 32u;       // DevCounters.err: an entry's context index >= the call's n_ctx

struct AdArgs {
    const Slot* slots;
    unsigned long long mask;
    const DevCounters* ctr;
};

__device__ __forceinline__ bool ad_find(const AdArgs& t, uint64_t n0, uint64_t n1, uint64_t tcd, uint32_t& ctx,
                                        uint32_t& flags) {
    uint32_t meta = 0;
    const bool f = probe(t.slots, t.mask, t.ctr->max_probe, uniform_hash(n0, n1, tcd), n0, n1, tcd, ctx, meta);
    flags = meta & 0xFFFFu;
    return f;
}

// Slot of each key (TryRemove / state updates): NONE32 if absent.
static __global__ void __launch_bounds__(BLOCK) k_ad_find(const gd_key* __restrict__ keys, uint32_t n, AdArgs t,
                                                   uint32_t* __restrict__ slot_of) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t n0 = keys[i].n0, n1 = keys[i].n1, tcd = keys[i].type_code_data;
    unsigned long long s = home_slot(uniform_hash(n0, n1, tcd), t.mask);
    uint32_t res = NONE32;
    for (uint32_t p = 0; p <= t.ctr->max_probe; ++p) {
        const Slot sl = t.slots[s];
        const uint32_t st = slot_state(sl.meta);
        if (st == SLOT_EMPTY) break;
        if (st == SLOT_LIVE && sl.n0 == n0 && sl.n1 == n1 && sl.tcd == tcd) {
            res = (uint32_t)s;
            break;
        }
        s = (s + 1) & t.mask;
    }
    slot_of[i] = res;
}

static __global__ void __launch_bounds__(BLOCK) k_ad_lookup(const gd_key* __restrict__ keys, uint32_t n, AdArgs t,
                                                     uint32_t* __restrict__ out_ctx, uint8_t* __restrict__ out_flags,
                                                     uint8_t* __restrict__ out_found) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t ctx = NONE32, fl = 0;
    const bool f = ad_find(t, keys[i].n0, keys[i].n1, keys[i].type_code_data, ctx, fl);
    out_ctx[i] = f ? ctx : NONE32;
    out_flags[i] = f ? (uint8_t)fl : 0;
    out_found[i] = f ? 1 : 0;
}

// Flag updates, batch order: the last item of a slot wins (`last` = 1 + its index, k_up_last).
static __global__ void __launch_bounds__(BLOCK) k_ad_setflags(const uint32_t* __restrict__ slot_of,
                                                       const uint8_t* __restrict__ flags, uint32_t n,
                                                       const uint32_t* __restrict__ last, Slot* slots,
                                                       uint8_t* __restrict__ out_found) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    if (s < SLOT_RETRY && last[s] == i + 1) slots[s].meta = make_meta(SLOT_LIVE, flags[i]);
    if (out_found) out_found[i] = s < SLOT_RETRY ? 1 : 0;
}

// ReceiveMessage per message.  ctx[i]: the bucket the message is enqueued in -- a context index
// < n_ctx, n_ctx for the null (system) context, NONE32 when it is not enqueued (rejection, drop,
// undecoded frame).  direction may be null (every message a Request); 0xFF = header absent =
// Request (Message.Direction's default, Message.cs:113-116).  frame_flags (nullable): a frame whose
// target address was not decoded completely goes back to C# (RECV_UNDECODED).  MARK_STATELESS: a
// message enqueued on a stateless-worker activation carries RECV_STATELESS_BIT for k_overload.
// An entry whose context index is not below n_ctx (gd_actdir_add stored it; n_ctx is per call) is a
// caller error: ERR_CTX_RANGE in *err (the call fails with GD_EINVAL) and the message is left
// un-enqueued (ctx NONE32, RECV_UNDECODED), so no later pass indexes past the n_ctx arrays.
template <bool MARK_STATELESS>
static __global__ void __launch_bounds__(BLOCK) k_receive(const gd_key* __restrict__ target_grain,
                                                   const gd_key* __restrict__ target_activation,
                                                   const uint8_t* __restrict__ direction,
                                                   const uint32_t* __restrict__ frame_flags, uint32_t n, uint32_t n_ctx,
                                                   AdArgs t, uint32_t* __restrict__ out_ctx,
                                                   uint8_t* __restrict__ out_status, uint32_t* __restrict__ err) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t ctx = NONE32;
    uint8_t st;
    bool ok = true;
    if (frame_flags) {
        const uint32_t f = frame_flags[i];
        ok = (f & FR_HAS_TARGET) && (f & FR_COMPLETE) && !(f & (FR_FALLBACK | FR_MALFORMED));
    }
    if (!ok) {
        st = RECV_UNDECODED;
    } else {
        const bool is_st = (uint32_t)(target_grain[i].type_code_data >> 56) == CAT_SYSTEM_TARGET;  // GrainId.IsSystemTarget
        const uint64_t* kp = reinterpret_cast<const uint64_t*>(target_activation + i);
        uint8_t d = direction ? direction[i] : 0;
        if (d == 0xFF) d = 0;
        uint32_t c = NONE32, fl = 0;
        const bool found = ad_find(t, kp[0], kp[1], kp[2], c, fl);
        if (is_st) {
            if (!found || !(fl & AD_SYSTEM_TARGET)) {
                st = RECV_REJECT_UNKNOWN;              // FindSystemTarget == null -> rejection (:99-110)
            } else if (d <= DIR_RESPONSE) {
                st = RECV_SYSTEM_TARGET;               // Request / Response work item (:111-124)
                ctx = c;
            } else {
                st = RECV_DROPPED;                     // "Invalid message" (:125-127)
            }
        } else if (found && !(fl & AD_SYSTEM_TARGET) && (fl & AD_VALID)) {
            st = RECV_ACTIVATION;                      // the activation's context (:136-152)
            ctx = c;
            if (MARK_STATELESS && (fl & AD_STATELESS_WORKER)) st |= RECV_STATELESS_BIT;
        } else {
            st = RECV_NULL_CONTEXT;                    // EnqueueReceiveMessage(msg, null, null) (:154-167)
            ctx = n_ctx;
        }
        if (ctx != NONE32 && ctx >= n_ctx && st != RECV_NULL_CONTEXT) {
            atomicOr(err, ERR_CTX_RANGE);
            ctx = NONE32;
            st = RECV_UNDECODED;
        }
    }
    out_ctx[i] = ctx;
    out_status[i] = st;
}

// CheckOverloaded's hard limit (ActivationData.cs:616-649) after the first bucketing, in message
// order: rank[i] = message i's output position, so j = rank[i] - offsets[c] is its place in its
// activation's arrival order; it is rejected iff it is not a response and
// j >= limit + 1 - request_count[c] (every earlier message was enqueued and counted by
// IncrementEnqueuedOnDispatcherCount until the first rejection; after it the count stays over the
// limit).  Rejected messages get ctx NONE32; the caller rebuckets.
static __global__ void __launch_bounds__(BLOCK) k_overload(const uint32_t* __restrict__ rank,
                                                    const uint32_t* __restrict__ offsets, uint32_t n,
                                                    const uint8_t* __restrict__ direction,
                                                    const uint32_t* __restrict__ request_count, int32_t hard_limit,
                                                    int32_t hard_limit_sw, uint32_t* __restrict__ ctx,
                                                    uint8_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint8_t st = status[i];
    if ((st & 0x7F) != RECV_ACTIVATION) return;
    const bool sw = st & RECV_STATELESS_BIT;
    if (sw) status[i] = RECV_ACTIVATION;
    uint8_t d = direction ? direction[i] : 0;
    if (d == 0xFF) d = 0;
    const int64_t limit = sw ? hard_limit_sw : hard_limit;
    if (d == DIR_RESPONSE || limit <= 0) return;       // responses are not checked (:140); no limit set (:627)
    const uint32_t c = ctx[i];
    const int64_t j = (int64_t)(rank[i] - offsets[c]);
    if (j >= limit + 1 - (int64_t)request_count[c]) {
        status[i] = RECV_REJECT_OVERLOADED;
        ctx[i] = NONE32;
    }
}

// gd_route_frames with an ActivationDirectory: a frame whose address is already complete
// (GD_ROUTE_ADDRESSED, Dispatcher.cs:718) gets the context of its TargetActivation when
// FindTarget finds a Valid activation, so the bucketing puts it in that activation's FIFO.
static __global__ void __launch_bounds__(BLOCK) k_frame_addressed_act(const uint8_t* __restrict__ status,
                                                               const gd_key* __restrict__ target_grain,
                                                               const gd_key* __restrict__ target_activation, uint32_t n,
                                                               AdArgs t, uint32_t* __restrict__ act) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || status[i] != ROUTE_ADDRESSED) return;
    if ((uint32_t)(target_grain[i].type_code_data >> 56) == CAT_SYSTEM_TARGET) return;   // FindSystemTarget's side
    const uint64_t* kp = reinterpret_cast<const uint64_t*>(target_activation + i);
    uint32_t c = NONE32, fl = 0;
    if (ad_find(t, kp[0], kp[1], kp[2], c, fl) && !(fl & AD_SYSTEM_TARGET) && (fl & AD_VALID)) act[i] = c;
}

}  // namespace gd
