"""CPU oracle for the silo receive path -- TEST INFRASTRUCTURE ONLY.

Restates, literally and sequentially, how a silo hands each arriving message to a scheduling
context:

* ``ActivationDirectory`` (src/Orleans.Runtime/Catalog/ActivationDirectory.cs)
    - ``activations`` / ``systemTargets``: two ``ConcurrentDictionary<ActivationId, ...>`` (:15-16);
    - ``FindTarget`` :41-45 and ``FindSystemTarget`` :47-51 (TryGetValue);
    - ``RecordNewTarget`` :86-93 / ``RecordNewSystemTarget`` :95-98 (TryAdd: the first add wins);
    - ``RemoveTarget`` :116-131 (TryRemove).
* ``IncomingMessageAgent.ReceiveMessage`` (src/Orleans.Runtime/Messaging/IncomingMessageAgent.cs:92-170):
    - system-target grain: ``FindSystemTarget(TargetActivation)``; none -> rejection response
      (Unrecoverable, :101-110); Request / Response -> that system target's context (:111-127); any
      other direction -> logged error, message dropped (:125-127);
    - otherwise ``FindTarget(TargetActivation)`` (:131): none -> ``EnqueueReceiveMessage(msg, null,
      null)`` = the null (system) context (:163-167); found but ``State != Valid`` -> null context
      (:154-160); Valid -> for non-responses ``CheckOverloaded`` (:140-149; a hard-limit hit is a
      rejection, Overloaded), then the activation's context (:152).
* ``ActivationData.CheckOverloaded`` (src/Orleans.Runtime/Catalog/ActivationData.cs:616-649): the
  stateless-worker or the plain hard limit; no limit (<= 0) -> never; else reject when
  ``GetRequestCount() > limit``.  ``EnqueueReceiveMessage`` (:172-190) increments the activation's
  ``EnqueuedOnDispatcherCount`` for every message it enqueues (responses too), which is part of
  ``GetRequestCount`` (:651-660); within one batch nothing decrements it (the agent thread enqueues
  the batch before a worker runs any of it: the state the GPU batch models).
* Enqueueing: ``scheduler.QueueWorkItem(closure, context)`` -> the context's ``WorkItemGroup`` FIFO
  (WorkItemGroup.cs:174-201); a null context -> the scheduler's system queue, also FIFO.

Output per message: (status, bucket).  Buckets: contexts 0..n_ctx-1 (activations and system
targets share the host's context index space), then bucket n_ctx = the null context, then bucket
n_ctx + 1 = messages that are not enqueued (rejections and dropped messages), each in arrival order.
The per-message ctx output is the bucket: a context index, n_ctx for the null context, or M32 when
the message is not enqueued.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import numpy as np

M32 = 0xFFFFFFFF
CAT_SYSTEM_TARGET = 1

# per-message receive statuses (GD_RECV_* in include/graindispatch.h)
RECV_ACTIVATION = 0          # enqueued on its activation's context
RECV_SYSTEM_TARGET = 1       # enqueued on a system target's context (Request/Response work item)
RECV_NULL_CONTEXT = 2        # EnqueueReceiveMessage(msg, null, null): no usable activation
RECV_REJECT_UNKNOWN = 3      # system target not active on this silo: rejection (Unrecoverable)
RECV_REJECT_OVERLOADED = 4   # CheckOverloaded hard limit: rejection (Overloaded)
RECV_DROPPED = 5             # system target message that is neither Request nor Response

# activation-directory entry flags (GD_ACTDIR_* in include/graindispatch.h)
AD_VALID = 1                 # ActivationData.State == ActivationState.Valid
AD_SYSTEM_TARGET = 2         # an entry of systemTargets, not of activations
AD_STATELESS_WORKER = 4      # ActivationData.IsStatelessWorker (the *_StatelessWorker limits)

DIR_REQUEST, DIR_RESPONSE, DIR_ONEWAY = 0, 1, 2
DIR_NULL = 0xFF              # Direction header absent: Message.Direction = default = Request (Message.cs:113-116)

Key = Tuple[int, int, int]


class ActivationDirectory:
    """ActivationId -> (context index, flags)."""

    def __init__(self):
        self.entries: Dict[Key, Tuple[int, int]] = {}

    def add(self, key: Key, ctx: int, flags: int) -> bool:
        """RecordNewTarget / RecordNewSystemTarget: TryAdd (first add wins)."""
        if key in self.entries:
            return False
        self.entries[key] = (ctx, flags)
        return True

    def remove(self, key: Key) -> bool:
        """RemoveTarget: TryRemove."""
        return self.entries.pop(key, None) is not None

    def set_flags(self, key: Key, flags: int) -> bool:
        """An activation's state change (ActivationData.SetState) as seen by the receive path."""
        if key not in self.entries:
            return False
        self.entries[key] = (self.entries[key][0], flags)
        return True

    def find(self, key: Key, system: bool) -> Optional[Tuple[int, int]]:
        """FindTarget (system=False) / FindSystemTarget (system=True): each looks in its own
        dictionary, so an entry of the other kind is not found."""
        e = self.entries.get(key)
        if e is None or bool(e[1] & AD_SYSTEM_TARGET) != system:
            return None
        return e


def receive_batch(target_grain: np.ndarray, target_activation: np.ndarray, direction: np.ndarray,
                  ad: ActivationDirectory, n_ctx: int, request_count: Optional[Sequence[int]] = None,
                  hard_limit: int = 0, hard_limit_stateless: int = 0):
    """ReceiveMessage for a batch in arrival order (literal loop).  request_count[c] =
    GetRequestCount() of context c when the batch starts (None: limits not checked, the
    default options).  Returns (status u8[n], ctx u32[n], perm u32[n], offsets u32[n_ctx + 3])."""
    tg = np.asarray(target_grain, dtype=np.uint64).reshape(-1, 3)
    ta = np.asarray(target_activation, dtype=np.uint64).reshape(-1, 3)
    n = tg.shape[0]
    status = np.zeros(n, np.uint8)
    ctx = np.full(n, M32, np.uint32)
    counts = None if request_count is None else [int(x) for x in request_count]
    queues = [[] for _ in range(n_ctx + 2)]
    for i in range(n):
        is_st = (int(tg[i, 2]) >> 56) == CAT_SYSTEM_TARGET          # GrainId.IsSystemTarget
        key = (int(ta[i, 0]), int(ta[i, 1]), int(ta[i, 2]))
        d = int(direction[i])
        d = DIR_REQUEST if d == DIR_NULL else d
        if is_st:
            e = ad.find(key, system=True)
            if e is None:
                status[i] = RECV_REJECT_UNKNOWN
            elif d in (DIR_REQUEST, DIR_RESPONSE):
                status[i] = RECV_SYSTEM_TARGET
                ctx[i] = e[0]
            else:
                status[i] = RECV_DROPPED
        else:
            e = ad.find(key, system=False)
            if e is None or not (e[1] & AD_VALID):
                status[i] = RECV_NULL_CONTEXT
                ctx[i] = n_ctx
            else:
                c, fl = e
                limit = hard_limit_stateless if fl & AD_STATELESS_WORKER else hard_limit
                if (d != DIR_RESPONSE and counts is not None and limit > 0 and counts[c] > limit):
                    status[i] = RECV_REJECT_OVERLOADED
                else:
                    status[i] = RECV_ACTIVATION
                    ctx[i] = c
                    if counts is not None:
                        counts[c] += 1                                 # IncrementEnqueuedOnDispatcherCount
        queues[int(ctx[i]) if ctx[i] != M32 else n_ctx + 1].append(i)
    perm = np.asarray([i for q in queues for i in q], dtype=np.uint32)
    offsets = np.zeros(n_ctx + 3, np.uint32)
    offsets[1:] = np.cumsum([len(q) for q in queues])
    return status, ctx, perm, offsets


def receive_batch_np(target_grain, target_activation, direction, keys: np.ndarray, ctxs: np.ndarray,
                     flags: np.ndarray, n_ctx: int, request_count=None, hard_limit: int = 0,
                     hard_limit_stateless: int = 0):
    """Vectorised receive_batch over a directory snapshot given as arrays (keys (m,3), ctx, flags;
    distinct keys).  Same outputs.  The overload rule in closed form: the j-th message (0-based, in
    arrival order, responses included) of a Valid activation c is rejected iff it is not a response
    and j >= limit + 1 - request_count[c] -- before the first rejection every message was enqueued
    (count = request_count[c] + j), after it the count never falls back under the limit."""
    tg = np.asarray(target_grain, dtype=np.uint64).reshape(-1, 3)
    ta = np.asarray(target_activation, dtype=np.uint64).reshape(-1, 3)
    n = tg.shape[0]
    d = np.asarray(direction, dtype=np.uint8).copy()
    d[d == DIR_NULL] = DIR_REQUEST
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    kv = np.ascontiguousarray(keys.astype(">u8")).view("V24").ravel()
    order = np.argsort(kv)
    skv = kv[order]
    qv = np.ascontiguousarray(ta.astype(">u8")).view("V24").ravel()
    pos = np.searchsorted(skv, qv) if len(skv) else np.zeros(n, np.int64)
    pos_c = np.minimum(pos, max(len(skv) - 1, 0))
    found = (skv[pos_c] == qv) if len(skv) else np.zeros(n, bool)
    ent = order[pos_c] if len(skv) else np.zeros(n, np.int64)
    e_ctx = np.where(found, np.asarray(ctxs, np.uint32)[ent] if len(skv) else 0, M32).astype(np.uint32)
    e_fl = np.where(found, np.asarray(flags, np.uint32)[ent] if len(skv) else 0, 0).astype(np.uint32)
    is_st = (tg[:, 2] >> np.uint64(56)).astype(np.uint32) == CAT_SYSTEM_TARGET
    ent_st = (e_fl & AD_SYSTEM_TARGET) != 0
    status = np.full(n, RECV_NULL_CONTEXT, np.uint8)
    ctx = np.full(n, n_ctx, np.uint32)
    st_ok = is_st & found & ent_st
    status[is_st & ~(found & ent_st)] = RECV_REJECT_UNKNOWN
    ctx[is_st] = M32
    rr = st_ok & ((d == DIR_REQUEST) | (d == DIR_RESPONSE))
    status[rr] = RECV_SYSTEM_TARGET
    ctx[rr] = e_ctx[rr]
    status[st_ok & ~rr] = RECV_DROPPED
    act = ~is_st & found & ~ent_st & ((e_fl & AD_VALID) != 0)
    status[act] = RECV_ACTIVATION
    ctx[act] = e_ctx[act]
    if request_count is not None:
        rc = np.asarray(request_count, dtype=np.int64)
        idx = np.nonzero(act)[0]
        c = e_ctx[idx].astype(np.int64)
        o = np.argsort(c, kind="stable")
        cs = c[o]
        first = np.searchsorted(cs, cs, side="left")
        j = np.empty(len(idx), np.int64)
        j[o] = np.arange(len(idx)) - first
        lim = np.where((e_fl[idx] & AD_STATELESS_WORKER) != 0, hard_limit_stateless, hard_limit).astype(np.int64)
        rej = (d[idx] != DIR_RESPONSE) & (lim > 0) & (j >= lim + 1 - rc[c])
        status[idx[rej]] = RECV_REJECT_OVERLOADED
        ctx[idx[rej]] = M32
    key = np.where(ctx != M32, ctx.astype(np.int64), n_ctx + 1)
    perm = np.argsort(key, kind="stable").astype(np.uint32)
    offsets = np.zeros(n_ctx + 3, np.uint32)
    offsets[1:] = np.cumsum(np.bincount(key, minlength=n_ctx + 2))
    return status, ctx, perm, offsets
