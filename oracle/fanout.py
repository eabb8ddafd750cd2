"""CPU oracle for SURVEY 8 f2 -- Chirper-style follower fan-out -- TEST INFRASTRUCTURE ONLY.

Restates, in Python/numpy, what one hop of Chirper's publish path does to the
message stream, so that the GPU fan-out (``gd_fanout_*``) can be checked bit for
bit.  Only ``tests/`` and the bench tools' CPU legs import it.

Reference behaviour (paths relative to the reference root):
  * ``ChirperAccount.PublishMessage``  Samples/Chirper/ChirperGrains/ChirperAccount.cs:106-147:
    for every follower in ``State.Followers.Values`` (:131-134), in the dictionary's
    enumeration order, send ``IChirperSubscriber.NewChirp(chirp)``.
  * ``AddFollower`` :213-221 (ContainsKey -> Remove, then ``Followers[userInfo] = follower``),
    ``RemoveFollower`` :223-232, driven by ``FollowUserId`` :158-164 (the loader's
    ``AddChirperFollower``, Samples/Chirper/NetworkLoader/ChirperNetworkLoader.cs:273-279).
  * Each NewChirp is a grain call to GrainId(typeCode(ChirperAccount), followerUserId):
    it is routed (LocalGrainDirectory.CalculateTargetSilo + directory probe) and enqueued
    on the follower's activation in arrival order -- exactly the cfg-2 path.

``State.Followers`` is a ``System.Collections.Generic.Dictionary<ChirperUserInfo, ...>``
(.NET BCL, netstandard2.0 / net461; not in the reference tree).  Its enumeration order is
the slot order of its entries array, with freed slots reused LIFO by later inserts
(the published BCL algorithm: ``Remove`` pushes the entry on ``freeList``; ``Insert``
takes ``freeList`` first, else appends at ``count``; the enumerator walks
``entries[0..count)`` skipping freed entries).  ``FollowersDict`` restates exactly that.

The multi-hop cascade (cfg 4: "3-hop message propagation (frontier expansion)") is a
synthetic extension: hop h's publishers are the grains that received at least one chirp
in hop h-1 and had not published yet (a BFS frontier), in activation order -- the order
in which the bucketing stage hands the activations their queues.  Seeds publish at hop 0.

Parity: pinned by the source text above (no numeric fixtures exist in the reference for
this sample) and by the small hand-checked cases in tests/test_fanout_oracle.py.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import numpy as np

import oracle as o

CHIRPER_ACCOUNT_CLASS = "Orleans.Samples.Chirper.Grains.ChirperAccount"


class FollowersDict:
    """``State.Followers`` enumeration order under AddFollower / RemoveFollower
    (ChirperAccount.cs:213-232) with .NET ``Dictionary`` slot reuse."""

    def __init__(self):
        self.slot_key: List[int] = []      # entries[i].key (None when freed)
        self.slot_next: List[int] = []     # entries[i].next on the free list
        self.where = {}                    # key -> slot
        self.free_list = -1
        self.free_count = 0

    def _insert(self, key: int):
        if self.free_count > 0:                         # Dictionary.Insert: reuse the free list head
            i = self.free_list
            self.free_list = self.slot_next[i]
            self.free_count -= 1
            self.slot_key[i] = key
        else:                                           # append at count
            i = len(self.slot_key)
            self.slot_key.append(key)
            self.slot_next.append(-1)
        self.where[key] = i

    def remove(self, key: int) -> bool:
        i = self.where.pop(key, None)
        if i is None:
            return False
        self.slot_key[i] = None                         # hashCode = -1
        self.slot_next[i] = self.free_list              # entries[i].next = freeList
        self.free_list = i
        self.free_count += 1
        return True

    def add_follower(self, key: int):
        """AddFollower (ChirperAccount.cs:213-221): a re-follow is Remove + add, which
        lands in the slot it just freed, so it keeps its position."""
        if key in self.where:
            self.remove(key)
        self._insert(key)

    def values(self) -> List[int]:
        return [k for k in self.slot_key if k is not None]


def build_follower_csr(n_nodes: int, ops: Iterable[Tuple[int, int, int]]):
    """CSR of the follower graph from a sequence of (publisher, follower, op) with
    op = +1 (FollowUserId -> AddFollower) or -1 (UnfollowUserId -> RemoveFollower).
    Row u lists u's followers in ``State.Followers`` enumeration order.
    Returns (row_off u32[n_nodes+1], dst u32[E])."""
    rows = {}
    for pub, fol, op in ops:
        d = rows.setdefault(int(pub), FollowersDict())
        if op > 0:
            d.add_follower(int(fol))
        else:
            d.remove(int(fol))
    deg = np.zeros(n_nodes, dtype=np.int64)
    for u, d in rows.items():
        deg[u] = len(d.values())
    row_off = np.zeros(n_nodes + 1, dtype=np.uint32)
    row_off[1:] = np.cumsum(deg).astype(np.uint32)
    dst = np.zeros(int(deg.sum()), dtype=np.uint32)
    for u, d in rows.items():
        v = d.values()
        dst[row_off[u]:row_off[u] + len(v)] = v
    return row_off, dst


def csr_from_rows(rows: Sequence[Sequence[int]]):
    """CSR from explicit follower lists (already in enumeration order)."""
    deg = np.asarray([len(r) for r in rows], dtype=np.int64)
    row_off = np.zeros(len(rows) + 1, dtype=np.uint32)
    row_off[1:] = np.cumsum(deg).astype(np.uint32)
    dst = np.asarray([f for r in rows for f in r], dtype=np.uint32)
    return row_off, dst


def expand(row_off: np.ndarray, dst: np.ndarray, frontier: np.ndarray):
    """One publish round: for each publisher u in frontier order, one NewChirp per
    follower in enumeration order (ChirperAccount.cs:131-134).  Publishers outside
    [0, n_nodes) publish nothing.  Returns (target u32[M], sender u32[M])."""
    row_off = np.asarray(row_off, dtype=np.int64)
    n_nodes = len(row_off) - 1
    fr = np.asarray(frontier, dtype=np.int64)
    ok = (fr >= 0) & (fr < n_nodes)
    fr_c = np.where(ok, fr, 0)
    beg = row_off[fr_c]
    deg = np.where(ok, row_off[fr_c + 1] - beg, 0)
    m = int(deg.sum())
    item = np.repeat(np.arange(len(fr)), deg)
    start = np.zeros(len(fr), dtype=np.int64)
    if len(fr):
        start[1:] = np.cumsum(deg)[:-1]
    pos = np.arange(m, dtype=np.int64) - start[item] + beg[item]
    target = np.asarray(dst, dtype=np.uint32)[pos] if m else np.zeros(0, np.uint32)
    sender = fr[item].astype(np.uint32)
    return target, sender


def expand_loop(row_off, dst, frontier):
    """Pure-Python loop form of ``expand`` (small cases; pins the vectorised one)."""
    t, s = [], []
    n_nodes = len(row_off) - 1
    for u in frontier:
        u = int(u)
        if not 0 <= u < n_nodes:
            continue
        for j in range(int(row_off[u]), int(row_off[u + 1])):
            t.append(int(dst[j]))
            s.append(u)
    return np.asarray(t, dtype=np.uint32), np.asarray(s, dtype=np.uint32)


def next_frontier(offsets: np.ndarray, n_act: int, visited: np.ndarray):
    """Activations that received at least one message this hop and have not published
    yet, ascending (the order the bucketing hands out queues).  Marks them visited."""
    off = np.asarray(offsets, dtype=np.int64)
    got = off[1:n_act + 1] > off[:n_act]
    new = got & ~visited[:n_act]
    visited[:n_act] |= new
    return np.nonzero(new)[0].astype(np.uint32)


def cascade(row_off, dst, seeds, hops: int, spec, directory, n_act: int, type_code: int,
            my_silo: int = 0, seed_silo: int = o.M32):
    """Reference result of ``hops`` publish rounds from ``seeds`` (activation index =
    node id).  Returns a list of per-hop dicts: target, sender, status, silo, act, perm,
    offsets, frontier (the publishers of that hop)."""
    visited = np.zeros(n_act, dtype=bool)
    frontier = np.asarray(seeds, dtype=np.uint32)
    visited[frontier[frontier < n_act]] = True
    out = []
    for _ in range(hops):
        target, sender = expand(row_off, dst, frontier)
        keys = o.grain_keys(type_code, target.astype(np.int64))
        st, silo, act, _, _ = o.route_batch_np(keys, spec, directory, my_silo=my_silo, seed_silo=seed_silo)
        perm, off = o.bucket_stable(act, n_act)
        out.append(dict(frontier=frontier, target=target, sender=sender, status=st, silo=silo, act=act,
                        perm=perm, offsets=off))
        frontier = next_frontier(off, n_act, visited)
    return out
