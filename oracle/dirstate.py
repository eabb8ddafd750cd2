"""CPU oracle for the directory partition under membership change -- TEST
INFRASTRUCTURE ONLY.

Restates, sequentially, what one ``GrainDirectoryPartition`` (src/Orleans.Runtime/GrainDirectory/
GrainDirectoryPartition.cs) holds for the grains the GPU path handles, and how it changes:

* ``IsValidSilo`` (:242-245): ``AddActivation`` (:274-302) and ``AddSingleActivation`` (:304-326)
  refuse an activation on a silo that is not a functional directory member; ``LookUpActivations``
  (:385-441) drops such addresses from the list it returns (with the grain's VersionTag).
* ``GrainInfo`` (:68-205): ``AddSingleActivation`` keeps the first registration (SingleInstance);
  ``AddActivation`` replaces the instance (refreshing the same activation on the same silo keeps
  the tag); ``RemoveActivation`` removes the grain with its last instance; every change draws a new
  ``VersionTag = rand.Next()``.
* ``LocalGrainDirectory.AdjustLocalDirectory`` (LocalGrainDirectory.cs:351-361): on a silo's
  removal every instance located on it is removed.
* ``GrainDirectoryPartition.Merge`` (:497-522) / ``GrainInfo.Merge`` (:139-179): absent grains are
  added as they come (with their tag); for a present single-instance grain the instance lists are
  unioned (a new tag if anything was added), then only the lowest ``ActivationId``
  (``UniqueKey.CompareTo``: TypeCodeData, N0, N1) stays and the rest go to
  ``Catalog.DeleteActivations``.

VersionTag: the reference's values are random; the library and this oracle use the same
deterministic 31-bit function of (the mutating call's sequence number, the grain's uniform hash),
drawn exactly where the reference draws one.  So the tag values are pinned only by this
restatement ("parity unpinned" for the values), while *when* a tag changes follows the source.
Batches: register = AddSingleActivation per item in order; upsert = AddActivation with the last item
of a grain applied (the batch's net change decides the tag); merge = one item per grain.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Tuple

import numpy as np

import oracle as o

M32 = 0xFFFFFFFF
ACT_MULTI = 0xFFFFFFFE
Key = Tuple[int, int, int]

MERGE_INSERTED, MERGE_KEPT, MERGE_SAME, MERGE_DROPPED, MERGE_HOST, MERGE_UNION = 0, 1, 2, 3, 4, 5


def fmix32(h: int) -> int:
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def version_tag(op: int, key: Key) -> int:
    h = o.jenkins_u64x3(key[2], key[0], key[1])
    return fmix32(h ^ ((op * 0x9E3779B9) & M32)) & 0x7FFFFFFF


def key_order(k: Key):
    """UniqueKey.CompareTo (UniqueKey.cs:255-265)."""
    return (k[2], k[0], k[1])


class DirectoryState:
    def __init__(self):
        self.entries: Dict[Key, list] = {}     # key -> [act, silo, tag, single]
        self.op = 0
        self.n_valid = 0
        self.valid: set = set()
        self.ids: Dict[int, Key] = {}          # activation index -> ActivationId

    # IsValidSilo
    def set_valid(self, valid: Iterable[int], n_silos: int):
        self.n_valid = n_silos
        self.valid = set(int(x) for x in valid)

    def silo_valid(self, s: int) -> bool:
        return self.n_valid == 0 or s >= self.n_valid or s in self.valid

    def register(self, keys, acts, silos):
        """AddSingleActivation per item, batch order.  Returns (act, silo, inserted) per item."""
        self.op += 1
        out = []
        for k, a, s in zip(keys, acts, silos):
            k = tuple(int(x) for x in k)
            a, s = int(a), int(s)
            if not self.silo_valid(s):
                out.append((M32, M32, 0))
                continue
            e = self.entries.get(k)
            if e is not None:
                out.append((e[0], e[1], 0))
                continue
            self.entries[k] = [a, s, version_tag(self.op, k), True]
            out.append((a, s, 1))
        return out

    def upsert(self, keys, acts, silos):
        """AddActivation, the last valid item of a grain applied.  Returns inserted per item."""
        self.op += 1
        last = {}
        keys = [tuple(int(x) for x in k) for k in keys]
        for i, (k, s) in enumerate(zip(keys, silos)):
            if self.silo_valid(int(s)):
                last[k] = i
        ins = [0] * len(keys)
        for k, i in last.items():
            a, s = int(acts[i]), int(silos[i])
            e = self.entries.get(k)
            if e is None:
                self.entries[k] = [a, s, version_tag(self.op, k), False]
                ins[i] = 1
            elif not (e[0] == a and e[1] == s):         # a refresh of the same instance changes nothing
                e[0], e[1], e[2], e[3] = a, s, version_tag(self.op, k), False
        return ins

    def unregister(self, keys, acts):
        """RemoveActivation(grain, act): the first matching item removes the grain."""
        out = []
        for k, a in zip(keys, acts):
            k = tuple(int(x) for x in k)
            e = self.entries.get(k)
            if e is not None and e[0] == int(a):
                del self.entries[k]
                out.append(1)
            else:
                out.append(0)
        return out

    def lookup_tagged(self, keys):
        """(act, silo, tag, found): found 0 absent, 1 valid address, 2 only an invalid silo."""
        out = []
        for k in keys:
            e = self.entries.get(tuple(int(x) for x in k))
            if e is None:
                out.append((M32, M32, 0, 0))
            elif e[0] == ACT_MULTI or self.silo_valid(e[1]):
                out.append((e[0], e[1], e[2], 1))
            else:
                out.append((M32, M32, e[2], 2))
        return out

    def remove_silos(self, silos):
        """AdjustLocalDirectory for every removed silo: (removed, multi)."""
        rm = set(int(s) for s in silos)
        removed = multi = 0
        for k in list(self.entries):
            e = self.entries[k]
            if e[1] in rm:
                if e[0] == ACT_MULTI:
                    multi += 1
                else:
                    del self.entries[k]
                    removed += 1
        return removed, multi

    def set_ids(self, acts, ids):
        for a, k in zip(acts, ids):
            self.ids[int(a)] = tuple(int(x) for x in k)

    def merge(self, keys, acts, silos, tags=None):
        """Merge of a partition (distinct grains).  Returns [(status, dropped act, dropped silo)].
        tags[i] bit 31 (GD_MERGE_TAG_MULTI_INSTANCE): the incoming GrainInfo is not SingleInstance."""
        self.op += 1
        out = []
        for i, k in enumerate(keys):
            k = tuple(int(x) for x in k)
            a, s = int(acts[i]), int(silos[i])
            e = self.entries.get(k)
            if e is None:                                   # partitionData.Add (:509-512): the GrainInfo as it is
                tag = (int(tags[i]) & 0x7FFFFFFF) if tags is not None else version_tag(self.op, k)
                multi_flag = tags is not None and (int(tags[i]) & 0x80000000) != 0
                self.entries[k] = [a, s, tag, a != ACT_MULTI and not multi_flag]
                out.append((MERGE_INSERTED, M32, M32))
            elif e[0] == ACT_MULTI or a == ACT_MULTI:
                out.append((MERGE_HOST, M32, M32))
            elif not e[3]:                                  # multi-instance grain with one instance: union (:141-152)
                if e[0] == a or self.ids[a] == self.ids[e[0]]:
                    out.append((MERGE_SAME, M32, M32))
                else:
                    e[0], e[2] = ACT_MULTI, version_tag(self.op, k)
                    out.append((MERGE_UNION, M32, M32))
            elif e[0] == a or self.ids[a] == self.ids[e[0]]:
                out.append((MERGE_SAME, M32, M32))          # ContainsKey(ActivationId) -> continue (:146)
            else:
                e[2] = version_tag(self.op, k)              # modified -> rand.Next()
                if key_order(self.ids[a]) < key_order(self.ids[e[0]]):
                    out.append((MERGE_KEPT, e[0], e[1]))
                    e[0], e[1] = a, s
                else:
                    out.append((MERGE_DROPPED, a, s))
        return out

    def register_handoff(self, keys, acts, silos):
        """ProcessSiloAddEvent's RegisterMany(singleActivation: true) on the receiver
        (GrainDirectoryHandoffManager.cs:212-233): AddSingleActivation per entry, reported as
        [(status, dropped act, dropped silo)] -- INSERTED, SAME (that ActivationId holds the grain),
        DROPPED (another activation holds it: first registration wins; or the silo is not valid),
        HOST (a multi-activation entry on either side)."""
        out = []
        keys = [tuple(int(x) for x in k) for k in keys]
        pre = [self.entries.get(k) for k in keys]
        pre = [None if e is None else list(e) for e in pre]
        res = self.register(keys, acts, silos)
        for k, a, s, e0, (ga, gs, ins) in zip(keys, acts, silos, pre, res):
            a = int(a)
            if a == ACT_MULTI or ga == ACT_MULTI:
                out.append((MERGE_HOST, M32, M32))
            elif ins:
                out.append((MERGE_INSERTED, M32, M32))
            elif ga == M32:
                out.append((MERGE_DROPPED, M32, M32))
            elif self.ids.get(ga) == self.ids.get(a):
                out.append((MERGE_SAME, M32, M32))
            else:
                out.append((MERGE_DROPPED, ga, gs))
        return out

    def as_arrays(self):
        """(keys (m,3) u64, acts, silos) of the live entries, for route_batch_np / DirectoryArrays,
        with IsValidSilo applied the way LookUpActivations applies it (invalid -> absent for routing)."""
        ks = [k for k, e in self.entries.items() if e[0] == ACT_MULTI or self.silo_valid(e[1])]
        keys = np.array(ks, dtype=np.uint64).reshape(-1, 3)
        acts = np.array([self.entries[k][0] for k in ks], dtype=np.uint32)
        silos = np.array([self.entries[k][1] for k in ks], dtype=np.uint32)
        return keys, acts, silos
