"""CPU oracle for the non-owner directory cache -- TEST INFRASTRUCTURE ONLY.

Restates, literally and sequentially, the reference's cache on the LocalLookup path:

* ``LRU<TKey, TValue>``  src/Orleans.Core/Utils/LRU.cs
    - ``Add`` :71-76: ``AdjustSize()`` first, then a new ``TimestampedValue`` whose ``Generation`` =
      ``Interlocked.Increment(ref nextGeneration)`` (:50-56), stored with ``AddOrUpdate``.
    - ``AdjustSize`` :165-182: ``while (cache.Count >= MaximumSize)``: ``generationToFree += 1``;
      remove the entry whose ``Generation == generationToFree`` if there is one.
    - ``TryGetValue`` :119-146: a hit sets ``Generation = ++nextGeneration``; the age check never
      fires for the directory cache (maxAge = TimeSpan.MaxValue, AdaptiveGrainDirectoryCache.cs:66).
    - ``RemoveKey`` :84-92.
* ``AdaptiveGrainDirectoryCache``  src/Orleans.Runtime/GrainDirectory/AdaptiveGrainDirectoryCache.cs
    - ``AddOrUpdate(key, value, version)`` :71-77 -> ``LRU.Add``; ``Remove`` :79-83; ``Clear`` :85-88;
    - ``LookUp`` :90-109: ``NumAccesses++``, ``TryGetValue``, on a hit ``NumHits++``, returns the
      value and the ETag (version);
    - ``KeyValues`` :111-127.
* ``LocalGrainDirectory.LocalLookup`` :797-837 / ``GetLocalCacheData`` :844-850: a grain whose owner
  (CalculateTargetSilo) is not this silo is looked up in the cache; a hit whose silo is not a
  valid (active) silo yields an empty address list, i.e. no usable address.

The generation numbers are part of the observable state here: the GPU cache must reproduce them
exactly (they decide every later eviction).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

Key = Tuple[int, int, int]


class DirectoryCacheOracle:
    def __init__(self, max_size: int):
        assert max_size > 0                       # LRU ctor :61-64
        self.max_size = max_size
        self.entries: Dict[Key, list] = {}        # key -> [generation, act, silo, version]
        self.by_gen: Dict[int, Key] = {}
        self.next_generation = 0
        self.generation_to_free = 0
        self.num_accesses = 0
        self.num_hits = 0

    # LRU.AdjustSize (:165-182)
    def _adjust_size(self):
        while len(self.entries) >= self.max_size:
            self.generation_to_free += 1
            k = self.by_gen.get(self.generation_to_free)
            if k is None:
                continue
            del self.by_gen[self.generation_to_free]
            del self.entries[k]

    def _new_gen(self) -> int:
        self.next_generation += 1
        return self.next_generation

    # AdaptiveGrainDirectoryCache.AddOrUpdate -> LRU.Add (:71-76)
    def add_or_update(self, key: Key, act: int, silo: int, version: int):
        self._adjust_size()
        g = self._new_gen()
        old = self.entries.get(key)
        if old is not None:
            del self.by_gen[old[0]]
        self.entries[key] = [g, act, silo, version]
        self.by_gen[g] = key

    # AdaptiveGrainDirectoryCache.Remove -> LRU.RemoveKey (:84-92)
    def remove(self, key: Key) -> bool:
        old = self.entries.pop(key, None)
        if old is None:
            return False
        del self.by_gen[old[0]]
        return True

    def clear(self):
        self.entries.clear()
        self.by_gen.clear()

    # AdaptiveGrainDirectoryCache.LookUp (:90-109) -> LRU.TryGetValue (:119-146)
    def lookup(self, key: Key) -> Optional[Tuple[int, int, int]]:
        self.num_accesses += 1
        e = self.entries.get(key)
        if e is None:
            return None
        del self.by_gen[e[0]]
        e[0] = self._new_gen()
        self.by_gen[e[0]] = key
        self.num_hits += 1
        return e[1], e[2], e[3]

    def key_values(self) -> Dict[Key, Tuple[int, int, int, int]]:
        """KeyValues (:111-127) plus each entry's generation: key -> (act, silo, version, gen)."""
        return {k: (e[1], e[2], e[3], e[0]) for k, e in self.entries.items()}


def local_lookup_route(keys, owners, local: set, valid: set, directory_lookup, cache: DirectoryCacheOracle):
    """LocalLookup for a batch in order (LocalGrainDirectory.cs:797-837).  owners[i] = ring owner
    of keys[i] (or None for messages handled outside the lookup: system targets, membership,
    KeyExt).  Returns per message (status, silo, act) with status 'OK' / 'MISS' / None (not a
    lookup), where `directory_lookup(key)` gives the owner partition's (act, silo) or None.  A miss
    reports the ring owner as its silo and no activation (the boundary's MISS convention)."""
    out = []
    for k, own in zip(keys, owners):
        if own is None:
            out.append((None, None, None))
            continue
        if own in local:
            r = directory_lookup(k)
            out.append(("OK", r[1], r[0]) if r is not None else ("MISS", own, None))
            continue
        r = cache.lookup(k)
        if r is None:
            out.append(("MISS", own, None))
        elif r[1] not in valid:                   # GetLocalCacheData: IsValidSilo filter -> empty list
            out.append(("MISS", own, None))
        else:
            out.append(("OK", r[1], r[0]))
    return out
