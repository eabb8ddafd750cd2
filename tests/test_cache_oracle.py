"""CPU checks of the directory-cache oracle (oracle/dircache.py) on hand-worked LRU sequences
(LRU.cs:71-76 Add, :119-146 TryGetValue, :165-182 AdjustSize)."""
import dircache as co


def test_lru_by_hand():
    c = co.DirectoryCacheOracle(3)
    for i, k in enumerate(["a", "b", "c"]):
        c.add_or_update(k, i, 0, 10 + i)                 # generations 1, 2, 3
    assert c.lookup("a") == (0, 0, 10)                   # a -> 4
    c.add_or_update("d", 3, 0, 13)                       # count 3 >= 3: evict generation 2 (b); d -> 5
    assert set(c.entries) == {"a", "c", "d"}
    assert c.key_values()["d"][3] == 5 and c.key_values()["a"][3] == 4
    c.add_or_update("c", 9, 1, 99)                       # AdjustSize still runs first: evicts c (gen 3) ...
    assert c.key_values()["c"] == (9, 1, 99, 6)          # ... then re-adds it
    assert set(c.entries) == {"a", "c", "d"}
    assert c.lookup("zz") is None
    assert (c.num_accesses, c.num_hits) == (2, 1)
    assert c.remove("a") and not c.remove("a")
    c.add_or_update("e", 1, 1, 1)                        # count 2 < 3: no eviction
    assert set(c.entries) == {"c", "d", "e"} and c.next_generation == 7
    c.clear()
    c.add_or_update("f", 1, 1, 1)
    assert c.key_values()["f"][3] == 8                   # Clear keeps nextGeneration


def test_lru_size_one():
    c = co.DirectoryCacheOracle(1)
    c.add_or_update("a", 0, 0, 0)
    c.add_or_update("a", 1, 0, 0)                        # evicts itself, re-added
    assert c.key_values() == {"a": (1, 0, 0, 2)}
    c.add_or_update("b", 2, 0, 0)
    assert c.key_values() == {"b": (2, 0, 0, 3)}


def test_local_lookup_route():
    c = co.DirectoryCacheOracle(4)
    c.add_or_update("r1", 7, 3, 0)
    c.add_or_update("r2", 8, 6, 0)                       # cached on silo 6, which is down
    d = {"m1": (5, 1)}
    out = co.local_lookup_route(["m1", "m2", "r1", "r2", "r3", "s"], [1, 1, 3, 6, 4, None], {1}, {1, 3, 4},
                                d.get, c)
    assert out == [("OK", 1, 5), ("MISS", 1, None), ("OK", 3, 7), ("MISS", 6, None), ("MISS", 4, None),
                   (None, None, None)]
    assert (c.num_accesses, c.num_hits) == (3, 2)
    assert c.key_values()["r2"][3] == 4                  # the invalid-silo hit still renews the entry


# LruTest.cs (test/NonSilo.Tests/General/LruTest.cs) restated on the oracle
def test_LruCountTest():
    c = co.DirectoryCacheOracle(10)
    assert len(c.entries) == 0
    c.add_or_update("1", 1, 0, 0)
    assert len(c.entries) == 1
    c.add_or_update("2", 2, 0, 0)
    assert len(c.entries) == 2


def test_LruMaximumSizeTest():
    c = co.DirectoryCacheOracle(10)
    for i in range(1, 16):
        c.add_or_update(str(i), i, 0, 0)
    assert len(c.entries) == 10
    assert all(str(i) not in c.entries for i in range(1, 6))


def test_LruUsageTest():
    c = co.DirectoryCacheOracle(10)
    for i in range(1, 11):
        c.add_or_update(str(i), i, 0, 0)
    for i in range(10, 0, -1):
        c.lookup(str(i))
    c.add_or_update("11", 11, 0, 0)
    assert len(c.entries) == 10 and "10" not in c.entries
    assert all(str(i) in c.entries for i in range(1, 10))
