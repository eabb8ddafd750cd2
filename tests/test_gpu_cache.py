"""GPU parity for the non-owner directory cache: AdaptiveGrainDirectoryCache over
LRU (AdaptiveGrainDirectoryCache.cs, LRU.cs) and the LocalLookup route (LocalGrainDirectory.cs:
797-850), through the C ABI, against oracle/dircache.py.  Entries, generations and statistics are
compared exactly after every batch."""
import numpy as np
import pytest

import dircache as co
import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _keys(ids):
    return o.grain_keys(TC, np.asarray(ids, dtype=np.int64))


def _check(e, oc):
    got = e.cache_entries()
    assert got == oc.key_values()
    st = e.cache_stats()
    assert st["count"] == len(oc.entries)
    assert st["next_generation"] == oc.next_generation
    assert st["accesses"] == oc.num_accesses and st["hits"] == oc.num_hits


@pytest.mark.parametrize("max_size", [1, 7, 64])
def test_cache_ops_vs_oracle(gd, max_size):
    rng = np.random.default_rng(100 + max_size)
    silos = o.bench_silos(8)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.cache_configure(max_size, [0], 8)
    oc = co.DirectoryCacheOracle(max_size)
    universe = 3 * max_size + 20
    for step in range(60):
        op = rng.integers(0, 3)
        k = int(rng.integers(1, 3 * max_size + 10))
        ids = rng.integers(0, universe, size=k)
        keys = _keys(ids)
        if op == 0:
            acts = rng.integers(0, 1 << 20, size=k).astype(np.uint32)
            sl = rng.integers(0, 8, size=k).astype(np.uint32)
            ver = rng.integers(-5, 1000, size=k).astype(np.int32)
            e.cache_add(keys, acts, sl, ver)
            for i in range(k):
                oc.add_or_update(tuple(int(x) for x in keys[i]), int(acts[i]), int(sl[i]), int(ver[i]))
        elif op == 1:
            found, act, silo, ver = e.cache_lookup(keys)
            for i in range(k):
                r = oc.lookup(tuple(int(x) for x in keys[i]))
                assert bool(found[i]) == (r is not None), (step, i)
                if r is not None:
                    assert (act[i], silo[i], ver[i]) == r
        else:
            rem = e.cache_remove(keys)
            for i in range(k):
                assert bool(rem[i]) == oc.remove(tuple(int(x) for x in keys[i]))
        _check(e, oc)
    e.cache_clear()
    oc.clear()
    _check(e, oc)
    e.close()


def test_cache_large_batches(gd):
    """A batch larger than the cache (every entry it adds early is evicted by its own later adds),
    tombstone compaction, and lookups in between."""
    M = 50000
    rng = np.random.default_rng(7)
    silos = o.bench_silos(8)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.cache_configure(M, [], 8)
    oc = co.DirectoryCacheOracle(M)
    for rnd in range(6):
        k = [30000, 120000, 40000, 70000, 5000, 90000][rnd]
        ids = rng.integers(0, 200000, size=k)
        keys = _keys(ids)
        acts = rng.integers(0, 1 << 30, size=k).astype(np.uint32)
        sl = rng.integers(0, 8, size=k).astype(np.uint32)
        ver = rng.integers(0, 1 << 30, size=k).astype(np.int32)
        e.cache_add(keys, acts, sl, ver)
        kt = [tuple(int(x) for x in r) for r in keys]
        for i in range(k):
            oc.add_or_update(kt[i], int(acts[i]), int(sl[i]), int(ver[i]))
        q = _keys(rng.integers(0, 200000, size=60000))
        found, act, silo, v = e.cache_lookup(q)
        for i, kk in enumerate(q):
            r = oc.lookup(tuple(int(x) for x in kk))
            assert bool(found[i]) == (r is not None)
            if r is not None:
                assert (act[i], silo[i], v[i]) == r
        _check(e, oc)
        if rnd == 2:
            rk = _keys(rng.integers(0, 200000, size=40000))
            gone = e.cache_remove(rk)
            assert gone.sum() > 0
            for i, kk in enumerate(rk):
                assert bool(gone[i]) == oc.remove(tuple(int(x) for x in kk))
            _check(e, oc)
    e.close()


@pytest.mark.parametrize("mode", ["D", "V"])
def test_local_lookup_route_vs_oracle(gd, mode):
    """gd_route in LocalLookup mode: owned grains from the partition, the rest from the cache
    (generation updates in batch order), invalid cached silos -> MISS."""
    rng = np.random.default_rng(31)
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    local, valid = {2, 5}, set(range(7))          # silo 7 is down
    G = 4000
    reg = _keys(np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    mine = np.nonzero(np.isin(owner, list(local)))[0]
    mine = mine[mine % 5 != 0]                     # some owned grains not registered
    e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=2, seed_silo=6)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg[mine], mine.astype(np.uint32), owner[mine])
    dirmap = {tuple(int(x) for x in reg[i]): (int(i), int(owner[i])) for i in mine}
    M = 700
    e.cache_configure(M, sorted(local), 8, sorted(valid))
    oc = co.DirectoryCacheOracle(M)
    remote = np.nonzero(~np.isin(owner, list(local)))[0]
    for rnd in range(5):
        add = rng.choice(remote, size=400)
        a_act = (add + 100000).astype(np.uint32)
        a_silo = rng.integers(0, 8, size=400).astype(np.uint32)
        a_ver = rng.integers(0, 50, size=400).astype(np.int32)
        e.cache_add(reg[add], a_act, a_silo, a_ver)
        for i, gi in enumerate(add):
            oc.add_or_update(tuple(int(x) for x in reg[gi]), int(a_act[i]), int(a_silo[i]), int(a_ver[i]))
        ids = rng.integers(0, G + 300, size=3000)
        keys = _keys(ids)
        keys[::211] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
        st, silo, act = e.route(keys)
        w_st, w_silo, w_act, w_owner, _ = o.route_batch_np(keys, spec, o.DirectoryArrays(np.zeros((0, 3), np.uint64),
                                                           [], []), my_silo=2, seed_silo=6)
        lookup = w_st == o.ST_MISS                 # everything the ring routes (not special categories)
        kt = [tuple(int(x) for x in r) for r in keys]
        want = co.local_lookup_route(kt, [int(w_owner[i]) if lookup[i] else None for i in range(len(kt))],
                                     local, valid, dirmap.get, oc)
        for i, (ws, wsi, wa) in enumerate(want):
            if ws is None:
                assert st[i] == w_st[i] and silo[i] == w_silo[i]
                continue
            assert st[i] == (o.ST_OK if ws == "OK" else o.ST_MISS), (rnd, i)
            assert silo[i] == wsi, (rnd, i)
            assert act[i] == (o.M32 if wa is None else wa), (rnd, i)
        _check(e, oc)
    # membership change: silo 5 no longer local -> its grains go through the cache
    e.cache_set_silos([2], 8, sorted(valid))
    st, silo, act = e.route(reg[mine])
    kt = [tuple(int(x) for x in r) for r in reg[mine]]
    want = co.local_lookup_route(kt, [int(owner[i]) for i in mine], {2}, valid, dirmap.get, oc)
    for i, (ws, wsi, wa) in enumerate(want):
        assert st[i] == (o.ST_OK if ws == "OK" else o.ST_MISS) and silo[i] == wsi
    _check(e, oc)
    e.close()


def test_lru_reference_tests(gd):
    """LruCountTest / LruMaximumSizeTest / LruUsageTest (test/NonSilo.Tests/General/LruTest.cs) on
    the GPU cache; keys "1".."n" are grains 1..n."""
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in o.bench_silos(4)])
    e.cache_configure(10, [0], 4)
    k = lambda i: _keys([i])  # noqa: E731
    assert e.cache_stats()["count"] == 0
    e.cache_add(k(1), [1], [1], [0])
    assert e.cache_stats()["count"] == 1
    e.cache_add(k(2), [2], [1], [0])
    assert e.cache_stats()["count"] == 2
    e.cache_clear()
    for i in range(1, 16):                                  # LruMaximumSizeTest
        e.cache_add(k(i), [i], [1], [0])
    ent = e.cache_entries()
    assert len(ent) == 10 and all(tuple(int(x) for x in k(i)[0]) not in ent for i in range(1, 6))
    e.cache_clear()
    for i in range(1, 11):                                  # LruUsageTest
        e.cache_add(k(i), [i], [1], [0])
    for i in range(10, 0, -1):
        assert e.cache_lookup(k(i))[0][0] == 1
    e.cache_add(k(11), [11], [1], [0])
    ent = e.cache_entries()
    assert len(ent) == 10 and tuple(int(x) for x in k(10)[0]) not in ent
    assert all(tuple(int(x) for x in k(i)[0]) in ent for i in range(1, 10))
    e.close()


def test_microbatch_in_cache_mode_survives_rehash(gd):
    """A micro-batch (gd_microbatch_run, use_graph=1) on a handle in LocalLookup mode, then a
    gd_cache_add large enough to rehash the cache table (its device memory moves), then the same
    micro-batch again: routes, runs and the LRU state match the oracle both times (the cache mode
    runs the micro-batch eagerly, so nothing replays freed pointers)."""
    rng = np.random.default_rng(5)
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    local, valid = {1, 4}, set(range(8))
    G = 120000
    reg = _keys(np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    mine = np.nonzero(np.isin(owner, list(local)))[0]
    e = gd.GrainDispatch(device=0, table_capacity=1 << 17, my_silo=1)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg[mine], mine.astype(np.uint32), owner[mine])
    dirmap = {tuple(int(x) for x in reg[i]): (int(i), int(owner[i])) for i in mine}
    M = 20000
    e.cache_configure(M, sorted(local), 8)
    oc = co.DirectoryCacheOracle(M)
    remote = np.nonzero(~np.isin(owner, list(local)))[0]

    def add(ids):
        a_act = (ids + 500000).astype(np.uint32)
        a_silo = (ids % 8).astype(np.uint32)
        a_ver = (ids % 97).astype(np.int32)
        e.cache_add(reg[ids], a_act, a_silo, a_ver)
        for i, gi in enumerate(ids):
            oc.add_or_update(tuple(int(x) for x in reg[gi]), int(a_act[i]), int(a_silo[i]), int(a_ver[i]))

    add(rng.choice(remote, size=300))
    cap0 = e.cache_stats()["capacity"]
    mb = gd.MicroBatch(e, 4096, G)
    n = 4096
    for rnd in range(3):
        ids = rng.integers(0, G, size=n)
        mb.keys[:n] = reg[ids]
        mb.run(n, use_graph=True)
        kt = [tuple(int(x) for x in r) for r in reg[ids]]
        want = co.local_lookup_route(kt, [int(owner[i]) for i in ids], local, valid, dirmap.get, oc)
        w_st = np.array([o.ST_OK if w[0] == "OK" else o.ST_MISS for w in want], np.uint8)
        w_silo = np.array([w[1] for w in want], np.uint32)
        w_act = np.array([o.M32 if w[2] is None else w[2] for w in want], np.uint32)
        np.testing.assert_array_equal(mb.status[:n], w_st)
        np.testing.assert_array_equal(mb.silo[:n], w_silo)
        np.testing.assert_array_equal(mb.act[:n], w_act)
        wp, wo = o.bucket_stable(w_act, G)
        np.testing.assert_array_equal(mb.perm[:n], wp)
        np.testing.assert_array_equal(mb.offsets(), wo)
        _check(e, oc)
        if rnd == 0:
            add(remote[: 60000])                 # past the rehash threshold: the cache table moves
            assert e.cache_stats()["capacity"] > cap0
    mb.close()
    e.close()
