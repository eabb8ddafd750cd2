"""KeyExt grains in the non-owner directory cache (SURVEY 8 f4 x a2), through the C ABI, against
oracle/dircache.py + oracle/keyext.py:

* AdaptiveGrainDirectoryCache over LRU<GrainId, entry> (AdaptiveGrainDirectoryCache.cs:71-127,
  LRU.cs) with GrainIds whose equality includes the KeyExt string (UniqueKey.cs:245-251): one LRU,
  one generation sequence for three-word and KeyExt entries, a KeyExt-category key with a null
  KeyExt being the three-word entry;
* LocalLookup (LocalGrainDirectory.cs:797-850) of string-keyed grains: owner by the KeyExt uniform
  hash (UniqueKey.cs:272-336), a local owner's grains from the KeyExt partition, the others from
  the cache (:93-110), hits of plain and KeyExt grains numbered in one batch order.

Entries (with their strings), generations and statistics are compared exactly after every batch."""
import numpy as np
import pytest

import dircache as co
import keyext as kx
import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)
STC = 0x2A2A2A2A
KX_TCD = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
GEO_TCD = o.type_code_data(o.CAT_GEO_CLIENT, 0)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _universe(rng, n_plain, n_str):
    """(keys u64[n,3], exts) mixing long-keyed grains (ext None), string grains (short, inline-size,
    register-path and long strings, empty, multi-byte UTF-8), compound keys (N1 != 0 + KeyExt),
    KeyExt-category keys with a null KeyExt and geo clients."""
    keys, exts = [], []
    for i in range(n_plain):
        keys.append(tuple(int(x) for x in o.grain_keys(TC, np.array([i]))[0]))
        exts.append(None)
    alphabet = list("abcxyz0189-_/") + ["é", "中", "\U0001F600"]
    for i in range(n_str):
        r = i % 6
        if r == 0:
            s = f"user-{i}".encode()
        elif r == 1:
            s = ("k" * int(rng.integers(20, 30)) + str(i)).encode()             # around the 24-B inline size
        elif r == 2:
            s = ("long/" + "".join(rng.choice(alphabet, size=int(rng.integers(60, 120)))) + str(i)).encode()
        elif r == 3:
            s = ("".join(rng.choice(alphabet, size=int(rng.integers(1, 12)))) + str(i)).encode()
        elif r == 4:
            s = b"" if i % 12 == 4 else None                                    # empty string / null KeyExt
        else:
            s = f"c{i}".encode()
        if r == 5:
            keys.append((0, i, KX_TCD))                                          # compound key: N1 + KeyExt
        elif r == 4 and s is None:
            keys.append((0, 1000 + i, KX_TCD))
        else:
            keys.append((0, 0, KX_TCD))
        exts.append(s)
    keys.append((7, 9, GEO_TCD))
    exts.append(b"eu-west")
    keys.append((7, 9, GEO_TCD))
    exts.append(b"us-east")
    return np.array(keys, np.uint64), exts


def _okey(k, x):
    k3 = tuple(int(v) for v in k)
    return k3 if x is None else k3 + (bytes(x),)


def _check(e, oc):
    assert e.cache_entries_ext() == oc.key_values()
    st = e.cache_stats()
    assert st["count"] == len(oc.entries)
    assert st["next_generation"] == oc.next_generation
    assert st["accesses"] == oc.num_accesses and st["hits"] == oc.num_hits


@pytest.mark.parametrize("max_size", [1, 7, 64, 400])
def test_cache_ops_mixed_keyext_vs_oracle(gd, max_size):
    rng = np.random.default_rng(300 + max_size)
    silos = o.bench_silos(8)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.cache_configure(max_size, [0], 8)
    oc = co.DirectoryCacheOracle(max_size)
    ukeys, uext = _universe(rng, 2 * max_size + 10, 3 * max_size + 30)
    U = len(ukeys)
    for step in range(50):
        op = int(rng.integers(0, 4))
        k = int(rng.integers(1, 2 * max_size + 12))
        ids = rng.integers(0, U, size=k)
        keys = ukeys[ids]
        exts = [uext[i] for i in ids]
        if op == 0:
            acts = rng.integers(0, 1 << 20, size=k).astype(np.uint32)
            sl = rng.integers(0, 8, size=k).astype(np.uint32)
            ver = rng.integers(-5, 1000, size=k).astype(np.int32)
            e.cache_add(keys, acts, sl, ver, exts=exts)
            for i in range(k):
                oc.add_or_update(_okey(keys[i], exts[i]), int(acts[i]), int(sl[i]), int(ver[i]))
        elif op == 1:
            found, act, silo, ver = e.cache_lookup(keys, exts=exts)
            for i in range(k):
                r = oc.lookup(_okey(keys[i], exts[i]))
                assert bool(found[i]) == (r is not None), (step, i)
                if r is not None:
                    assert (act[i], silo[i], ver[i]) == r, (step, i)
        elif op == 2:
            rem = e.cache_remove(keys, exts=exts)
            for i in range(k):
                assert bool(rem[i]) == oc.remove(_okey(keys[i], exts[i])), (step, i)
        else:
            # the plain forms on the same cache: a KeyExt-category key is its null-KeyExt entry
            found, act, silo, ver = e.cache_lookup(keys)
            for i in range(k):
                r = oc.lookup(_okey(keys[i], None))
                assert bool(found[i]) == (r is not None), (step, i)
                if r is not None:
                    assert (act[i], silo[i], ver[i]) == r, (step, i)
        _check(e, oc)
    e.cache_clear()
    oc.clear()
    _check(e, oc)
    e.close()


def test_cache_keyext_heap_compaction(gd):
    """Long strings through a small LRU: evictions free their heap bytes and the heap is compacted
    (moved strings still compare equal) as adds run past its capacity, several times over."""
    rng = np.random.default_rng(11)
    M = 300
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in o.bench_silos(4)])
    e.cache_configure(M, [], 4)
    oc = co.DirectoryCacheOracle(M)
    names = [(f"tenant-{i % 97}/" + "p" * (40 + i % 300) + f"/{i}").encode() for i in range(6000)]
    keys = np.tile(np.array([[0, 0, KX_TCD]], np.uint64), (len(names), 1))
    for rnd in range(12):
        ids = rng.integers(0, len(names), size=700)
        acts = (ids + rnd).astype(np.uint32)
        e.cache_add(keys[ids], acts, (ids % 4).astype(np.uint32), (ids % 50).astype(np.int32),
                    exts=[names[i] for i in ids])
        for j, i in enumerate(ids):
            oc.add_or_update(_okey(keys[i], names[i]), int(acts[j]), int(i % 4), int(i % 50))
        q = rng.integers(0, len(names), size=500)
        found, act, silo, ver = e.cache_lookup(keys[q], exts=[names[i] for i in q])
        for j, i in enumerate(q):
            r = oc.lookup(_okey(keys[i], names[i]))
            assert bool(found[j]) == (r is not None) and (r is None or (act[j], silo[j], ver[j]) == r)
        _check(e, oc)
    e.close()


@pytest.mark.parametrize("mode", ["D", "V"])
def test_local_lookup_route_keyext_vs_oracle(gd, mode):
    """gd_route_ext / gd_route_bucket_ext in LocalLookup mode over batches mixing long-keyed grains,
    string grains (local owner: the KeyExt partition; remote: the cache), null KeyExts, geo
    clients, system targets and GD_KEYEXT_HOST items; an invalid cached silo is MISS."""
    rng = np.random.default_rng(77)
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    local, valid = {2, 5}, set(range(7))            # silo 7 is down
    ukeys, uext = _universe(rng, 1500, 3000)
    U = len(ukeys)
    owner = np.zeros(U, np.int64)
    for i in range(U):
        n0, n1, tcd = (int(x) for x in ukeys[i])
        h = kx.ext_uniform_hash(n0, n1, tcd, uext[i]) if (tcd >> 56) in (o.CAT_KEYEXT_GRAIN, o.CAT_GEO_CLIENT) \
            else o.jenkins_u64x3(tcd, n0, n1)
        owner[i] = int(o.ring_owner_np(spec, np.array([h], np.uint32))[0])
    e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=2, seed_silo=6)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    # this silo's partition: some of the locally owned grains, plain ones and KeyExt ones
    mine = [i for i in range(U) if owner[i] in local and i % 5 != 0]
    plain_mine = [i for i in mine if uext[i] is None and (int(ukeys[i][2]) >> 56) == o.CAT_GRAIN]
    plain_set = set(plain_mine)
    ext_mine = [i for i in mine if i not in plain_set]
    e.register(ukeys[plain_mine], np.array(plain_mine, np.uint32) + 7, owner[plain_mine].astype(np.uint32))
    e.register_ext(ukeys[ext_mine], [uext[i] for i in ext_mine], np.array(ext_mine, np.uint32) + 7,
                   owner[ext_mine].astype(np.uint32))
    part = {_okey(ukeys[i], None if i in plain_set else uext[i]): (i + 7, int(owner[i])) for i in mine}
    M = 900
    e.cache_configure(M, sorted(local), 8, sorted(valid))
    oc = co.DirectoryCacheOracle(M)
    remote = [i for i in range(U) if owner[i] not in local]
    sys_key = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
    for rnd in range(5):
        add = rng.choice(remote, size=500)
        a_act = (add + 100000).astype(np.uint32)
        a_silo = rng.integers(0, 8, size=500).astype(np.uint32)
        a_ver = rng.integers(0, 50, size=500).astype(np.int32)
        e.cache_add(ukeys[add], a_act, a_silo, a_ver, exts=[uext[i] for i in add])
        for j, i in enumerate(add):
            oc.add_or_update(_okey(ukeys[i], uext[i]), int(a_act[j]), int(a_silo[j]), int(a_ver[j]))
        ids = rng.integers(0, U, size=4000)
        keys = ukeys[ids].copy()
        exts = [uext[i] for i in ids]
        kind = ["lookup"] * len(ids)
        for j in range(0, len(ids), 173):
            keys[j] = sys_key
            exts[j] = None
            kind[j] = "system"
        for j in range(5, len(ids), 191):
            if (int(keys[j][2]) >> 56) == o.CAT_KEYEXT_GRAIN:
                exts[j] = gd.GD_KEYEXT_HOST
                kind[j] = "host"
        if rnd % 2 == 0:
            st, silo, act = e.route_ext(keys, exts)
        else:
            n_act = 200000
            st, silo, act, perm, off = e.route_bucket_ext(keys, exts, n_act)
        okeys = [_okey(keys[j], exts[j]) if kind[j] == "lookup" else None for j in range(len(ids))]
        owners = [int(owner[ids[j]]) if kind[j] == "lookup" else None for j in range(len(ids))]
        want = co.local_lookup_route(okeys, owners, local, valid, part.get, oc)
        for j, (ws, wsi, wa) in enumerate(want):
            if kind[j] == "system":
                assert st[j] == o.ST_SYSTEM_TARGET and silo[j] == 2, (rnd, j)
                continue
            if kind[j] == "host":
                assert st[j] == o.ST_KEYEXT, (rnd, j)
                continue
            assert st[j] == (o.ST_OK if ws == "OK" else o.ST_MISS), (rnd, j, okeys[j])
            assert silo[j] == wsi, (rnd, j)
            assert act[j] == (o.M32 if wa is None else wa), (rnd, j)
        if rnd % 2 == 1:
            wp, wo = o.bucket_stable(act, n_act)
            np.testing.assert_array_equal(perm, wp)
            np.testing.assert_array_equal(off, wo)
        _check(e, oc)
    e.close()
