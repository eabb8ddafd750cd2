"""GPU parity for the directory under membership change, through the C ABI, against
oracle/dirstate.py and oracle/dircache.py:

* IsValidSilo on registration, upsert, lookup and every route path (GrainDirectoryPartition.cs:242-245,
  :279, :310, :431);
* VersionTags through register / upsert / unregister / merge / rehash sequences (the tag changes
  exactly where GrainInfo draws rand.Next());
* silo leave sequences in ring modes D, R and V: ring rebuilt without the silo, AdjustLocalDirectory
  (LocalGrainDirectory.cs:340-361), then routing against the oracle;
* the handoff merge (GrainDirectoryPartition.Merge + GrainInfo.Merge: lowest ActivationId stays);
* AdjustLocalCache (:371-385) in LocalLookup mode.
"""
import numpy as np
import pytest

import dircache as co
import dirstate as ds
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


def _check_state(e, st, universe):
    act, silo, tag, found = e.lookup_tagged(universe)
    want = st.lookup_tagged(universe)
    np.testing.assert_array_equal(found, [w[3] for w in want])
    np.testing.assert_array_equal(act, [w[0] for w in want])
    np.testing.assert_array_equal(silo, [w[1] for w in want])
    np.testing.assert_array_equal(tag, [w[2] for w in want])
    assert e.stats()["table_live"] == len(st.entries)


def test_valid_silos_register_lookup_route(gd):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    e = gd.GrainDispatch(device=0, table_capacity=1 << 12, my_silo=1)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    st = ds.DirectoryState()
    rng = np.random.default_rng(4)
    G = 1500
    universe = _keys(np.arange(G))
    acts = np.arange(G, dtype=np.uint32)
    asilo = rng.integers(0, 10, size=G).astype(np.uint32)      # silos 8, 9: outside the mask (valid)
    # every silo valid, then silos 2 and 5 down
    out = e.register(universe[:500], acts[:500], asilo[:500])
    want = st.register(universe[:500], acts[:500], asilo[:500])
    np.testing.assert_array_equal(out[2], [w[2] for w in want])
    e.set_valid_silos([0, 1, 3, 4, 6, 7], 8)
    st.set_valid([0, 1, 3, 4, 6, 7], 8)
    out = e.register(universe[300:], acts[300:] + 7, asilo[300:])   # refused where the silo is invalid
    want = st.register(universe[300:], acts[300:] + 7, asilo[300:])
    np.testing.assert_array_equal(out[0], [w[0] for w in want])
    np.testing.assert_array_equal(out[1], [w[1] for w in want])
    np.testing.assert_array_equal(out[2], [w[2] for w in want])
    ins = e.upsert(universe[100:200], acts[100:200] + 1000, (asilo[100:200] + 1) % 10)
    np.testing.assert_array_equal(ins, st.upsert(universe[100:200], acts[100:200] + 1000, (asilo[100:200] + 1) % 10))
    _check_state(e, st, universe)
    # routes: an entry on an invalid silo is a MISS (empty address list)
    q = _keys(rng.integers(0, G + 100, size=20000))
    s_, si, a_ = e.route(q)
    k, a, sl = st.as_arrays()
    w = o.route_batch_np(q, spec, o.DirectoryArrays(k, a, sl), my_silo=1)
    np.testing.assert_array_equal(s_, w[0])
    np.testing.assert_array_equal(si, w[1])
    np.testing.assert_array_equal(a_, w[2])
    assert (w[0] == o.ST_MISS).sum() > 0
    # back to every silo valid
    e.set_valid_silos([], 0)
    st.set_valid([], 0)
    _check_state(e, st, universe)
    e.close()


def test_version_tags_sequence(gd):
    """register / upsert / unregister / merge in random batches, a rehash in the middle: every tag
    and value equals the oracle's after every call."""
    rng = np.random.default_rng(8)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in o.bench_silos(4)])
    st = ds.DirectoryState()
    U = 3000
    universe = _keys(np.arange(U))
    ids = np.zeros((1 << 16, 3), np.uint64)
    ids[:, 0] = rng.integers(0, 1 << 62, size=1 << 16, dtype=np.int64).astype(np.uint64)
    ids[:, 1] = rng.integers(0, 1 << 62, size=1 << 16, dtype=np.int64).astype(np.uint64)
    ids[rng.random(1 << 16) < 0.1, 0] = 7                       # N0 ties: N1 decides
    e.activation_ids_set(np.arange(1 << 16), ids)
    st.set_ids(np.arange(1 << 16), ids)
    for step in range(40):
        op = int(rng.integers(0, 4))
        k = int(rng.integers(1, 900))
        sel = rng.integers(0, U, size=k)
        keys = universe[sel]
        acts = rng.integers(0, 1 << 16, size=k).astype(np.uint32)
        silos = rng.integers(0, 4, size=k).astype(np.uint32)
        if op == 0:
            out = e.register(keys, acts, silos)
            want = st.register(keys, acts, silos)
            np.testing.assert_array_equal(out[2], [w[2] for w in want])
            np.testing.assert_array_equal(out[0], [w[0] for w in want])
        elif op == 1:
            if rng.random() < 0.3:
                acts[rng.random(k) < 0.3] = ds.ACT_MULTI
            np.testing.assert_array_equal(e.upsert(keys, acts, silos), st.upsert(keys, acts, silos))
        elif op == 2:
            cur = np.array([st.entries.get(tuple(int(x) for x in kk), [0])[0] for kk in keys], np.uint32)
            cur[rng.random(k) < 0.3] += 1
            np.testing.assert_array_equal(e.unregister(keys, cur), st.unregister(keys, cur))
        else:
            sel = np.unique(sel)
            keys = universe[sel]
            k = len(sel)
            acts = rng.integers(0, 1 << 16, size=k).astype(np.uint32)
            same = rng.random(k) < 0.2
            acts[same] = [st.entries.get(tuple(int(x) for x in kk), [a])[0] for kk, a in zip(keys[same], acts[same])]
            tags = rng.integers(0, 1 << 31, size=k).astype(np.int32) if rng.random() < 0.5 else None
            acts[acts == ds.ACT_MULTI] = 5
            silos = silos[:k]
            got = e.merge(keys, acts, silos, tags)
            want = st.merge(keys, acts, silos, tags)
            np.testing.assert_array_equal(got[0], [w[0] for w in want])
            np.testing.assert_array_equal(got[1], [w[1] for w in want])
            np.testing.assert_array_equal(got[2], [w[2] for w in want])
        if step == 20:
            e.rehash(1 << 14)
        _check_state(e, st, universe)
    e.close()


def test_merge_rules_and_duplicates(gd):
    """Hand-built conflicts: lower incoming ActivationId kept, higher dropped, same activation,
    multi-activation grains left to the host, and a batch naming a grain twice is refused whole."""
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in o.bench_silos(4)])
    st = ds.DirectoryState()
    ids = np.array([[5, 1, 0], [5, 0, 0], [4, 9, 0], [9, 9, 0], [0, 0, 1], [7, 7, 0]], np.uint64)
    e.activation_ids_set(np.arange(6), ids)
    st.set_ids(np.arange(6), ids)
    g = _keys([10, 11, 12, 13, 14])
    e.register(g[:4], [0, 0, 3, 3], [1, 1, 2, 2])
    st.register(g[:4], [0, 0, 3, 3], [1, 1, 2, 2])
    e.upsert(g[4:], [ds.ACT_MULTI], [1])
    st.upsert(g[4:], [ds.ACT_MULTI], [1])
    # grain 10: id (5,0) < (5,1) -> incoming kept; 11: (0,0,tcd 1) has the larger TypeCodeData -> dropped;
    # 12: id (4,9) < (9,9) -> kept; 13: same activation; 14: multi -> host; 15: new
    mk = _keys([10, 11, 12, 13, 14, 15])
    got = e.merge(mk, [1, 4, 2, 3, 5, 5], [3, 3, 0, 2, 0, 1])
    want = st.merge(mk, [1, 4, 2, 3, 5, 5], [3, 3, 0, 2, 0, 1])
    assert got[0].tolist() == [ds.MERGE_KEPT, ds.MERGE_DROPPED, ds.MERGE_KEPT, ds.MERGE_SAME, ds.MERGE_HOST,
                               ds.MERGE_INSERTED]
    assert got[0].tolist() == [w[0] for w in want]
    assert got[1].tolist() == [w[1] for w in want] and got[2].tolist() == [w[2] for w in want]
    assert (got[1][0], got[2][0]) == (0, 1) and (got[1][1], got[2][1]) == (4, 3)
    universe = _keys(np.arange(8, 20))
    _check_state(e, st, universe)
    # multi-instance grains (AddActivation) holding one instance: another instance -> the lists are
    # unioned (GD_MERGE_UNION, the entry becomes GD_ACT_MULTI with a new tag); the same one -> SAME
    mi = _keys([18, 19])
    e.upsert(mi, [5, 4], [1, 2])
    st.upsert(mi, [5, 4], [1, 2])
    got = e.merge(mi, [2, 4], [0, 2])
    want = st.merge(mi, [2, 4], [0, 2])
    assert got[0].tolist() == [ds.MERGE_UNION, ds.MERGE_SAME] == [w[0] for w in want]
    _check_state(e, st, universe)
    live = e.stats()["table_live"]
    with pytest.raises(gd.GrainDispatchError):
        e.merge(_keys([16, 17, 16]), [1, 2, 3], [0, 0, 0])
    st.op += 1                                      # a refused call still takes its sequence number
    assert e.stats()["table_live"] == live
    _check_state(e, st, universe)
    e.close()


def _ring_without(mode, silos, gone):
    """Ring of the remaining silos, owners given as original silo indices (AddServer over them)."""
    keep = [i for i in range(len(silos)) if i not in gone]
    spec = o.ring_spec([silos[i] for i in keep], mode)
    return keep, o.RingSpec(spec.mode, spec.points, [keep[x] for x in spec.owners])


@pytest.mark.parametrize("mode", ["D", "R", "V"])
def test_silo_leave_sequence(gd, mode):
    """Silos 3, 6, 0 leave one after another: each time the ring is rebuilt without them
    (RemoveServer), AdjustLocalDirectory drops the entries on the dead silo, and the next batch
    routes exactly as the oracle's directory over the remaining silos."""
    silos = o.bench_silos(8)
    G = 20000
    reg = _keys(np.arange(G))
    rng = np.random.default_rng(12)
    asilo = rng.integers(0, 8, size=G).astype(np.uint32)         # activations anywhere in the cluster
    e = gd.GrainDispatch(device=0, table_capacity=1 << 16, my_silo=1, seed_silo=2)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, np.arange(G), asilo)
    st = ds.DirectoryState()
    st.register(reg, np.arange(G), asilo)
    gone = []
    for leaver in (3, 6, 0):
        gone.append(leaver)
        keep, spec = _ring_without(mode, silos, gone)
        e.ring_set(mode, np.asarray(spec.points, np.int64) if mode != "V" else np.asarray(spec.points, np.uint32),
                   np.asarray(spec.owners, np.uint32))
        r = e.remove_silos([leaver])
        wr, wm = st.remove_silos([leaver])
        assert (r["removed"], r["multi"]) == (wr, wm) and wr > 0
        q = _keys(rng.integers(0, G + 500, size=30000))
        s_, si, a_ = e.route(q)
        k, a, sl = st.as_arrays()
        w = o.route_batch_np(q, spec, o.DirectoryArrays(k, a, sl), my_silo=1, seed_silo=2)
        np.testing.assert_array_equal(s_, w[0])
        np.testing.assert_array_equal(si, w[1])
        np.testing.assert_array_equal(a_, w[2])
        assert not np.isin(si[s_ == o.ST_OK], gone).any()
        _check_state(e, st, reg[::7])
    e.close()


def test_handoff_after_leave_two_partitions(gd):
    """Two handles hold the partitions of silos {0..3} and {4..7}.  A silo of A whose range passes to
    a silo of B leaves: the entries whose owner under the new ring is no longer kept move from A
    (gd_dir_split) and merge into B (gd_dir_merge), where B already holds some of those grains with
    other activations; both sides equal the oracle's partitions afterwards."""
    mode = "D"
    silos = o.bench_silos(8)
    G = 12000
    reg = _keys(np.arange(G))
    rng = np.random.default_rng(21)
    spec = o.ring_spec(silos, mode)
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    ids = np.zeros((2 * G, 3), np.uint64)
    ids[:, 0] = rng.integers(0, 1 << 62, size=2 * G, dtype=np.int64).astype(np.uint64)
    ids[:, 1] = rng.integers(0, 1 << 62, size=2 * G, dtype=np.int64).astype(np.uint64)
    A = gd.GrainDispatch(device=0, table_capacity=1 << 15, my_silo=0)
    B = gd.GrainDispatch(device=0, table_capacity=1 << 15, my_silo=4)
    sa, sb = ds.DirectoryState(), ds.DirectoryState()
    for h, s_ in ((A, sa), (B, sb)):
        h.ring_set_silos(mode, [(x.ip, x.port, x.gen) for x in silos])
        h.activation_ids_set(np.arange(2 * G), ids)
        s_.set_ids(np.arange(2 * G), ids)
    mine_a = owner < 4
    A.register(reg[mine_a], np.nonzero(mine_a)[0], owner[mine_a])
    sa.register(reg[mine_a], np.nonzero(mine_a)[0], owner[mine_a])
    mine_b = ~mine_a
    B.register(reg[mine_b], np.nonzero(mine_b)[0], owner[mine_b])
    sb.register(reg[mine_b], np.nonzero(mine_b)[0], owner[mine_b])
    # the leaver: a silo of A whose range passes (at least partly) to a silo of B
    leaver = None
    for c in range(4):
        _, ns = _ring_without(mode, silos, [c])
        oc = owner == c
        no = o.ring_owner_np(ns, o.jenkins_u64x3_np(reg[oc, 2], reg[oc, 0], reg[oc, 1]))
        if (no >= 4).any():
            leaver = c
            break
    assert leaver is not None
    # B already registered a competing activation (index G + g) for some grains owned by the leaver
    comp = np.nonzero(owner == leaver)[0][::3]
    B.register(reg[comp], comp + G, np.full(len(comp), 5, np.uint32))
    sb.register(reg[comp], comp + G, np.full(len(comp), 5, np.uint32))
    keep, nspec = _ring_without(mode, silos, [leaver])
    for h in (A, B):
        h.ring_set(mode, np.asarray(nspec.points, np.int64), np.asarray(nspec.owners, np.uint32))
    mk, ma, ms = A.split([x for x in range(4) if x != leaver], move=True)
    nown = o.ring_owner_np(nspec, o.jenkins_u64x3_np(mk[:, 2], mk[:, 0], mk[:, 1]))
    assert len(mk) > 0 and np.isin(nown, [4, 5, 6, 7]).all()
    for kk in mk:
        del sa.entries[tuple(int(x) for x in kk)]
    got = B.merge(mk, ma, ms)
    want = sb.merge(mk, ma, ms)
    np.testing.assert_array_equal(got[0], [w[0] for w in want])
    np.testing.assert_array_equal(got[1], [w[1] for w in want])
    np.testing.assert_array_equal(got[2], [w[2] for w in want])
    assert {int(x) for x in np.unique(got[0])} >= {ds.MERGE_INSERTED, ds.MERGE_KEPT, ds.MERGE_DROPPED}
    # AdjustLocalDirectory on both sides
    for h, s_ in ((A, sa), (B, sb)):
        r = h.remove_silos([leaver])
        assert r["removed"] == s_.remove_silos([leaver])[0]
        _check_state(h, s_, reg)
    A.close()
    B.close()


def test_adjust_local_cache(gd):
    """LocalLookup mode: after silo 6 leaves, cache entries pointing at silo 6 and entries for grains a
    local silo now owns are removed (LRU.RemoveKey: generations untouched)."""
    silos = o.bench_silos(8)
    G = 6000
    reg = _keys(np.arange(G))
    rng = np.random.default_rng(33)
    local = {1, 2}
    e = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=1)
    e.ring_set_silos("V", [(s.ip, s.port, s.gen) for s in silos])
    M = 3000
    e.cache_configure(M, sorted(local), 8)
    oc = co.DirectoryCacheOracle(M)
    ids = rng.integers(0, G, size=2500)
    a_act = (ids + 100).astype(np.uint32)
    a_silo = rng.integers(0, 8, size=2500).astype(np.uint32)
    e.cache_add(reg[ids], a_act, a_silo, np.zeros(2500, np.int32))
    for i, gi in enumerate(ids):
        oc.add_or_update(tuple(int(x) for x in reg[gi]), int(a_act[i]), int(a_silo[i]), 0)
    keep, nspec = _ring_without("V", silos, [6])
    e.ring_set("V", np.asarray(nspec.points, np.uint32), np.asarray(nspec.owners, np.uint32))
    r = e.remove_silos([6])
    n_rm = 0
    for kk, v in list(oc.key_values().items()):
        own = int(o.ring_owner_np(nspec, o.jenkins_u64x3_np(np.array([kk[2]], np.uint64), np.array([kk[0]], np.uint64),
                                                             np.array([kk[1]], np.uint64)))[0])
        if own in local or v[1] == 6:
            oc.remove(kk)
            n_rm += 1
    assert r["cache_removed"] == n_rm > 0
    assert e.cache_entries() == oc.key_values()
    e.close()
