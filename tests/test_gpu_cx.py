"""The compact probe index (gd_cx.h, GD_OPT_PROBE): a derived copy of the directory table for the route
probe, rebuilt after every change of the table.  Routes through it must equal routes through the
directory table itself (GD_OPT_PROBE 0) and the oracle, after every kind of directory change
(registration, RemoveActivation, AddActivation / multi-activation upserts, silo removal, handoff
Merge, split-and-move, clear, rehash), with the IsValidSilo filter, and when the table is not
eligible (an N0 != 0 key, more than 256 TypeCodeData) or the batch holds keys the index cannot
hold (N0 != 0, unknown types, special categories)."""
import os

import numpy as np
import pytest

import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _pair(gd, mode, cap, cx_mode="2", **kw):
    """(engine with the index: GD_OPT_PROBE = cx_mode -- 2 group reads, 3 slot reads, 1 measured choice;
    engine without: 0)."""
    silos = o.bench_silos(8)
    out = []
    for cx in (cx_mode, "0"):
        e = gd.GrainDispatch(device=0, table_capacity=cap, options={"probe": int(cx)}, **kw)
        e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
        out.append(e)
    return out, o.ring_spec(silos, mode)


def _same(a, b, keys, n_act=None):
    if n_act is None:
        ra, rb = a.route(keys), b.route(keys)
    else:
        ra, rb = a.route_bucket(keys, n_act), b.route_bucket(keys, n_act)
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(x, y)
    return ra


def _both(engines, fn):
    return [fn(e) for e in engines]


@pytest.mark.parametrize("mode,cx_mode", [("D", "2"), ("R", "2"), ("V", "2"), ("D", "1"), ("V", "3")])
def test_cx_matches_directory_through_changes(gd, mode, cx_mode):
    rng = np.random.default_rng(41)
    (a, b), spec = _pair(gd, mode, 1 << 14, cx_mode)
    tc2 = o.grain_type_code("UnitTests.OtherGrain")
    G = 5000
    reg = np.concatenate([o.grain_keys(TC, np.arange(G)), o.grain_keys(tc2, np.arange(G // 2))])
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    acts = np.arange(len(reg), dtype=np.uint32) + 3

    def batch(n=20000):
        ids = rng.integers(0, len(reg) + 300, size=n)
        k = np.concatenate([reg, o.grain_keys(TC, np.arange(G, G + 300))])[ids]
        k[::97, 0] = 5                                                   # N0 != 0: never registered
        k[::89, 2] = np.uint64(o.type_code_data(o.CAT_GRAIN, 0x777))     # a type nobody registered
        k[::211] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), np.uint64)
        return k

    _both((a, b), lambda e: e.register(reg[: G], acts[: G], owner[: G]))
    q = batch()
    st, silo, act = _same(a, b, q)
    want = o.route_batch_np(q, spec, o.DirectoryArrays(reg[:G], acts[:G], owner[:G]))
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    _same(a, b, batch(), n_act=len(reg) + 10)
    _both((a, b), lambda e: e.register(reg[G:], acts[G:], owner[G:]))        # a second type
    _same(a, b, batch(), n_act=len(reg) + 10)
    _both((a, b), lambda e: e.unregister(reg[: G: 3], acts[: G: 3]))
    _same(a, b, batch())
    up = rng.choice(len(reg), size=400, replace=False)
    ua = acts[up].copy()
    ua[::2] = gd.GD_ACT_MULTI if hasattr(gd, "GD_ACT_MULTI") else 0xFFFFFFFE
    _both((a, b), lambda e: e.upsert(reg[up], ua, owner[up]))
    _same(a, b, batch())
    _both((a, b), lambda e: e.set_valid_silos([s for s in range(8) if s != 3], 8))
    _same(a, b, batch())
    _both((a, b), lambda e: e.remove_silos([5]))
    _same(a, b, batch())
    _both((a, b), lambda e: e.set_valid_silos([], 0))
    mk = o.grain_keys(TC, np.arange(G - 100, G + 200))
    ms = rng.integers(0, 8, size=len(mk)).astype(np.uint32)
    n_ids = 90000 + len(mk)                                              # Merge compares ActivationIds
    ids = np.zeros((n_ids, 3), np.uint64)
    ids[:, 1] = rng.permutation(n_ids).astype(np.uint64)
    _both((a, b), lambda e: e.activation_ids_set(np.arange(n_ids), ids))
    _both((a, b), lambda e: e.merge(mk, np.arange(len(mk), dtype=np.uint32) + 90000, ms))
    _same(a, b, batch())
    _both((a, b), lambda e: e.split([0, 1, 2, 3], move=True))
    _same(a, b, batch())
    _both((a, b), lambda e: e.rehash(1 << 15))
    _same(a, b, batch(), n_act=len(reg) + 10)
    _both((a, b), lambda e: e.clear())
    _same(a, b, batch())
    _both((a, b), lambda e: e.register(reg, acts, owner))
    _same(a, b, batch(), n_act=len(reg) + 10)
    a.close()
    b.close()


def test_cx_ineligible_tables_fall_back(gd):
    """An N0 != 0 grain (a Guid key) or more than 256 types: the route keeps the directory probe,
    and the index returns once the table is eligible again."""
    rng = np.random.default_rng(9)
    (a, b), spec = _pair(gd, "D", 1 << 14)
    G = 3000
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    guid = np.array([[0x1234, 77, reg[0, 2]]], np.uint64)
    gown = o.ring_owner_np(spec, o.jenkins_u64x3_np(guid[:, 2], guid[:, 0], guid[:, 1])).astype(np.uint32)
    _both((a, b), lambda e: e.register(reg, np.arange(G), owner))
    _both((a, b), lambda e: e.register(guid, [999], gown))
    q = np.concatenate([reg[rng.integers(0, G, size=5000)], guid])
    st, silo, act = _same(a, b, q)
    assert act[-1] == 999 and st[-1] == o.ST_OK
    _both((a, b), lambda e: e.unregister(guid, [999]))
    st, _, act = _same(a, b, q)
    assert st[-1] == o.ST_MISS
    # 300 types of one grain number each
    many = np.concatenate([o.grain_keys(o.grain_type_code(f"T.Grain{t}"), np.array([t])) for t in range(300)])
    mown = o.ring_owner_np(spec, o.jenkins_u64x3_np(many[:, 2], many[:, 0], many[:, 1])).astype(np.uint32)
    _both((a, b), lambda e: e.register(many, np.arange(300) + 5000, mown))
    q2 = np.concatenate([q, many])
    st, _, act = _same(a, b, q2)
    assert (st[-300:] == o.ST_OK).all() and (act[-300:] == np.arange(300) + 5000).all()
    _both((a, b), lambda e: e.unregister(many[:100], np.arange(100) + 5000))   # 200 types + Ping: eligible
    st, _, act = _same(a, b, q2)
    assert (st[-300:-200] == o.ST_MISS).all() and (st[-200:] == o.ST_OK).all()
    a.close()
    b.close()


@pytest.mark.parametrize("mode,act_base", [("D", 0), ("V", 0), ("D", 1 << 26)])
def test_cx8_matches_directory_through_changes(gd, mode, act_base):
    """The 8-B index (GD_OPT_PROBE = 4: one type, N1 < 2^32, activation and silo numbers sharing a u32
    -- act_base moves the activations to 27 bits, BASELINE cfg 3's range) gives
    the directory probe's routes through every directory change -- registration, RemoveActivation,
    multi-activation upserts (GD_ACT_MULTI), IsValidSilo, silo removal, Merge, split-and-move, rehash,
    clear -- and through the changes that make it ineligible and eligible again (a second type, an
    N1 past 2^32) or change its bit split (an activation past 2^24): keys it cannot hold (other types,
    N0 != 0, large N1) miss without a probe or fall back to the 16-B index."""
    rng = np.random.default_rng(43)
    (a, b), spec = _pair(gd, mode, 1 << 14, "4")
    G = 6000
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    acts = (np.arange(G, dtype=np.uint32) * 7 + 1 + act_base).astype(np.uint32)

    def batch(n=20000, extra=None):
        pool = np.concatenate([reg, o.grain_keys(TC, np.arange(G, G + 400))] + ([extra] if extra is not None else []))
        k = pool[rng.integers(0, len(pool), size=n)]
        k[::97, 0] = 5                                                   # N0 != 0
        k[::89, 2] = np.uint64(o.type_code_data(o.CAT_GRAIN, 0x777))     # another type
        k[::83, 1] += np.uint64(1 << 32)                                 # N1 past 2^32
        return k

    _both((a, b), lambda e: e.register(reg, acts, owner))
    q = batch()
    st, silo, act = _same(a, b, q)
    want = o.route_batch_np(q, spec, o.DirectoryArrays(reg, acts, owner))
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    _same(a, b, batch(), n_act=int(acts.max()) + 10)
    _both((a, b), lambda e: e.unregister(reg[::3], acts[::3]))
    _same(a, b, batch())
    up = rng.choice(G, size=400, replace=False)
    ua = acts[up].copy()
    ua[::2] = 0xFFFFFFFE                                                 # GD_ACT_MULTI
    _both((a, b), lambda e: e.upsert(reg[up], ua, owner[up]))
    _same(a, b, batch())
    _both((a, b), lambda e: e.set_valid_silos([s for s in range(8) if s != 3], 8))
    _same(a, b, batch())
    _both((a, b), lambda e: e.remove_silos([5]))
    _same(a, b, batch())
    _both((a, b), lambda e: e.set_valid_silos([], 0))
    # ineligible: an N1 past 2^32, then an activation past 2^24, then a second type; eligible again after
    big = o.grain_keys(TC, np.array([(1 << 32) + 9]))
    bown = o.ring_owner_np(spec, o.jenkins_u64x3_np(big[:, 2], big[:, 0], big[:, 1])).astype(np.uint32)
    _both((a, b), lambda e: e.register(big, [42], bown))
    st, _, act = _same(a, b, batch(extra=big))
    _both((a, b), lambda e: e.unregister(big, [42]))
    far = o.grain_keys(TC, np.array([G + 1000]))
    fown = o.ring_owner_np(spec, o.jenkins_u64x3_np(far[:, 2], far[:, 0], far[:, 1])).astype(np.uint32)
    _both((a, b), lambda e: e.register(far, [1 << 24], fown))
    _same(a, b, batch(extra=far))
    _both((a, b), lambda e: e.unregister(far, [1 << 24]))
    other = o.grain_keys(o.grain_type_code("UnitTests.OtherGrain"), np.arange(50))
    oown = o.ring_owner_np(spec, o.jenkins_u64x3_np(other[:, 2], other[:, 0], other[:, 1])).astype(np.uint32)
    _both((a, b), lambda e: e.register(other, np.arange(50) + 90000, oown))
    _same(a, b, batch(extra=other))
    _both((a, b), lambda e: e.unregister(other, np.arange(50) + 90000))
    _same(a, b, batch())
    _both((a, b), lambda e: e.split([0, 1, 2, 3], move=True))
    _same(a, b, batch())
    _both((a, b), lambda e: e.rehash(1 << 15))
    _same(a, b, batch(), n_act=int(acts.max()) + 10)
    _both((a, b), lambda e: e.clear())
    _same(a, b, batch())
    _both((a, b), lambda e: e.register(reg, acts, owner))
    st, silo, act = _same(a, b, q)
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(act, want[2])
    a.close()
    b.close()


def _owner(spec, k):
    return o.ring_owner_np(spec, o.jenkins_u64x3_np(k[:, 2], k[:, 0], k[:, 1])).astype(np.uint32)


@pytest.mark.parametrize("mode,probe", [("D", "4"), ("V", "2"), ("D", "3"), ("D", "1")])
def test_index_kept_current_through_churn(gd, mode, probe):
    """Round 6: AddSingleActivation / RemoveActivation / AddActivation batches re-project the slots they
    touch (k_cx_sync), so the index stays current without a rebuild (GrainDirectoryPartition.cs:304-363
    are O(1) dictionary updates).  Every round -- 1 % unregistered, 1 % new grains registered, a few
    upserts -- routes equal the directory probe and the oracle, and the index was built once."""
    rng = np.random.default_rng(61)
    (a, b), spec = _pair(gd, mode, 1 << 15, probe)
    G = 12000
    reg = o.grain_keys(TC, np.arange(G))
    acts = np.arange(G, dtype=np.uint32) * 3 + 1
    live = {tuple(k): (int(x), int(s)) for k, x, s in zip(reg, acts, _owner(spec, reg))}
    _both((a, b), lambda e: e.register(reg, acts, _owner(spec, reg)))
    nxt = G

    def check(n=20000):
        keys = np.array(list(live.keys()), np.uint64).reshape(-1, 3)
        pool = np.concatenate([keys, o.grain_keys(TC, np.arange(nxt, nxt + 500))])
        q = pool[rng.integers(0, len(pool), size=n)]
        q[::101, 0] = 9                                                   # N0 != 0
        vals = np.array(list(live.values()), np.uint32).reshape(-1, 2)
        want = o.route_batch_np(q, spec, o.DirectoryArrays(keys, vals[:, 0], vals[:, 1]))
        st, silo, act = _same(a, b, q)
        np.testing.assert_array_equal(st, want[0])
        np.testing.assert_array_equal(silo, want[1])
        np.testing.assert_array_equal(act, want[2])

    check()
    builds = a.index_stats()["builds"]
    assert builds >= 1 or probe == "1"
    for r in range(5):
        keys = np.array(list(live.keys()), np.uint64).reshape(-1, 3)
        gone = keys[rng.choice(len(keys), size=len(keys) // 100, replace=False)]
        gacts = np.array([live[tuple(k)][0] for k in gone], np.uint32)
        _both((a, b), lambda e: e.unregister(gone, gacts))
        for k in gone:
            del live[tuple(k)]
        new = o.grain_keys(TC, np.arange(nxt, nxt + G // 100))
        nacts = (np.arange(len(new), dtype=np.uint32) + nxt) * 3 + 1
        _both((a, b), lambda e: e.register(new, nacts, _owner(spec, new)))
        for k, x, s in zip(new, nacts, _owner(spec, new)):
            live[tuple(k)] = (int(x), int(s))
        nxt += len(new)
        keys = np.array(list(live.keys()), np.uint64).reshape(-1, 3)
        up = keys[rng.choice(len(keys), size=50, replace=False)]
        uacts = rng.integers(0, 1 << 20, size=len(up)).astype(np.uint32)
        uacts[::5] = 0xFFFFFFFE                                           # GD_ACT_MULTI
        usil = rng.integers(0, 8, size=len(up)).astype(np.uint32)
        _both((a, b), lambda e: e.upsert(up, uacts, usil))
        for k, x, s in zip(up, uacts, usil):
            live[tuple(k)] = (int(x), int(s))
        check()
    st = a.index_stats()
    assert st["current"] == 1 and st["synced_slots"] > 0
    assert st["builds"] == builds, st                                     # no rebuild through the churn
    a.close()
    b.close()


@pytest.mark.parametrize("probe", ["4", "2", "1"])
def test_index_mixed_directory(gd, probe):
    """8 grain classes and 1 % Guid-keyed grains (UniqueKey.cs:135-143) keep the
    index: the 8-B index holds the 8 classes, the Guid keys are probed in the directory per message;
    routes equal the oracle.  Then a ninth class and activations past the 8-B layout's width arrive
    through registration (not held / redirect entries) and routes still equal the oracle."""
    from orleans_amd.workloads import mixed_grain_keys
    rng = np.random.default_rng(62)
    (a, b), spec = _pair(gd, "D", 1 << 16, probe)
    tcds = [o.type_code_data(o.CAT_GRAIN, o.grain_type_code(f"Mixed.Grain{c}")) for c in range(8)]
    G = 20000
    reg = mixed_grain_keys(tcds, G)
    acts = np.arange(G, dtype=np.uint32) + 5
    own = _owner(spec, reg)
    _both((a, b), lambda e: e.register(reg, acts, own))
    extra = mixed_grain_keys(tcds, G + 300)[G:]
    q = np.concatenate([reg, extra])[rng.integers(0, G + 300, size=40000)]
    want = o.route_batch_np(q, spec, o.DirectoryArrays(reg, acts, own))
    st, silo, act = _same(a, b, q)
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    s = a.index_stats()
    if probe != "1":
        assert s["types8"] == 8 and s["n0_live"] == G // 100, s
    # a ninth class, and activations wider than the layout's field
    t9 = o.type_code_data(o.CAT_GRAIN, o.grain_type_code("Mixed.Grain9"))
    k9 = mixed_grain_keys([t9], 500)
    wide = o.grain_keys(o.grain_type_code("Mixed.Grain0"), np.arange(10 ** 7, 10 ** 7 + 200))
    wide[:, 2] = tcds[0]
    nk = np.concatenate([k9, wide])
    na = np.concatenate([np.arange(500, dtype=np.uint32) + 7, np.arange(200, dtype=np.uint32) + (1 << 30)])
    nown = _owner(spec, nk)
    _both((a, b), lambda e: e.register(nk, na, nown))
    allk = np.concatenate([reg, nk])
    q = np.concatenate([allk, extra])[rng.integers(0, len(allk) + 300, size=40000)]
    want = o.route_batch_np(q, spec, o.DirectoryArrays(allk, np.concatenate([acts, na]), np.concatenate([own, nown])))
    st, silo, act = _same(a, b, q)
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    a.close()
    b.close()


@pytest.mark.parametrize("n_new,report", [(3000, True), (60_000, True), (300_000, True), (60_000, False)])
def test_async_directory_batches_vs_oracle(gd, n_new, report):
    """Asynchronous AddSingleActivation / RemoveActivation batches (gd_dir_register_device_async,
    gd_dir_unregister_device) of every size against the oracle's directory: first registration wins
    over duplicate keys inside a batch, a grain already registered is reported, not inserted, the first
    matching item of a removal batch removes and a wrong activation removes nothing; routes equal the
    oracle and the live count follows.  300,000 new grains in a 2M-slot table collide on their first
    free slots often enough to need more than three claim passes (REG_PASSES).  report=False: the removals
    ask for no out_removed, so they take the one-launch CAS form (k_unreg_cas); the directory's end state
    (routes, live count) must be the same."""
    import torch
    dev = torch.device("cuda:0")
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    rng = np.random.default_rng(n_new)
    G = 50_000
    e = gd.GrainDispatch(device=0, table_capacity=1 << 21, options={"probe": 4})
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    reg = o.grain_keys(TC, np.arange(G))
    acts = np.arange(G, dtype=np.uint32)
    own = _owner(spec, reg)
    e.register(reg, acts, own)
    live = {tuple(k): (int(x), int(s)) for k, x, s in zip(reg, acts, own)}
    e.route(o.grain_keys(TC, rng.integers(0, G, size=20000)))            # builds the probe index
    for rnd in range(3):
        # removals: 1 % of the live grains, each twice (the first removes), and some wrong activations
        lk = np.array(list(live.keys()), np.uint64).reshape(-1, 3)
        pick = rng.permutation(len(lk))
        gone = lk[pick[:len(lk) // 100]]
        still = lk[pick[len(lk) // 100:len(lk) // 100 + n_new // 50]]     # live through the round
        gacts = np.array([live[tuple(x)][0] for x in gone], np.uint32)
        wrong = lk[pick[-200:]]
        wacts = np.array([live[tuple(x)][0] ^ 1 for x in wrong], np.uint32)
        uk = np.concatenate([gone, gone, wrong])
        ua = np.concatenate([gacts, gacts, wacts])
        # new grains, every 7th repeated inside the batch with another value (the first wins), and grains
        # already registered (reported, not inserted)
        new_ids = np.arange(G + rnd * n_new, G + (rnd + 1) * n_new)
        rep = new_ids[::7]
        k = np.concatenate([o.grain_keys(TC, np.concatenate([new_ids, rep])), still])
        ids = np.concatenate([new_ids, rep, still[:, 1].astype(np.int64)])
        v = np.stack([(ids * 5 + rnd).astype(np.uint32), _owner(spec, k)], 1)
        v[n_new:n_new + len(rep), 0] += 1                                 # the repeats' other value
        dk = torch.from_numpy(uk.view(np.int64)).to(dev)
        da = torch.from_numpy(ua.view(np.int32)).to(dev)
        rm = torch.empty(len(ua), dtype=torch.uint8, device=dev)
        e.unregister_device(dk.data_ptr(), da.data_ptr(), len(ua), rm.data_ptr() if report else None)
        rk = torch.from_numpy(k.view(np.int64)).to(dev)
        rv = torch.from_numpy(v.view(np.int32)).to(dev)
        ov = torch.empty((len(k), 2), dtype=torch.int32, device=dev)
        oi = torch.empty(len(k), dtype=torch.uint8, device=dev)
        e.register_device_async(rk.data_ptr(), rv.data_ptr(), len(k), ov.data_ptr(), oi.data_ptr())
        e.synchronize()
        rm, ov, oi = rm.cpu().numpy(), ov.cpu().numpy().view(np.uint32), oi.cpu().numpy()
        if report:
            assert rm[:len(gone)].all() and not rm[len(gone):].any()
        for x in gone:
            del live[tuple(x)]
        assert oi[:n_new].all() and not oi[n_new:].any()                  # each new grain once, first wins
        np.testing.assert_array_equal(ov[:n_new, 0], v[:n_new, 0])
        np.testing.assert_array_equal(ov[n_new:n_new + len(rep), 0], v[:n_new:7, 0])
        np.testing.assert_array_equal(ov[n_new + len(rep):, 0],
                                      np.array([live[tuple(x)][0] for x in still], np.uint32))
        for key, val in zip(k[:n_new], v[:n_new]):
            live[tuple(key)] = (int(val[0]), int(val[1]))
        keys = np.array(list(live.keys()), np.uint64).reshape(-1, 3)
        vals = np.array(list(live.values()), np.uint32).reshape(-1, 2)
        q = np.concatenate([keys[rng.integers(0, len(keys), size=30000)], gone[:500]])
        want = o.route_batch_np(q, spec, o.DirectoryArrays(keys, vals[:, 0], vals[:, 1]))
        st, silo, act = e.route(q)
        np.testing.assert_array_equal(st, want[0])
        np.testing.assert_array_equal(silo, want[1])
        np.testing.assert_array_equal(act, want[2])
        assert e.stats()["table_live"] == len(live)
    e.close()


def test_pure_index_form_follows_the_directory(gd):
    """k_route_m's PURE form (gd_engine.h cx8_pure: one grain class, every live entry held by the 8-B
    index, none redirected -- no directory fallback compiled in) runs only while that holds as of the last
    counter read-back with no batch enqueued since: Guid-keyed grains registered asynchronously right
    before a route are found (the batch itself turns the form off), and after read-backs that show the
    index impure they keep being found; routes equal the oracle throughout."""
    import torch
    dev = torch.device("cuda:0")
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    rng = np.random.default_rng(17)
    G = 40_000
    e = gd.GrainDispatch(device=0, table_capacity=1 << 17, options={"probe": 4})
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    reg = o.grain_keys(TC, np.arange(G))
    own = _owner(spec, reg)
    e.register(reg, np.arange(G, dtype=np.uint32), own)
    live = {tuple(k): (int(i), int(s)) for i, (k, s) in enumerate(zip(reg, own))}

    def check():
        keys = np.array(list(live.keys()), np.uint64).reshape(-1, 3)
        vals = np.array(list(live.values()), np.uint32).reshape(-1, 2)
        q = keys[rng.integers(0, len(keys), size=20000)]
        want = o.route_batch_np(q, spec, o.DirectoryArrays(keys, vals[:, 0], vals[:, 1]))
        st, silo, act = e.route(q)
        np.testing.assert_array_equal(st, want[0])
        np.testing.assert_array_equal(silo, want[1])
        np.testing.assert_array_equal(act, want[2])

    check()                                                                # pure: one class, all held
    e.stats()
    guid = o.grain_keys(TC, np.arange(G, G + 200))
    guid[:, 0] = rng.integers(1, 1 << 62, size=len(guid)).astype(np.uint64)   # N0 != 0: not in the index
    gv = np.stack([np.arange(G, G + 200, dtype=np.uint32), _owner(spec, guid)], 1)
    dk = torch.from_numpy(guid.view(np.int64)).to(dev)
    dvv = torch.from_numpy(gv.view(np.int32)).to(dev)
    e.register_device_async(dk.data_ptr(), dvv.data_ptr(), len(guid))
    for k, v in zip(guid, gv):
        live[tuple(k)] = (int(v[0]), int(v[1]))
    check()                                                                # no read-back since the batch
    e.stats()                                                              # read-back: impure now
    check()
    assert e.index_stats()["out8"] >= 200
    e.close()
