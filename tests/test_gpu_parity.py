"""GPU parity: libgraindispatch (through the C ABI) against the CPU oracle.

Every result is compared bit-for-bit (integer path).  Sizes stay where the
oracle finishes in seconds, except the full-size property checks at the end.
"""
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


def _engine(gd, silos, mode="D", cap=1 << 12, my_silo=0, seed_silo=o.M32, buckets=30):
    e = gd.GrainDispatch(device=0, table_capacity=cap, my_silo=my_silo, seed_silo=seed_silo)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos], buckets)
    return e


def _silo_tuples(silos):
    return [(s.ip, s.port, s.gen) for s in silos]


# ----------------------------------------------------------------------------- ring
RING_SETS = {
    "bench8": o.bench_silos(8),
    "one": o.bench_silos(1),
    "two": o.bench_silos(2),
    "s64": [o.Silo(f"10.1.{i // 250}.{i % 250 + 1}", 11111 + (i % 3), 1 + (i % 5)) for i in range(64)],
    # RingTests_Standalone silos: 127.0.0.1:0 gen 1..5, all-negative consistent hashes
    "loopback5": [o.Silo("127.0.0.1", 0, g) for g in range(1, 6)],
    "ipv6": [o.Silo("fe80::1", 11111, 3), o.Silo("2001:db8::42", 30000, 7), o.Silo("::ffff:10.0.0.9", 11111, 1)],
}


def _edge_hashes(points):
    hs = [0, 1, 0x7FFFFFFF, 0x80000000, 0x80000001, 0xFFFFFFFF]
    for p in points:
        p &= o.M32
        hs += [(p - 1) & o.M32, p, (p + 1) & o.M32]
    rng = np.random.default_rng(7)
    return np.concatenate([np.asarray(hs, dtype=np.uint32),
                           rng.integers(0, 1 << 32, size=20000, dtype=np.uint64).astype(np.uint32)])


@pytest.mark.parametrize("mode", ["D", "R", "V"])
@pytest.mark.parametrize("name", sorted(RING_SETS))
def test_ring_lookup_hashes(gd, mode, name):
    silos = RING_SETS[name]
    spec = o.ring_spec(silos, mode)
    e = _engine(gd, silos, mode)
    hs = _edge_hashes(spec.points)
    got = e.ring_lookup_hashes(hs)
    want = o.ring_owner_np(spec, hs)
    np.testing.assert_array_equal(got, want.astype(np.uint32))
    # and the scan-form oracle (the reference loop itself) on the edge cases
    for h in hs[:64]:
        if mode == "D":
            pos = o.ring_d_lookup(spec.points, int(h))
        elif mode == "R":
            pos = o.ring_r_lookup(spec.points, int(h))
        else:
            pos = o.ring_v_lookup(spec.points, int(h))
        assert spec.owners[pos] == got[list(hs).index(h)]
    e.close()


def test_ring_ties_mode_d(gd):
    """Equal consistent hashes: the scan from the end picks the LAST equal entry
    (LocalGrainDirectory.cs:521-529); insertion puts newcomers before equals."""
    pts = np.array([-100, 5, 5, 5, 900], dtype=np.int64)
    own = np.array([3, 0, 1, 2, 4], dtype=np.uint32)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.ring_set("D", pts, own)
    hs = np.array([4, 5, 6, 899, 900, 0xFFFFFF9C, 0xFFFFFF9B, 0x7FFFFFFF, 0x80000000], dtype=np.uint32)
    got = e.ring_lookup_hashes(hs)
    want = [own[o.ring_d_lookup(pts.tolist(), int(h))] for h in hs]
    assert got.tolist() == want
    assert got[1] == 2 and got[0] == 3 and got[6] == 4
    e.close()


def test_ring_rejects_unsorted(gd):
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    with pytest.raises(gd.GrainDispatchError):
        e.ring_set("D", np.array([5, 1], dtype=np.int64), np.array([0, 1], dtype=np.uint32))
    with pytest.raises(gd.GrainDispatchError):
        e.ring_set("V", np.array([5, 5], dtype=np.uint32), np.array([0, 1], dtype=np.uint32))
    with pytest.raises(gd.GrainDispatchError):
        e.route(o.grain_keys(TC, np.arange(4)))  # no ring installed
    e.close()


# ----------------------------------------------------------------------------- directory
def test_register_first_wins_and_lookup(gd):
    silos = o.bench_silos(8)
    e = _engine(gd, silos, cap=1 << 12)
    rng = np.random.default_rng(11)
    ks = rng.integers(0, 500, size=2000)                       # many duplicates in the batch
    keys = o.grain_keys(TC, ks)
    acts = np.arange(2000, dtype=np.uint32) + 7
    sil = (np.arange(2000) % 8).astype(np.uint32)
    got_act, got_silo, ins = e.register(keys, acts, sil)
    part = o.DirectoryPartition()
    for i in range(2000):
        a, s, new = part.add_single_activation(tuple(int(x) for x in keys[i]), int(acts[i]), int(sil[i]))
        assert (got_act[i], got_silo[i], ins[i]) == (a, s, int(new)), i
    # a second batch re-registering: all get the existing address back
    got_act2, got_silo2, ins2 = e.register(keys[:300], acts[:300] + 10000, sil[:300])
    assert ins2.sum() == 0
    np.testing.assert_array_equal(got_act2, got_act[:300])
    # lookup hits and misses
    probe = o.grain_keys(TC, np.arange(0, 800))
    la, ls, lf = e.lookup(probe)
    for i in range(800):
        v = part.lookup(tuple(int(x) for x in probe[i]))
        if v is None:
            assert lf[i] == 0 and la[i] == o.M32 and ls[i] == o.M32
        else:
            assert lf[i] == 1 and (la[i], ls[i]) == v
    assert e.stats()["table_live"] == len(part.data)
    e.close()


def test_unregister_semantics(gd):
    e = _engine(gd, o.bench_silos(8), cap=1 << 12)
    keys = o.grain_keys(TC, np.arange(100))
    e.register(keys, np.arange(100), np.zeros(100))
    part = o.DirectoryPartition()
    for i in range(100):
        part.add_single_activation(tuple(int(x) for x in keys[i]), i, 0)
    # wrong activation ids do not remove; duplicates: only the first removes
    ukeys = np.concatenate([keys[:10], keys[:10], keys[20:30]])
    uacts = np.concatenate([np.arange(10), np.arange(10), np.arange(20, 30) + 1])
    rem = e.unregister(ukeys, uacts)
    want = [int(part.remove_activation(tuple(int(x) for x in ukeys[i]), int(uacts[i]))) for i in range(30)]
    assert rem.tolist() == want
    la, ls, lf = e.lookup(keys)
    for i in range(100):
        v = part.lookup(tuple(int(x) for x in keys[i]))
        assert bool(lf[i]) == (v is not None)
    # re-register a removed grain: a new entry, in the first tombstone of its chain (round 6: the
    # claim probes past tombstones for the key, then reuses the first one)
    a, s, ins = e.register(keys[:5], np.arange(5) + 500, np.ones(5))
    assert ins.tolist() == [1] * 5 and a.tolist() == list(range(500, 505))
    st = e.stats()
    assert st["table_live"] == 95 and st["table_tombstones"] == 5
    e.close()


def test_rehash_growth(gd):
    e = _engine(gd, o.bench_silos(8), cap=1024)
    keys = o.grain_keys(TC, np.arange(5000))
    a, s, ins = e.register(keys, np.arange(5000), np.arange(5000) % 8)
    assert ins.all()
    assert e.stats()["table_capacity"] >= 8192
    la, ls, lf = e.lookup(keys)
    assert lf.all() and np.array_equal(la, np.arange(5000))
    e.rehash(1 << 15)
    la, ls, lf = e.lookup(keys)
    assert lf.all() and np.array_equal(ls, np.arange(5000) % 8)
    e.clear()
    assert e.lookup(keys)[2].sum() == 0
    e.close()


# ----------------------------------------------------------------------------- route
def _special_keys():
    ks = [
        o.UniqueKey(0, 77, o.type_code_data(o.CAT_SYSTEM_TARGET, 12)).as_tuple(),   # system target
        o.MEMBERSHIP_TABLE_ID.as_tuple(),                                             # membership grain
        o.UniqueKey(0, 5, o.type_code_data(o.CAT_KEYEXT_GRAIN, TC)).as_tuple(),      # KeyExt
        o.UniqueKey(3, 4, o.type_code_data(o.CAT_GEO_CLIENT, 0)).as_tuple(),         # geo client
        o.guid_key("0d2b3e5a-1111-4c3b-9f4e-aa0000000001", o.CAT_GRAIN, TC).as_tuple(),  # guid grain
        o.UniqueKey(0, 1, o.type_code_data(o.CAT_CLIENT, 0)).as_tuple(),              # client
        o.UniqueKey(0, 0, 0).as_tuple(),
        (o.M64, o.M64, o.type_code_data(o.CAT_GRAIN, -1)),                            # negative type code
    ]
    return np.array(ks, dtype=np.uint64)


@pytest.mark.parametrize("mode", ["D", "R", "V"])
def test_route_matches_oracle(gd, mode):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    e = _engine(gd, silos, mode, cap=1 << 14, my_silo=3, seed_silo=5)
    reg_k = o.grain_keys(TC, np.arange(3000))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg_k[:, 2], reg_k[:, 0], reg_k[:, 1]))
    e.register(reg_k, np.arange(3000), owner)
    special = _special_keys()
    e.register(special[4:5], [99999], [6])                      # a registered guid grain
    rng = np.random.default_rng(5)
    keys = np.concatenate([o.grain_keys(TC, rng.integers(0, 6000, size=20000)), special,
                           o.grain_keys(-123456, rng.integers(-50, 50, size=500))])
    d = o.DirectoryArrays(np.concatenate([reg_k, special[4:5]]), np.append(np.arange(3000), 99999),
                          np.append(owner, 6))
    want = o.route_batch_np(keys, spec, d, my_silo=3, seed_silo=5)
    st, silo, act = e.route(keys)
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    # CalculateTargetSilo only (no probe)
    np.testing.assert_array_equal(e.ring_owner(keys), want[3])
    # the per-message reference loop on the special rows
    dd = {tuple(int(x) for x in d_k): (int(a), int(s)) for d_k, a, s in
          zip(np.concatenate([reg_k, special[4:5]]), np.append(np.arange(3000), 99999), np.append(owner, 6))}
    loop = o.route_batch(special, spec, dd, my_silo=3, seed_silo=5)
    np.testing.assert_array_equal(st[20000:20008], loop[0])
    np.testing.assert_array_equal(silo[20000:20008], loop[1])
    e.close()


def test_route_empty_and_tiny(gd):
    e = _engine(gd, o.bench_silos(8))
    st, silo, act = e.route(np.zeros((0, 3), dtype=np.uint64))
    assert len(st) == 0
    st, silo, act = e.route(o.grain_keys(TC, [42]))
    assert st[0] == o.ST_MISS and act[0] == o.M32
    e.close()


# ----------------------------------------------------------------------------- bucket
@pytest.mark.parametrize("n,n_act", [(0, 0), (0, 10), (1, 1), (5, 0), (4095, 8), (4096, 8), (4097, 17),
                                     (12345, 255), (12345, 256), (70000, 1 << 20), (100000, 3),
                                     (65536, 65535), (200001, 1 << 24)])
def test_bucket_matches_oracle(gd, n, n_act):
    rng = np.random.default_rng(n * 31 + n_act)
    acts = rng.integers(0, max(1, n_act + n_act // 8 + 1), size=n).astype(np.uint32)
    if n:
        acts[rng.random(n) < 0.01] = o.M32                    # unrouted messages
    e = _engine(gd, o.bench_silos(8))
    perm, off = e.bucket(acts, n_act)
    wp, wo = o.bucket_stable(acts, n_act)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()


@pytest.mark.parametrize("shape", ["first", "last", "ends", "trailing_only"])
@pytest.mark.parametrize("n_act", [1 << 20, 100_000, 16_383, 3])
def test_bucket_starts_empty_runs(gd, shape, n_act):
    """Bucket starts across long runs of empty activations: the reverse min-scan's carries
    (k_starts_rangescan's digit-base carry, or the device-wide scan) must cross whole empty digit
    ranges, and an empty tail takes n."""
    n = 50_000
    rng = np.random.default_rng(n_act + len(shape))
    if shape == "first":
        acts = np.zeros(n, np.uint32)
    elif shape == "last":
        acts = np.full(n, n_act - 1, np.uint32)
    elif shape == "ends":
        acts = np.where(rng.random(n) < 0.5, 0, n_act - 1).astype(np.uint32)
    else:
        acts = np.full(n, o.M32, np.uint32)                     # every message unrouted
    e = _engine(gd, o.bench_silos(8))
    perm, off = e.bucket(acts, n_act)
    wp, wo = o.bucket_stable(acts, n_act)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()


def test_bucket_fifo_loop_small(gd):
    rng = np.random.default_rng(2)
    acts = rng.integers(0, 9, size=3000).astype(np.uint32)
    e = _engine(gd, o.bench_silos(8))
    perm, off = e.bucket(acts, 7)
    wp, wo = o.bucket_fifo_loop(acts, 7)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()


def test_bucket_skewed(gd):
    """Zipf-like skew: one activation takes most of the batch (hot grain)."""
    rng = np.random.default_rng(9)
    n = 300000
    acts = np.where(rng.random(n) < 0.7, 12345, rng.integers(0, 1 << 17, size=n)).astype(np.uint32)
    e = _engine(gd, o.bench_silos(8))
    perm, off = e.bucket(acts, 1 << 17)
    wp, wo = o.bucket_stable(acts, 1 << 17)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()


def test_route_bucket_fused(gd):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    e = _engine(gd, silos, "D", cap=1 << 15)
    G = 10000
    reg_k = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg_k[:, 2], reg_k[:, 0], reg_k[:, 1]))
    e.register(reg_k, np.arange(G), owner)
    rng = np.random.default_rng(3)
    keys = o.grain_keys(TC, rng.integers(0, G + 500, size=250000))
    st, silo, act, perm, off = e.route_bucket(keys, G)
    d = o.DirectoryArrays(reg_k, np.arange(G), owner)
    want = o.route_batch_np(keys, spec, d)
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    wp, wo = o.bucket_stable(want[2], G)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()


# ----------------------------------------------------------------------------- device API + full size
BALANCED_GENS = [138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820]   # bench.py SILO_SETS["balanced"]


@pytest.mark.parametrize("silo_set", ["literal", "balanced"])
def test_full_size_cfg2_properties(gd, silo_set):
    """BASELINE config 2 at full size (16M messages over 1M grains): route checked
    against the known directory (act == grain index, silo == ring owner), a
    100k sample against the oracle, and the bucketing by size-independent
    properties (permutation, sorted, stable, offsets = counts).  Both silo sets bench.py
    reports: SURVEY 8(d)'s literal generation-1 silos and the balanced generations the
    benchmark line is timed on."""
    import torch
    silos = o.bench_silos(8) if silo_set == "literal" else \
        [o.Silo(f"10.0.0.{i + 1}", 11111, gen) for i, gen in enumerate(BALANCED_GENS)]
    spec = o.ring_spec(silos, "D")
    G, N = 1 << 20, 1 << 24
    e = _engine(gd, silos, "D", cap=2 * G)
    reg_k = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg_k[:, 2], reg_k[:, 0], reg_k[:, 1])).astype(np.uint32)
    e.register(reg_k, np.arange(G), owner)
    rng = np.random.default_rng(0x5EED0001)
    ks = rng.integers(0, G, size=N)
    keys = torch.from_numpy(o.grain_keys(TC, ks).view(np.int64)).cuda()
    dev = torch.device("cuda:0")
    silo = torch.empty(N, dtype=torch.int32, device=dev)
    act = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    off = torch.empty(G + 2, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)          # not torch's null stream (handle 0 = the library's own stream)
    stream.wait_stream(torch.cuda.current_stream())
    e.set_stream(stream.cuda_stream)
    e.route_bucket_device(keys.data_ptr(), N, G, silo.data_ptr(), act.data_ptr(), st.data_ptr(),
                          perm.data_ptr(), off.data_ptr())
    torch.cuda.synchronize()
    st_h = st.cpu().numpy()
    act_h = act.cpu().numpy().view(np.uint32)
    silo_h = silo.cpu().numpy().view(np.uint32)
    assert (st_h == 0).all()
    np.testing.assert_array_equal(act_h, ks.astype(np.uint32))
    np.testing.assert_array_equal(silo_h, owner[ks])
    samp = rng.choice(N, size=100000, replace=False)
    d = o.DirectoryArrays(reg_k, np.arange(G), owner)
    want = o.route_batch_np(o.grain_keys(TC, ks[samp]), spec, d)
    np.testing.assert_array_equal(silo_h[samp], want[1])
    perm_h = perm.cpu().numpy().view(np.uint32).astype(np.int64)
    off_h = off.cpu().numpy().view(np.uint32).astype(np.int64)
    # permutation
    seen = np.zeros(N, dtype=bool)
    seen[perm_h] = True
    assert seen.all()
    a_sorted = act_h[perm_h].astype(np.int64)
    assert (np.diff(a_sorted) >= 0).all()
    same = np.diff(a_sorted) == 0
    assert (np.diff(perm_h)[same] > 0).all()                  # stable: FIFO inside each activation
    counts = np.bincount(act_h, minlength=G + 1)
    np.testing.assert_array_equal(np.diff(off_h), counts)
    assert off_h[0] == 0 and off_h[-1] == N
    e.close()


# ----------------------------------------------------------------------------- micro-batch graphs (f3)
def _check_runs(mb, n, want_act, n_act):
    wp, wo = o.bucket_stable(want_act, n_act)
    assert np.array_equal(mb.perm[:n], wp)
    assert np.array_equal(mb.offsets(), wo)
    r = mb.n_runs
    clamped = np.minimum(want_act.astype(np.int64), n_act)
    ua, first = np.unique(clamped, return_index=True) if n else (np.zeros(0, np.int64), np.zeros(0, np.int64))
    assert r == len(ua)
    assert np.array_equal(mb.run_act[:r], ua)
    assert mb.run_start[r] == n
    assert np.array_equal(np.diff(mb.run_start[:r + 1]), np.bincount(clamped, minlength=n_act + 1)[ua])


MB_VARIANTS = {  # GD_OPT_MB_* options, read at gd_microbatch_create
    "zero_copy": {},
    "zero_copy_one_sorter": {"mb_split": 1},
    "staged_copies": {"mb_zerocopy": 0},
}


@pytest.mark.parametrize("variant,mode", [("zero_copy", "D"), ("zero_copy", "R"), ("zero_copy", "V"),
                                          ("zero_copy_one_sorter", "V"), ("staged_copies", "V"),
                                          ("ballot_ranks", "D")])
def test_microbatch_graph_matches_eager_and_oracle(gd, monkeypatch, variant, mode):
    if variant == "ballot_ranks":                # every rank by ballots (GD_CFG_NO_LANE_ORDER)
        monkeypatch.setattr(gd, "FORCE_NO_LANE_ORDER", True)
    for k, v in MB_VARIANTS.get(variant, {}).items():
        monkeypatch.setitem(gd.DEFAULT_OPTIONS, k, v)
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    G = 50000
    e = _engine(gd, silos, mode, cap=1 << 17)
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    e.register(reg, np.arange(G), owner)
    d = o.DirectoryArrays(reg, np.arange(G), owner)
    mb = gd.MicroBatch(e, 8192, G)
    rng = np.random.default_rng(55)
    routed0, routed = e.stats()["routed"], 0
    for n in (4096, 8192, 1000, 4096, 1, 0, 4097, 2, 6000):
        hot = rng.integers(0, 64, size=n)                           # skewed: many messages per activation
        keys = o.grain_keys(TC, np.where(rng.random(n) < 0.5, hot, rng.integers(0, G + 300, size=n)))
        mb.keys[:n] = keys
        for use_graph in (True, False):
            mb.run(n, use_graph)
            routed += n
            assert e.stats()["routed"] - routed0 == routed      # every replay counts its messages
            want = o.route_batch_np(keys, spec, d)
            assert np.array_equal(mb.status[:n], want[0]) and np.array_equal(mb.silo[:n], want[1])
            assert np.array_equal(mb.act[:n], want[2])
            _check_runs(mb, n, want[2], G)
    mb.close()
    e.close()


def test_microbatch_graph_recaptured_after_ring_and_table_change(gd):
    """Cached graphs bake in the ring snapshot and table pointers; a ring swap or a rehash
    must not replay a stale graph."""
    silos = o.bench_silos(8)
    G = 3000
    e = _engine(gd, silos, "D", cap=1 << 12)
    reg = o.grain_keys(TC, np.arange(G))
    spec = o.ring_spec(silos, "D")
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    e.register(reg, np.arange(G), owner)
    mb = gd.MicroBatch(e, 2048, 4 * G)
    rng = np.random.default_rng(9)
    keys = o.grain_keys(TC, rng.integers(0, 4 * G, size=2048))
    mb.keys[:] = keys
    mb.run(2048, True)
    # ring change: 3 silos only
    spec3 = o.ring_spec(silos[:3], "D")
    e.ring_set_silos("D", _silo_tuples(silos[:3]))
    # table growth: register 9000 more grains (forces a rehash of the 4096-slot table)
    reg2 = o.grain_keys(TC, np.arange(G, 4 * G))
    own2 = o.ring_owner_np(spec3, o.jenkins_u64x3_np(reg2[:, 2], reg2[:, 0], reg2[:, 1]))
    e.register(reg2, np.arange(G, 4 * G), own2)
    assert e.stats()["table_capacity"] > (1 << 12)
    mb.run(2048, True)
    d = o.DirectoryArrays(np.concatenate([reg, reg2]), np.arange(4 * G), np.concatenate([owner, own2]))
    want = o.route_batch_np(keys, spec3, d)
    assert np.array_equal(mb.status[:2048], want[0]) and np.array_equal(mb.silo[:2048], want[1])
    assert np.array_equal(mb.act[:2048], want[2])
    _check_runs(mb, 2048, want[2], 4 * G)
    mb.close()
    e.close()


def test_microbatch_limits(gd):
    e = _engine(gd, o.bench_silos(2), "D")
    with pytest.raises(gd.GrainDispatchError):
        gd.MicroBatch(e, 8193, 10)
    mb = gd.MicroBatch(e, 8192, 10)
    keys = o.grain_keys(TC, np.arange(8192))
    mb.keys[:] = keys
    mb.run(8192, True)
    assert mb.n_runs == 1 and mb.run_act[0] == 10 and mb.run_start[1] == 8192    # all misses: trailing bucket
    assert np.array_equal(mb.perm, np.arange(8192))
    with pytest.raises(gd.GrainDispatchError):
        mb.run(8193, True)
    mb.close()
    e.close()


# ----------------------------------------------------------------------------- header decode (f1)
import json  # noqa: E402
import os  # noqa: E402
import struct  # noqa: E402
import sys  # noqa: E402

import headers as H  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import frames_synth as FS  # noqa: E402


def _assert_decoded(got, want, rows=None):
    for k in want:
        if k in got:
            g = got[k] if rows is None else got[k][rows]
            np.testing.assert_array_equal(g, want[k], err_msg=k)


def test_decode_frames_golden(gd):
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")))["frames"]
    buf = bytes.fromhex(g["buffer_hex"])
    e = gd.GrainDispatch(device=0, table_capacity=1 << 10)
    got = e.decode_frames(buf, g["offsets"])
    assert got["flags"].tolist() == g["flags"] and got["mask"].tolist() == g["mask"]
    assert [[str(int(x)) for x in k] for k in got["target_grain"]] == g["target_grain"]
    assert [bytes(x).hex() for x in got["target_silo"]] == g["target_silo_hex"]
    assert [str(int(x)) for x in got["correlation_id"]] == g["correlation_id"]
    _assert_decoded(got, H.decode_frames(buf, g["offsets"]))
    e.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_decode_frames_random_vs_oracle(gd, seed):
    rng = np.random.default_rng(seed)
    n = 20000 + seed * 37                                          # not a multiple of 64
    keys = o.grain_keys(TC, rng.integers(0, 1 << 20, size=n))
    buf, off = H.random_frames(n, keys, rng, p_fallback=0.03, p_complete=0.08, p_malformed=0.02)
    if seed == 2:                                                  # shuffled, unaligned frame order
        off = off[rng.permutation(n)]
    e = gd.GrainDispatch(device=0, table_capacity=1 << 10)
    got = e.decode_frames(buf, off)
    _assert_decoded(got, H.decode_frames(buf, off))
    e.close()


def test_decode_frames_edges(gd):
    e = gd.GrainDispatch(device=0, table_capacity=1 << 10)
    k = (7, 8, o.type_code_data(o.CAT_GRAIN, TC))
    frames = [
        H.encode_frame({"target_grain": (k, None), "debug_context": "d" * 600}),          # past the LDS window
        H.encode_frame({"target_grain": (k, "ext" * 70), "category": 1}),                 # long KeyExt
        H.encode_frame({"sending_grain": ((1, 2, 3), "s" * 300), "target_grain": (k, None),
                        "target_activation": ((5, 6, 0), None), "target_silo": (bytes(16), 9, 9)}),
        H.encode_frame({"target_grain": (k, None)}, b"body"),
        H.encode_frame({"category": 0}),                                                  # no target grain
        H.encode_frame({"target_observer": b"\x01" * 9, "target_grain": (k, None), "target_silo": (bytes(16), 1, 1)}),
    ]
    # every alignment of every frame, back to back
    for pad in range(4):
        buf = b"\xee" * pad
        offs = []
        for f in frames:
            offs.append(len(buf))
            buf += f
        got = e.decode_frames(buf, offs)
        _assert_decoded(got, H.decode_frames(buf, offs))
    # the last frame cut at every length (tail bytes not a whole dword; past-the-end offsets)
    last = H.encode_frame({"target_grain": (k, "tail"), "correlation_id": 5, "direction": 2}, b"xyz")
    head = frames[3] + b"\x00"
    for cut in range(len(last) + 1):
        buf = head + last[:cut]
        offs = [0, len(head), len(buf), len(buf) + 1, 1 << 62]
        got = e.decode_frames(buf, offs)
        want = H.decode_frames(buf, offs)
        _assert_decoded(got, want)
        assert (got["flags"][1] == H.F_HAS_TARGET | H.F_TARGET_KEYEXT) == (cut == len(last))
    # corrupted lengths
    bad = bytearray(frames[3])
    struct.pack_into("<i", bad, 0, -5)
    bad2 = bytearray(frames[0])
    struct.pack_into("<i", bad2, 12, -2)                                   # DebugContext length -2
    buf = bytes(bad) + bytes(bad2)
    got = e.decode_frames(buf, [0, len(bad)])
    assert got["flags"].tolist() == [H.F_MALFORMED, H.F_MALFORMED]
    # empty batch
    got = e.decode_frames(b"", [])
    assert got["flags"].shape == (0,)
    e.close()


def _frames_engine(gd, G=5000):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    e = _engine(gd, silos, "D", cap=1 << 14, my_silo=3, seed_silo=5)
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    e.register(reg, np.arange(G), owner)
    return e, spec, o.DirectoryArrays(reg, np.arange(G), owner)


def test_route_frames_vs_oracle(gd):
    G = 5000
    e, spec, d = _frames_engine(gd, G)
    rng = np.random.default_rng(11)
    n = 12000
    keys = np.concatenate([o.grain_keys(TC, rng.integers(0, G + 500, size=n - 8)), _special_keys()])
    buf, off = H.random_frames(n, keys, rng, p_fallback=0.03, p_complete=0.1, p_malformed=0.02)
    dec, st, silo, act, perm, offs = e.route_frames(buf, off, n_act=G, fields=["mask"])
    f, wst, wsilo, wact = H.route_frames_np(buf, off, spec, d)
    wst2, wsilo2, wact2 = o.route_batch_np(f["target_grain"], spec, d, my_silo=3, seed_silo=5)[:3]
    routed = wst < H.ROUTE_ADDRESSED
    wst[routed], wsilo[routed], wact[routed] = wst2[routed], wsilo2[routed], wact2[routed]
    np.testing.assert_array_equal(st, wst)
    np.testing.assert_array_equal(silo, wsilo)
    np.testing.assert_array_equal(act, wact)
    np.testing.assert_array_equal(dec["flags"], f["flags"])
    np.testing.assert_array_equal(dec["target_grain"], f["target_grain"])
    np.testing.assert_array_equal(dec["mask"], f["mask"])
    wp, wo = o.bucket_stable(wact, G)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(offs, wo)
    assert {int(x) for x in np.unique(st)} >= {0, 1, 2, 3, 4, 5, 6}
    # without bucketing
    _, st2, silo2, act2 = e.route_frames(buf, off)
    np.testing.assert_array_equal(st2, st)
    np.testing.assert_array_equal(act2, act)
    e.close()


def test_route_frames_device_full_size(gd):
    """2^22 frames of the cfg2 distribution straight from a device receive buffer: decode ->
    route -> bucket equals route_bucket on the keys; a sample against the oracle."""
    import torch
    G, N = 1 << 20, 1 << 22
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    e = _engine(gd, silos, "D", cap=1 << 22)
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    e.register(reg, np.arange(G), owner)
    rng = np.random.default_rng(0xF1)
    keys = reg[rng.integers(0, G, size=N)]
    buf, off, fl = FS.build_frames(keys, rng)
    dev = torch.device("cuda:0")
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    flags = torch.empty(N, dtype=torch.int32, device=dev)
    tg = torch.empty((N, 3), dtype=torch.int64, device=dev)
    corr = torch.empty(N, dtype=torch.int64, device=dev)
    silo = torch.empty(N, dtype=torch.int32, device=dev)
    act = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    offs = torch.empty(G + 2, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    e.set_stream(s.cuda_stream)
    e.route_frames_device(d_buf.data_ptr(), len(buf), d_off.data_ptr(), N, G,
                          {"flags": flags.data_ptr(), "target_grain": tg.data_ptr(),
                           "correlation_id": corr.data_ptr()},
                          silo.data_ptr(), act.data_ptr(), st.data_ptr(), perm.data_ptr(), offs.data_ptr())
    e.synchronize()
    assert (flags.cpu().numpy() == H.F_HAS_TARGET).all()
    np.testing.assert_array_equal(tg.cpu().numpy().view(np.uint64), keys)
    np.testing.assert_array_equal(corr.cpu().numpy(), np.arange(1, N + 1))
    e.set_stream(None)
    wst, wsilo, wact, wperm, woff = e.route_bucket(keys, G)
    np.testing.assert_array_equal(st.cpu().numpy(), wst)
    np.testing.assert_array_equal(silo.cpu().numpy().view(np.uint32), wsilo)
    np.testing.assert_array_equal(act.cpu().numpy().view(np.uint32), wact)
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wperm)
    np.testing.assert_array_equal(offs.cpu().numpy().view(np.uint32), woff)
    rows = rng.integers(0, N, size=3000)
    d = o.DirectoryArrays(reg, np.arange(G), owner)
    want = o.route_batch_np(keys[rows], spec, d)
    np.testing.assert_array_equal(wst[rows], want[0])
    np.testing.assert_array_equal(wact[rows], want[2])
    sample = H.decode_frames(buf[int(off[rows[0]]):int(off[rows[0]]) + 100 * fl].tobytes(),
                             np.arange(100, dtype=np.uint64) * np.uint64(fl))
    np.testing.assert_array_equal(sample["target_grain"], keys[rows[0]:rows[0] + 100])
    e.close()


# ----------------------------------------------------------------------------- membership change (f4)
def _sorted_rows(keys, *cols):
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    order = np.lexsort((keys[:, 2], keys[:, 1], keys[:, 0]))
    return (keys[order],) + tuple(np.asarray(c)[order] for c in cols)


@pytest.mark.parametrize("mode", ["D", "R", "V"])
def test_dir_split_vs_oracle(gd, mode):
    silos8, silos9 = o.bench_silos(8), o.bench_silos(9)
    spec8, spec9 = o.ring_spec(silos8, mode), o.ring_spec(silos9, mode)
    e = _engine(gd, silos8, mode, cap=1 << 16, my_silo=2, seed_silo=6)
    G = 20000
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec8, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    special = _special_keys()[:3]          # system target, membership grain, KeyExt grain
    keys = np.concatenate([reg, special])
    acts = np.arange(G + 3, dtype=np.uint32)
    silos = np.concatenate([owner, [2, 6, 1]]).astype(np.uint32)
    e.register(keys, acts, silos)
    d = o.DirectoryArrays(keys, acts, silos)
    e.ring_set_silos(mode, _silo_tuples(silos9))                      # silo 8 joins
    keep = [0, 1, 2, 3, 8]
    wk, wa, ws, rest = o.split_directory(d, spec9, keep, my_silo=2, seed_silo=6)
    # copy (modifyOrigin false): same entries, table untouched
    ck, ca, cs = e.split(keep, move=False)
    gk, ga, gs = _sorted_rows(ck, ca, cs)
    np.testing.assert_array_equal(gk, wk)
    np.testing.assert_array_equal(ga, wa)
    np.testing.assert_array_equal(gs, ws)
    assert e.stats()["table_live"] == G + 3
    # move: the same entries leave; everything else stays findable
    mk, ma, ms = e.split(keep, move=True)
    np.testing.assert_array_equal(_sorted_rows(mk)[0], wk)
    st = e.stats()
    assert st["table_live"] == G + 3 - len(wk) and st["table_tombstones"] == len(wk)
    _, _, found = e.lookup(keys)
    kv = {tuple(int(x) for x in k) for k in wk}
    assert all(bool(f) != (tuple(int(x) for x in k) in kv) for k, f in zip(keys, found))
    # specials: system target owned by my silo (2, kept), membership by the seed (6, not kept),
    # KeyExt never selected
    assert tuple(int(x) for x in special[0]) not in kv
    assert tuple(int(x) for x in special[1]) in kv
    assert tuple(int(x) for x in special[2]) not in kv
    # nothing left to move
    assert len(e.split(keep, move=True)[0]) == 0
    # merge into the partition that now owns them: inserted, then a second merge conflicts
    e2 = _engine(gd, silos9, mode, cap=1 << 16, my_silo=2, seed_silo=6)
    a2, s2, ins = e2.register(mk, ma, ms)
    assert ins.all()
    a3, s3, ins2 = e2.register(mk, ma + 100000, ms)                    # same grains, other activations
    assert not ins2.any()
    np.testing.assert_array_equal(a3, ma)                              # existing entries kept
    e.close()
    e2.close()


def test_dir_split_device_and_full_size(gd):
    import torch
    silos8, silos9 = o.bench_silos(8), o.bench_silos(9)
    spec9 = o.ring_spec(silos9, "D")
    G = 1 << 20
    e = _engine(gd, silos8, "D", cap=1 << 21)
    reg = o.grain_keys(TC, np.arange(G))
    spec8 = o.ring_spec(silos8, "D")
    owner = o.ring_owner_np(spec8, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    e.register(reg, np.arange(G), owner)
    e.ring_set_silos("D", _silo_tuples(silos9))
    keep = [s for s in range(9) if s % 2 == 0]
    mask = gd.GrainDispatch.keep_mask(keep, 9)
    n = e.split_device(mask, False, None, None, 0)
    d = o.DirectoryArrays(reg, np.arange(G), owner)
    wk, wa, ws, _ = o.split_directory(d, spec9, keep)
    assert n == len(wk)
    dev = torch.device("cuda:0")
    k = torch.empty((n, 3), dtype=torch.int64, device=dev)
    v = torch.empty((n, 2), dtype=torch.int32, device=dev)
    with pytest.raises(gd.GrainDispatchError):
        e.split_device(mask, True, k.data_ptr(), v.data_ptr(), n - 1)     # too small: nothing moved
    assert e.stats()["table_live"] == G
    assert e.split_device(mask, True, k.data_ptr(), v.data_ptr(), n) == n
    torch.cuda.synchronize()
    gk, gv = _sorted_rows(k.cpu().numpy().view(np.uint64), v.cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(gk, wk)
    np.testing.assert_array_equal(gv[:, 0], wa)
    np.testing.assert_array_equal(gv[:, 1], ws)
    assert e.stats()["table_live"] == G - n
    e.close()


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 100003])
def test_pack_by_shard_vs_oracle(gd, n):
    """gd_pack_by_shard_device (the exchange partition, OutboundMessageQueue.cs:54-131 per target
    silo): stable partition of the 24-B headers by owner silo % n_shards, origin indices alongside;
    system targets / KeyExt go to my silo's rank, the membership grain to the seed's."""
    import torch
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    rng = np.random.default_rng(n + 5)
    keys = o.grain_keys(TC, rng.integers(-5000, 5000, size=n))
    if n > 10:
        keys[::7] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
        keys[3::11] = np.array(o.MEMBERSHIP_TABLE_ID.as_tuple(), dtype=np.uint64)
        keys[5::13, 2] = np.uint64(o.type_code_data(o.CAT_KEYEXT_GRAIN, 77))
    e = _engine(gd, silos, "D", my_silo=3, seed_silo=6)
    dev = torch.device("cuda", 0)
    tk = torch.from_numpy(keys.view(np.int64).copy()).to(dev)
    st, silo, act, owner, h = o.route_batch_np(keys, spec, o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []),
                                               my_silo=3, seed_silo=6)
    owner = np.where(st == o.ST_KEYEXT, 3, owner).astype(np.int64)
    for shards in (1, 2, 3, 8, 13, 256):
        sk = torch.empty_like(tk)
        si = torch.empty(n, dtype=torch.int32, device=dev)
        cnt = torch.empty(shards, dtype=torch.int32, device=dev)
        e.pack_by_shard_device(tk.data_ptr(), n, shards, sk.data_ptr(), si.data_ptr(), cnt.data_ptr())
        torch.cuda.synchronize()
        dest = (owner % shards).astype(np.uint32)
        perm, off = o.bucket_stable(dest, shards)
        np.testing.assert_array_equal(si.cpu().numpy().view(np.uint32), perm)
        np.testing.assert_array_equal(sk.cpu().numpy().view(np.uint64).reshape(-1, 3), keys[perm])
        np.testing.assert_array_equal(cnt.cpu().numpy(), np.diff(off[:shards + 1]))
    e.close()


@pytest.mark.parametrize("mode", ["D", "V"])
def test_upsert_and_multi_activation_grains(gd, mode):
    """gd_dir_upsert (the host's mirror of GrainDirectoryPartition.AddActivation for multi-instance
    grains, GrainDirectoryPartition.cs:274-302): overwrite in batch order (the last item of a grain
    wins); a grain marked GD_ACT_MULTI routes as GD_ROUTE_MULTI_ACT with the owner silo, no
    activation, trailing bucket (RandomPlacementDirector.cs:33-53 stays in C#)."""
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    e = _engine(gd, silos, mode, cap=1 << 13, my_silo=2)
    G = 2000
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg[:1000], np.arange(1000), own[:1000])               # first-wins registrations
    final = {tuple(int(x) for x in reg[i]): (i, int(own[i])) for i in range(1000)}
    rng = np.random.default_rng(4)
    idx = rng.integers(0, G, size=6000)                                 # many duplicates, old and new grains
    acts = rng.integers(0, 50000, size=6000).astype(np.uint32)
    acts[rng.random(6000) < 0.2] = gd.GD_ACT_MULTI
    ss = rng.integers(0, 8, size=6000).astype(np.uint32)
    before = e.stats()["table_live"]
    ins = e.upsert(reg[idx], acts, ss)
    new_keys = set()
    for j, i in enumerate(idx):
        k = tuple(int(x) for x in reg[i])
        if k not in final:
            new_keys.add(k)
        final[k] = (int(acts[j]), int(ss[j]))
    assert e.stats()["table_live"] == before + len(new_keys)
    assert int(ins.sum()) == len(new_keys)
    fk = np.array(list(final.keys()), dtype=np.uint64)
    d = o.DirectoryArrays(fk, [v[0] for v in final.values()], [v[1] for v in final.values()])
    msgs = o.grain_keys(TC, rng.integers(0, G + 100, size=50000))
    st, silo, act, perm, off = e.route_bucket(msgs, 50000)
    wst, wsilo, wact, _, _ = o.route_batch_np(msgs, spec, d, my_silo=2)
    np.testing.assert_array_equal(st, wst)
    np.testing.assert_array_equal(silo, wsilo)
    np.testing.assert_array_equal(act, wact)
    assert (wst == o.ST_MULTI_ACT).sum() > 1000
    wp, wo = o.bucket_stable(wact, 50000)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    # the scalar restatement agrees on the multi-activation rule
    st2, silo2, act2, _, _ = o.route_batch(msgs[:3000], spec, final, 2, o.M32)
    np.testing.assert_array_equal(st2, wst[:3000])
    np.testing.assert_array_equal(act2, wact[:3000])
    e.close()


def test_randomized_configurations(gd):
    """Random shapes through route + bucket against the oracle: ring modes and sizes (1..70 silos,
    V-ring bucket counts), table capacities far below the grain count (growth/rehash), n_act
    around powers of two (radix digit widths and pass counts change there), unregistered and
    special-category keys, empty, tiny and tile-straddling batches."""
    rng = np.random.default_rng(20261016)
    special = _special_keys()
    for trial in range(24):
        mode = "DRV"[trial % 3]
        n_silos = int(rng.choice([1, 2, 3, 8, 13, 70]))
        silos = [o.Silo(f"10.{trial}.{i // 200}.{i % 200 + 1}", 11111 + i % 7, 1 + int(rng.integers(0, 9)))
                 for i in range(n_silos)]
        buckets = int(rng.choice([1, 3, 30]))
        spec = o.ring_spec(silos, mode, buckets)
        G = int(rng.choice([1, 17, 255, 256, 257, 4095, 4097, 65535, 65537]))
        n_act = G + int(rng.integers(0, 3))
        my_silo, seed_silo = int(rng.integers(0, n_silos)), int(rng.integers(0, n_silos))
        e = gd.GrainDispatch(device=0, table_capacity=int(rng.choice([16, 1024, 1 << 17])),
                             my_silo=my_silo, seed_silo=seed_silo)
        e.ring_set_silos(mode, _silo_tuples(silos), buckets)
        reg = o.grain_keys(TC, rng.permutation(G * 3)[:G])
        own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
        acts = rng.permutation(n_act)[:G].astype(np.uint32)
        e.register(reg, acts, own)
        n = int(rng.choice([0, 1, 63, 64, 4095, 4096, 4097, 100000]))
        pick = rng.integers(0, G + max(1, G // 4), size=n)
        keys = np.where((pick < G)[:, None], reg[np.minimum(pick, G - 1)], o.grain_keys(TC, G * 3 + pick))
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        if n > 64:
            keys[5::31] = special[rng.integers(0, len(special), size=len(keys[5::31]))]
        st, silo, act, perm, off = e.route_bucket(keys, n_act)
        d = o.DirectoryArrays(reg, acts, own)
        wst, wsilo, wact, _, _ = o.route_batch_np(keys, spec, d, my_silo=my_silo, seed_silo=seed_silo)
        msg = f"trial {trial}: mode {mode} silos {n_silos} G {G} n_act {n_act} n {n}"
        np.testing.assert_array_equal(st, wst, err_msg=msg)
        np.testing.assert_array_equal(silo, wsilo, err_msg=msg)
        np.testing.assert_array_equal(act, wact, err_msg=msg)
        wp, wo = o.bucket_stable(wact, n_act)
        np.testing.assert_array_equal(perm, wp, err_msg=msg)
        np.testing.assert_array_equal(off, wo, err_msg=msg)
        if 0 < n <= 4096:                                   # the hipGraph micro-batch path too
            mb = gd.MicroBatch(e, 4096, n_act)
            mb.keys[:n] = keys
            mb.run(n, use_graph=bool(trial & 1))
            np.testing.assert_array_equal(mb.status[:n], wst, err_msg=msg)
            np.testing.assert_array_equal(mb.act[:n], wact, err_msg=msg)
            np.testing.assert_array_equal(mb.perm[:n], wp, err_msg=msg)
            np.testing.assert_array_equal(mb.offsets(), wo, err_msg=msg)
            mb.close()
        e.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_route_bucket_host_pipelined(gd, pinned, monkeypatch):
    """gd_route_bucket's pipelined host path (chunked H2D / probe / D2H on three streams, then the
    bucketing of the whole batch), forced on with small chunks (GD_OPT_HOST_CHUNK), from pageable and
    from gd_host_alloc'd pinned buffers; a ragged last chunk."""
    import ctypes as C
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "host_chunk", 4096)
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "V")
    e = _engine(gd, silos, "V", cap=1 << 15, my_silo=2)
    G = 9000
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg, np.arange(G), own)
    n = 4096 * 7 + 123
    keys = o.grain_keys(TC, np.random.default_rng(17).integers(0, G + 900, size=n))
    keys[::37] = _special_keys()[np.arange(len(keys[::37])) % 8]
    bufs = []

    def arr(shape, dt):
        if not pinned:
            return np.zeros(shape, dt)
        p = C.c_void_p()
        nb = int(np.prod(shape)) * np.dtype(dt).itemsize
        assert gd.lib.gd_host_alloc(nb, C.byref(p)) == 0
        bufs.append(p)
        return np.ctypeslib.as_array((C.c_uint8 * nb).from_address(p.value)).view(dt).reshape(shape)

    k = arr((n, 3), np.uint64)
    k[:] = keys
    silo, act, perm = arr(n, np.uint32), arr(n, np.uint32), arr(n, np.uint32)
    st, off = arr(n, np.uint8), arr(G + 2, np.uint32)
    for _ in range(2):                                  # the streams and events are reused
        e._c(gd.lib.gd_route_bucket(e.h, k.ctypes.data, n, G, silo.ctypes.data, act.ctypes.data, st.ctypes.data,
                                    perm.ctypes.data, off.ctypes.data))
        wst, wsilo, wact, _, _ = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), own), my_silo=2)
        np.testing.assert_array_equal(st, wst)
        np.testing.assert_array_equal(silo, wsilo)
        np.testing.assert_array_equal(act, wact)
        wp, wo = o.bucket_stable(wact, G)
        np.testing.assert_array_equal(perm, wp)
        np.testing.assert_array_equal(off, wo)
        silo[:], act[:], st[:] = 7, 7, 7                 # gd_route: routes only, same pipeline
        e._c(gd.lib.gd_route(e.h, k.ctypes.data, n, silo.ctypes.data, act.ctypes.data, st.ctypes.data))
        np.testing.assert_array_equal(st, wst)
        np.testing.assert_array_equal(silo, wsilo)
        np.testing.assert_array_equal(act, wact)
    e.close()
    for p in bufs:
        assert gd.lib.gd_host_free(p) == 0


@pytest.mark.parametrize("cap", [1 << 21, 1 << 24])
def test_route_index_size_forms_vs_oracle(gd, cap):
    """k_route's two launch forms, picked by the probe index's size (eng_core.hip route_mode): a
    cache-sized index (one message a thread, non-temporal key stream) and a large one (two messages a
    thread), on a ragged batch with misses, system targets and N0 != 0 keys, against the oracle."""
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    G, N = 100_000, 1_000_003
    e = _engine(gd, silos, "D", cap=cap)
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg, np.arange(G), owner)
    rng = np.random.default_rng(0x5EED0301)
    keys = o.grain_keys(TC, rng.integers(0, G + G // 4, size=N))      # a fifth unregistered: misses
    keys[::97, 0] = rng.integers(1, 1 << 40, size=keys[::97].shape[0], dtype=np.uint64)   # N0 != 0
    st, silo, act = e.route(keys)
    want = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), owner))
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    assert (st == o.ST_OK).sum() > N // 2 and (st != o.ST_OK).sum() > N // 10
    e.close()
