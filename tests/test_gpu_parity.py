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
    # re-register a removed grain: a new entry (tombstones are probed past)
    a, s, ins = e.register(keys[:5], np.arange(5) + 500, np.ones(5))
    assert ins.tolist() == [1] * 5 and a.tolist() == list(range(500, 505))
    st = e.stats()
    assert st["table_live"] == 95 and st["table_tombstones"] == 10
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
def test_full_size_cfg2_properties(gd):
    """BASELINE config 2 at full size (16M messages over 1M grains): route checked
    against the known directory (act == grain index, silo == ring owner), a
    100k sample against the oracle, and the bucketing by size-independent
    properties (permutation, sorted, stable, offsets = counts)."""
    import torch
    silos = o.bench_silos(8)
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
    e.set_stream(torch.cuda.current_stream().cuda_stream)
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
