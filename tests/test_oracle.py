"""CPU tests of the oracle: the reference's own structural tests restated, the
frozen golden vectors, and the independent C restatement (oracle/cpu_ref.c)
agreeing bit-for-bit."""
import hashlib
import json
import os
import random
import struct

import numpy as np
import pytest

import oracle as o

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


# --------------------------------------------------------------- reference tests, restated
def test_id_hash_correctness():
    """Identifiertests.ID_HashCorrectness (test/NonSilo.Tests/General/Identifiertests.cs:278-293):
    the byte[] Jenkins equals the 3 x ulong Jenkins on 1,000 random 24-byte inputs."""
    r = random.Random(278)
    for _ in range(1000):
        b = bytes(r.getrandbits(8) for _ in range(24))
        u1, u2, u3 = struct.unpack("<QQQ", b)
        assert o.jenkins_bytes(b) == o.jenkins_u64x3(u1, u2, u3)


def test_silo_uniform_hash_layout():
    """Identifiertests.SiloAddressGetUniformHashCodes (:51-68): the point for extraBit i is
    Jenkins over Write(SiloAddress) + Write(int i) in the wire layout."""
    s = o.Silo("127.0.0.1", 8080, 26)
    wire = b"\x00" * 12 + bytes([127, 0, 0, 1]) + struct.pack("<i", 8080) + struct.pack("<i", 26)
    assert s.wire_bytes() == wire
    for i, h in enumerate(s.uniform_hashes(3)):
        assert h == o.jenkins_bytes(wire + struct.pack("<i", i))


def test_unique_key_to_byte_array():
    """Identifiertests.UniqueKeyToByteArray (:32-48): N0 | N1 | TCD | int32 len | UTF-8 KeyExt."""
    k = o.UniqueKey(0x0102030405060708, 0x1112131415161718, o.type_code_data(o.CAT_KEYEXT_GRAIN, 7), "hello world")
    b = k.to_byte_array()
    assert b[:24] == struct.pack("<QQQ", k.n0, k.n1, k.tcd)
    assert b[24:28] == struct.pack("<i", 11) and b[28:] == b"hello world"
    assert o.UniqueKey(1, 2, 3).to_byte_array()[24:] == struct.pack("<i", -1)
    # KeyExt grains hash the byte form, others the 3 x u64 form (UniqueKey.cs:279-286)
    assert k.uniform_hash() == o.jenkins_bytes(b)
    plain = o.UniqueKey(5, 6, o.type_code_data(o.CAT_GRAIN, 9))
    assert plain.uniform_hash() == o.jenkins_u64x3(plain.tcd, plain.n0, plain.n1)


def test_sha256_fips_vectors():
    """FIPS 180-4 known answers for the SHA-256 under CalculateIdHash (Utils.cs:184-203)."""
    assert hashlib.sha256(b"abc").hexdigest() == \
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert hashlib.sha256(b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq").hexdigest() == \
        "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"
    # XOR-fold of the big-endian int32 words, signed
    d = hashlib.sha256("abc".encode("utf-16-le")).digest()
    x = 0
    for i in range(0, 32, 4):
        x ^= int.from_bytes(d[i:i + 4], "big")
    assert o.calculate_id_hash("abc") == (x - (1 << 32) if x >= 1 << 31 else x)


def test_type_code_data_sign_extension():
    """GrainId.GetGrainId(long typeCode, ..): a negative int type code is sign-extended before
    the 0x00FFFFFFFFFFFFFF mask (UniqueKey.cs:116)."""
    assert o.type_code_data(o.CAT_GRAIN, -1) == (3 << 56) | 0x00FFFFFFFFFFFFFF
    assert o.type_code_data(o.CAT_GRAIN, 5) == (3 << 56) | 5
    k = o.grain_id_long(-123, -1)
    assert k.n0 == 0 and k.n1 == o.M64 and k.category == o.CAT_GRAIN


def _ranges_r(silos):
    """ConsistentRingProvider ranges: (pred hash, my hash] as uint over the ring in
    AddServer order (ConsistentRingProvider.cs:112-124, :139-147)."""
    order = o.ring_d_build(silos)
    hs = [silos[i].consistent_hash() & o.M32 for i in order]
    if len(hs) == 1:
        return {order[0]: [(0, 0)]}
    return {order[i]: [(hs[i - 1], hs[i])] for i in range(len(hs))}


def _tiles(ranges):
    """RangeBreakable check (RingTests_Standalone.cs:171-261): the ranges cover the
    ring exactly once; sampled at every boundary +/- 1 and random points."""
    pts = set([0, 1, o.M32, o.M32 - 1])
    for rs in ranges.values():
        for b, e in rs:
            for x in (b - 1, b, b + 1, e - 1, e, e + 1):
                pts.add(x & o.M32)
    r = random.Random(5)
    pts.update(r.getrandbits(32) for _ in range(2000))
    for p in pts:
        n = sum(1 for rs in ranges.values() for b, e in rs
                if (b == e) or o.in_range(b, e, p))
        assert n == 1, (p, n)


@pytest.mark.parametrize("fails,joins", [((), ()), ((0,), ()), ((0, 1), ()), ((4,), ()), ((2, 3), ()),
                                         ((), (0,)), ((), (1, 3)), ((0,), (4,)), ((4,), (0,))])
def test_ring_standalone_tiling(fails, joins):
    """RingStandalone_Basic/Failures/Joins/Mixed (RingTests_Standalone.cs:15-70): silos
    127.0.0.1:0 gen 1..5; after failures and joins the ranges still tile the ring."""
    silos = [o.Silo("127.0.0.1", 0, g) for g in range(1, 6)]
    by_hash = sorted(range(5), key=lambda i: silos[i].consistent_hash())
    live = [i for i in range(5) if by_hash.index(i) not in fails]
    order = [i for i in live if by_hash.index(i) not in joins] + [i for i in live if by_hash.index(i) in joins]
    ss = [silos[i] for i in order]
    _tiles(_ranges_r(ss))


def test_ring_v_ranges_tile_and_match_lookup():
    """VirtualBucketsRingProvider.CalculateRange (:176-200): silo owns (prev, point] of each
    of its buckets; the lookup (:257-293) returns that owner."""
    silos = o.bench_silos(8)
    pts, own = o.ring_v_build(silos, 30)
    ranges = {}
    for i in range(len(pts)):
        ranges.setdefault(own[i], []).append((pts[i - 1], pts[i]))
    _tiles(ranges)
    r = random.Random(9)
    for _ in range(3000):
        k = r.getrandbits(32)
        owner = own[o.ring_v_lookup(pts, k)]
        assert any(o.in_range(b, e, k) for b, e in ranges[owner])


def test_ring_r_quirk():
    """ConsistentRingProvider.IsSiloNextInTheRing compares (long)int >= (long)uint: negative
    silo hashes never match, so keys above every non-negative point wrap to ring[0]."""
    silos = [o.Silo("127.0.0.1", 0, g) for g in range(1, 6)]           # all hashes negative
    sp = o.ring_spec(silos, "R")
    assert all(p < 0 for p in sp.points)
    for k in (0, 1, 12345, 0x7FFFFFFF, 0x80000000, o.M32):
        assert o.ring_r_lookup(sp.points, k) == 0


def test_ring_d_ties():
    """AddServer puts a newcomer before equal hashes; the lookup scans from the end."""
    pts = [-100, 5, 5, 5, 900]
    assert o.ring_d_lookup(pts, 5) == 3
    assert o.ring_d_lookup(pts, 4) == 0
    assert o.ring_d_lookup(pts, (-101) & o.M32) == 4          # below the first -> last silo


def test_np_lookups_equal_reference_scans():
    r = np.random.default_rng(4)
    for silos in (o.bench_silos(8), [o.Silo("127.0.0.1", 0, g) for g in range(1, 6)], o.bench_silos(1)):
        for mode in "DRV":
            sp = o.ring_spec(silos, mode)
            hs = np.concatenate([r.integers(0, 1 << 32, size=500, dtype=np.uint64).astype(np.uint32),
                                 np.array([(p + d) & o.M32 for p in sp.points for d in (-1, 0, 1)], dtype=np.uint32)])
            got = o.ring_owner_np(sp, hs)
            scan = {"D": o.ring_d_lookup, "R": o.ring_r_lookup, "V": o.ring_v_lookup}[mode]
            want = [sp.owners[scan(sp.points, int(h))] for h in hs]
            assert got.tolist() == want


# --------------------------------------------------------------- directory + bucketing semantics
def test_directory_first_wins_and_remove():
    d = o.DirectoryPartition()
    k = (0, 1, 2)
    assert d.add_single_activation(k, 5, 1) == (5, 1, True)
    assert d.add_single_activation(k, 6, 2) == (5, 1, False)
    assert not d.remove_activation(k, 6)
    assert d.remove_activation(k, 5)
    assert d.lookup(k) is None
    assert d.add_single_activation(k, 6, 2) == (6, 2, True)


def test_bucket_stable_equals_fifo_loop():
    r = np.random.default_rng(3)
    for n, a in [(0, 0), (1, 0), (50, 3), (1000, 17), (5000, 600)]:
        acts = r.integers(0, a + 3, size=n).astype(np.uint32)
        p1, o1 = o.bucket_stable(acts, a)
        p2, o2 = o.bucket_fifo_loop(acts, a)
        assert np.array_equal(p1, p2) and np.array_equal(o1, o2)


def test_route_np_equals_loop():
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    reg = o.grain_keys(tc, np.arange(500))
    for mode in "DRV":
        spec = o.ring_spec(o.bench_silos(8), mode)
        own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
        keys = np.concatenate([o.grain_keys(tc, np.random.default_rng(1).integers(0, 900, size=2000)),
                               np.array([o.MEMBERSHIP_TABLE_ID.as_tuple(),
                                         o.UniqueKey(0, 3, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(),
                                         o.UniqueKey(0, 3, o.type_code_data(o.CAT_GEO_CLIENT, 1)).as_tuple()],
                                        dtype=np.uint64)])
        a = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(500), own), 2, 6)
        dd = {tuple(int(x) for x in reg[i]): (i, int(own[i])) for i in range(500)}
        b = o.route_batch(keys, spec, dd, 2, 6)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


# --------------------------------------------------------------- golden vectors
def test_golden_identity():
    for hexb, h in GOLDEN["jenkins_bytes"]:
        assert o.jenkins_bytes(bytes.fromhex(hexb)) == h
    for a, b, c, h in GOLDEN["jenkins_u64x3"]:
        assert o.jenkins_u64x3(int(a), int(b), int(c)) == h
    for t, h in GOLDEN["calculate_id_hash"]:
        assert o.calculate_id_hash(t) == h
    for s in GOLDEN["silos"]:
        silo = o.Silo(s["ip"], s["port"], s["gen"])
        assert silo.consistent_hash() == s["consistent_hash"]
        assert silo.uniform_hashes(30) == s["uniform_hashes_30"]


def test_golden_rings():
    sets = {"bench8": o.bench_silos(8),
            "mixed10": [o.Silo(s["ip"], s["port"], s["gen"]) for s in GOLDEN["silos"]],
            "loopback5": [o.Silo("127.0.0.1", 0, k) for k in range(1, 6)]}
    for key, want in GOLDEN["rings"].items():
        name, mode = key.split("/")
        sp = o.ring_spec(sets[name], mode)
        assert [int(p) for p in sp.points] == want["points"] and sp.owners == want["owners"], key


def test_golden_route_and_bucket():
    r = GOLDEN["route"]
    spec = o.ring_spec(o.bench_silos(8), "D")
    reg = np.array([[int(x) for x in k] for k in r["directory"]["keys"]], dtype=np.uint64)
    d = o.DirectoryArrays(reg, r["directory"]["acts"], r["directory"]["silos"])
    msgs = np.array([[int(x) for x in k] for k in r["messages"]], dtype=np.uint64)
    st, silo, act, own, h = o.route_batch_np(msgs, spec, d, r["my_silo"], r["seed_silo"])
    assert st.tolist() == r["status"] and silo.tolist() == r["silo"] and act.tolist() == r["act"]
    assert own.tolist() == r["owner"] and h.tolist() == r["hash"]
    b = GOLDEN["bucket"]
    perm, off = o.bucket_stable(np.array(b["acts"], dtype=np.uint32), b["n_act"])
    assert perm.tolist() == b["perm"] and off.tolist() == b["offsets"]


# --------------------------------------------------------------- the C restatement agrees
@pytest.mark.parametrize("faithful", [True, False])
@pytest.mark.parametrize("mode", ["D", "R", "V"])
def test_c_restatement_matches_oracle(faithful, mode):
    import cpu_ref
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    G = 20000
    spec = o.ring_spec(o.bench_silos(8), mode)
    reg = o.grain_keys(tc, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    d = cpu_ref.CpuDirectory(faithful, G)
    a, s, ins = d.register(np.concatenate([reg, reg[:100]]), np.arange(G + 100), np.concatenate([own, own[:100]]))
    assert ins[:G].all() and not ins[G:].any() and np.array_equal(a[G:], np.arange(100))
    keys = np.concatenate([o.grain_keys(tc, np.random.default_rng(2).integers(0, G + 3000, size=100000)),
                           np.array([o.MEMBERSHIP_TABLE_ID.as_tuple()], dtype=np.uint64)])
    st, silo, act = d.route(mode, spec.points, spec.owners, keys, my_silo=1, seed_silo=4, nthreads=3)
    want = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), own), 1, 4)
    assert np.array_equal(st, want[0]) and np.array_equal(silo, want[1]) and np.array_equal(act, want[2])
    perm, off = cpu_ref.bucket(act, G, faithful=faithful, nthreads=3)
    wp, wo = o.bucket_stable(act, G)
    assert np.array_equal(perm, wp) and np.array_equal(off, wo)


@pytest.mark.parametrize("n,n_act", [(0, 10), (1, 1), (1000, 7), (100_000, 1000), (1 << 20, 1 << 20),
                                     (1 << 19, 100_000_000), (300_017, 5_000_000)])
def test_c_fast_bucket_two_level_matches_oracle(n, n_act):
    """cpu_bucket fast mode (the CPU baseline's parallel two-level partition: high-digit scatter, then
    a counting sort per bucket) = the stable partition, on 1, 3 and 8 threads, with unrouted and
    clamped activations and Zipf-hot keys."""
    import cpu_ref
    rng = np.random.default_rng(n + n_act)
    for kind in ("uniform", "zipf"):
        a = (rng.integers(0, n_act + 3, size=n) if kind == "uniform" else (rng.zipf(1.1, size=n) - 1) % (n_act + 3))
        a = a.astype(np.uint32)
        a[rng.random(n) < 0.1] = o.M32
        wp, wo = o.bucket_stable(a, n_act)
        for thr in (1, 3, 8):
            perm, off = cpu_ref.bucket(a, n_act, faithful=False, nthreads=thr)
            np.testing.assert_array_equal(perm, wp, err_msg=f"{kind} {thr}")
            np.testing.assert_array_equal(off, wo, err_msg=f"{kind} {thr}")


def test_c_bucket_runs_matches_stable_partition():
    """cpu_bucket_runs (the micro-batch form of the CPU bucketing, cfg 5 baseline) = the stable
    partition restricted to the activations present, across reused scratch."""
    import cpu_ref
    rng = np.random.default_rng(12)
    br = cpu_ref.BucketRuns(1000, 5000)
    for n in (0, 1, 17, 4096, 5000):
        acts = rng.integers(0, 1100, size=n).astype(np.uint32)
        acts[rng.random(n) < 0.05] = o.M32
        perm, ra, rs = br(acts)
        wp, wo = o.bucket_stable(acts, 1000)
        np.testing.assert_array_equal(perm, wp)
        c = np.minimum(acts.astype(np.int64), 1000)
        ua = np.unique(c)
        np.testing.assert_array_equal(ra, ua)
        np.testing.assert_array_equal(np.diff(rs), np.bincount(c, minlength=1001)[ua])
        assert rs[0] == 0 and rs[-1] == n
    assert not br.counts.any()


def test_type_codes_match_the_reference_assertions():
    """Known answers the reference's own tests hold: the GrainId of GetGrain<ITestGrain>(k) has
    BaseTypeCode 1146670029 and that of GetGrain<ICollectionTestGrain>(k) 1381240679
    (test/DefaultCluster.Tests/CodeGenTests/CodeGeneratorTests_RequiringSilo.cs:32,47).  The class's type
    code is GrainInterfaceUtils.GetTypeCode = Utils.CalculateIdHash(class full name) (no
    [TypeCodeOverride]; GrainInterfaceUtils.cs:400-415, Utils.cs:184-203), it goes into the key's
    TypeCodeData (GrainId.GetGrainId(typeCode, long), GrainId.cs:72-77, UniqueKey.cs:112-128) and
    BaseTypeCode reads its low 32 bits back (UniqueKey.cs:11,36-39).  This pins the SHA-256-of-UTF-16LE
    fold and the key layout every routed message carries."""
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))
    for row in kat["grain_class_type_codes"]:
        tc = o.grain_type_code(row["class"])
        assert tc == row["base_type_code"], row["class"]
        key = o.grain_keys(tc, np.array([12345]))[0]
        assert int(key[2]) >> 56 == o.CAT_GRAIN
        assert int(key[2]) & 0xFFFFFFFF == row["base_type_code"]
