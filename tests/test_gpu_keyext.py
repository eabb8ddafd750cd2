"""KeyExt grains on the GPU (gd_*_ext, gd_keyext.h) against the oracle (oracle/keyext.py):
device Jenkins over ToByteArray for every tail length and multi-byte UTF-8, the KeyExt
directory (first-wins registration, RemoveActivation, tombstones, growth, heap compaction) and
routing + bucketing of batches mixing KeyExt grains with ordinary ones, in ring modes D/R/V."""
import json
import os

import numpy as np
import pytest

import oracle as o
import keyext as kx

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "keyext.json")))
TC = o.grain_type_code(o.PING_GRAIN_CLASS)
STC = GOLD["type_code"]


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _engine(gd, mode="D", my_silo=0, cap=1 << 12):
    silos = o.bench_silos(8)
    e = gd.GrainDispatch(device=0, table_capacity=cap, my_silo=my_silo)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    return e, o.ring_spec(silos, mode)


def _dev_ext(exts):
    """oracle ext items -> binding items (EXT_HOST -> GD_KEYEXT_HOST)."""
    from orleans_amd import graindispatch as g
    return [g.GD_KEYEXT_HOST if (isinstance(e, str) and e == kx.EXT_HOST) else e for e in exts]


def test_device_hash_golden_and_random(gd):
    e, _ = _engine(gd)
    items = [(int(a), int(b), int(c), None if x is None else bytes.fromhex(x), h) for a, b, c, x, h in GOLD["hashes"]]
    keys = np.array([[a, b, c] for a, b, c, _, _ in items], dtype=np.uint64)
    got = e.uniform_hashes_ext(keys, [x for _, _, _, x, _ in items])
    assert got.tolist() == [h for *_, h in items]
    rng = np.random.default_rng(5)
    n = 3000
    keys = rng.integers(0, 2 ** 63, size=(n, 3), dtype=np.uint64)
    keys[:, 2] = (keys[:, 2] & np.uint64(0x00FFFFFFFFFFFFFF)) | np.uint64(o.CAT_KEYEXT_GRAIN << 56)
    alphabet = list("abcxyz0189 -_/") + ["é", "中", "\U0001F600", "Ω"]
    exts = ["".join(rng.choice(alphabet, size=int(rng.integers(0, 90)))).encode("utf-8") for _ in range(n)]
    exts[::17] = [None] * len(exts[::17])
    got = e.uniform_hashes_ext(keys, exts)
    want = [kx.ext_uniform_hash(int(a), int(b), int(c), x) for (a, b, c), x in zip(keys, exts)]
    assert got.tolist() == want
    e.close()


def test_register_lookup_unregister(gd):
    e, _ = _engine(gd)
    d = kx.KeyExtDirectory()
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
    geo = o.type_code_data(o.CAT_GEO_CLIENT, 0)
    # batch 1: duplicates inside the batch (first wins), null KeyExt for a geo client, unicode
    names = [b"alice", b"bob", b"alice", "zé中".encode(), b"bob", b"carol", b""]
    keys = [(0, 0, tcd)] * 6 + [(0, 0, tcd)]
    keys += [(1, 2, geo), (1, 2, geo)]
    names += [None, b"eu"]
    acts = np.arange(len(keys), dtype=np.uint32) + 10
    silos = np.arange(len(keys), dtype=np.uint32) % 8
    ga, gs, gi = e.register_ext(np.array(keys, np.uint64), names, acts, silos)
    for i, (k, x) in enumerate(zip(keys, names)):
        a, s, ins = d.add_single_activation(k, x, int(acts[i]), int(silos[i]))
        assert (ga[i], gs[i], gi[i]) == (a, s, int(ins)), i
    # lookups incl. absent keys and same words with another KeyExt / null
    q = keys + [(0, 0, tcd), (0, 0, tcd), (1, 2, geo)]
    qn = names + [b"dave", None, b"us"]
    f, la, ls = e.lookup_ext(np.array(q, np.uint64), qn)
    for i, (k, x) in enumerate(zip(q, qn)):
        v = d.lookup(k, x)
        assert bool(f[i]) == (v is not None) and (v is None or (la[i], ls[i]) == v), i
    # RemoveActivation: wrong activation keeps the entry, right one removes it
    rm = e.unregister_ext(np.array([keys[0], keys[1], keys[1]], np.uint64), [b"alice", b"bob", b"bob"],
                          [999, 11, 11])
    assert rm.tolist() == [0, 1, 0]
    assert d.remove_activation(keys[1], b"bob", 11)
    f, la, _ = e.lookup_ext(np.array([keys[0], keys[1]], np.uint64), [b"alice", b"bob"])
    assert f.tolist() == [1, 0] and la[0] == 10
    # re-register over the tombstone
    ga, _, gi = e.register_ext(np.array([keys[1]], np.uint64), [b"bob"], [77], [3])
    assert gi.tolist() == [1] and ga.tolist() == [77]
    assert e.ext_stats()["live"] == len(d.data) + 1 - 0   # bob is back
    e.close()


def test_growth_tombstones_and_heap_compaction(gd):
    e, _ = _engine(gd)
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
    d = kx.KeyExtDirectory()
    n = 40000
    names = [f"grain/{i:06d}/" + "x" * (i % 37) for i in range(n)]
    keys = np.tile(np.array([[0, 0, tcd]], np.uint64), (n, 1))
    for lo in range(0, n, 10000):                  # several batches: the table grows (rehash) on the way
        sl = slice(lo, lo + 10000)
        e.register_ext(keys[sl], names[sl], np.arange(lo, lo + 10000), np.full(10000, 4))
    for i, nm in enumerate(names):
        d.add_single_activation(tuple(keys[i]), nm.encode(), i, 4)
    rm = e.unregister_ext(keys[::2], names[::2], np.arange(0, n, 2))
    assert rm.all()
    for i in range(0, n, 2):
        d.remove_activation(tuple(keys[i]), names[i].encode(), i)
    st = e.ext_stats()
    assert st["live"] == n // 2
    heap_before = st["heap_bytes"]
    # enough new entries to force a rehash: tombstones dropped, the heap compacted
    more = [f"late/{i}" for i in range(3 * n)]
    mk = np.tile(np.array([[0, 0, tcd]], np.uint64), (len(more), 1))
    e.register_ext(mk, more, np.arange(len(more)) + n, np.full(len(more), 1))
    for i, nm in enumerate(more):
        d.add_single_activation(tuple(mk[i]), nm.encode(), i + n, 1)
    st = e.ext_stats()
    assert st["live"] == len(d.data)
    assert st["heap_bytes"] < heap_before + sum(len(m) for m in more)   # removed strings are gone
    q = names[:200] + more[:200]
    qk = np.tile(np.array([[0, 0, tcd]], np.uint64), (len(q), 1))
    f, la, _ = e.lookup_ext(qk, q)
    for i, nm in enumerate(q):
        v = d.lookup(tuple(qk[i]), nm.encode())
        assert bool(f[i]) == (v is not None) and (v is None or la[i] == v[0])
    e.close()


@pytest.mark.parametrize("mode", ["D", "R", "V"])
def test_route_bucket_mixed_batch(gd, mode):
    """Ordinary grains, string grains (registered or not), compound keys, geo clients with and
    without KeyExt, GD_KEYEXT_HOST items, system targets and the membership grain in one batch."""
    e, spec = _engine(gd, mode, my_silo=3, cap=1 << 14)
    rng = np.random.default_rng(11)
    G = 3000
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg, np.arange(G), own)
    d = kx.KeyExtDirectory()
    S = 2000
    snames = [f"user-{i}" + ("é" if i % 5 == 0 else "") for i in range(S)]
    sk = np.tile(np.array([[0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)]], np.uint64), (S, 1))
    sk[S // 2:, 1] = np.arange(S - S // 2, dtype=np.uint64)          # compound long key + extension
    reg_idx = np.arange(0, S, 2)
    acts = G + reg_idx
    ss = (reg_idx * 7) % 8
    e.register_ext(sk[reg_idx], [snames[i] for i in reg_idx], acts, ss)
    for j, i in enumerate(reg_idx):
        d.add_single_activation(tuple(sk[i]), snames[i].encode(), int(acts[j]), int(ss[j]))
    geo_k = np.array([[9, 9, o.type_code_data(o.CAT_GEO_CLIENT, 0)]], np.uint64)
    e.register_ext(geo_k, [None], [G + S], [6])
    d.add_single_activation(tuple(geo_k[0]), None, G + S, 6)
    n = 60000
    kind = rng.integers(0, 10, size=n)
    keys = o.grain_keys(TC, rng.integers(0, G + 100, size=n))
    exts = [None] * n
    for i in np.nonzero(kind >= 5)[0]:
        j = int(rng.integers(0, S))
        keys[i] = sk[j]
        exts[i] = snames[j].encode()
    for i in np.nonzero(kind == 4)[0]:
        keys[i] = geo_k[0]
        exts[i] = None if i % 2 else b"other-cluster"
    host = np.nonzero(kind == 3)[0][::3]
    for i in host:
        keys[i] = sk[0]
        exts[i] = kx.EXT_HOST
    keys[::101] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
    keys[50::103] = np.array(o.MEMBERSHIP_TABLE_ID.as_tuple(), dtype=np.uint64)
    for i in list(range(0, n, 101)) + list(range(50, n, 103)):
        exts[i] = None
    n_act = G + S + 1
    st, silo, act, perm, off = e.route_bucket_ext(keys, _dev_ext(exts), n_act)
    wst, wsilo, wact, _, _ = kx.route_batch_ext(keys, exts, spec, o.DirectoryArrays(reg, np.arange(G), own), d,
                                                my_silo=3, seed_silo=o.M32)
    np.testing.assert_array_equal(st, wst)
    np.testing.assert_array_equal(silo, wsilo)
    np.testing.assert_array_equal(act, wact)
    wp, wo = o.bucket_stable(wact, n_act)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    n_host = sum(1 for x in exts if isinstance(x, str) and x == kx.EXT_HOST)
    assert (st == o.ST_OK).sum() > n // 3 and (st == o.ST_KEYEXT).sum() == n_host > 1000
    # route without ext: every KeyExt message stays at GD_ROUTE_KEYEXT (the gd_route contract)
    st0, _, _ = e.route(keys)
    assert ((st0 == o.ST_KEYEXT) == np.isin(keys[:, 2] >> np.uint64(56), [6, 7])).all()
    e.close()


def test_golden_route(gd):
    r = GOLD["route"]
    e, spec = _engine(gd, "D", my_silo=r["my_silo"])
    names = [f"user-{i:04d}" for i in range(64)]
    k = [kx.string_grain(STC, nm) for nm, _, _ in r["directory"]]
    e.register_ext(np.array([x[0] for x in k], np.uint64), [x[1] for x in k], [a for _, a, _ in r["directory"]],
                   [s for _, _, s in r["directory"]])
    keys, exts = [], []
    for (idx,) in r["messages"]:
        kk, ee = kx.string_grain(STC, names[idx if idx is not None else 3])
        keys.append(kk)
        exts.append(gd.GD_KEYEXT_HOST if idx is None else ee)
    st, silo, act = e.route_ext(np.array(keys, np.uint64), exts)
    assert st.tolist() == r["status"] and silo.tolist() == r["silo"] and act.tolist() == r["act"]
    e.close()


def test_bad_ranges_and_errors(gd):
    e, _ = _engine(gd)
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
    keys = np.array([[0, 0, tcd]] * 3, np.uint64)
    x = gd.KeyExtBatch([b"abc", b"de", b"f"])
    x.offset[1] = 1 << 40                                       # outside the buffer
    x.struct = gd.gd_key_ext(x.blob.ctypes.data, x.offset.ctypes.data, x.length.ctypes.data, 6)
    st, silo, act = e.route_ext(keys, x)
    assert st.tolist() == [o.ST_MISS, o.ST_KEYEXT, o.ST_MISS]
    with pytest.raises(gd.GrainDispatchError):
        e.register_ext(keys, x, [1, 2, 3], [0, 0, 0])           # bad range: GD_EINVAL, nothing applied
    assert e.ext_stats()["live"] == 0
    with pytest.raises(gd.GrainDispatchError):                  # not a KeyExt category
        e.register_ext(o.grain_keys(TC, np.arange(1)), [b"x"], [1], [0])
    with pytest.raises(gd.GrainDispatchError):                  # GD_KEYEXT_HOST cannot be registered
        e.register_ext(keys[:1], [gd.GD_KEYEXT_HOST], [1], [0])
    e.close()


def test_device_entry_point(gd):
    import torch
    e, spec = _engine(gd, "V")
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
    names = [f"n{i}" for i in range(500)]
    keys = np.tile(np.array([[0, 0, tcd]], np.uint64), (500, 1))
    e.register_ext(keys[:250], names[:250], np.arange(250), np.full(250, 2))
    x = gd.KeyExtBatch(names)
    dev = torch.device("cuda", 0)
    tk = torch.from_numpy(keys.view(np.int64).copy()).to(dev)
    tb = torch.from_numpy(x.blob).to(dev)
    to = torch.from_numpy(x.offset.view(np.int64)).to(dev)
    tl = torch.from_numpy(x.length).to(dev)
    silo = torch.empty(500, dtype=torch.int32, device=dev)
    act = torch.empty(500, dtype=torch.int32, device=dev)
    st = torch.empty(500, dtype=torch.uint8, device=dev)
    perm = torch.empty(500, dtype=torch.int32, device=dev)
    off = torch.empty(252, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    e.set_stream(s.cuda_stream)
    with torch.cuda.stream(s):
        e.route_bucket_ext_device(tk.data_ptr(), tb.data_ptr(), to.data_ptr(), tl.data_ptr(), int(x.struct.bytes_len),
                                  500, 250, silo.data_ptr(), act.data_ptr(), st.data_ptr(), perm.data_ptr(),
                                  off.data_ptr())
    torch.cuda.synchronize()
    a = act.cpu().numpy().view(np.uint32)
    assert a[:250].tolist() == list(range(250)) and (a[250:] == o.M32).all()
    assert (st.cpu().numpy()[250:] == o.ST_MISS).all()
    wp, wo = o.bucket_stable(a, 250)
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wp)
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), wo)
    e.close()


@pytest.mark.parametrize("mode", ["D", "V"])
def test_route_frames_ext(gd, mode):
    """gd_route_frames_ext: frames whose TargetGrain is a string-keyed grain are routed with the
    KeyExt string read from the frame buffer (oracle/headers.py route_frames_ext_np), next to
    ordinary, complete, fallback and malformed frames; bucketing over the result."""
    import headers as H
    e, spec = _engine(gd, mode, cap=1 << 13)
    rng = np.random.default_rng(23)
    G = 1000
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg, np.arange(G), own)
    d = kx.KeyExtDirectory()
    names = [f"device/{i}" + ("ü" * (i % 3)) + "q" * (i % 41) for i in range(600)]    # inline and heap strings
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
    e.register_ext(np.tile(np.array([[0, 0, tcd]], np.uint64), (300, 1)), names[:300], np.arange(300) + G,
                   np.arange(300) % 8)
    for i in range(300):
        d.add_single_activation((0, 0, tcd), names[i].encode(), G + i, i % 8)
    n = 5000
    keys = o.grain_keys(TC, rng.integers(0, G + 50, size=n))
    exts = [None] * n
    for i in np.nonzero(rng.random(n) < 0.5)[0]:
        keys[i] = (0, 0, tcd)
        exts[i] = names[int(rng.integers(0, 600))]
    buf, offs = H.random_frames(n, keys, rng, p_fallback=0.05, p_complete=0.05, p_malformed=0.03, target_exts=exts)
    f, wst, wsilo, wact = H.route_frames_ext_np(buf, offs, spec, o.DirectoryArrays(reg, np.arange(G), own), d)
    n_act = G + 300
    _, st, silo, act, perm, off = e.route_frames(buf, offs, n_act, keyext=True)
    np.testing.assert_array_equal(st, wst)
    np.testing.assert_array_equal(silo, wsilo)
    np.testing.assert_array_equal(act, wact)
    wp, wo = o.bucket_stable(wact, n_act)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    assert ((wst == o.ST_OK) & (keys[:, 2] == np.uint64(tcd))).sum() > 500
    _, st0, _, _ = e.route_frames(buf, offs)           # gd_route_frames: KeyExt targets stay KEYEXT
    assert ((st0 == o.ST_KEYEXT) == ((wst != H.ROUTE_ADDRESSED) & (wst != H.ROUTE_UNDECODED) &
                                    (f["target_grain"][:, 2] == np.uint64(tcd)))).all()
    e.close()


@pytest.mark.parametrize("mode", ["D", "V"])
def test_split_ext_membership_change(gd, mode):
    """gd_dir_split_ext: after a ring change, the KeyExt entries whose new owner (the stored
    uniform hash under the new ring) is not kept leave the partition with their strings
    (GrainDirectoryPartition.Split, GrainDirectoryPartition.cs:532-570; handoff predicate
    GrainDirectoryHandoffManager.cs:212-218); merged elsewhere with gd_dir_register_ext."""
    silos = o.bench_silos(8)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 12)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, STC)
    names = [f"player/{i}" + "ö" * (i % 5) + "y" * (i % 33) for i in range(3000)]
    keys = np.tile(np.array([[0, 0, tcd]], np.uint64), (3000, 1))
    keys[::7, 1] = np.arange(0, 3000, 7, dtype=np.uint64)                 # compound keys too
    exts = [n.encode() for n in names]
    exts[5] = None
    keys[5] = (1, 2, o.type_code_data(o.CAT_GEO_CLIENT, 0))               # a geo client, null KeyExt
    acts = np.arange(3000, dtype=np.uint32)
    e.register_ext(keys, exts, acts, acts % 8)
    new = silos[:6] + [o.Silo("10.0.0.99", 11111, 3)]                       # silos 6, 7 leave, one joins
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in new])
    spec = o.ring_spec(new, mode)
    keep = [0, 1, 2]
    owner = o.ring_owner_np(spec, np.array([kx.ext_uniform_hash(int(a), int(b), int(c), x)
                                            for (a, b, c), x in zip(keys, exts)], dtype=np.uint32))
    want = {(tuple(int(v) for v in keys[i]), exts[i], int(acts[i]), int(acts[i] % 8))
            for i in range(3000) if int(owner[i]) not in keep}
    k, a, s, x = e.split_ext(keep, len(new), move=True)
    got = {(tuple(int(v) for v in k[i]), x[i], int(a[i]), int(s[i])) for i in range(len(a))}
    assert got == want and len(a) == len(want) > 1000
    assert e.ext_stats()["live"] == 3000 - len(want)
    f, _, _ = e.lookup_ext(keys, exts)
    assert (f.astype(bool) == np.array([int(o_) in keep for o_ in owner])).all()
    k2, a2, _, _ = e.split_ext(keep, len(new), move=True)                   # nothing left to move
    assert len(a2) == 0
    other = gd.GrainDispatch(device=0, table_capacity=1 << 12)              # the merge on the receiver
    other.ring_set_silos(mode, [(s_.ip, s_.port, s_.gen) for s_ in new])
    _, _, ins = other.register_ext(k, x, a, s)
    assert ins.all()
    f2, a3, _ = other.lookup_ext(k, x)
    assert f2.all() and (a3 == a).all()
    other.close()
    e.close()
