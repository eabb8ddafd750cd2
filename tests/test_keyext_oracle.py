"""KeyExt grains on CPU: the oracle (oracle/keyext.py) against its frozen fixtures
(tests/golden/keyext.json), against the oracle's own UniqueKey.ToByteArray restatement and the
library's host Jenkins (gd_jenkins_hash_bytes, no GPU needed), plus directory semantics."""
import json
import os
import struct

import numpy as np

import oracle as o
import keyext as kx

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "keyext.json")))


def _items():
    for n0, n1, t, e, h in GOLD["hashes"]:
        yield int(n0), int(n1), int(t), None if e is None else bytes.fromhex(e), h


def test_golden_keyext_hashes():
    for n0, n1, t, e, h in _items():
        assert kx.ext_uniform_hash(n0, n1, t, e) == h


def test_hash_is_jenkins_over_to_byte_array():
    """UniqueKey.GetUniformHashCode (UniqueKey.cs:272-293) = Jenkins(ToByteArray) for a KeyExt
    key; the ToByteArray layout is the wire layout (Identifiertests.UniqueKeyToByteArray,
    Identifiertests.cs:32-48): N0 | N1 | TCD | int32 length | UTF-8."""
    for n0, n1, t, e, h in _items():
        if e is None:
            assert h == o.jenkins_u64x3(t, n0, n1)
            continue
        uk = o.UniqueKey(n0, n1, t, e.decode("utf-8"))
        b = uk.to_byte_array()
        assert b == struct.pack("<QQQi", n0, n1, t, len(e)) + e
        assert uk.uniform_hash() == h


def test_library_host_jenkins_agrees():
    from orleans_amd import graindispatch as g
    for n0, n1, t, e, h in _items():
        if e is not None:
            assert g.jenkins_bytes(struct.pack("<QQQi", n0, n1, t, len(e)) + e) == h


def test_golden_keyext_route():
    r = GOLD["route"]
    tc = GOLD["type_code"]
    names = [f"user-{i:04d}" for i in range(64)]
    d = kx.KeyExtDirectory()
    for nm, a, s in r["directory"]:
        k, e = kx.string_grain(tc, nm)
        d.add_single_activation(k, e, a, s)
    keys, exts = [], []
    for (idx,) in r["messages"]:
        k, e = kx.string_grain(tc, names[idx if idx is not None else 3])
        keys.append(k)
        exts.append(kx.EXT_HOST if idx is None else e)
    st, silo, act, own, h = kx.route_batch_ext(np.array(keys, dtype=np.uint64), exts, o.ring_spec(o.bench_silos(8), "D"),
                                               o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []), d,
                                               my_silo=r["my_silo"])
    assert st.tolist() == r["status"] and silo.tolist() == r["silo"] and act.tolist() == r["act"]
    assert own.tolist() == r["owner"] and h.tolist() == r["hash"]


def test_keyext_directory_semantics():
    """AddSingleActivation first-wins, RemoveActivation only for the matching activation
    (GrainDirectoryPartition.cs:304-363); KeyExt is part of the key (UniqueKey.cs:245-251)."""
    d = kx.KeyExtDirectory()
    k = (0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, 9))
    assert d.add_single_activation(k, b"a", 1, 2) == (1, 2, True)
    assert d.add_single_activation(k, b"a", 5, 6) == (1, 2, False)
    assert d.add_single_activation(k, b"b", 5, 6) == (5, 6, True)
    assert d.add_single_activation(k, None, 7, 0) == (7, 0, True)
    assert not d.remove_activation(k, b"a", 99)
    assert d.remove_activation(k, b"a", 1)
    assert d.lookup(k, b"a") is None and d.lookup(k, b"b") == (5, 6) and d.lookup(k, None) == (7, 0)


def test_pack_ext_layout():
    blob, off, ln = kx.pack_ext([b"ab", None, kx.EXT_HOST, "é".encode(), b""])
    assert bytes(blob) == b"ab\xc3\xa9"
    assert ln.tolist() == [2, -1, -2, 2, 0] and off.tolist()[:1] == [0] and off[3] == 2
