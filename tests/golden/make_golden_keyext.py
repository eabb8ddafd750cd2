"""Generate tests/golden/keyext.json from the oracle (oracle/keyext.py): KeyExt-grain uniform
hashes (Jenkins over UniqueKey.ToByteArray, UniqueKey.cs:272-336) for every tail length of the
byte variant, multi-byte UTF-8, null KeyExt, geo clients; and a routed batch against a KeyExt
directory.  Frozen oracle outputs (the reference holds no numeric vectors for these), inputs
synthetic.

usage: python tests/golden/make_golden_keyext.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as o  # noqa: E402
import keyext as kx  # noqa: E402

STRINGS = ["a", "hello world", "user-0001", "grainé中\U0001F600", "  x", "Ω" * 13, "k" * 64, "z" * 257,
           "chirper/alice", "0123456789a", "0123456789ab", "0123456789abc"]


def main():
    rng = np.random.default_rng(20261017)
    tc = o.grain_type_code("UnitTests.GrainInterfaces.IStringKeyGrain")
    items = []
    for L in range(0, 40):                       # every length mod 12, around the 28-byte head
        items.append((0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, tc), bytes(rng.integers(32, 127, size=L,
                                                                                         dtype=np.uint8))))
    for s in STRINGS:
        items.append((0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, tc), s.encode("utf-8")))
    for _ in range(6):                           # compound keys: Guid / long key + extension
        n0, n1 = (int(x) for x in rng.integers(0, 2 ** 63, size=2, dtype=np.uint64))
        items.append((n0, n1, o.type_code_data(o.CAT_KEYEXT_GRAIN, -tc), b"ext-%d" % (n0 % 1000)))
    items.append((3, 4, o.type_code_data(o.CAT_GEO_CLIENT, 0), None))      # geo client, null KeyExt
    items.append((5, 6, o.type_code_data(o.CAT_GEO_CLIENT, 0), b"us-west"))
    g = {"_comment": "frozen outputs of oracle/keyext.py; regenerate with make_golden_keyext.py",
         "type_code": tc,
         "hashes": [[str(n0), str(n1), str(t), None if e is None else e.hex(), kx.ext_uniform_hash(n0, n1, t, e)]
                    for n0, n1, t, e in items]}
    # routed batch: ring bench8/D, half of the string grains registered, my silo 2
    spec = o.ring_spec(o.bench_silos(8), "D")
    names = [f"user-{i:04d}" for i in range(64)]
    d = kx.KeyExtDirectory()
    for i, nm in enumerate(names[:32]):
        k, e = kx.string_grain(tc, nm)
        d.add_single_activation(k, e, 500 + i, i % 8)
    keys, exts = [], []
    for j in range(80):
        k, e = kx.string_grain(tc, names[int(rng.integers(0, 64))])
        keys.append(k)
        exts.append(e)
    keys[7], exts[7] = kx.string_grain(tc, names[3])[0], kx.EXT_HOST
    keys = np.array(keys, dtype=np.uint64)
    st, silo, act, own, h = kx.route_batch_ext(keys, exts, spec, o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []),
                                               d, my_silo=2)
    g["route"] = {"ring": "bench8/D", "my_silo": 2,
                  "directory": [[nm, 500 + i, i % 8] for i, nm in enumerate(names[:32])],
                  "messages": [[None if isinstance(e, str) else names.index(e.decode())] for e in exts],
                  "status": st.tolist(), "silo": silo.tolist(), "act": act.tolist(), "owner": own.tolist(),
                  "hash": h.tolist()}
    with open(os.path.join(HERE, "keyext.json"), "w") as f:
        json.dump(g, f, indent=0)


if __name__ == "__main__":
    main()
