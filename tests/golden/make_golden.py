"""Generate tests/golden/golden.json from the oracle (oracle/oracle.py).

The reference (C#) cannot run here and its tests hold no numeric vectors for
these hashes, so these fixtures are the oracle's own outputs, frozen: they pin
the oracle (and every later refactor of it) and give the GPU tests fixed
inputs/outputs.  Inputs are synthetic; nothing here is copied from the reference.

usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as o  # noqa: E402
import headers as H  # noqa: E402

SILOS = [o.Silo("10.0.0.1", 11111, 1), o.Silo("10.0.0.2", 11111, 1), o.Silo("127.0.0.1", 0, 1),
         o.Silo("127.0.0.1", 0, 5), o.Silo("127.0.0.1", 8080, 26), o.Silo("192.168.1.200", 30000, 123456789),
         o.Silo("fe80::1", 11111, 3), o.Silo("2001:db8::42", 22222, 7), o.Silo("::ffff:10.0.0.9", 11111, 1),
         o.Silo("10.0.0.3", 11111, -2)]
TEXTS = ["", "a", "BenchmarkGrains.Ping.PingGrain", "UnitTests.GrainInterfaces.ITestGrain",
         "Orleans.Runtime.IMembershipTableGrain", "grainé中\U0001F600", "x" * 200]


def main():
    rng = np.random.default_rng(20261015)
    g = {"_comment": "frozen outputs of oracle/oracle.py; regenerate with make_golden.py"}
    blobs = [bytes(rng.integers(0, 256, size=n, dtype=np.uint8)) for n in
             [0, 1, 2, 3, 4, 5, 7, 8, 11, 12, 13, 23, 24, 25, 28, 35, 36, 37, 100]]
    g["jenkins_bytes"] = [[b.hex(), o.jenkins_bytes(b)] for b in blobs]
    u = rng.integers(0, 2 ** 63, size=(32, 3), dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=(32, 3),
                                                                                               dtype=np.uint64)
    g["jenkins_u64x3"] = [[str(int(a)), str(int(b)), str(int(c)), o.jenkins_u64x3(int(a), int(b), int(c))]
                          for a, b, c in u]
    g["calculate_id_hash"] = [[t, o.calculate_id_hash(t)] for t in TEXTS]
    g["silos"] = [{"ip": s.ip, "port": s.port, "gen": s.gen, "consistent_hash": s.consistent_hash(),
                   "uniform_hashes_30": s.uniform_hashes(30)} for s in SILOS]
    rings = {}
    for name, silos in (("bench8", o.bench_silos(8)), ("mixed10", SILOS),
                        ("loopback5", [o.Silo("127.0.0.1", 0, k) for k in range(1, 6)])):
        for mode in "DRV":
            sp = o.ring_spec(silos, mode)
            rings[f"{name}/{mode}"] = {"points": [int(p) for p in sp.points], "owners": sp.owners}
    g["rings"] = rings
    # a small addressing batch (ring D over bench8, seed silo 5, my silo 3)
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    reg = o.grain_keys(tc, np.arange(32))
    spec = o.ring_spec(o.bench_silos(8), "D")
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    special = np.array([o.UniqueKey(0, 77, o.type_code_data(o.CAT_SYSTEM_TARGET, 12)).as_tuple(),
                        o.MEMBERSHIP_TABLE_ID.as_tuple(),
                        o.UniqueKey(0, 5, o.type_code_data(o.CAT_KEYEXT_GRAIN, tc)).as_tuple()], dtype=np.uint64)
    msgs = np.concatenate([o.grain_keys(tc, rng.integers(0, 48, size=61)), special])
    d = o.DirectoryArrays(reg, np.arange(32) + 1000, owner)
    st, silo, act, own, h = o.route_batch_np(msgs, spec, d, my_silo=3, seed_silo=5)
    g["route"] = {"type_code": tc, "ring": "bench8/D", "my_silo": 3, "seed_silo": 5,
                  "directory": {"keys": [[str(int(x)) for x in k] for k in reg], "acts": list(range(1000, 1032)),
                                "silos": [int(x) for x in owner]},
                  "messages": [[str(int(x)) for x in k] for k in msgs],
                  "status": st.tolist(), "silo": silo.tolist(), "act": act.tolist(), "owner": own.tolist(),
                  "hash": h.tolist()}
    acts = rng.integers(0, 40, size=300).astype(np.uint32)
    acts[::17] = o.M32
    perm, off = o.bucket_stable(acts, 37)
    g["bucket"] = {"acts": acts.tolist(), "n_act": 37, "perm": perm.tolist(), "offsets": off.tolist()}
    # frames (oracle/headers.py encoder) and their decode, incl. fallback/malformed cases
    frng = np.random.default_rng(20261016)
    fkeys = o.grain_keys(tc, frng.integers(0, 48, size=40))
    fkeys[5] = o.UniqueKey(0, 5, o.type_code_data(o.CAT_KEYEXT_GRAIN, tc)).as_tuple()
    buf, offs = H.random_frames(40, fkeys, frng, p_fallback=0.1, p_complete=0.15, p_malformed=0.08)
    dec = H.decode_frames(buf, offs)
    fst, fsilo, fact = H.route_frames_np(buf, offs, spec, d)[1:]
    g["frames"] = {"buffer_hex": buf.hex(), "offsets": [int(x) for x in offs],
                   "flags": dec["flags"].tolist(), "mask": dec["mask"].tolist(),
                   "target_grain": [[str(int(x)) for x in k] for k in dec["target_grain"]],
                   "sending_grain": [[str(int(x)) for x in k] for k in dec["sending_grain"]],
                   "target_silo_hex": [bytes(x).hex() for x in dec["target_silo"]],
                   "correlation_id": [str(int(x)) for x in dec["correlation_id"]],
                   "category": dec["category"].tolist(), "direction": dec["direction"].tolist(),
                   "route_status": fst.tolist(), "route_silo": fsilo.tolist(), "route_act": fact.tolist()}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=0)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
