"""Debug: LocalLookup of a string grain owned locally (C++ PerSiloLocalLookupStringKeys)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import oracle as o
import keyext as kx
from orleans_amd import graindispatch as gd

sil = o.bench_silos(4)
e = gd.GrainDispatch(device=0, table_capacity=4096, my_silo=0)
e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in sil])
spec = o.ring_spec(sil, "D")
e.set_valid_silos([0, 1, 2, 3], 4)
stc = o.calculate_id_hash("UnitTests.StringKeyGrain")
tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, stc)
mine, theirs = [], []
for k in range(400):
    s = f"user/{k}".encode()
    h = kx.ext_uniform_hash(0, 0, tcd, s)
    own = int(o.ring_owner_np(spec, np.array([h], np.uint32))[0])
    (mine if own == 0 else theirs).append(s)
print("mine", len(mine), "theirs", len(theirs))
key = np.array([[0, 0, tcd]], np.uint64)
print("register", e.register_ext(key, [mine[0]], [0], [0]))
print("whole-node route", e.route_ext(key, [mine[0]]))
e.cache_configure(100, [0], 4, [0, 1, 2, 3])
print("cache route mine0", e.route_ext(key, [mine[0]]))
print("cache route mine1", e.route_ext(key, [mine[1]]))
print("cache route theirs0", e.route_ext(key, [theirs[0]]))
print("stats", e.cache_stats())
