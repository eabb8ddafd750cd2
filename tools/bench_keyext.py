#!/usr/bin/env python3
"""String-keyed grains (IGrainWithStringKey, GrainId.cs:86-91) on one MI355X.

The cfg-2 shape with KeyExt grains: 2^20 grains "user-%07d" of one string-key grain type, every
one registered (gd_dir_register_ext) with one activation on its owner silo; step = 16M messages
uniform over them through gd_route_bucket_ext_device: the 24-B route kernel marks them KEYEXT,
k_route_keyext hashes N0|N1|TCD|len|UTF-8 (Jenkins bytes), finds the owner on the ring, probes
the 64-B KeyExt slots and compares the string in the heap; then the bucketing.
Prints one JSON line (per-kernel times from the library's HIP events).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g    # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1 << 24)
    ap.add_argument("--grains", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--profile-steps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    tc = g.calculate_id_hash("UnitTests.GrainInterfaces.IStringKeyGrain")
    tcd = (6 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    G, n = args.grains, args.msgs
    names = [f"user-{i:07d}" for i in range(G)]
    gkeys = np.zeros((G, 3), dtype=np.uint64)
    gkeys[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=0, table_capacity=1 << 10, my_silo=0)
    e.ring_set_silos("D", SILOS)
    t0 = time.perf_counter()
    hashes = e.uniform_hashes_ext(gkeys, names)
    owner = np.zeros(G, np.uint32)
    owner[:] = e.ring_lookup_hashes(hashes)
    e.register_ext(gkeys, names, np.arange(G, dtype=np.uint32), owner)
    t_reg = time.perf_counter() - t0
    rng = np.random.default_rng(0x5EED0001)
    pick = rng.integers(0, G, size=n)
    # the batch's KeyExt strings in message order, as a receive buffer holds them (12 bytes each)
    blob = np.frombuffer(np.array(names, dtype="S12")[pick].tobytes(), dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * np.uint64(12)
    ln = np.full(n, 12, np.int32)
    kk = np.zeros((n, 3), dtype=np.uint64)
    kk[:, 2] = np.uint64(tcd)
    keys = torch.from_numpy(kk.view(np.int64)).to(dev)
    tb = torch.from_numpy(blob.copy()).to(dev)
    to = torch.from_numpy(off.view(np.int64)).to(dev)
    tl = torch.from_numpy(ln).to(dev)
    silo = torch.empty(n, dtype=torch.int32, device=dev)
    act = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    offs = torch.empty(G + 2, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)

    def step():
        e.route_bucket_ext_device(keys.data_ptr(), tb.data_ptr(), to.data_ptr(), tl.data_ptr(), blob.size, n, G,
                                  silo.data_ptr(), act.data_ptr(), st.data_ptr(), perm.data_ptr(), offs.data_ptr())

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    a = act.cpu().numpy().view(np.uint32)
    ok = bool((a == pick.astype(np.uint32)).all() and (st.cpu().numpy() == 0).all())
    e.set_kernel_timing(True)
    e.kernel_times_reset()
    with torch.cuda.stream(stream):
        for _ in range(args.profile_steps):
            step()
    torch.cuda.synchronize()
    kt = e.kernel_times()
    kernels = {k: round(ms / args.profile_steps, 4) for k, (c, ms) in kt.items() if c}
    ms_kx = kernels.get("k_route_keyext", 0.0)
    # per message: status 1 + len 4 + off 8 + key 24 + string 12 + one 64-B slot (string inline) + 9 out
    alg = n * (1 + 4 + 8 + 24 + 12 + 64 + 9)
    print(json.dumps({
        "metric": "routed messages/sec, string-keyed grains (KeyExt), route + bucket",
        "value": round(n * args.steps / wall, 1), "unit": "messages/s", "ms_per_step": round(wall / args.steps * 1e3, 4),
        "config": {"msgs": n, "grains": G, "key": "12-byte UTF-8 string keys 'user-%07d'", "ring_mode": "D"},
        "all_routed_to_the_registered_activation": ok, "register_seconds": round(t_reg, 2),
        "k_route_keyext": {"ms": ms_kx, "alg_GBps": round(alg / (ms_kx * 1e-3) / 1e9, 1) if ms_kx else None},
        "kernels_ms_per_step": kernels}))
    e.close()


if __name__ == "__main__":
    main()
