#!/usr/bin/env python3
"""A/B of the route kernel that also counts the one-pass MSD digits (option fuse_hist) at the cfg-2
shape: bit-exact outputs with the option on and off, then interleaved timing.  Prints JSON lines.
The option was removed after this A/B; the script needs that experiment's build."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g    # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    dev = torch.device("cuda", 0)
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    keys_all = np.zeros((G, 3), dtype=np.uint64)
    keys_all[:, 1] = np.arange(G, dtype=np.uint64)
    keys_all[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=0, table_capacity=2 * G)
    e.ring_set_silos("D", SILOS)
    owner = e.ring_owner(keys_all)
    e.register(keys_all, np.arange(G, dtype=np.uint32), owner)
    rng = np.random.default_rng(0x5EED0001)
    kk = np.zeros((n, 3), dtype=np.uint64)
    kk[:, 1] = rng.integers(0, G, size=n, dtype=np.int64).astype(np.uint64)
    kk[:, 2] = np.uint64(tcd)
    keys = torch.from_numpy(kk.view(np.int64)).to(dev)
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)
    outs = {}
    for f in (0, 1):
        o = [torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
             torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
             torch.empty(G + 2, dtype=torch.int32, device=dev)]
        outs[f] = o

    def step(f):
        e.set_option("fuse_hist", f)
        e.tune_set("probe_keys", 3)
        s, a, st, p, off = outs[f]
        e.route_bucket_device(keys.data_ptr(), n, G, s.data_ptr(), a.data_ptr(), st.data_ptr(), p.data_ptr(),
                              off.data_ptr())

    with torch.cuda.stream(stream):
        for f in (0, 1):
            step(f)
        torch.cuda.synchronize()
        same = all(bool(torch.equal(x, y)) for x, y in zip(outs[0], outs[1]))
        print(json.dumps({"bit_exact": same}), flush=True)
        if not same:
            sys.exit(1)
        res = {0: [], 1: []}
        for r in range(6):
            for f in (0, 1):
                for _ in range(10):
                    step(f)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(50):
                    step(f)
                b.record(stream)
                b.synchronize()
                res[f].append(a.elapsed_time(b) / 50)
        print(json.dumps({"n": n, "grains": G, "ms_off": sorted(res[0]), "ms_on": sorted(res[1]),
                          "median_off": float(np.median(res[0])), "median_on": float(np.median(res[1]))}), flush=True)


if __name__ == "__main__":
    main()
