#!/usr/bin/env python3
"""k_route against its memory bound (gd_route_bound_device) on cfg 2's directory and batch: per-launch ms
from the library's HIP events, interleaved rounds.  One JSON line.  (profiles/r06_route_bound_forms.json
holds the forms the bound was chosen from: 1, 2 and 4 messages a thread, NT or temporal keys, with and
without the ring-staging barrier -- since folded into the one form the library keeps.)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g                      # noqa: E402
from orleans_amd.workloads import grain_keys_torch              # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    G, N = 1 << 20, 1 << 24
    dev = torch.device("cuda:0")
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0, kernel_timing=False)
    e.tune_set("probe_keys", 3)
    e.ring_set_silos("D", SILOS)
    allk = grain_keys_torch(tcd, torch.arange(G, device=dev), dev)
    own = torch.empty(G, dtype=torch.int32, device=dev)
    e.ring_owner_device(allk.data_ptr(), G, own.data_ptr())
    vals = torch.stack([torch.arange(G, device=dev, dtype=torch.int32), own], 1).contiguous()
    e.register_device(allk.data_ptr(), vals.data_ptr(), G)
    ks = torch.from_numpy(np.random.default_rng(0x5EED0001).integers(0, G, size=N)).to(dev)
    keys = grain_keys_torch(tcd, ks, dev)
    silo = torch.empty(N, dtype=torch.int32, device=dev)
    act = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    args = (keys.data_ptr(), N, silo.data_ptr(), act.data_ptr(), st.data_ptr())
    e.route_device(*args)
    torch.cuda.synchronize()
    res = {}

    def timed(name, fn, reps=5):
        fn()
        torch.cuda.synchronize()
        e.set_kernel_timing(1)
        e.kernel_times_reset()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        t = e.kernel_times()
        e.set_kernel_timing(False)
        k = "k_route_bound" if name.startswith("bound") else "k_route"
        res.setdefault(name, []).append(round(t[k][1] / t[k][0], 4))

    for _ in range(3):
        timed("route", lambda: e.route_device(*args))
        timed("bound", lambda: e.route_bound_device(*args))
    print(json.dumps(res), flush=True)
    e.close()


if __name__ == "__main__":
    main()
