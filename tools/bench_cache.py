#!/usr/bin/env python3
"""LocalLookup mode with the non-owner directory cache on one MI355X.

The per-silo deployment of Orleans: this GPU is silo 0 of 8 and holds only its own directory
partition (LocalGrainDirectory.cs:806-821); every other grain is looked up in the
AdaptiveGrainDirectoryCache (LRU, max 1,000,000 entries, :823-836), pre-filled here with the
remote grains' addresses as remote lookups would leave it (LocalGrainDirectory.cs:920).
Step = cfg-2 batch (16M messages uniform over 2^20 grains) through gd_route_bucket_device: ring
lookup, partition or cache probe, LRU generation update in batch order, bucketing.
Prints one JSON line.
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
    ap.add_argument("--cache-max", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--profile-steps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    G = args.grains
    keys_all = np.zeros((G, 3), dtype=np.uint64)
    keys_all[:, 1] = np.arange(G, dtype=np.uint64)
    keys_all[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0)
    e.ring_set_silos("D", SILOS)
    owner = e.ring_owner(keys_all)
    mine = np.nonzero(owner == 0)[0]
    remote = np.nonzero(owner != 0)[0]
    e.register(keys_all[mine], mine.astype(np.uint32), owner[mine])
    e.cache_configure(args.cache_max, [0], 8)
    fill = remote[: args.cache_max]
    e.cache_add(keys_all[fill], fill.astype(np.uint32), owner[fill], np.zeros(len(fill), np.int32))
    rng = np.random.default_rng(0x5EED0001)
    ks = rng.integers(0, G, size=args.msgs, dtype=np.int64)
    kk = np.zeros((args.msgs, 3), dtype=np.uint64)
    kk[:, 1] = ks.astype(np.uint64)
    kk[:, 2] = np.uint64(tcd)
    keys = torch.from_numpy(kk.view(np.int64)).to(dev)
    n = args.msgs
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    silo = torch.empty(n, dtype=torch.int32, device=dev)
    act = torch.empty(n, dtype=torch.int32, device=dev)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    off = torch.empty(G + 2, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)

    def step():
        e.route_bucket_device(keys.data_ptr(), n, G, silo.data_ptr(), act.data_ptr(), st.data_ptr(),
                              perm.data_ptr(), off.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ok = int((st == 0).sum().item())
    stats = e.cache_stats()
    kernels = {}
    if args.profile_steps:
        e.set_kernel_timing(True)
        e.kernel_times_reset()
        for _ in range(args.profile_steps):
            step()
        torch.cuda.synchronize()
        for name, (launches, ms) in e.kernel_times().items():
            kernels[name] = {"launches_per_step": launches // args.profile_steps,
                             "ms_per_step": round(ms / args.profile_steps, 4)}
        e.set_kernel_timing(False)
    kr = kernels.get("k_route_cached", {}).get("ms_per_step")
    line = {
        "metric": "routed messages/sec (LocalLookup: partition or LRU cache + bucket, one silo of 8)",
        "value": round(n * args.steps / wall, 1), "unit": "messages/s", "n_gpus": 1,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "steps": args.steps,
        "config": {"workload": f"cfg2 messages; silo 0 owns {len(mine)} grains, cache holds {len(fill)} "
                               f"(max {args.cache_max})"},
        "routed_ok_last_step": ok, "cache": stats,
        "k_route_cached_GBps": round(n * (24 + 64 + 9) / (kr * 1e-3) / 1e9, 1) if kr else None,
        "kernels": kernels,
    }
    print(json.dumps(line), flush=True)
    e.close()


if __name__ == "__main__":
    main()
