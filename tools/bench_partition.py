#!/usr/bin/env python3
"""Exchange partition (SURVEY 8 a14 / e) on one MI355X: gd_pack_by_shard_device over a resident
batch of 16M cfg 2 keys, for 1, 2, 4 and 8 destination ranks, with the LDS-light gather kernel
(k_shard_gather, default) and the staged-key kernel (GD_SHARD_GATHER=0).  Per-kernel times from
the library's HIP events; one JSON line per (variant, shards)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g   # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]   # bench.py "balanced"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1 << 24)
    ap.add_argument("--grains", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    ks = np.random.default_rng(0x5EED0001).integers(0, args.grains, size=args.msgs, dtype=np.int64)
    keys = np.zeros((args.msgs, 3), np.uint64)
    keys[:, 1] = ks.view(np.uint64)
    keys[:, 2] = np.uint64(tcd)
    d_keys = torch.from_numpy(keys.view(np.int64)).to(dev)
    n = args.msgs
    out_k = torch.empty_like(d_keys)
    out_i = torch.empty(n, dtype=torch.int32, device=dev)
    ref = {}
    for variant, env in (("gather", "1"), ("staged", "0")):
        os.environ["GD_SHARD_GATHER"] = env
        e = g.GrainDispatch(device=0, table_capacity=1 << 12, my_silo=0)
        e.ring_set_silos("D", SILOS)
        s = torch.cuda.Stream(dev)
        e.set_stream(s.cuda_stream)
        for shards in (1, 2, 4, 8):
            counts = torch.empty(shards, dtype=torch.int32, device=dev)

            def once():
                e.pack_by_shard_device(d_keys.data_ptr(), n, shards, out_k.data_ptr(), out_i.data_ptr(),
                                       counts.data_ptr())
            once()
            torch.cuda.synchronize()
            e.set_kernel_timing(True)
            e.kernel_times_reset()
            for _ in range(args.reps):
                once()
            torch.cuda.synchronize()
            kt = {k: round(ms / args.reps * 1e3, 2) for k, (c, ms) in e.kernel_times().items() if c}
            e.set_kernel_timing(False)
            digest = (int(out_i[::4099].to(torch.int64).sum().item()), int(out_k[::8191].sum().item()),
                      counts.tolist())
            if shards in ref:
                same = ref[shards] == digest
            else:
                ref[shards], same = digest, True
            print(json.dumps({"variant": variant, "shards": shards, "msgs": n, "us_per_kernel": kt,
                              "same_output_as_gather": same}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
