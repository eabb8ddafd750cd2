#!/usr/bin/env python3
"""cfg 5 micro-batch latency, graph replay against eager launches.  Builds cfg 2's
directory (2^20 grains), then times `--runs` 4,096-message micro-batches each way and prints p50 / p99 per
mode.  Under `rocprofv3 --kernel-trace` the kernels of both modes are traced (the replays first); the
trace's per-run spans say where a replay's extra microseconds go (launch vs. kernel time).
  python tools/mb_trace.py [--runs N] [--json OUT]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g                      # noqa: E402
from orleans_amd.workloads import grain_keys_torch              # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=2000)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    G, B = 1 << 20, 4096
    dev = torch.device("cuda:0")
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0, kernel_timing=False)
    e.ring_set_silos("D", SILOS)
    keys = grain_keys_torch(tcd, torch.arange(G, device=dev), dev)
    own = torch.empty(G, dtype=torch.int32, device=dev)
    e.ring_owner_device(keys.data_ptr(), G, own.data_ptr())
    vals = torch.stack([torch.arange(G, device=dev, dtype=torch.int32), own], 1).contiguous()
    e.register_device(keys.data_ptr(), vals.data_ptr(), G)
    # one large route so the probe index is built (the micro-batches read it when it is current)
    big = grain_keys_torch(tcd, torch.randint(0, G, (1 << 20,), device=dev), dev)
    o = [torch.empty(1 << 20, dtype=torch.int32, device=dev) for _ in range(2)] + [torch.empty(1 << 20, dtype=torch.uint8, device=dev)]
    e.route_device(big.data_ptr(), 1 << 20, o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr())
    torch.cuda.synchronize()
    rng = np.random.default_rng(0x5EED0005)
    kk = np.zeros((64, B, 3), np.uint64)
    kk[:, :, 1] = rng.integers(0, G, size=(64, B))
    kk[:, :, 2] = np.uint64(tcd)
    out = {"index": e.index_stats()}
    for poll in (1, 0):                        # GD_OPT_MB_POLL: completion by the sort's pinned count, or not
        e.set_option("mb_poll", poll)
        mb = g.MicroBatch(e, B, G)
        ref = None
        for use_graph in (True, False):
            for i in range(50):
                mb.keys[:] = kk[i % 64]
                mb.run(B, use_graph)
            lat = np.empty(args.runs)
            for i in range(args.runs):
                mb.keys[:] = kk[i % 64]
                t0 = time.perf_counter()
                mb.run(B, use_graph)
                lat[i] = (time.perf_counter() - t0) * 1e6
            # the last run's outputs, read right after the run returned
            got = (mb.perm[:B].copy(), mb.status[:B].copy())
            ref = ref or got
            assert all((a == b).all() for a, b in zip(got, ref))
            out[f"{'graph' if use_graph else 'eager'}_poll{poll}"] = {
                "p50": round(float(np.percentile(lat, 50)), 2), "p99": round(float(np.percentile(lat, 99)), 2)}
        mb.close()
    e.close()
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
