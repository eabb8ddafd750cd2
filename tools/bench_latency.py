#!/usr/bin/env python3
"""BASELINE config 5: micro-batch latency of the fused route+bucket.

4,096-message batches of the cfg2 distribution (uniform over 2^20 registered grains,
8 silos, ring D), each batch = keys in pinned host memory -> k_mb_route (reads them in
place) -> k_mb_sort_runs -> results written straight to pinned host memory (zero-copy;
GD_OPT_MB_ZEROCOPY 0 for the staged H2D / D2H form), replayed as one hipGraph
(gd_microbatch_run(..., use_graph=1)) or launched eagerly.  Reports p50/p99/max wall
latency per batch over --batches batches, and checks a sample of graph replays bit-exact
against the library's gd_route_bucket.  bench.py reports the same measurement with the CPU
restatement's p50/p99 beside it (secondary.cfg5_latency_us, cpu_baseline.cfg5_latency_us).

usage: python tools/bench_latency.py [--batches 10000] [--size 4096]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g  # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=10000)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--grains", type=int, default=1 << 20)
    ap.add_argument("--check", type=int, default=20, help="graph replays checked against gd_route_bucket")
    args = ap.parse_args()
    G, B = args.grains, args.size
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + (tc & 0x00FFFFFFFFFFFFFF)
    allk = np.zeros((G, 3), dtype=np.uint64)
    allk[:, 1] = np.arange(G, dtype=np.uint64)
    allk[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=0, table_capacity=2 * G)
    e.ring_set_silos("D", SILOS)
    owner = e.ring_owner(allk)
    e.register(allk, np.arange(G, dtype=np.uint32), owner)
    mb = g.MicroBatch(e, B, G)
    rng = np.random.default_rng(0x5EED0005)
    pool = allk[rng.integers(0, G, size=(64, B))]           # 64 distinct batches, cycled
    res = {}
    for use_graph in (True, False):
        lat = np.empty(args.batches)
        for w in range(50):                                 # warmup (captures the graph)
            mb.keys[:] = pool[w % 64]
            mb.run(B, use_graph)
        for i in range(args.batches):
            mb.keys[:] = pool[i % 64]
            t0 = time.perf_counter()
            mb.run(B, use_graph)
            lat[i] = time.perf_counter() - t0
        us = lat * 1e6
        res["graph" if use_graph else "eager"] = {
            "p50_us": round(float(np.percentile(us, 50)), 1), "p99_us": round(float(np.percentile(us, 99)), 1),
            "max_us": round(float(us.max()), 1), "mean_us": round(float(us.mean()), 1),
            "msgs_per_s": round(B / lat.mean(), 1)}
    # consistency on a sample: the graph replay must equal the library's own fused call on the
    # same keys (oracle parity of that path is tests/test_gpu_parity.py::test_microbatch_*)
    for i in range(args.check):
        mb.keys[:] = pool[i % 64]
        mb.run(B, True)
        st, silo, act, perm, off = e.route_bucket(pool[i % 64], G)
        assert np.array_equal(mb.status, st) and np.array_equal(mb.silo, silo) and np.array_equal(mb.act, act)
        assert np.array_equal(mb.perm, perm) and np.array_equal(mb.offsets(), off)
    out = {"metric": "micro-batch route+bucket latency (cfg5)", "batch": B, "batches": args.batches,
           "grains": G, "consistency_checked_batches": args.check, **res}
    print(json.dumps(out), flush=True)
    mb.close()
    e.close()


if __name__ == "__main__":
    main()
