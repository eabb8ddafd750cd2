#!/usr/bin/env python3
"""A/B: serial route -> bucket per batch vs a 2-deep pipeline where batch k+1's route (latency-
bound random probes) runs on one stream while batch k's bucketing (LDS/issue-bound) runs on
another.  Same handle; route outputs double-buffered; checks the pipelined results equal the
serial ones.  cfg2 workload.

usage: python tools/ab_pipeline.py [--batches 40] [--rounds 3]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g  # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    N, G = 1 << 24, 1 << 20
    dev = torch.device("cuda:0")
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + (tc & 0x00FFFFFFFFFFFFFF)
    allk = np.zeros((G, 3), dtype=np.uint64)
    allk[:, 1] = np.arange(G, dtype=np.uint64)
    allk[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=0, table_capacity=2 * G)
    e.ring_set_silos("D", SILOS)
    e.register(allk, np.arange(G, dtype=np.uint32), e.ring_owner(allk))
    rng = np.random.default_rng(0x5EED0001)
    keys = [torch.from_numpy(allk[rng.integers(0, G, size=N)].view(np.int64)).to(dev) for _ in range(2)]
    mk = lambda dt, n=N: [torch.empty(n, dtype=dt, device=dev) for _ in range(2)]
    silo, act, perm = mk(torch.int32), mk(torch.int32), mk(torch.int32)
    st = mk(torch.uint8)
    offs = mk(torch.int32, G + 2)
    s_r, s_b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    r_done = [torch.cuda.Event() for _ in range(2)]
    b_done = [torch.cuda.Event() for _ in range(2)]

    def route(b):
        e.route_device(keys[b].data_ptr(), N, silo[b].data_ptr(), act[b].data_ptr(), st[b].data_ptr())

    def bucket(b):
        e.bucket_device(act[b].data_ptr(), N, G, perm[b].data_ptr(), offs[b].data_ptr())

    def serial(k):
        e.set_stream(s_r.cuda_stream)
        for i in range(k):
            route(i % 2)
            bucket(i % 2)

    def pipelined(k):
        for i in range(k):
            b = i % 2
            e.set_stream(s_r.cuda_stream)
            s_r.wait_event(b_done[b])          # buffers of batch i-2 consumed
            route(b)
            r_done[b].record(s_r)
            e.set_stream(s_b.cuda_stream)
            s_b.wait_event(r_done[b])
            bucket(b)
            b_done[b].record(s_b)

    res = {"serial": [], "pipelined": []}
    for _ in range(args.rounds):
        for name, fn in (("serial", serial), ("pipelined", pipelined)):
            fn(4)
            torch.cuda.synchronize()
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(torch.cuda.current_stream())
            s_r.wait_stream(torch.cuda.current_stream())
            s_b.wait_stream(torch.cuda.current_stream())
            fn(args.batches)
            torch.cuda.current_stream().wait_stream(s_r)
            torch.cuda.current_stream().wait_stream(s_b)
            z.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(z) / args.batches)
    # results of the last pipelined batches equal a serial run of the same batch
    torch.cuda.synchronize()
    got = [perm[b].cpu().numpy().copy() for b in range(2)]
    e.set_stream(None)
    want = [e.route_bucket(keys[b].cpu().numpy().view(np.uint64), G)[3] for b in range(2)]
    ok = all(np.array_equal(got[b].view(np.uint32), want[b]) for b in range(2))
    for k, v in res.items():
        print(f"{k:10s} ms/batch {np.median(v):.4f}  -> {N / np.median(v) / 1e6:.2f} G msgs/s   ({v})")
    print("pipelined results identical:", ok)
    e.close()


if __name__ == "__main__":
    main()
