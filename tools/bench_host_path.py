#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer entry point (gd_route_bucket) on the cfg-2 workload.

The C# host hands the library pinned managed arrays: keys in (24 B a message),
silo / act / status / perm / offsets out (17 B a message + the offsets).  This times that whole
call -- H2D copy, route, bucketing, D2H copies, synchronisation -- with the buffers in pinned
host memory (what `fixed` + a registered array gives) and, for comparison, pageable memory.
It is not the bench value (bench.py times the device entry with inputs resident in HBM).
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


def grain_keys(tcd: int, ks: np.ndarray) -> np.ndarray:
    out = np.zeros((len(ks), 3), dtype=np.uint64)
    out[:, 1] = ks.astype(np.int64).view(np.uint64)
    out[:, 2] = np.uint64(tcd)
    return out


def pinned(shape, dtype):
    t = torch.empty(int(np.prod(shape)) * np.dtype(dtype).itemsize, dtype=torch.uint8, pin_memory=True)
    return t, t.numpy().view(dtype).reshape(shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1 << 24)
    ap.add_argument("--grains", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--label", default="")
    args = ap.parse_args()
    torch.cuda.init()
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    G, n = args.grains, args.msgs
    e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0)
    e.ring_set_silos("D", SILOS)
    gk = grain_keys(tcd, np.arange(G))
    e.register(gk, np.arange(G, dtype=np.uint32), e.ring_owner(gk))
    rng = np.random.default_rng(0x5EED0001)
    ks = rng.integers(0, G, size=n, dtype=np.int64)
    out = {"metric": "routed messages/sec, host buffers (PCIe-inclusive gd_route_bucket)", "unit": "messages/s",
           "msgs": n, "grains": G, "label": args.label, "GD_HOST_CHUNK": os.environ.get("GD_HOST_CHUNK", "default")}
    for kind in ("pinned", "pageable"):
        hold = []
        if kind == "pinned":
            for shape, dt in (((n, 3), np.uint64), ((n,), np.uint32), ((n,), np.uint32), ((n,), np.uint8),
                              ((n,), np.uint32), ((G + 2,), np.uint32)):
                t, a = pinned(shape, dt)
                hold.append(t)
                hold.append(a)
            keys, silo, act, st, perm, off = hold[1::2]
        else:
            keys = np.empty((n, 3), np.uint64)
            silo, act, perm = (np.empty(n, np.uint32) for _ in range(3))
            st = np.empty(n, np.uint8)
            off = np.empty(G + 2, np.uint32)
        keys[:] = grain_keys(tcd, ks)
        ptr = lambda a: a.ctypes.data

        def step():
            e._c(g.lib.gd_route_bucket(e.h, ptr(keys), n, G, ptr(silo), ptr(act), ptr(st), ptr(perm), ptr(off)))

        def route_only():
            e._c(g.lib.gd_route(e.h, ptr(keys), n, ptr(silo), ptr(act), ptr(st)))

        def timed(fn):
            for _ in range(args.warmup):
                fn()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                fn()
            return (time.perf_counter() - t0) / args.steps

        dt = timed(step)
        assert int((st == 0).sum()) == n
        dr = timed(route_only)
        out[kind] = {"value": n / dt, "ms_per_call": dt * 1e3, "pcie_GBps": n * (24 + 17) / dt / 1e9,
                     "route_only": {"value": n / dr, "ms_per_call": dr * 1e3, "pcie_GBps": n * (24 + 9) / dr / 1e9}}
    out["value"] = out["pinned"]["value"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
