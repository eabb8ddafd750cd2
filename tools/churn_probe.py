#!/usr/bin/env python3
"""Where a churn step's time goes: cfg 2's batch routed + bucketed (a) on the static
directory, (b) on a directory with 1 % of its grains removed once (the misses' unrouted bucket), (c) under
churn (1 % unregistered + 1 % registered a step, enqueued), (d) the directory batches alone.  Per-kernel
times from the library's HIP events (gd_set_kernel_timing) over a few extra steps of each.  One JSON line.
  python tools/churn_probe.py [--cfg3]   (--cfg3: 64M Zipf(1.1) messages over 100M grains, a 2^28-slot table)"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g                      # noqa: E402
from orleans_amd.workloads import grain_keys_torch, zipf_keys_torch   # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]


def main():
    cfg3 = "--cfg3" in sys.argv[1:]
    G, N = (100_000_000, 1 << 26) if cfg3 else (1 << 20, 1 << 24)
    cap = 1 << 28 if cfg3 else 2 * G
    dev = torch.device("cuda:0")
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    e = g.GrainDispatch(device=0, table_capacity=cap, my_silo=0, kernel_timing=False)
    e.tune_set("probe_keys", 3)
    e.tune_set("bucket", 1)
    e.tune_set("probe_n1", 3)
    e.ring_set_silos("D", SILOS)
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)
    B = G // 100
    perm = torch.randperm(G, generator=torch.Generator(device=dev).manual_seed(7), device=dev)
    with torch.cuda.stream(stream):
        chunk = 1 << 25
        for c0 in range(0, G, chunk):
            c1 = min(G, c0 + chunk)
            ck = grain_keys_torch(tcd, torch.arange(c0, c1, device=dev), dev)
            own = torch.empty(c1 - c0, dtype=torch.int32, device=dev)
            e.ring_owner_device(ck.data_ptr(), c1 - c0, own.data_ptr())
            vals = torch.stack([torch.arange(c0, c1, device=dev, dtype=torch.int32), own], 1).contiguous()
            e.register_device(ck.data_ptr(), vals.data_ptr(), c1 - c0)
            del ck, own, vals
        if cfg3:
            keys = zipf_keys_torch(tcd, G, N, 0x5EED0003, dev)
        else:
            ks = torch.from_numpy(np.random.default_rng(0x5EED0001).integers(0, G, size=N)).to(dev)
            keys = grain_keys_torch(tcd, ks, dev)
        K, A, V = [], [], []
        for i in range(40):
            a = perm[i * B:(i + 1) * B]
            k = grain_keys_torch(tcd, a, dev)
            own = torch.empty(B, dtype=torch.int32, device=dev)
            e.ring_owner_device(k.data_ptr(), B, own.data_ptr())
            K.append(k)
            A.append(a.to(torch.int32).contiguous())
            V.append(torch.stack([a.to(torch.int32), own], 1).contiguous())
        # two output sets, alternating: with the bucket stream a batch's bucketing still reads its act
        # while the next batch's route writes
        outs = [[torch.empty(N, dtype=torch.int32, device=dev), torch.empty(N, dtype=torch.int32, device=dev),
                 torch.empty(N, dtype=torch.uint8, device=dev), torch.empty(N, dtype=torch.int32, device=dev),
                 torch.empty(G + 2, dtype=torch.int32, device=dev)] for _ in range(2)]
    torch.cuda.synchronize()
    nb = [0]

    def rb():
        silo, act, st, pm, off = outs[nb[0] & 1]
        nb[0] += 1
        e.route_bucket_device(keys.data_ptr(), N, G, silo.data_ptr(), act.data_ptr(), st.data_ptr(), pm.data_ptr(),
                              off.data_ptr())

    def timed(fn, steps=40, warm=5):
        for s in range(warm):
            fn(s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(warm, warm + steps):
            fn(s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        torch.cuda.synchronize()
        e.set_kernel_timing(1)
        e.kernel_times_reset()
        for s in range(warm + steps, warm + steps + 3):
            fn(s)
        torch.cuda.synchronize()
        kt = {k: round(v[1] / 3, 4) for k, v in e.kernel_times().items()}
        e.set_kernel_timing(False)
        return {"ms_per_step": round(ms, 4), "kernels_ms_per_step": kt}

    out = {}
    with torch.cuda.stream(stream):
        out["static"] = timed(lambda s: rb())
        e.unregister_device(K[39].data_ptr(), A[39].data_ptr(), B)
        out["static_1pct_missing"] = timed(lambda s: rb())
        e.register_device(K[39].data_ptr(), V[39].data_ptr(), B)

        def churn(s):
            i = s % 39
            e.unregister_device(K[i].data_ptr(), A[i].data_ptr(), B)
            if s:
                j = (s - 1) % 39
                e.register_device_async(K[j].data_ptr(), V[j].data_ptr(), B)
            rb()
        out["churn"] = timed(churn)
        e.register_device(K[(5 + 40 + 3 - 1) % 39].data_ptr(), V[(5 + 40 + 3 - 1) % 39].data_ptr(), B)

        def dir_only(s):
            i = s % 39
            e.unregister_device(K[i].data_ptr(), A[i].data_ptr(), B)
            e.register_device_async(K[i].data_ptr(), V[i].data_ptr(), B)
        out["directory_batches_only"] = timed(dir_only)
        # the same with each batch's bucketing on a second stream (gd_set_bucket_stream): the directory
        # batches (their own scratch, no fence on the bucket stream) overlap the previous bucketing
        bs = torch.cuda.Stream(dev)
        e.set_bucket_stream(bs.cuda_stream)

        def rb_p():
            rb()

        out["static_pipelined"] = timed(lambda s: rb_p())
        out["churn_pipelined"] = timed(churn)
        stream.wait_stream(bs)
        torch.cuda.synchronize()
        e.set_bucket_stream(None)
    e.synchronize()
    # one window's RemoveActivation then AddSingleActivation, synchronous: how many claim passes the
    # registration needed (each relaunch follows a non-zero deferred count)
    with torch.cuda.stream(stream):
        e.unregister_device(K[3].data_ptr(), A[3].data_ptr(), B)
        torch.cuda.synchronize()
        e.set_kernel_timing(1)
        e.kernel_times_reset()
        e.register_device(K[3].data_ptr(), V[3].data_ptr(), B)
        torch.cuda.synchronize()
        out["sync_register_kernels"] = {k: [v[0], round(v[1], 4)] for k, v in e.kernel_times().items() if v[0]}
        e.set_kernel_timing(False)
    out["index"] = e.index_stats()
    out["stats"] = e.stats()
    print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()
