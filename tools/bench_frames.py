#!/usr/bin/env python3
"""SURVEY 8 f1 bench: decode -> route -> bucket straight from a device receive buffer.

Workload: --frames request frames (tools/frames_synth.py layout, 170 B each with the default
40-B body) whose TargetGrain is drawn uniformly from --grains registered grains (cfg2
distribution: 8 silos, ring D).  Buffer and frame offsets are resident in HBM before timing.
Reports, per step, the whole pipeline (gd_route_frames_device with bucketing) and the
decode kernel alone, plus per-kernel averages from the library's HIP events.

Algorithmic bytes of k_decode_frames per frame: 8 (offset) + 8 + header_len (frame prefix and
header, read once) + 4 + 24 (flags + TargetGrain written) = 166 B at header_len 122.

usage: python tools/bench_frames.py [--frames 16777216] [--steps 10] [--warmup 3]
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
sys.path.insert(0, os.path.join(ROOT, "tools"))
from orleans_amd import graindispatch as g  # noqa: E402
import frames_synth as FS  # noqa: E402

SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]
PEAK_HBM = 8000.0  # GB/s, MI355X_MICROARCH.md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 24)
    ap.add_argument("--grains", type=int, default=1 << 20)
    ap.add_argument("--body", type=int, default=40)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    N, G = args.frames, args.grains
    dev = torch.device("cuda:0")
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + (tc & 0x00FFFFFFFFFFFFFF)
    allk = np.zeros((G, 3), dtype=np.uint64)
    allk[:, 1] = np.arange(G, dtype=np.uint64)
    allk[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=0, table_capacity=2 * G, kernel_timing=False)
    e.ring_set_silos("D", SILOS)
    e.register(allk, np.arange(G, dtype=np.uint32), e.ring_owner(allk))
    rng = np.random.default_rng(0x5EED0002)
    keys = allk[rng.integers(0, G, size=N)]
    t0 = time.time()
    buf, off, fl = FS.build_frames(keys, rng, body_len=args.body)
    build_s = time.time() - t0
    d_buf = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    del buf
    flags = torch.empty(N, dtype=torch.int32, device=dev)
    tg = torch.empty((N, 3), dtype=torch.int64, device=dev)
    silo = torch.empty(N, dtype=torch.int32, device=dev)
    act = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    offs = torch.empty(G + 2, dtype=torch.int32, device=dev)
    fields = {"flags": flags.data_ptr(), "target_grain": tg.data_ptr()}
    s = torch.cuda.Stream(device=dev)
    e.set_stream(s.cuda_stream)

    def pipeline():
        e.route_frames_device(d_buf.data_ptr(), d_buf.numel(), d_off.data_ptr(), N, G, fields, silo.data_ptr(),
                              act.data_ptr(), st.data_ptr(), perm.data_ptr(), offs.data_ptr())

    def decode():
        e.decode_frames_device(d_buf.data_ptr(), d_buf.numel(), d_off.data_ptr(), N, fields)

    res = {}
    with torch.cuda.stream(s):
        for name, fn in (("pipeline", pipeline), ("decode", decode)):
            for _ in range(args.warmup):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(args.steps):
                fn()
            b.record(s)
            torch.cuda.synchronize()
            res[name] = a.elapsed_time(b) / args.steps
        e.set_kernel_timing(True)
        e.kernel_times_reset()
        for _ in range(args.steps):
            pipeline()
        e.synchronize()
        kt = e.kernel_times()
        e.set_kernel_timing(False)
    assert (flags.cpu().numpy() == g.FRAME_HAS_TARGET).all()
    assert np.array_equal(tg.cpu().numpy().view(np.uint64), keys)
    ker = {k: round(ms / max(n, 1) * 1e3, 1) for k, (n, ms) in kt.items()}
    dec_us = ker.get("k_decode_frames", res["decode"] * 1e3)
    alg_b = 8 + 8 + FS.HEADER_LEN + 4 + 24
    out = {"metric": "frames decoded+routed+bucketed per second (f1)", "frames": N, "grains": G,
           "frame_bytes": fl, "steps": args.steps, "pipeline_ms": round(res["pipeline"], 4),
           "frames_per_s": round(N / (res["pipeline"] * 1e-3), 1), "decode_ms": round(res["decode"], 4),
           "decode_frames_per_s": round(N / (res["decode"] * 1e-3), 1),
           "kernel_us": ker, "decode_alg_bytes_per_frame": alg_b,
           "decode_achieved_GBps": round(alg_b * N / (dec_us * 1e-6) / 1e9, 1),
           "decode_frac_of_hbm_peak": round(alg_b * N / (dec_us * 1e-6) / 1e9 / PEAK_HBM, 3),
           "buffer_GBps": round(fl * N / (dec_us * 1e-6) / 1e9, 1), "host_build_s": round(build_s, 1)}
    print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()
