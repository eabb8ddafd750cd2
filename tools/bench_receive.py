#!/usr/bin/env python3
"""Silo receive path on one MI355X: IncomingMessageAgent.ReceiveMessage for a batch.

A silo hosting --acts activations (ActivationDirectory entries, 2% of them not Valid, 10% stateless
workers) plus 64 system targets receives --msgs messages from its peers: TargetActivation uniform
over the activations (1% unknown activation ids, 1% system-target messages), Direction 70% Request,
20% Response, 10% OneWay, per-activation request counts at the batch start uniform in [0, 4) and
the hard limits (5, 3) on, so CheckOverloaded rejects messages too.  Step = one batch through
gd_receive_device (FindTarget / FindSystemTarget, Valid check, null-context fallback, overload
rejections, stable per-context bucketing), inputs resident in HBM.  Prints one JSON line.
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

PEAK_HBM_GBS = 8000.0
CAT_GRAIN, CAT_SYSTEM_TARGET = 3, 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1 << 24)
    ap.add_argument("--acts", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--no-limits", action="store_true", help="hard limits off (the reference's default options)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    A, N, S = args.acts, args.msgs, 64
    rng = np.random.default_rng(0x5EED00A1)
    ids = np.zeros((A + S, 3), np.uint64)
    ids[:, 0] = rng.integers(0, 1 << 63, size=A + S, dtype=np.int64).astype(np.uint64)
    ids[:, 1] = rng.integers(0, 1 << 63, size=A + S, dtype=np.int64).astype(np.uint64)
    flags = np.where(rng.random(A) < 0.98, g.ACTDIR_VALID, 0) | \
        np.where(rng.random(A) < 0.10, g.ACTDIR_STATELESS_WORKER, 0)
    flags = np.concatenate([flags, np.full(S, g.ACTDIR_VALID | g.ACTDIR_SYSTEM_TARGET)]).astype(np.uint8)
    n_ctx = A + S
    e = g.GrainDispatch(device=0, table_capacity=1 << 12, my_silo=0)
    added = e.actdir_add(ids, np.arange(n_ctx, dtype=np.uint32), flags)
    assert added.all()

    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd_grain = (CAT_GRAIN << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    tcd_st = (CAT_SYSTEM_TARGET << 56) + 12
    gen = torch.Generator(device=dev).manual_seed(0x5EED00A2)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    which = torch.randint(0, A, (N,), device=dev, generator=gen)
    sys_msg = torch.rand(N, device=dev, generator=gen) < 0.01
    which = torch.where(sys_msg, A + torch.randint(0, S, (N,), device=dev, generator=gen), which)
    ta = d_ids[which].contiguous()
    unknown = torch.rand(N, device=dev, generator=gen) < 0.01
    ta[unknown, 0] ^= 0x5A5A5A5A
    tg = torch.zeros((N, 3), dtype=torch.int64, device=dev)
    tg[:, 1] = which
    tg[:, 2] = torch.where(sys_msg, torch.tensor(tcd_st, device=dev),
                           torch.tensor(tcd_grain - (1 << 64) if tcd_grain >= 1 << 63 else tcd_grain, device=dev))
    u = torch.rand(N, device=dev, generator=gen)
    direction = torch.where(u < 0.7, 0, torch.where(u < 0.9, 1, 2)).to(torch.uint8)
    rc = torch.randint(0, 4, (n_ctx,), device=dev, generator=gen).to(torch.int32)

    ctx = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    off = torch.empty(n_ctx + 3, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)
    torch.cuda.synchronize()

    def step():
        e.receive_device(tg.data_ptr(), ta.data_ptr(), direction.data_ptr(), N, n_ctx, ctx.data_ptr(),
                         st.data_ptr(), perm.data_ptr(), off.data_ptr(), None if args.no_limits else rc.data_ptr(),
                         5, 3)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    counts = torch.bincount(st.to(torch.int64), minlength=7).tolist()
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
    kr = kernels.get("k_receive", {}).get("ms_per_step")
    # k_receive per message: TargetGrain's TypeCodeData (8 B), TargetActivation (24 B), Direction (1),
    # one 32-B slot probe, ctx (4) + status (1) out = 70 B
    line = {
        "metric": "received messages/sec (ReceiveMessage: FindTarget + overload check + per-context bucket)",
        "value": round(N * args.steps / wall, 1), "unit": "messages/s", "n_gpus": 1,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "steps": args.steps, "data": "synthetic",
        "config": {"workload": f"{N} messages to {A} activations + {S} system targets, "
                               + ("no hard limits" if args.no_limits else "hard limits (5, 3)")},
        "status_counts": {"activation": counts[0], "system_target": counts[1], "null_context": counts[2],
                          "reject_unknown": counts[3], "reject_overloaded": counts[4], "dropped": counts[5]},
        "k_receive": {"alg_bytes_per_msg": 70,
                      "GBps": round(N * 70 / (kr * 1e-3) / 1e9, 1) if kr else None,
                      "frac_hbm": round(N * 70 / (kr * 1e-3) / 1e9 / PEAK_HBM_GBS, 4) if kr else None},
        "kernels": kernels,
    }
    print(json.dumps(line), flush=True)
    e.close()


if __name__ == "__main__":
    main()
