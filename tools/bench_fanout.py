#!/usr/bin/env python3
"""BASELINE cfg 4: Chirper-style follower fan-out, 10M-grain power-law graph, 3-hop cascade.

One "step" = one whole cascade: `--hops` publish rounds from `--seeds` publishers, each round =
expand the frontier's follower lists (ChirperAccount.cs:131-134) -> route every NewChirp (ring
owner + directory probe) -> bucket per activation -> next frontier.  Value = messages routed
(all hops, all ranks) / max-over-ranks wall time of the cascade, graph and directory resident
in HBM.

  N = 1  fused expand+route kernel (k_fan_route) per hop.
  N > 1  directory sharded by ring owner; (target, sender) pairs exchanged with one
         all-to-all-v per hop (orleans_amd.fanout.ShardedFanout over RCCL).

Prints one JSON line on rank 0.  Launch N > 1 as bench.py is launched
(torch.distributed.run --nproc-per-node N ... tools/bench_fanout.py --gpus N).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from orleans_amd import graindispatch as g                                       # noqa: E402
from orleans_amd.fanout import (CHIRPER_ACCOUNT_CLASS, DeviceFanoutEngine, FanoutCascade,  # noqa: E402
                                ShardedFanout, upload_graph)
from orleans_amd.workloads import power_law_graph                                # noqa: E402

PEAK_HBM_GBS = 8000.0
SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in
         enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]   # bench.py "balanced"


def kernel_bytes(name, msgs, n_front, n_act, passes, keep_target, n_hops):
    """Algorithmic HBM bytes over all launches of a kernel."""
    if name == "k_fan_route":
        # dst read 4 + one slot 32 + sender/silo/act 12 + status 1 (+ target 4); per publisher 16
        return msgs * (49 + (4 if keep_target else 0)) + n_front * 16
    if name == "k_route_nodes":
        return msgs * (4 + 32 + 9)
    if name == "k_fan_expand":
        return msgs * (4 + 8) + n_front * 16
    if name == "k_radix_scatter":
        return msgs * (12 + 16 * (passes - 1))
    if name == "k_radix_hist":
        return msgs * 4 * passes
    if name == "k_bucket_starts":
        return msgs * 4 + n_hops * (n_act + 2) * 4
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--mean-deg", type=float, default=10.0)
    ap.add_argument("--max-deg", type=int, default=1 << 16)
    ap.add_argument("--seeds", type=int, default=1 << 16)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default="D", choices=["D", "R", "V"])
    ap.add_argument("--profile-steps", type=int, default=2)
    ap.add_argument("--no-target", action="store_true", help="do not write the target node per message")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearse-one-gpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo" if args.rehearse_one_gpu else "nccl",
                                **({} if args.rehearse_one_gpu else {"device_id": dev}))
    else:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29573")
        dist.init_process_group("gloo", rank=0, world_size=1)

    t_setup = time.perf_counter()
    n = args.nodes
    ro, dst = power_law_graph(n, args.mean_deg, seed=0x5EED0004, max_deg=args.max_deg)
    tc = g.calculate_id_hash(CHIRPER_ACCOUNT_CLASS)
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)

    # directory: node u = GrainId(tc, u), activation u, on its owner silo; this rank keeps the
    # grains whose owner silo it hosts
    keys = np.zeros((n, 3), dtype=np.uint64)
    keys[:, 1] = np.arange(n, dtype=np.uint64)
    keys[:, 2] = np.uint64(tcd)
    e = g.GrainDispatch(device=local, table_capacity=1 << int(np.ceil(np.log2(2 * n / world + 1))),
                        my_silo=rank % 8)
    pts, own = e.ring_set_silos(args.mode, SILOS)
    owner = e.ring_owner(keys)
    mine = np.nonzero(owner % world == rank)[0]
    e.register(keys[mine], mine.astype(np.uint32), owner[mine])
    del keys
    eng = DeviceFanoutEngine(e, dev, tc, keep_target=not args.no_target)
    graph = upload_graph(ro, dst, dev)
    seeds = np.random.default_rng(0x5EED0004).choice(n, size=args.seeds, replace=False).astype(np.uint32)
    t_seeds = torch.from_numpy(seeds.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    if world == 1:
        runner = FanoutCascade(eng, graph, n)
    else:
        runner = ShardedFanout(eng, graph, n, stage_via_cpu=args.rehearse_one_gpu)

    def step():
        return runner.run(t_seeds, args.hops)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    msgs_local = 0
    for _ in range(args.steps):
        hops = step()
        msgs_local += sum(h.messages for h in hops)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall, msgs_local], dtype=torch.float64)
    tw = t.clone()
    dist.all_reduce(tw, op=dist.ReduceOp.MAX)
    ts = t.clone()
    dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    wall_max, msgs_total = float(tw[0]), float(ts[1])
    hop_msgs = [h.messages for h in hops]
    hop_front = [int(h.frontier.shape[0]) for h in hops]

    kernels, roofline = {}, None
    if args.profile_steps > 0:
        e.set_kernel_timing(True)
        e.kernel_times_reset()
        for _ in range(args.profile_steps):
            step()
        torch.cuda.synchronize()
        kt = e.kernel_times()
        e.set_kernel_timing(False)
        passes = (max(1, n.bit_length()) + 7) // 8
        msgs_step = sum(hop_msgs)
        for name, (launches, ms) in kt.items():
            if not launches:
                continue
            per = ms / args.profile_steps
            b = kernel_bytes(name, msgs_step, sum(hop_front), n, passes, not args.no_target, len(hops))
            gbs = b / (per * 1e-3) / 1e9 if b and per > 0 else None
            kernels[name] = {"launches_per_step": launches // args.profile_steps, "ms_per_step": round(per, 4),
                             "alg_GBps": round(gbs, 1) if gbs else None,
                             "frac_hbm": round(gbs / PEAK_HBM_GBS, 4) if gbs else None}
        dom = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
        d = kernels[dom]
        roofline = {"bound": "hbm", "kernel": dom, "achieved": d["alg_GBps"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": d["frac_hbm"], "traffic": None,
                    "avg_launch_ms": round(d["ms_per_step"] / max(1, d["launches_per_step"]), 5)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, hops, tcd, ro, dst, owner, pts, own, n)

    if rank == 0:
        line = {
            "metric": "routed messages/sec (fan-out cascade: expand+lookup+bucket, whole node)",
            "value": round(msgs_total / wall_max, 1), "unit": "messages/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u32/u64 integer",
            "data": f"synthetic power-law follower graph (alpha 2.5, mean {args.mean_deg}, cap {args.max_deg}), "
                    f"seed 0x5EED0004",
            "config": {"workload": f"cfg4: {n} grains, {int(ro[-1])} follower edges, {args.seeds} seeds, "
                                   f"{args.hops} hops", "ring_mode": args.mode,
                       "parallelism": f"shard{world}" + ("-rehearsal" if args.rehearse_one_gpu else "")},
            "messages_per_step": int(msgs_total / args.steps), "hop_messages_rank0": hop_msgs,
            "hop_publishers_rank0": hop_front, "setup_s": round(setup_s, 1),
            "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    e.close()
    dist.destroy_process_group()


def cpu_baseline(args, hops, tcd, ro, dst, owner, pts, own, n):
    """C restatement (oracle/cpu_ref.c, faithful mode, 1 thread) routing + bucketing a bounded
    sample of the cascade's last hop; the expansion itself is a numpy gather (not timed)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref  # test-infrastructure checker, timed here as the CPU baseline only
    last = hops[-1]
    t = last.target.cpu().numpy().view(np.uint32)
    sample = min(t.size, 1 << 21)
    keys = np.zeros((sample, 3), dtype=np.uint64)
    keys[:, 1] = t[:sample]
    keys[:, 2] = np.uint64(tcd)
    all_keys = np.zeros((n, 3), dtype=np.uint64)
    all_keys[:, 1] = np.arange(n, dtype=np.uint64)
    all_keys[:, 2] = np.uint64(tcd)
    d = cpu_ref.CpuDirectory(True, n)
    d.register(all_keys, np.arange(n, dtype=np.uint32), owner)
    done, t0 = 0, time.perf_counter()
    while True:
        st, silo, act = d.route(args.mode, pts, own, keys, nthreads=1)
        cpu_ref.bucket(act, n, faithful=True, nthreads=1)
        done += sample
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    v = done / (time.perf_counter() - t0)
    return {"value": round(v, 1), "unit": "messages/s", "cores": 1, "kind": "port",
            "sample": f"{done} NewChirp messages ({sample}-message prefix of the last hop, repeated) through the C "
                      f"restatement in faithful mode (linear ring scan, chained map, per-activation FIFO)"}


if __name__ == "__main__":
    main()
