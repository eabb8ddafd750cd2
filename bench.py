#!/usr/bin/env python3
"""Routed messages/sec for the Orleans grain-dispatch hot path on MI355X.

One step = one batch of message headers through ring lookup + directory probe
+ per-activation bucketing (libgraindispatch, gfx950), inputs resident in HBM.

  N = 1  BASELINE.json config 2: 16,777,216 messages, uniform over 1,048,576
         grains (GrainId = Ping grain type code + long key), 8 silos
         10.0.0.{1..8}:11111@1, directory ring mode D (LocalGrainDirectory),
         table load 0.5, every grain registered with one activation on its owner.
  N > 1  weak scaling: the same 16M messages per GPU over 2^20 x N grains;
         silo s lives on GPU s % N; each GPU owns its silos' directory
         partition; a stable partition by owner + all-to-all-v (RCCL over xGMI)
         moves headers to their owner, which probes and buckets them.

Prints ONE JSON line on rank 0 (see DESIGN.md for the byte model behind the
roofline object).
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from orleans_amd import graindispatch as g          # noqa: E402
from orleans_amd.sharded import DeviceEngine, LibraryRouter, ShardedRouter, same_result  # noqa: E402
from orleans_amd.workloads import grain_keys_torch, zipf_keys_torch  # noqa: E402

PEAK_HBM_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# 8 silos 10.0.0.{1..8}:11111.  "literal" = generation 1; its ring gives
# one silo 35.7% of the directory.  "balanced" (default) = generations found by
# tools/balanced_silos.py so that every silo owns 1/8 of the hash space -- Orleans
# generations are arbitrary timestamps (SiloAddress.cs:72-76); routing is unchanged.
SILO_SETS = {
    "literal": [(f"10.0.0.{i + 1}", 11111, 1) for i in range(8)],
    "balanced": [(f"10.0.0.{i + 1}", 11111, g) for i, g in
                 enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])],
}
PING_GRAIN_CLASS = "BenchmarkGrains.Ping.PingGrain"


def grain_keys(type_code_data: int, ks: np.ndarray) -> np.ndarray:
    out = np.zeros((ks.shape[0], 3), dtype=np.uint64)
    out[:, 1] = ks.astype(np.int64).view(np.uint64)
    out[:, 2] = np.uint64(type_code_data)
    return out


def radix_layout(n: int, n_act: int):
    """(passes, digit bits, packed) of libgraindispatch's LSD bucketing for n messages over n_act
    activations (eng_core.hip bucket_lsd): <= 8-bit digits; records packed to 6 B between the passes
    when the key bits above the first digit fit a u16 and the message index fits a u32 beside the
    first digit."""
    key_bits = max(1, int(n_act).bit_length())
    passes = (key_bits + 7) // 8
    bits = max(4, -(-key_bits // passes))
    ib = max(1, int(max(n, 1) - 1).bit_length())
    packed = passes >= 2 and bits <= 8 and key_bits - bits <= 16 and ib + bits <= 32
    return passes, bits, packed


MSD_CAP, MSD_MID_CAP, CH_CAP, L2_SMALL = 24576, 8192, 8192, 1024     # gd_msd.h / gd_msd2.h


def bucket_form(names) -> str:
    """The bucketing form a step ran, from its kernel names: "msd3" (the three-pass two-level form,
    gd_msd2.h), "msd" (the one-pass two-level form, gd_msd.h) or "lsd" (the LSD radix passes)."""
    if "k_seg_scatter" in names:
        return "msd3"
    if "k_msd_local" in names:
        return "msd"
    return "lsd"


def l2_classes(acts: np.ndarray, n_act: int, t_small: int = L2_SMALL) -> dict:
    """The three-pass form's level-2 work (gd_msd2.h k_l2_classify) for one batch: per class, the
    messages and activations it owns; chunks and ranges of the hot class."""
    k = np.minimum(acts.astype(np.int64), n_act) >> 10
    R = (n_act >> 10) + 1
    S = np.bincount(k, minlength=R)
    per = np.full(R, 1024, np.int64)
    per[-1] = n_act + 1 - (R - 1) * 1024
    small, hot = S <= t_small, S > MSD_CAP
    mid = ~small & (S <= MSD_MID_CAP)
    staged = ~small & ~mid & ~hot
    return {"small": (int(S[small].sum()), int(per[small].sum())),
            "mid": (int(S[mid].sum()), int(per[mid].sum())),
            "staged": (int(S[staged].sum()), int(per[staged].sum())),
            "hot": (int(S[hot].sum()), int(per[hot].sum())), "chunks": int(((S[hot] + CH_CAP - 1) // CH_CAP).sum()),
            "hot_ranges": int(hot.sum()), "ranges": R}


def bucket_bytes(form: str, n: int, n_act: int, acts=None) -> dict:
    """Algorithmic HBM bytes of one bucketing of n messages over n_act activations, per kernel name
    (all its launches), for the form the library ran (DESIGN 5 byte tables).  Every form writes the
    permutation (4 B a message) and the n_act + 2 bucket starts (4 B each)."""
    off = (n_act + 2) * 4
    if form == "lsd":
        passes, _, packed = radix_layout(n, n_act)
        if passes == 1:
            sc = n * 8.0
        else:
            sc = n * (10 + 12 * (passes - 2) + 10) if packed else n * (12 + 16 * (passes - 2) + 12)
        # the first histogram fills the starts, the last scatter lowers them, one range scan reads and
        # writes them
        return {"k_radix_hist": (n * (4 + 2 * (passes - 1)) if packed else n * 4 * passes) + off,
                "k_radix_scatter": sc, "k_starts_rangescan": 2 * off}
    if form == "msd":
        # one MSD pass (activation read twice, 6-B record written), the in-LDS range sort (record read,
        # index written in order, every start written once)
        return {"k_radix_hist": n * 4.0, "k_radix_scatter": n * 10.0, "k_msd_local": n * 10.0 + off}
    # msd3: pass A (activation read twice, 8-B record written), pass B (key read for the histogram,
    # the record read, a 6-B record written; its [segment][digit][tile] counts flat-scanned), level 2
    # (record read, index written in order, starts written once, per class)
    kb = max(1, (n_act >> 10).bit_length())
    a = kb // 2
    tiles = -(-n // 8192) + (n_act >> (10 + a)) + 1
    cnt = (1 << a) * tiles * 4.0
    # pass A's records: 6 B (u16 + the index word's spare bits) when the index leaves room, else 8 B
    hb, ib = max(0, a + 10 - 16), max(1, int(max(n, 1) - 1).bit_length())
    rec = 6.0 if hb == 0 or ib + hb <= 32 else 8.0
    c = l2_classes(acts, n_act) if acts is not None else None
    out = {"k_radix_hist": n * 4.0, "k_radix_scatter": n * (4.0 + rec),
           "k_seg_hist": n * (2.0 if rec == 6.0 else 4.0) + cnt,
           "k_scan_reduce": cnt, "k_scan_down": 2 * cnt, "k_seg_scatter": n * (rec + 6.0) + cnt,
           "k_l2_classify": ((n_act >> 10) + 1) * 12.0}
    if c is None:
        out["k_l2_small"] = n * 10.0 + off      # unknown split: all charged to one kernel
        return out
    out.update({"k_l2_small": c["small"][0] * 10.0 + c["small"][1] * 4.0,
                "k_msd_local_mid": c["mid"][0] * 10.0 + c["mid"][1] * 4.0,
                "k_msd_local": c["staged"][0] * 10.0 + c["staged"][1] * 4.0,
                "k_l2_chunk_hist": c["hot"][0] * 2.0 + c["chunks"] * 4096.0,
                "k_l2_chunk_scan": c["chunks"] * 8192.0 + c["hot_ranges"] * 4096.0,
                "k_l2_chunk_scatter": c["hot"][0] * 10.0 + c["hot"][1] * 4.0 + c["chunks"] * 8192.0})
    if (n_act + 1) % 1024:
        out["k_l2_small"] += 8.0                # offsets[n_act + 1]
    return out


# The kernels of a bucketing stage (every form), for the stage total
BUCKET_KERNELS = ("k_radix_hist", "k_radix_rowscan", "k_radix_scatter", "k_msd_local", "k_msd_local_mid",
                  "k_starts_rangescan",
                  "k_scan_reduce", "k_scan_down", "k_fill", "k_seg_table", "k_seg_hist", "k_seg_scatter",
                  "k_l2_classify", "k_l2_small", "k_l2_chunk_hist", "k_l2_chunk_ptot", "k_l2_chunk_scan",
                  "k_l2_chunk_scatter")


def kernel_bytes(name: str, n: int, n_act: int, form: str = "lsd", acts=None) -> float:
    """Algorithmic HBM bytes of one step for a kernel (all launches of it), per DESIGN.md's byte
    tables: the route (key 24 + one 32-B directory slot + silo/act/status 9 B) and the
    bucketing form's kernels (bucket_bytes)."""
    if name == "k_route":
        return n * (24 + 32 + 4 + 4 + 1)
    return float(bucket_bytes(form, n, n_act, acts).get(name, 0.0))


def load_pmc(tag: str, kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary profiles/pmc_<tag>_<kernel>.json
    (tools/pmc_traffic.py), or None."""
    d = load_pmc_entry(tag, kernel)
    return d.get("hbm_bytes_per_launch") if d else None


def load_pmc_entry(tag: str, kernel: str):
    path = os.path.join(ROOT, "profiles", f"pmc_{tag}_{kernel}.json")
    if not tag or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def roofline_of(kt: dict, steps: int, n: int, n_act: int, acts, tag, world: int = 1, bytes_fn=None,
                nonstage=None):
    """(kernels, roofline) from in-library HIP-event kernel times kt {name: (launches, ms)} over `steps`
    steps of one workload: per kernel its algorithmic GB/s and fraction of HBM peak; the dominant
    kernel's roofline with its PMC traffic (profiles/pmc_*.json at this workload, N = 1) and the ratio
    of that traffic to the algorithmic bytes; the bucketing kernels (the MSD scatter and the level-2
    range sort, or the LSD scatter) on their implementation bytes -- `frac` -- with SURVEY 8(d)'s
    16 B/record/pass model beside them; and the whole bucketing stage against the 12-B contract.
    bytes_fn(name, form): a kernel's bytes a step when a step is not one batch (the cfg 4 cascade);
    nonstage: {name: bytes a step} of those launched outside the bucketing (cfg 4's degree scans)."""
    kt = dict(kt)
    stage_ev = kt.pop("stage:bucket", None)       # one event pair around each whole bucketing (timing 2)
    form = bucket_form(kt)
    kernels = {}
    for name, (launches, ms) in kt.items():
        if launches == 0:
            continue
        per_step_ms = ms / steps
        b = bytes_fn(name, form) if bytes_fn else kernel_bytes(name, n, n_act, form, acts)
        gbs = b / (per_step_ms * 1e-3) / 1e9 if b and per_step_ms > 0 else None
        kernels[name] = {"launches_per_step": launches // steps, "ms_per_step": round(per_step_ms, 4),
                         "alg_bytes_per_step": b or None, "alg_GBps": round(gbs, 1) if gbs else None,
                         "frac_hbm": round(gbs / PEAK_HBM_GBS, 4) if gbs else None}
    if not kernels:
        return kernels, None
    pmc_tag = tag if world == 1 else None
    # every kernel's committed PMC figures at this workload (N = 1): HBM bytes as the counters saw
    # them, their rate over this run's launch time, and the LDS bank-conflict ratio
    for name, d in kernels.items():
        p = load_pmc_entry(pmc_tag, name)
        if not p or d["ms_per_step"] <= 0:
            continue
        t = d["ms_per_step"] / max(1, d["launches_per_step"]) * 1e-3
        d["pmc_bytes_per_launch"] = round(p["hbm_bytes_per_launch"])
        d["frac_pmc"] = round(p["hbm_bytes_per_launch"] / t / 1e9 / PEAK_HBM_GBS, 4)
        if d["alg_bytes_per_step"]:
            d["traffic_ratio"] = round(p["hbm_bytes_per_launch"] * max(1, d["launches_per_step"])
                                       / d["alg_bytes_per_step"], 3)
        if p.get("lds_conflict_ratio") is not None:
            d["lds_conflict_ratio"] = p["lds_conflict_ratio"]

    def entry(name):
        d = kernels[name]
        launches = max(1, d["launches_per_step"])
        t = d["ms_per_step"] / launches * 1e-3
        alg = (d["alg_bytes_per_step"] or 0.0) / launches
        traffic = load_pmc(pmc_tag, name) if pmc_tag else None
        return {"kernel": name, "achieved": d["alg_GBps"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": d["frac_hbm"], "traffic": traffic, "alg_bytes_per_launch": alg,
                "traffic_ratio": round(traffic / alg, 3) if traffic and alg else None,
                "frac_pmc": round(traffic / t / 1e9 / PEAK_HBM_GBS, 4) if traffic and t > 0 else None,
                "avg_launch_ms": round(t * 1e3, 5), "launches_per_step": launches}

    dom = max((k for k in kernels if not k.startswith("rccl_")), key=lambda k: kernels[k]["ms_per_step"])
    roofline = dict(entry(dom), bound="hbm")
    if dom == "k_route":
        roofline["bytes_model"] = "SURVEY 8(d): key 24 + one 32-B directory slot + silo/act/status 9 B"
    bk = {}
    for name in ("k_radix_scatter", "k_msd_local", "k_msd_local_mid", "k_seg_scatter", "k_l2_small",
                 "k_l2_chunk_scatter"):
        if name in kernels and kernels[name]["alg_bytes_per_step"]:
            e = entry(name)
            launches = e["launches_per_step"]
            if name in ("k_radix_scatter", "k_seg_scatter"):
                # SURVEY 8(d)'s model: 16 B per record per radix pass, side field
                sm = 16.0 * n / max(1, kernels[name]["launches_per_step"])
                e["frac_survey_model"] = round(sm / (e["avg_launch_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
            bk[name] = e
    if bk:
        roofline["bucketing_kernel"] = dict(form=form, bytes_model="implementation bytes (DESIGN 5); frac_pmc on "
                                            "the PMC counters' bytes where profiles/ holds them", **bk)
    stage = [k for k in BUCKET_KERNELS if k in kernels]
    sum_ms = sum(kernels[k]["ms_per_step"] for k in stage)
    # the stage's time: events around the whole bucketing (no events between its kernels, which add
    # ~5 us a launch to the per-kernel sum), else the per-kernel sum
    st_ms = stage_ev[1] / steps if stage_ev and stage_ev[0] else sum_ms
    st_b = sum((kernels[k]["alg_bytes_per_step"] or 0.0) - (nonstage or {}).get(k, 0.0) for k in stage)
    roofline["bucketing_stage"] = {
        "form": form, "kernels": stage, "ms_per_step": round(st_ms, 4), "kernel_sum_ms_per_step": round(sum_ms, 4),
        "timing": "stage events (gd_set_kernel_timing 2)" if stage_ev and stage_ev[0] else "per-kernel events, summed",
        "impl_bytes_per_message": round(st_b / max(1, n), 2), "contract_bytes_per_message": 12,
        "frac_impl": round(st_b / (st_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4) if st_ms > 0 else None,
        "frac_contract": round(12.0 * n / (st_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4) if st_ms > 0 else None}
    return kernels, roofline


def zipf_keys(tcd: int, n_grains: int, n: int, seed: int, dev) -> torch.Tensor:
    """(n, 3) int64 keys on `dev`: grain k ~ Zipf(s=1.1) over ranks 0..n_grains-1 by inverse CDF
    (SURVEY 8 d cfg 3), sampled on the GPU (orleans_amd/workloads.py)."""
    return zipf_keys_torch(tcd, n_grains, n, seed, dev)


def setup_workload(args, workload, world, rank, local, dev, tcd, msgs, grains):
    """Directory + resident message batch + router for one workload on this rank.

    The directory is built in HBM: grain keys generated on the GPU, ring owner by
    gd_ring_owner_device, this rank's grains (owner silo % world == rank) registered with
    gd_dir_register_device (act = running index over this rank's grains, silo = owner)."""
    if workload == "cfg3":
        # BASELINE cfg 3 (SURVEY 8 d): 67,108,864 messages for the whole node, k ~ Zipf(1.1) over
        # 100,000,000 grains, directory sharded by mode-D owner
        G_total = grains * world if grains else 100_000_000
        N = msgs or (1 << 26) // world
        Gr = -(-G_total // world)
    else:
        N, Gr = msgs or 1 << 24, grains or 1 << 20
        G_total = Gr * world
    cap = 2 * Gr if workload == "cfg2" else 1 << int(np.ceil(np.log2(2 * Gr)))
    e = g.GrainDispatch(device=local, table_capacity=cap, my_silo=rank % 8, kernel_timing=False)
    pin_choices(e, args, workload)
    silos = SILO_SETS[args.silos]
    pts, own = e.ring_set_silos(args.mode, silos)
    engine = DeviceEngine(e, dev, pipeline=args.pipeline and world == 1)
    stream = engine.stream
    counts = torch.zeros(world, dtype=torch.int64, device=dev)
    n_act = 0
    chunk = 1 << 25
    with torch.cuda.stream(stream):
        for c0 in range(0, G_total, chunk):
            c1 = min(G_total, c0 + chunk)
            rk = grain_keys_torch(tcd, torch.arange(c0, c1, device=dev), dev)
            owner = torch.empty(c1 - c0, dtype=torch.int32, device=dev)
            e.ring_owner_device(rk.data_ptr(), c1 - c0, owner.data_ptr())
            sel = (owner % world) == rank
            counts += torch.bincount((owner % world).long(), minlength=world)
            m = int(sel.sum().item())
            if m:
                vals = torch.stack([torch.arange(n_act, n_act + m, device=dev, dtype=torch.int32), owner[sel]],
                                   dim=1).contiguous()
                mk = rk[sel].contiguous()
                e.register_device(mk.data_ptr(), vals.data_ptr(), m)
                del vals, mk
            n_act += m
            del rk, owner, sel
        # ---- synthetic message batch, resident in HBM ----------------------------------
        if workload == "cfg3":
            keys = zipf_keys(tcd, G_total, N, 0x5EED0003 + rank, dev)
        else:
            rng = np.random.default_rng(0x5EED0001 + rank)
            ks = rng.integers(0, G_total, size=N, dtype=np.int64)
            keys = torch.from_numpy(grain_keys(tcd, ks).view(np.int64)).to(dev)
            del ks
    torch.cuda.synchronize()
    owner_share = float(counts.max().item()) / G_total
    # the same share under the other silo set (generation 1 literal vs balanced), from a sample
    by_set = {}
    for name, ss in SILO_SETS.items():
        sp, so = g.ring_build(args.mode, ss)
        e2 = g.GrainDispatch(device=local, table_capacity=1024)
        e2.ring_set(args.mode, sp, so)
        sample = np.random.default_rng(5).integers(0, G_total, size=1 << 20)
        o2 = e2.ring_owner(grain_keys(tcd, sample))
        e2.close()
        by_set[name] = round(float(np.bincount(o2 % world, minlength=world).max()) / len(sample), 4)

    router = ShardedRouter(engine, stage_via_cpu=args.rehearse_one_gpu)
    exchange = "none" if world == 1 else (
        "rehearsal: gloo all_to_all on host-staged copies (every rank on cuda:0)" if args.rehearse_one_gpu
        else "torch.distributed all_to_all_single (RCCL)")
    if not args.rehearse_one_gpu and ((world > 1 and args.exchange != "torch") or args.exchange == "library"):
        # the in-library exchange, checked bit for bit against the torch exchange on the first batch;
        # every rank reaches the agreement all-reduce, whatever happened on it (no rank left waiting)
        ok, err = False, None
        try:
            lib_router = LibraryRouter(engine)
            with torch.cuda.stream(stream):
                r_lib, r_torch = lib_router.route_bucket(keys, n_act), router.route_bucket(keys, n_act)
                if engine.bstream is not None:   # pipeline mode: the buckets are done on the bucket stream
                    stream.wait_stream(engine.bstream)
                ok = same_result(r_lib, r_torch)
                torch.cuda.synchronize()
        except Exception as ex:   # noqa: BLE001 -- reported in the JSON line, torch exchange used instead
            if args.exchange == "library":
                raise
            err = f"{ex!r}"[:200]
        agree = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MIN)
        if int(agree.item()) == 1:
            # keys are resident and complete: batch i+1's exchange overlaps batch i's probe + bucket
            # timed batches: messages are known by (sender, index); the probe reads the compact
            # 8-B headers as they arrive and no 24-B key copy is rebuilt (GD_MULTI_NO_KEYS)
            router = lib_router
            lib_router.keys_ready = True
            lib_router.no_keys = True
            exchange = ("libgraindispatch gd_route_multi_device (grouped RCCL send/recv, compact headers, "
                        "GD_MULTI_NO_KEYS); first batch bit-identical to the torch.distributed exchange")
        elif err is not None:
            exchange = f"torch.distributed all_to_all_single (RCCL); library exchange failed here: {err}"
        else:
            exchange = "torch.distributed all_to_all_single (RCCL); library exchange disagreed on batch 1 (some rank)"
            assert args.exchange != "library", "library exchange disagrees with the torch exchange"
    agree = e if world > 1 and router is not None and isinstance(router, LibraryRouter) and args.tune == "measured" \
        else None
    return {"e": e, "engine": engine, "router": router, "stream": stream, "keys": keys, "N": N, "n_act": n_act,
            "agree": agree,
            "G_total": G_total, "cap": cap, "pts": pts, "own": own, "exchange": exchange,
            "owner_share_max": round(owner_share, 4), "owner_share_by_set": by_set}


# Untimed steps before the W warmup steps: libgraindispatch times its probe variants (compact index in
# group reads, directory, index in slot reads) on the first 2 x 3 eligible launches of each launch kind
# and size, then keeps the fastest (eng_core.hip cx_choose).  These steps let that
# measurement finish before the timed region with any --warmup (the driver uses 5): every timed step
# then runs the variant the library keeps.
SETTLE_STEPS = 8
# --tune pinned: the variants each workload's measured runs settle on, fixed with
# gd_tune_set before the first launch -- no settle steps, the same variant on every rank
PINNED = {"cfg2": {"probe_keys": 3, "probe_n1": 3, "bucket": 1},
          "cfg3": {"probe_keys": 3, "probe_n1": 3, "bucket": 1},
          "cfg4": {"probe_fanout": 2, "probe_nodes": 2, "bucket": 1}}


def silos_note(which: str) -> str:
    if which == "literal":
        return "8 x 10.0.0.{1..8}:11111 generation 1 (SURVEY 8(d)'s literal silo set)"
    return ("8 x 10.0.0.{1..8}:11111, balanced generations (tools/balanced_silos.py: each silo owns 1/8 of the "
            "ring; SURVEY 8(d) names generation 1 -- --silos literal -- whose ring gives one silo 35.7 %; "
            "generations are arbitrary timestamps, SiloAddress.cs:72-76, and the per-message work is the same)")


def comm_info(w) -> dict:
    """The library communicator's own view (gd_comm_info: RCCL's ncclCommCount / ncclCommUserRank)."""
    try:
        return w["e"].comm_info()
    except Exception as ex:   # noqa: BLE001 -- reporting only
        return {"error": f"{ex!r}"[:120]}


def settle_steps(args) -> int:
    return 0 if args.tune == "pinned" else SETTLE_STEPS


def pin_choices(e, args, workload: str):
    if args.tune == "pinned":
        for kind, v in PINNED[workload].items():
            e.tune_set(kind, v)


def timed_steps(router, keys, n_act, stream, steps, warmup, settle=SETTLE_STEPS, agree=None):
    """W untimed steps (after `settle` steps for the library's measured choices, then gd_tune_agree
    on `agree`'s communicator at N > 1), then exactly K steps bracketed by barrier + synchronize; max
    over ranks."""
    with torch.cuda.stream(stream):
        for _ in range(settle):
            router.route_bucket(keys, n_act)
        if agree is not None:
            torch.cuda.synchronize()
            try:
                agree.tune_agree()
            except Exception as ex:   # noqa: BLE001 -- speed only: every rank keeps its own choices
                print(f"gd_tune_agree failed: {ex!r}", file=sys.stderr, flush=True)
        for _ in range(warmup):
            router.route_bucket(keys, n_act)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        res = None
        for _ in range(steps):
            res = router.route_bucket(keys, n_act)
        bstream = getattr(getattr(router, "engine", None), "bstream", None)
        if bstream is not None:
            stream.wait_stream(bstream)   # the last batch's bucketing ran on the bucket stream
        ev1.record(stream)
        torch.cuda.synchronize()
        # this rank's K steps end when its device is done; the closing barrier aligns the ranks and the
        # max over ranks below takes the slowest
        wall = time.perf_counter() - t0
        dist.barrier()
        torch.cuda.synchronize()
    t = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), ev0.elapsed_time(ev1), res


T_START = time.perf_counter()

# The one printed line must reach the driver whole: it keeps only the tail (~8 KB) of stdout, and round 4's
# 21.5-KB line (every kernel table inline) was cut and went unparsed.  The line carries the headline and
# compact roofline / baseline / secondary summaries; the full record (per-kernel tables of every config)
# goes to --full-out.
LINE_CAP = 6000


def _pick(d, keys) -> dict:
    return {k: d[k] for k in keys if d and d.get(k) is not None}


ROOF_KEYS = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "traffic_ratio", "frac_pmc",
             "avg_launch_ms", "launches_per_step", "alg_bytes_per_launch")


def compact_roofline(rf, kernels, with_table=True):
    """The line's roofline: the dominant kernel (BASELINE's fields: achieved / peak / frac / traffic, plus
    frac_pmc and the traffic ratio), the bucketing stage's summary, its weakest kernel by name (lowest
    frac_pmc -- else frac -- of the kernels taking >= 10 % of the stage), and (with_table) every stage
    kernel as [ms a step, frac, frac_pmc, traffic_ratio]."""
    if not rf:
        return rf
    out = _pick(rf, ROOF_KEYS)
    if out.get("traffic") is not None:
        out["traffic"] = round(out["traffic"])
    for k in ("probe_variant", "probe_index_frac_impl"):
        if rf.get(k) is not None:
            out[k] = rf[k]
    if rf.get("route_bound"):
        out["route_bound_ms"] = rf["route_bound"].get("ms_per_launch")
        out["route_bound_frac"] = rf["route_bound"].get("frac_of_bound")
    if rf.get("fan_bound"):
        out["fan_bound_ms"] = rf["fan_bound"].get("ms_per_launch")
        out["fan_bound_frac"] = rf["fan_bound"].get("frac_of_bound")
    if rf.get("random_probe_ceiling"):
        out["random_probe_ceiling_frac"] = rf["random_probe_ceiling"].get("frac_of_ceiling")
        out["random_probe_io_ceiling_frac"] = rf["random_probe_ceiling"].get("frac_of_io_ceiling")
    if rf.get("probe_index"):
        out["probe_index_frac_impl"] = rf["probe_index"].get("frac_impl")
    st = rf.get("bucketing_stage")
    if st:
        out["bucketing_stage"] = _pick(st, ("form", "ms_per_step", "impl_bytes_per_message", "frac_impl",
                                            "frac_contract"))
        stage_ms = st.get("ms_per_step") or 0.0
        weakest, wkey = None, None
        table = {}
        for name in st.get("kernels", []):
            d = (kernels or {}).get(name)
            if not d or not d.get("frac_hbm"):
                continue
            table[name] = [d["ms_per_step"], d["frac_hbm"], d.get("frac_pmc"), d.get("traffic_ratio")]
            key = d.get("frac_pmc") or d["frac_hbm"]
            if d["ms_per_step"] >= 0.1 * stage_ms and (wkey is None or key < wkey):
                weakest, wkey = name, key
        if weakest:
            d = kernels[weakest]
            out["weakest_bucketing_kernel"] = dict(
                kernel=weakest, **_pick(d, ("ms_per_step", "launches_per_step", "frac_hbm", "frac_pmc",
                                            "traffic_ratio", "lds_conflict_ratio")))
        if with_table and table:
            out["bucketing_kernels"] = dict(cols="ms_per_step,frac,frac_pmc,traffic_ratio", **table)
    return out


def compact_cpu(c):
    if not c:
        return c
    out = _pick(c, ("value", "unit", "cores", "kind", "mode"))
    out["sample"] = (c.get("sample") or "")[:240]
    return out


def compact_secondary(sec: dict) -> dict:
    out = {}
    for name, v in (sec or {}).items():
        if name == "cfg5_latency_us":
            out[name] = {k: v[k] for k in ("batch", "graph", "eager", "zero_copy") if k in v}
        elif name == "cfg1_ping_shape":
            out[name] = _pick(v, ("value", "ms_per_step", "workload"))
        elif name.endswith("_churn"):
            out[name] = _pick(v, ("value", "ms_per_step", "static_ms_per_step", "churn_vs_static", "pipelined",
                                  "unregistered_per_step", "index_builds_timed", "slots_reprojected_timed",
                                  "last_full_build_ms", "table_tombstones", "routed_ok_fraction_last_step"))
        elif name == "cfg2_mixed":
            out[name] = _pick(v, ("value", "ms_per_step", "k_route_ms", "k_route_vs_single_class", "index_types8",
                                  "guid_grains", "routed_ok_fraction"))
        elif name == "host_path":
            out[name] = _pick(v, ("value", "ms_per_call", "pcie_GBps", "workload"))
        elif name == "cfg2_other_silo_set":
            out[name] = _pick(v, ("silos", "value", "ms_per_step", "owner_share_max", "exchange"))
        else:
            d = _pick(v, ("value", "unit", "ms_per_step", "steps", "workload", "n_gpus", "scaling",
                          "messages_per_step"))
            if isinstance(d.get("workload"), str):
                d["workload"] = d["workload"][:160]
            if v.get("config", {}).get("workload"):
                d["workload"] = v["config"]["workload"][:160]
            d["roofline"] = compact_roofline(v.get("roofline"), v.get("kernels"), with_table=False)
            if v.get("cpu_baseline"):
                d["cpu_baseline"] = compact_cpu(v["cpu_baseline"])
            out[name] = d
    return out


def compact_line(full: dict, full_path=None) -> dict:
    """The printed line from the full record (LINE_CAP bytes at most: secondary tables are dropped first,
    then the main stage table)."""
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "settle_steps", "tune",
                                 "ms_per_step", "gpu_event_ms_per_step", "higher_is_better", "scaling",
                                 "vs_baseline", "dtype", "data") if k in full}
    cfg = dict(full.get("config") or {})
    if isinstance(cfg.get("silos"), str):
        cfg["silos"] = cfg["silos"][:90]
    line["config"] = cfg
    for k in ("routed_ok_last_step_rank0", "rehearsal_one_gpu", "messages_per_step", "comm", "exchange_ms_per_rank"):
        if k in full:
            line[k] = full[k]
    if isinstance(full.get("exchange"), str):
        line["exchange"] = full["exchange"][:120]
    line["roofline"] = compact_roofline(full.get("roofline"), full.get("kernels"))
    line["cpu_baseline"] = compact_cpu(full.get("cpu_baseline"))
    if full.get("secondary"):
        line["secondary"] = compact_secondary(full["secondary"])
    if full_path:
        line["full_record"] = full_path
    if "bench_wall_s" in full:
        line["bench_wall_s"] = full["bench_wall_s"]
    if len(json.dumps(line)) > LINE_CAP and line["roofline"]:
        line["roofline"].pop("bucketing_kernels", None)
    for name in list((line.get("secondary") or {}).keys()):
        if len(json.dumps(line)) <= LINE_CAP:
            break
        sec = line["secondary"][name]
        if isinstance(sec, dict) and isinstance(sec.get("roofline"), dict):
            sec["roofline"] = {k: sec["roofline"][k] for k in ("kernel", "frac", "frac_pmc")
                               if k in sec["roofline"]}
    return line


def emit(full: dict, args):
    """Writes the full record to --full-out, prints the compact line (one JSON line, <= LINE_CAP bytes)."""
    path = args.full_out
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
    except OSError as ex:
        print(f"bench: full record not written: {ex!r}", file=sys.stderr, flush=True)
        path = None
    line = compact_line(full, os.path.relpath(path, ROOT) if path else None)
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "cfg3", "cfg4"],
                    help="cfg2: 16M uniform msgs/GPU over 2^20 grains/GPU (weak scaling); cfg3: 64M Zipf(1.1) "
                         "msgs over 100M grains for the whole node (strong scaling); cfg4: Chirper fan-out "
                         "cascade over a 10M-grain power-law follower graph")
    ap.add_argument("--msgs", type=int, default=None, help="messages per GPU per step (cfg2 default 2^24)")
    ap.add_argument("--grains", type=int, default=None, help="grains per GPU (cfg2 default 2^20)")
    ap.add_argument("--mode", default="D", choices=["D", "R", "V"])
    ap.add_argument("--silos", default="balanced", choices=sorted(SILO_SETS))
    ap.add_argument("--cpu-seconds", type=float, default=24.0, help="bounded CPU baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=5, help="extra steps with per-kernel events")
    ap.add_argument("--exchange", default="auto", choices=["auto", "library", "torch"],
                    help="N>1: RCCL exchange inside libgraindispatch (gd_route_multi_device) or torch.distributed "
                         "all_to_all_single; auto = library once it matches torch bit for bit on the first batch")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary configs (N>1: cfg3 strong scaling; N=1: cfg3 and cfg4 on one GPU)")
    ap.add_argument("--msgs3", type=int, default=None, help="secondary cfg3: messages per GPU (default 2^26 / N)")
    ap.add_argument("--grains3", type=int, default=None, help="secondary cfg3: grains per GPU (default 1e8 / N)")
    ap.add_argument("--latency-batches", type=int, default=10000,
                    help="N=1 cfg2: 4,096-message micro-batches timed for the cfg5 latency line (0: skip)")
    ap.add_argument("--nodes", type=int, default=10_000_000, help="cfg4: grains (follower-graph nodes)")
    ap.add_argument("--mean-deg", type=float, default=10.0, help="cfg4: mean follower count")
    ap.add_argument("--max-deg", type=int, default=1 << 16, help="cfg4: follower-count cap")
    ap.add_argument("--seeds", type=int, default=1 << 16, help="cfg4: publishers of the first hop")
    ap.add_argument("--hops", type=int, default=3, help="cfg4: publish rounds per cascade")
    ap.add_argument("--no-target", action="store_true", help="cfg4: do not write the target node per message")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0, gloo, host-staged all-to-all")
    ap.add_argument("--full-out", default=os.path.join(ROOT, "gpurun_out", "bench_full.json"),
                    help="where the full record (every kernel table) is written; the printed line is its summary")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a handle option for every handle (graindispatch.OPTIONS: GD_OPT_*), e.g. bucket=2")
    ap.add_argument("--pipeline", action="store_true",
                    help="N=1: each batch's bucketing on a second stream (gd_set_bucket_stream), overlapping the "
                         "next batch's route")
    ap.add_argument("--tune", default="pinned", choices=["measured", "pinned"],
                    help="pinned (default): the variants each workload's measured runs settle on, fixed up front "
                         "(gd_tune_set: the 8-B index's group reads, two-level bucketing), no settle steps, the "
                         "same on every rank; measured: the library times its variants on the first launches "
                         "(settle steps, then gd_tune_agree across ranks at N > 1; the exchange pipeline runs "
                         "unoverlapped while it times, DESIGN 10)")
    args = ap.parse_args()
    for kv in args.opt:
        k, v = kv.split("=", 1)
        g.DEFAULT_OPTIONS[k] = int(v)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus or "WORLD_SIZE" not in os.environ, "--gpus must match WORLD_SIZE"
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and args.rehearse_one_gpu:
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=dev)
    else:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        # gloo's connect message goes to fd 1: keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=0, world_size=1)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    if args.workload == "cfg4":
        return run_cfg4(args, world, rank, local, dev)

    tc = g.calculate_id_hash(PING_GRAIN_CLASS)
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    w = setup_workload(args, args.workload, world, rank, local, dev, tcd, args.msgs, args.grains)
    e, N, n_act, G_total, cap, router, stream, keys = (w["e"], w["N"], w["n_act"], w["G_total"], w["cap"],
                                                        w["router"], w["stream"], w["keys"])
    exchange = w["exchange"]
    wall_max, gpu_ms, res = timed_steps(router, keys, n_act, stream, args.steps, args.warmup, settle_steps(args),
                                        w["agree"])
    value = N * args.steps * world / wall_max
    secondary = {}
    if world > 1 and args.workload == "cfg2" and not args.no_secondary:
        # BASELINE cfg 3 is the node-level configuration: 64M Zipf(1.1) messages over 100M grains
        # for the whole node (strong scaling), measured by the same harness beside the weak line
        w3 = setup_workload(args, "cfg3", world, rank, local, dev, tcd, args.msgs3, args.grains3)
        wall3, gpu3, r3 = timed_steps(w3["router"], w3["keys"], w3["n_act"], w3["stream"],
                                      max(10, args.steps // 10), max(3, args.warmup // 4), settle_steps(args),
                                      w3["agree"])
        steps3 = max(10, args.steps // 10)
        k3, rf3 = secondary_roofline(w3, r3, args, "cfg3", world)
        secondary["cfg3_strong"] = {
            "roofline": rf3, "kernels": k3,
            "value": round(w3["N"] * steps3 * world / wall3, 1), "unit": "messages/s",
            "ms_per_step": round(wall3 / steps3 * 1e3, 4), "steps": steps3,
            "workload": workload_name("cfg3", world, w3["N"], w3["G_total"]), "msgs_per_gpu": w3["N"],
            "scaling": "strong", "exchange": w3["exchange"], "owner_share_max": w3["owner_share_max"],
            "owner_share_max_by_silo_set": w3["owner_share_by_set"]}
        w3["e"].close()
        del w3

    if world == 1 and args.workload == "cfg2" and not args.no_secondary:
        # BASELINE cfg 3 on one GPU (64M Zipf(1.1) messages over 100M grains) and cfg 4 (the Chirper
        # fan-out cascade), each with its bounded CPU baseline; the cfg 2 handle stays open
        w3 = setup_workload(args, "cfg3", 1, 0, local, dev, tcd, args.msgs3, args.grains3)
        steps3 = max(10, args.steps // 10)
        wall3, gpu3, r3 = timed_steps(w3["router"], w3["keys"], w3["n_act"], w3["stream"], steps3,
                                      max(3, args.warmup // 4), settle_steps(args))
        k3, rf3 = secondary_roofline(w3, r3, args, "cfg3", 1)
        c3 = None
        if not args.no_cpu_baseline:
            c3 = cpu_baseline_cfg3(args, w3, tcd)
        secondary["cfg3"] = {
            "value": round(w3["N"] * steps3 / wall3, 1), "unit": "messages/s",
            "ms_per_step": round(wall3 / steps3 * 1e3, 4), "steps": steps3,
            "workload": workload_name("cfg3", 1, w3["N"], w3["G_total"]), "msgs_per_gpu": w3["N"],
            "roofline": rf3, "kernels": k3, "cpu_baseline": c3}
        secondary["cfg3_churn"] = churn_line(w3, args, wall3 / steps3 * 1e3, "cfg3", steps3, 3)
        w3["e"].close()
        del w3
        torch.cuda.empty_cache()
        secondary["cfg4"] = measure_cfg4(args, 1, 0, local, dev, steps=max(5, args.steps // 20),
                                         warmup=max(2, args.warmup // 5), profile_steps=2,
                                         with_cpu=not args.no_cpu_baseline)

    # received (owner-side) message count, for the byte model
    m_recv = int(res.status.shape[0])
    st_ok = int((res.status == 0).sum().item())

    # ---- per-kernel durations (separate steps, HIP events around every launch) -----
    acts_np = res.act.cpu().numpy().view(np.uint32)
    kt = profile_kernels(e, router, keys, n_act, stream, args.profile_steps)
    kernels, roofline = roofline_of(kt, max(1, args.profile_steps), m_recv, n_act, acts_np, args.workload, world)
    # the library exchange's RCCL rounds on every rank (HIP events around each grouped round, the
    # profiled steps): VERDICT r05 item 5
    ex_ms = sum(v[1] for k, v in kt.items() if k.startswith("rccl_")) / max(1, args.profile_steps)
    ex_ms_ranks = gather_floats(ex_ms, world, dev)

    # ---- N > 1: the same line on the other silo set (SURVEY 8(d)'s literal generation-1 set and the
    # balanced one), with each set's largest owner share -------------------------------------------
    if world > 1 and args.workload == "cfg2" and not args.no_secondary:
        secondary["cfg2_other_silo_set"] = other_silo_set_line(args, world, rank, local, dev, tcd)
    if roofline and roofline["kernel"] == "k_route":
        route_extras(roofline, e, m_recv, args.workload, world, isinstance(router, LibraryRouter), keys, stream)

    # ---- the directory under churn, a mixed directory, the host-buffer path (cfg 2, N = 1) -------
    if world == 1 and args.workload == "cfg2" and not args.no_secondary:
        secondary["cfg2_churn"] = churn_line(w, args, wall_max / args.steps * 1e3, "cfg2", args.steps,
                                             args.warmup)
        single = (roofline or {}).get("avg_launch_ms") if (roofline or {}).get("kernel") == "k_route" else None
        secondary["cfg2_mixed"] = mixed_line(args, tcd, dev, max(10, args.steps // 4), max(3, args.warmup // 2),
                                             single)
        secondary["host_path"] = host_path_line(e, tcd, G_total, n_act)

    # ---- BASELINE cfg 5: 4,096-message micro-batch latency on this directory ---------
    if world == 1 and args.workload == "cfg2" and args.latency_batches > 0:
        secondary["cfg5_latency_us"] = micro_batch_latency(e, tcd, G_total, n_act, args.latency_batches)

    # ---- BASELINE cfg 1's shape on the GPU: 1M calls over 10k grains, one silo ---------
    if world == 1 and args.workload == "cfg2" and args.latency_batches > 0:
        secondary["cfg1_ping_shape"] = ping_shape(tcd, dev, args.mode)

    # ---- CPU baseline: the C restatement (oracle/cpu_ref.c), bounded sample ---------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "cfg2":
        owner = e.ring_owner(grain_keys(tcd, np.arange(G_total, dtype=np.int64)))
        cpu = cpu_baseline(args, tcd, G_total, w["pts"], w["own"], owner)

    if rank == 0:
        line = {
            "metric": "routed messages/sec (lookup+bucket, whole node)",
            "value": round(value, 1),
            "unit": "messages/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup, "settle_steps": settle_steps(args), "tune": args.tune,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.workload == "cfg2" else "strong",
            "vs_baseline": None,
            "dtype": "u32/u64 integer",
            "data": "synthetic GrainIds (no dataset); " + (
                "uniform keys, seed 0x5EED0001+rank" if args.workload == "cfg2" else
                "Zipf(1.1) keys by inverse CDF on the GPU, seed 0x5EED0003+rank"),
            "config": {"workload": workload_name(args.workload, world, N, G_total),
                       "msgs_per_gpu": N, "grains_total": G_total, "ring_mode": args.mode,
                       "silos": silos_note(args.silos),
                       "owner_share_max": w["owner_share_max"],
                       "owner_share_max_by_silo_set": w["owner_share_by_set"],
                       "table_load": round(n_act / cap, 3), "parallelism": f"shard{world}",
                       "batch_pipeline": bool(w["engine"].bstream is not None)},
            "routed_ok_last_step_rank0": st_ok,
            "rehearsal_one_gpu": bool(args.rehearse_one_gpu),
            "exchange": exchange,
            # the library exchange's RCCL rounds per rank (HIP events); null on the torch / rehearsal exchange
            "exchange_ms_per_rank": ([round(x, 4) for x in ex_ms_ranks]
                                     if world > 1 and isinstance(router, LibraryRouter) else None),
            "comm": comm_info(w),
            "roofline": roofline,
            "kernels": kernels,
            "cpu_baseline": cpu,
        }
        if secondary:
            line["secondary"] = secondary
        line["bench_wall_s"] = round(time.perf_counter() - T_START, 1)
        emit(line, args)
    e.close()
    dist.destroy_process_group()


def secondary_roofline(w, res, args, tag: str, world: int):
    """(kernels, roofline) of a secondary workload's steps (its own profiled steps)."""
    m = int(res.status.shape[0])
    acts = res.act.cpu().numpy().view(np.uint32)
    kt = profile_kernels(w["e"], w["router"], w["keys"], w["n_act"], w["stream"], 3)
    k, rf = roofline_of(kt, 3, m, w["n_act"], acts, tag, world)
    if rf and rf["kernel"] == "k_route":
        route_extras(rf, w["e"], m, tag, world, isinstance(w["router"], LibraryRouter), w["keys"], w["stream"])
    return k, rf


def profile_kernels(e, router, keys, n_act, stream, steps: int) -> dict:
    """{kernel: (launches, total ms)} over `steps` extra steps with HIP events around every launch in
    the library (gd_set_kernel_timing; events inside the timed region would perturb it)."""
    if steps <= 0:
        return {}
    kt = {}
    for mode in (1, 2):            # every launch, then the stages alone ("stage:bucket")
        e.set_kernel_timing(mode)
        e.kernel_times_reset()
        with torch.cuda.stream(stream):
            for _ in range(steps):
                router.route_bucket(keys, n_act)
        torch.cuda.synchronize()
        t = e.kernel_times()
        kt.update(t if mode == 1 else {k: v for k, v in t.items() if k.startswith("stage:")})
    e.set_kernel_timing(False)
    return kt


def route_extras(roofline: dict, e, m_recv: int, tag: str, world: int, exchange: bool = False, keys=None,
                 stream=None):
    """k_route's side fields: the probe variant the library runs (gd_tune_get) and, when it reads a
    compact index (gd_cx.h), the index's own bytes a message.  exchange: the probe reads the library
    exchange's N1 headers (GD_TUNE_PROBE_N1), at any world size.  keys (24-B keys, world 1, 8-B index):
    the route's memory bound measured live on the same index and key stream (route_bound)."""
    kind = "probe_n1" if exchange or world > 1 else "probe_keys"
    v = e.tune_get(kind, m_recv)
    roofline["probe_variant"] = PROBE_VARIANTS.get(v, str(v))
    t_l = roofline["avg_launch_ms"] * 1e-3
    slot = {0: 16, 2: 16, 3: 8}.get(v)
    if v == 3 and world == 1 and not exchange and keys is not None:
        rb = route_bound(e, keys, stream, roofline["avg_launch_ms"])
        if rb:
            roofline["route_bound"] = rb
    if slot:
        # per message: key 24 + one index slot + silo/act/status 9
        impl = m_recv * (24 + slot + 9)
        roofline["probe_index"] = {"slot_bytes": slot, "impl_bytes_per_launch": impl,
                                   "frac_impl": round(impl / t_l / 1e9 / PEAK_HBM_GBS, 4) if t_l > 0 else None}


def route_bound(e, keys, stream, launch_ms: float, reps: int = 5):
    """gd_route_bound_device over the route's own 8-B index and key stream, `reps` launches timed by the
    library's HIP events on its stream (as k_route is): k_route's launch shape, key reads, one 64-B
    group read a message and its 9-B writes, with no ring search, walk or fallback (gd_kernels.h
    k_route_bound).  frac_of_bound = bound / k_route: 1.0 would be a route with nothing but its memory
    traffic left."""
    n = int(keys.shape[0])
    dev = keys.device
    silo = torch.empty(n, dtype=torch.int32, device=dev)
    act = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    try:
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            e.route_bound_device(keys.data_ptr(), n, silo.data_ptr(), act.data_ptr(), st.data_ptr())   # warm
            torch.cuda.synchronize()
            e.set_kernel_timing(1)
            e.kernel_times_reset()
            for _ in range(reps):
                e.route_bound_device(keys.data_ptr(), n, silo.data_ptr(), act.data_ptr(), st.data_ptr())
            torch.cuda.synchronize()
            t = e.kernel_times().get("k_route_bound")
    except (g.GrainDispatchError, AttributeError):
        return None
    finally:
        e.set_kernel_timing(False)
    if not t or t[0] == 0 or launch_ms <= 0:
        return None
    ms = t[1] / t[0]
    return {"ms_per_launch": round(ms, 4), "frac_of_bound": round(ms / launch_ms, 3),
            "source": "gd_route_bound_device, live: same index, keys, grid and writes; one 64-B index read a "
                      "message, no ring / walk / fallback"}


def fan_bound(e, step, reps: int):
    """GD_OPT_FAN_BOUND: every hop's k_fan_route over the 8-B index preceded by k_fan_bound on the same
    inputs (the staged publishers, follower lists, home hash, one 64-B index group read a message and the
    same result writes into scratch; no ring search, no walk -- gd_fanout.h k_fan_route<..., BOUND>), both
    timed by the library's HIP events over `reps` cascades.  frac_of_bound = bound / k_fan_route over the
    same launches."""
    try:
        e.set_option("fan_bound", 1)
        e.set_kernel_timing(1)
        e.kernel_times_reset()
        for _ in range(max(1, reps)):
            step()
        torch.cuda.synchronize()
        t = e.kernel_times()
    except (g.GrainDispatchError, AttributeError, KeyError):
        return None
    finally:
        e.set_kernel_timing(False)
        try:
            e.set_option("fan_bound", 0)
        except (g.GrainDispatchError, KeyError):
            pass
    b, r = t.get("k_fan_bound"), t.get("k_fan_route")
    if not b or not r or b[0] != r[0] or r[1] <= 0:
        return None
    return {"ms_per_launch": round(b[1] / b[0], 4), "route_ms_per_launch": round(r[1] / r[0], 4),
            "frac_of_bound": round(b[1] / r[1], 3),
            "source": "GD_OPT_FAN_BOUND, live: the hop's own frontier, graph, index and grid; expansion reads, "
                      "one 64-B index group read a message and the result writes, no ring search / walk"}


# The random-probe ceiling of the 8-B index (tools/ubench_fanprobe.hip, profiles/r05_ubench_fanprobe.txt):
# probes a ms of one 64-B group (4 x 16-B loads) at random into an index of the workload's size, with a
# 4-B key stream in and 8 B out -- no hash, ring or compare work.  cfg 2: 2^21 slots (16 MB) at load 0.5,
# 16M probes, 0.2567 ms; cfg 4: 2^25 slots (268 MB) at load 0.3, 43M probes, 0.8226 ms.  EA requests:
# 1.0 64-B request a probe (TCC_EA0_RDREQ_32B_sum = 0: a 32-B read still moves 64 B).
PROBE_CEILING_PER_MS = {"cfg2": 16777216 / 0.2567, "cfg4": 43000000 / 0.8226}
# the same probe with k_route's own streams beside it (24-B keys in, silo / act / status out: g4io)
PROBE_IO_CEILING_PER_MS = {"cfg2": 16777216 / 0.3186, "cfg4": 43000000 / 0.9481}


def probe_ceiling(tag: str, probes: float, launch_ms: float):
    rate, rate_io = PROBE_CEILING_PER_MS.get(tag), PROBE_IO_CEILING_PER_MS.get(tag)
    if not rate or launch_ms <= 0:
        return None
    ms, ms_io = probes / rate, probes / rate_io
    return {"ms_per_launch": round(ms, 4), "frac_of_ceiling": round(ms / launch_ms, 3),
            "with_io_ms_per_launch": round(ms_io, 4), "frac_of_io_ceiling": round(ms_io / launch_ms, 3),
            "source": "profiles/r05_ubench_fanprobe.txt, r05_ubench_probe_io_{21,25}.txt (8-B index, random 64-B "
                      "group reads; g4io adds the route's 24-B key reads and 9-B result writes)"}


# gd_tune_get variants of the 24-B-key / N1 probes (eng_core.hip cx_choose)
PROBE_VARIANTS = {0: "16-B index, 64-B group reads", 1: "directory table, 32-B slots",
                  2: "16-B index, 16-B slot reads", 3: "8-B index, 64-B group reads", -1: "still measuring"}


def ping_shape(tcd: int, dev, mode: str, G: int = 10_000, N: int = 1 << 20, steps: int = 200) -> dict:
    """BASELINE cfg 1's shape (PingBenchmark: 1M calls over 10k grains, one silo) through
    gd_route_bucket_device, inputs resident in HBM; the CPU restatement's rate for the same shape
    is cpu_baseline.cfg1_ping_shape."""
    e1 = g.GrainDispatch(device=dev.index or 0, table_capacity=1 << 15, my_silo=0, kernel_timing=False)
    e1.ring_set_silos(mode, SILO_SETS["literal"][:1])
    reg = grain_keys(tcd, np.arange(G, dtype=np.int64))
    e1.register(reg, np.arange(G, dtype=np.uint32), np.zeros(G, np.uint32))
    ks = np.random.default_rng(0x5EED0101).integers(0, G, size=N, dtype=np.int64)
    keys = torch.from_numpy(grain_keys(tcd, ks).view(np.int64)).to(dev)
    silo = torch.empty(N, dtype=torch.int32, device=dev)
    act = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    off = torch.empty(G + 2, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream())
    e1.set_stream(stream.cuda_stream)

    def one():
        e1.route_bucket_device(keys.data_ptr(), N, G, silo.data_ptr(), act.data_ptr(), st.data_ptr(),
                               perm.data_ptr(), off.data_ptr())
    for _ in range(10):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ok = int((st == 0).sum().item())
    e1.close()
    return {"value": round(N * steps / wall, 1), "unit": "messages/s", "ms_per_step": round(wall / steps * 1e3, 4),
            "steps": steps, "workload": f"{N} calls uniform over {G} grains, 1 silo, ring {mode}",
            "routed_ok_last_step": ok}


def micro_batch_latency(e, tcd: int, G: int, n_act: int, batches: int, B: int = 4096) -> dict:
    """BASELINE cfg 5: wall latency of one 4,096-message batch (uniform over the registered grains)
    from keys in pinned host memory to statuses / silos / activations / per-activation runs back in
    host memory (gd_microbatch_run: one hipGraph replay, or eager launches), p50 / p99 over
    ``batches`` batches after 50 warmup batches.  The CPU restatement's p50 / p99 for the same batch
    is cpu_baseline.cfg5_latency_us."""
    mb = g.MicroBatch(e, B, n_act)
    rng = np.random.default_rng(0x5EED0005)
    pool = grain_keys(tcd, rng.integers(0, G, size=64 * B, dtype=np.int64)).reshape(64, B, 3)
    out = {"batch": B, "batches": batches,
           "path": "pinned host keys -> route -> one-workgroup radix sort + runs -> pinned host results"}
    for use_graph in (True, False):
        lat = np.empty(batches)
        for i in range(50):
            mb.keys[:] = pool[i % 64]
            mb.run(B, use_graph)
        for i in range(batches):
            mb.keys[:] = pool[i % 64]
            t0 = time.perf_counter()
            mb.run(B, use_graph)
            lat[i] = time.perf_counter() - t0
        us = lat * 1e6
        out["graph" if use_graph else "eager"] = {"p50": round(float(np.percentile(us, 50)), 1),
                                                  "p99": round(float(np.percentile(us, 99)), 1),
                                                  "max": round(float(us.max()), 1)}
    out["zero_copy"] = bool(e.get_option("mb_zerocopy"))
    mb.close()
    return out


def gather_floats(x: float, world: int, dev) -> list:
    """x from every rank, in rank order (all_gather; on the GPU under RCCL)."""
    if world == 1:
        return [x]
    on_gpu = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_gpu else "cpu")
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def other_silo_set_line(args, world, rank, local, dev, tcd) -> dict:
    """The cfg 2 line on the other silo set: the balanced set gives every silo 1/8
    of the ring; SURVEY 8(d)'s literal generation-1 set gives one silo 35.7 %, so its owner rank receives
    that share of every batch.  Same harness, fewer steps."""
    import copy
    a2 = copy.copy(args)
    a2.silos = "literal" if args.silos == "balanced" else "balanced"
    w2 = setup_workload(a2, "cfg2", world, rank, local, dev, tcd, args.msgs, args.grains)
    steps = max(10, args.steps // 4)
    wall, _, _ = timed_steps(w2["router"], w2["keys"], w2["n_act"], w2["stream"], steps, max(3, args.warmup // 4),
                             settle_steps(args), w2["agree"])
    out = {"silos": a2.silos, "value": round(w2["N"] * steps * world / wall, 1), "unit": "messages/s",
           "ms_per_step": round(wall / steps * 1e3, 4), "steps": steps,
           "owner_share_max": w2["owner_share_max"], "exchange": w2["exchange"][:80]}
    w2["e"].close()
    del w2
    torch.cuda.empty_cache()
    return out


def churn_line(w, args, static_ms: float, tag: str, steps: int, warmup: int) -> dict:
    """the directory under continuous registration (Catalog.cs:540-552,1270-1277 ->
    GrainDirectoryPartition.AddSingleActivation / RemoveActivation, :304-363).  Every step removes 1 % of
    the grains (gd_dir_unregister_device) and registers the 1 % removed the step before again
    (gd_dir_register_device_async), then routes and buckets the workload's batch -- all enqueued on the
    handle's stream, timed together exactly like the static steps.  The probe indexes are re-projected for
    the touched slots (k_cx_sync), not rebuilt; index builds during the timed steps are reported."""
    e, router, keys, stream, n_act, G = w["e"], w["router"], w["keys"], w["stream"], w["n_act"], w["G_total"]
    dev = keys.device
    B = max(1, G // 100)
    nwin = max(2, min(G // B, steps + warmup + 1))
    tcd = int(keys[0, 2].item()) & 0xFFFFFFFFFFFFFFFF
    K, A, V = [], [], []
    with torch.cuda.stream(stream):
        for i in range(nwin):
            ks = torch.arange(i * B, (i + 1) * B, device=dev, dtype=torch.int64)
            k = grain_keys_torch(tcd, ks, dev)
            own = torch.empty(B, dtype=torch.int32, device=dev)
            e.ring_owner_device(k.data_ptr(), B, own.data_ptr())
            a = ks.to(torch.int32)                       # world 1: grain k's activation is k (setup_workload)
            K.append(k)
            A.append(a)
            V.append(torch.stack([a, own], 1).contiguous())
    torch.cuda.synchronize()
    before = e.index_stats()

    def churn_batches(s_):
        i = s_ % nwin
        e.unregister_device(K[i].data_ptr(), A[i].data_ptr(), B)
        if s_:
            j = (s_ - 1) % nwin
            e.register_device_async(K[j].data_ptr(), V[j].data_ptr(), B)

    def step(s_):
        churn_batches(s_)
        return router.route_bucket(keys, n_act)

    def step_p(s_):                                    # pipeline mode (below): the same on the second router
        churn_batches(s_)
        return r2.route_bucket(keys, n_act)

    with torch.cuda.stream(stream):
        for s_ in range(warmup):
            step(s_)
        torch.cuda.synchronize()
        mid = e.index_stats()
        t0 = time.perf_counter()
        res = None
        for s_ in range(warmup, warmup + steps):
            res = step(s_)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    e.synchronize()                                    # any deferred device error of the async batches
    after = e.index_stats()
    st = e.stats()
    ok = int((res.status == 0).sum().item())
    ms = wall / steps * 1e3
    # the same in pipeline mode (gd_set_bucket_stream): each batch's bucketing on a second stream, so the
    # directory batches (their own scratch: no wait for the bucket stream) overlap the previous bucketing;
    # the static steps timed the same way beside them
    pipe = {}
    if w["engine"].bstream is None:
        eng2 = DeviceEngine(e, dev, stream=stream, pipeline=True)
        r2 = ShardedRouter(eng2)
        s0 = warmup + steps
        for tag_, fn in (("static", lambda s_: r2.route_bucket(keys, n_act)), ("churn", step_p)):
            with torch.cuda.stream(stream):
                for s_ in range(warmup):
                    fn(s0 + s_)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for s_ in range(warmup, warmup + steps):
                    fn(s0 + s_)
                torch.cuda.synchronize()
                pipe[tag_] = (time.perf_counter() - t0) / steps * 1e3
            if tag_ == "churn":
                s0 += warmup + steps
        e.set_bucket_stream(None)
        e.synchronize()
    # restore the directory: the last removed window comes back
    last = (s0 - 1) % nwin if pipe else (warmup + steps - 1) % nwin
    e.register_device(K[last].data_ptr(), V[last].data_ptr(), B)
    return {"value": round(w["N"] * steps / wall, 1), "unit": "messages/s", "ms_per_step": round(ms, 4),
            "steps": steps, "static_ms_per_step": round(static_ms, 4),
            "churn_vs_static": round(ms / static_ms, 3) if static_ms else None,
            "pipelined": {"static_ms_per_step": round(pipe["static"], 4), "churn_ms_per_step": round(pipe["churn"], 4),
                          "churn_vs_static": round(pipe["churn"] / pipe["static"], 3)} if pipe else None,
            "unregistered_per_step": B, "registered_per_step": B,
            "index_builds_timed": after["builds"] - mid["builds"],
            "index_builds_total": after["builds"] - before["builds"],
            "slots_reprojected_timed": after["synced_slots"] - mid["synced_slots"],
            "last_full_build_ms": round(after["last_build_ms"], 3),
            "table_live": st["table_live"], "table_tombstones": st["table_tombstones"],
            "routed_ok_fraction_last_step": round(ok / w["N"], 4),
            "workload": f"{tag} batch + 1% of the grains unregistered and 1% registered a step "
                        "(gd_dir_unregister_device + gd_dir_register_device_async on the stream)"}


def mixed_line(args, tcd_ping: int, dev, steps: int, warmup: int, single_route_ms: float) -> dict:
    """cfg 2's shape over a mixed directory -- 2^20 grains of 8 grain classes, every
    100th Guid-keyed (N0 != 0, UniqueKey.cs:135-143; orleans_amd.workloads.mixed_grain_keys), 16M
    messages uniform over them.  The 8-B index holds the 8 classes, the Guid keys' messages probe the
    directory per message.  k_route's time is compared with the single-class line's."""
    from orleans_amd.workloads import mixed_grain_keys
    G, N = 1 << 20, 1 << 24
    tcds = [(3 << 56) + ((g.calculate_id_hash(f"BenchmarkGrains.Mixed.Grain{c}") & 0xFFFFFFFFFFFFFFFF)
                         & 0x00FFFFFFFFFFFFFF) for c in range(8)]
    e = g.GrainDispatch(device=dev.index or 0, table_capacity=2 * G, my_silo=0, kernel_timing=False)
    e.tune_set("probe_keys", 3)
    e.tune_set("bucket", 1)
    pts, own = e.ring_set_silos(args.mode, SILO_SETS[args.silos])
    reg = mixed_grain_keys(tcds, G)
    owner = e.ring_owner(reg)
    e.register(reg, np.arange(G, dtype=np.uint32), owner)
    idx = np.random.default_rng(0x5EED0007).integers(0, G, size=N)
    keys = torch.from_numpy(reg[idx].view(np.int64)).to(dev)
    engine = DeviceEngine(e, dev)
    router = ShardedRouter(engine)
    stream = engine.stream
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            router.route_bucket(keys, G)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = None
        for _ in range(steps):
            res = router.route_bucket(keys, G)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    ok = int((res.status == 0).sum().item())
    kt = profile_kernels(e, router, keys, G, stream, 3)
    kr = kt.get("k_route")
    route_ms = kr[1] / kr[0] if kr and kr[0] else None
    ist = e.index_stats()
    e.close()
    return {"value": round(N * steps / wall, 1), "unit": "messages/s", "ms_per_step": round(wall / steps * 1e3, 4),
            "steps": steps, "k_route_ms": round(route_ms, 4) if route_ms else None,
            "k_route_vs_single_class": round(route_ms / single_route_ms, 3) if route_ms and single_route_ms else None,
            "index_types8": ist["types8"], "guid_grains": ist["n0_live"],
            "routed_ok_fraction": round(ok / N, 4),
            "workload": f"{N} msgs uniform over {G} grains of 8 classes, 1% Guid-keyed (N0 != 0), ring {args.mode}"}


def host_path_line(e, tcd: int, G: int, n_act: int, steps: int = 5, warmup: int = 2) -> dict:
    """what a C# caller sees -- gd_route_bucket on pinned host buffers (the
    P/Invoke entry point): cfg 2's 16M keys in (24 B a message), silo / act / status /
    perm out (13 B) and the offsets, H2D / D2H copies overlapped with the kernels in chunks."""
    N = 1 << 24
    hold = []

    def pinned(shape, dt):
        t = torch.empty(int(np.prod(shape)) * np.dtype(dt).itemsize, dtype=torch.uint8, pin_memory=True)
        hold.append(t)
        return t.numpy().view(dt).reshape(shape)
    keys = pinned((N, 3), np.uint64)
    silo, act, perm = (pinned((N,), np.uint32) for _ in range(3))
    st = pinned((N,), np.uint8)
    off = pinned((n_act + 2,), np.uint32)
    keys[:] = grain_keys(tcd, np.random.default_rng(0x5EED0001).integers(0, G, size=N, dtype=np.int64))
    ptr = lambda a: a.ctypes.data                       # noqa: E731

    def one():
        e._c(g.lib.gd_route_bucket(e.h, ptr(keys), N, n_act, ptr(silo), ptr(act), ptr(st), ptr(perm), ptr(off)))
    for _ in range(warmup):
        one()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    dt = (time.perf_counter() - t0) / steps
    ok = int((st == 0).sum())
    return {"value": round(N / dt, 1), "unit": "messages/s", "ms_per_call": round(dt * 1e3, 3), "steps": steps,
            "pcie_GBps": round(N * (24 + 17) / dt / 1e9, 2), "routed_ok": ok,
            "workload": "cfg2 keys in pinned host memory -> gd_route_bucket -> pinned host results (PCIe-inclusive)"}


def workload_name(w: str, world: int, n: int, g_total: int) -> str:
    if w == "cfg3":
        return (f"cfg3: {n * world} msgs Zipf(1.1) over {g_total} grains, directory sharded by ring owner over "
                f"{world} GPU(s)" + (", RCCL all-to-all-v" if world > 1 else ""))
    if world == 1:
        return "cfg2: 16M msgs uniform over 1M grains, 8 silos, ring D"
    return f"cfg2 per GPU (16M msgs/GPU over {g_total} grains), directory sharded by ring owner, RCCL all-to-all-v"


def usable_cores() -> int:
    """CPUs this process may actually run on: the affinity set, capped by a cgroup v2 CPU quota.
    (os.cpu_count() reports the whole host -- 256 on the GPU box -- not the job's share.)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _timed(fn, budget: float, unit: int):
    """Repeat fn() (each call = `unit` messages) for about `budget` seconds: (messages/s, messages)."""
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += unit
        if time.perf_counter() - t0 >= budget:
            break
    return done / (time.perf_counter() - t0), done


def cpu_baseline(args, tcd, G_total, pts, own, owner):
    """The C restatement (oracle/cpu_ref.c, test infrastructure) timed on this host's cores, on
    bounded samples of the bench workload: route (ring + directory probe) + per-activation bucketing
    of the same messages.  faithful = the reference's data structures (linear ring scan under
    lock(membershipCache), chained Dictionary under lock(lockable), per-activation FIFO append on the
    single IncomingMessageAgent thread); fast = binary search, open addressing, parallel counting
    sort.  `value` is the strongest CPU configuration measured (fast, all usable cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref  # test-infrastructure checker, timed here as the CPU baseline only

    cores = usable_cores()
    host = os.cpu_count() or 1
    budget = args.cpu_seconds / 6
    sample = 1 << 22
    rng = np.random.default_rng(0x5EED0001)
    keys = grain_keys(tcd, rng.integers(0, G_total, size=sample, dtype=np.int64))
    all_keys = grain_keys(tcd, np.arange(G_total, dtype=np.int64))
    res = {}
    runs = [("faithful_1", True, 1, 1), ("faithful_n", True, cores, 1), ("fast_1", False, 1, 1),
            ("fast_n", False, cores, cores)]
    if host != cores:
        runs.append(("fast_host", False, host, host))
    dirs = {}
    for label, faithful, thr_route, thr_bucket in runs:
        d = dirs.get(faithful)
        if d is None:
            d = dirs[faithful] = cpu_ref.CpuDirectory(faithful, G_total)
            d.register(all_keys, np.arange(G_total, dtype=np.uint32), owner)

        def one(d=d, faithful=faithful, thr_route=thr_route, thr_bucket=thr_bucket):
            st, silo, act = d.route(args.mode, pts, own, keys, nthreads=thr_route)
            cpu_ref.bucket(act, G_total, faithful=faithful, nthreads=thr_bucket)
        v, done = _timed(one, budget, sample)
        res[label] = {"value": round(v, 1), "route_threads": thr_route, "bucket_threads": thr_bucket,
                      "messages": done}
    dirs.clear()
    # BASELINE cfg 1's shape (PingBenchmark: 1M calls over 10k grains, one silo), same restatement
    G1, N1 = 10_000, 1 << 20
    k1 = grain_keys(tcd, np.random.default_rng(0x5EED0101).integers(0, G1, size=N1, dtype=np.int64))
    reg1 = grain_keys(tcd, np.arange(G1, dtype=np.int64))
    cfg1 = {}
    for label, faithful, thr in (("faithful_1", True, 1), ("fast_n", False, cores)):
        d = cpu_ref.CpuDirectory(faithful, G1)
        d.register(reg1, np.arange(G1, dtype=np.uint32), np.zeros(G1, np.uint32))

        def one1(d=d, faithful=faithful, thr=thr):
            _, _, act = d.route("D", np.zeros(1, np.uint32), np.zeros(1, np.uint32), k1, nthreads=thr)
            cpu_ref.bucket(act, G1, faithful=faithful, nthreads=thr)
        v, done = _timed(one1, budget / 2, N1)
        cfg1[label] = {"value": round(v, 1), "threads": thr, "messages": done}
        del d
    # BASELINE cfg 5's latency path: one 4096-message micro-batch, faithful, single thread
    d = cpu_ref.CpuDirectory(True, G_total)
    d.register(all_keys, np.arange(G_total, dtype=np.uint32), owner)
    runs = cpu_ref.BucketRuns(G_total, 4096)
    lat = []
    t_end = time.perf_counter() + budget / 2
    i = 0
    while time.perf_counter() < t_end or len(lat) < 50:
        kb = np.ascontiguousarray(keys[(i * 4096) % sample:(i * 4096) % sample + 4096])
        t0 = time.perf_counter()
        _, _, act = d.route(args.mode, pts, own, kb, nthreads=1)
        runs(act)
        lat.append(time.perf_counter() - t0)
        i += 1
    del d
    lat_us = np.asarray(lat) * 1e6
    best = res["fast_n"]
    return {"value": best["value"], "unit": "messages/s", "cores": cores, "kind": "port", "mode": "fast_n",
            "sample": f"{best['messages']} messages (cfg2 distribution, {sample}-message batches repeated) through "
                      f"the C restatement (oracle/cpu_ref.c) in fast mode (binary-search ring, open addressing, "
                      f"parallel two-level stable partition) on {cores} threads = this job's usable cores "
                      f"(affinity + cgroup quota; os.cpu_count() = {host})",
            "modes": res, "host_cpus": host,
            "cfg1_ping_shape": cfg1,
            "cfg5_latency_us": {"batch": 4096, "n_batches": len(lat),
                                "mode": "faithful route (linear ring scan + chained map under locks) + per-activation "
                                        "FIFO runs of the batch (cpu_bucket_runs), 1 thread",
                                "p50": round(float(np.percentile(lat_us, 50)), 1),
                                "p99": round(float(np.percentile(lat_us, 99)), 1)}}


def cpu_baseline_cfg3(args, w3, tcd):
    """cfg 3's CPU baseline: the C restatement (oracle/cpu_ref.c, test infrastructure) routing +
    bucketing a bounded prefix of the GPU's own Zipf(1.1) batch.  The CPU directory holds the
    sample's distinct grains only (registering all 100M would take minutes and ~8 GB): a smaller
    table than the GPU's 8.6 GB one, which favours the CPU."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref  # test-infrastructure checker, timed here as the CPU baseline only

    cores = usable_cores()
    sample = 1 << 21
    keys = w3["keys"][:sample].cpu().numpy().view(np.uint64).copy()
    ks = keys[:, 1].astype(np.int64)
    grains = np.unique(ks)
    reg = grain_keys(tcd, grains)
    owner = w3["e"].ring_owner(reg)
    res = {}
    for label, faithful, thr in (("faithful_1", True, 1), ("fast_n", False, cores)):
        d = cpu_ref.CpuDirectory(faithful, len(grains))
        d.register(reg, grains.astype(np.uint32), owner)

        def one(d=d, faithful=faithful, thr=thr):
            _, _, act = d.route(args.mode, w3["pts"], w3["own"], keys, nthreads=thr)
            cpu_ref.bucket(act, w3["n_act"], faithful=faithful, nthreads=thr)
        v, done = _timed(one, args.cpu_seconds / 4, sample)
        res[label] = {"value": round(v, 1), "threads": thr, "messages": done}
        del d
    # the faster mode is the baseline (fast: binary-search ring, open addressing, the parallel two-level
    # partition of cpu_ref.c -- O(n + n_act) work over all threads)
    label = max(res, key=lambda k: res[k]["value"])
    best = res[label]
    return {"value": best["value"], "unit": "messages/s", "cores": best["threads"], "kind": "port",
            "mode": label,
            "sample": f"{best['messages']} messages (the first {sample} of the GPU's Zipf(1.1) batch, repeated; "
                      f"{len(grains)} distinct grains registered on the CPU of the 100M) through the C restatement "
                      f"in {'faithful' if label.startswith('faithful') else 'fast'} mode on {best['threads']} "
                      f"thread(s), the faster of the two modes", "modes": res, "usable_cores": cores}


# ---- BASELINE cfg 4: Chirper-style follower fan-out cascade -------------------------------------

def fan_kernel_bytes(name, msgs, n_front, keep_target):
    """Algorithmic HBM bytes over all launches of a cfg 4 expansion / route kernel in one cascade
    (DESIGN.md 5.3); the bucketing kernels follow bucket_bytes per hop."""
    if name == "k_fan_route":
        # dst read 4 + one slot 32 + sender/silo/act 12 + status 1 (+ target 4); per publisher 16
        return msgs * (49 + (4 if keep_target else 0)) + n_front * 16
    if name == "k_route_nodes":
        return msgs * (4 + 32 + 9)
    if name == "k_fan_expand":
        return msgs * (4 + 8) + n_front * 16
    return 0.0


def hop_form(e, m: int, n_act: int) -> str:
    """The bucketing form the library keeps for m messages over n_act activations (gd_tune_get,
    GD_TUNE_BUCKET; the two-level forms only from 2^20 messages)."""
    if m < (1 << 20):
        return "lsd"
    q, sub = m // ((n_act >> 10) + 1), 0
    while sub < 31 and (q >> sub) > 1:
        sub += 1
    v = e.tune_get("bucket", m, sub)
    if v != 1:
        return "lsd"
    return "msd" if (n_act >> 10) + 1 <= 1056 else "msd3"


def run_cfg4(args, world, rank, local, dev):
    """--workload cfg4: the cascade line (measure_cfg4) printed on rank 0."""
    line = measure_cfg4(args, world, rank, local, dev, args.steps, args.warmup, args.profile_steps,
                        with_cpu=not args.no_cpu_baseline)
    if rank == 0:
        line["bench_wall_s"] = round(time.perf_counter() - T_START, 1)
        emit(line, args)
    dist.destroy_process_group()


def measure_cfg4(args, world, rank, local, dev, steps, warmup, profile_steps, with_cpu):
    """One step = one whole cascade: `--hops` publish rounds from `--seeds` publishers, each round =
    expand the frontier's follower lists (ChirperAccount.cs:131-134) -> route every NewChirp (ring
    owner + directory probe) -> bucket per activation -> next frontier.  Value = messages routed
    (all hops, all ranks) / max-over-ranks wall time of the cascade, graph and directory resident in
    HBM.  N = 1: fused expand+route kernel (k_fan_route) per hop.  N > 1: directory sharded by ring
    owner, (target, sender) pairs exchanged with one grouped RCCL send/recv round per hop inside the
    library (gd_fanout_multi_device, LibraryFanout)."""
    from orleans_amd.fanout import (CHIRPER_ACCOUNT_CLASS, DeviceFanoutEngine, LibraryCascade, LibraryFanout,
                                    partition_graph_np, upload_graph)
    from orleans_amd.workloads import power_law_graph

    t_setup = time.perf_counter()
    n = args.nodes
    ro, dst = power_law_graph(n, args.mean_deg, seed=0x5EED0004, max_deg=args.max_deg)
    tc = g.calculate_id_hash(CHIRPER_ACCOUNT_CLASS)
    tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
    # directory: node u = GrainId(tc, u), activation u, on its owner silo; this rank keeps the
    # grains whose owner silo it hosts
    keys = grain_keys(tcd, np.arange(n, dtype=np.int64))
    e = g.GrainDispatch(device=local, table_capacity=1 << int(np.ceil(np.log2(2 * n / world + 1))),
                        my_silo=rank % 8)
    pin_choices(e, args, "cfg4")
    pts, own = e.ring_set_silos(args.mode, SILO_SETS[args.silos])
    owner = e.ring_owner(keys)
    mine = np.nonzero(owner % world == rank)[0]
    # N > 1 (or --exchange library at N = 1: the same path over a one-rank RCCL communicator): the
    # follower graph is partitioned (gd_fanout_multi_part_device), this rank keeps the rows of the
    # grains it owns, row i = activation i (ascending node ids); else node u = activation u
    sharded = world > 1 or args.exchange == "library"
    e.register(keys[mine], (np.arange(mine.size) if sharded else mine).astype(np.uint32), owner[mine])
    del keys
    eng = DeviceFanoutEngine(e, dev, tc, keep_target=not args.no_target)
    node_of = None
    n_act = n
    if sharded:
        ro_l, dst_l, no = partition_graph_np(ro, dst, mine)
        graph = upload_graph(ro_l, dst_l, dev)
        node_of = torch.from_numpy(no.view(np.int32) if no.size else np.zeros(1, np.int32)).to(dev)
        n_act = int(mine.size)
        graph_edges_rank = int(dst_l.size)
        del ro_l, dst_l, no
    else:
        graph = upload_graph(ro, dst, dev)
        graph_edges_rank = int(dst.size)
    seeds = np.random.default_rng(0x5EED0004).choice(n, size=args.seeds, replace=False).astype(np.uint32)
    t_seeds = torch.from_numpy(seeds.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    # N > 1: the sharded cascade inside the library (gd_fanout_multi_device), bit-exact against
    # oracle/fanout.py in tests/test_gpu_fanout_multi.py (W = 8 and 3 in process)
    assert not (world > 1 and args.rehearse_one_gpu), "cfg4 at N > 1 runs the library's RCCL cascade only"
    # N = 1: the whole cascade inside the library (gd_fanout_cascade_device, one read-back a hop)
    runner = LibraryFanout(eng, graph, n_act, node_of=node_of) if sharded else LibraryCascade(eng, graph, n)
    exchange = "none" if not sharded else ("libgraindispatch gd_fanout_multi_part_device (partitioned follower "
                                           "graph; grouped RCCL send/recv of (target, sender) per hop)")

    def step():
        return runner.run(t_seeds, args.hops)

    for _ in range(settle_steps(args)):              # cascades: the measured choices per hop size (3 fan-out
        #                                              probe variants x 2 launches each, then the pick)
        step()
    if world > 1 and args.tune == "measured" and runner is not None and isinstance(runner, LibraryFanout):
        torch.cuda.synchronize()
        try:
            e.tune_agree()
        except Exception as ex:   # noqa: BLE001 -- speed only: every rank keeps its own choices
            print(f"gd_tune_agree failed: {ex!r}", file=sys.stderr, flush=True)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    msgs_local = 0
    for _ in range(steps):
        hops = step()
        msgs_local += sum(h.messages for h in hops)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0                  # this rank's steps; the max over ranks below
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([wall, msgs_local], dtype=torch.float64)
    tw, ts = t.clone(), t.clone()
    dist.all_reduce(tw, op=dist.ReduceOp.MAX)
    dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    wall_max, msgs_total = float(tw[0]), float(ts[1])
    hop_msgs = [h.messages for h in hops]
    hop_front = [h.n_frontier if hasattr(h, "n_frontier") else int(h.frontier.shape[0]) for h in hops]

    kernels, roofline = {}, None
    if profile_steps > 0:
        hop_acts = ([f["act"] for f in runner.fetch(hops)] if isinstance(runner, LibraryCascade)
                    else [None for _ in hops])
        kt = {}
        for mode in (1, 2):        # every launch, then the stages alone ("stage:bucket")
            e.set_kernel_timing(mode)
            e.kernel_times_reset()
            for _ in range(profile_steps):
                step()
            torch.cuda.synchronize()
            t = e.kernel_times()
            kt.update(t if mode == 1 else {k: v for k, v in t.items() if k.startswith("stage:")})
        e.set_kernel_timing(False)
        msgs_step = sum(hop_msgs)

        fan_scan = {"k_fan_degree": 16.0 * sum(hop_front), "k_scan_down": 8.0 * sum(hop_front)}

        def cfg4_bytes(name, _form):
            if name in ("k_fan_route", "k_route_nodes", "k_fan_expand"):
                return fan_kernel_bytes(name, msgs_step, sum(hop_front), not args.no_target)
            # each hop's publishers: their degrees (frontier 4 B, two row offsets 8 B, the degree 4 B),
            # then the degrees' inclusive scan (read + write 8 B); the grids cover the frontier's bound
            # (min(n_act, the previous hop's messages)), the bytes count the publishers
            fan = fan_scan.get(name, 0.0)
            # the bucketing kernels: each hop's batch in the form the library keeps for its shape
            return fan + float(sum(bucket_bytes(hop_form(e, m, n_act), m, n_act, a).get(name, 0.0)
                                   for m, a in zip(hop_msgs, hop_acts) if m))
        kernels, roofline = roofline_of(kt, profile_steps, msgs_step, n_act, None, "cfg4", world,
                                        bytes_fn=cfg4_bytes, nonstage=fan_scan)
        if roofline:
            roofline["hop_bucket_forms"] = [hop_form(e, m, n_act) for m in hop_msgs]
            if roofline.get("kernel") == "k_fan_route" and world == 1:
                pc = probe_ceiling("cfg4", msgs_step / roofline["launches_per_step"], roofline["avg_launch_ms"])
                if pc:
                    roofline["random_probe_ceiling"] = pc
                fb = fan_bound(e, step, profile_steps)
                if fb:
                    roofline["fan_bound"] = fb

    cpu = None
    if rank == 0 and world == 1 and with_cpu and isinstance(runner, LibraryCascade):
        cpu = cpu_baseline_cfg4(args, runner.fetch(hops)[-1]["target"], tcd, owner, pts, own, n)

    line = {
            "metric": "routed messages/sec (fan-out cascade: expand+lookup+bucket, whole node)",
            "value": round(msgs_total / wall_max, 1), "unit": "messages/s", "n_gpus": world,
            "steps": steps, "warmup": warmup,
            "ms_per_step": round(wall_max / steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u32/u64 integer",
            "data": f"synthetic power-law follower graph (alpha 2.5, mean {args.mean_deg}, cap {args.max_deg}), "
                    f"seed 0x5EED0004",
            "config": {"workload": f"cfg4: {n} grains, {int(ro[-1])} follower edges, {args.seeds} seeds, "
                                   f"{args.hops} hops", "ring_mode": args.mode,
                       "silos": silos_note(args.silos),
                       "parallelism": f"shard{world}" + ("-rehearsal" if args.rehearse_one_gpu else "")},
            "comm": e.comm_info(),
            "messages_per_step": int(msgs_total / steps), "hop_messages_rank0": hop_msgs,
            "hop_publishers_rank0": hop_front, "setup_s": round(setup_s, 1), "exchange": exchange,
            "graph_edges_rank0": graph_edges_rank, "graph_edges_total": int(dst.size),
            "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
        }
    e.close()
    del graph, eng
    torch.cuda.empty_cache()
    return line


def cpu_baseline_cfg4(args, t, tcd, owner, pts, own, n):
    """cfg 4's CPU baseline: the C restatement (oracle/cpu_ref.c, test infrastructure) routing +
    bucketing a bounded sample of the cascade's last hop, in faithful mode on 1 thread and fast mode
    on all usable cores; the faster is the baseline.  The follower expansion itself is a numpy gather
    and is not timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref  # test-infrastructure checker, timed here as the CPU baseline only
    t = np.asarray(t, dtype=np.uint32)                 # the last hop's targets
    sample = min(t.size, 1 << 21)
    keys = grain_keys(tcd, t[:sample].astype(np.int64))
    cores = usable_cores()
    reg = grain_keys(tcd, np.arange(n, dtype=np.int64))
    res = {}
    for label, faithful, thr in (("faithful_1", True, 1), ("fast_n", False, cores)):
        d = cpu_ref.CpuDirectory(faithful, n)
        d.register(reg, np.arange(n, dtype=np.uint32), owner)

        def one(d=d, faithful=faithful, thr=thr):
            _, _, act = d.route(args.mode, pts, own, keys, nthreads=thr)
            cpu_ref.bucket(act, n, faithful=faithful, nthreads=thr)
        v, done = _timed(one, args.cpu_seconds / 4, sample)
        res[label] = {"value": round(v, 1), "threads": thr, "messages": done}
        del d
    label = max(res, key=lambda k: res[k]["value"])
    best = res[label]
    return {"value": best["value"], "unit": "messages/s", "cores": best["threads"], "kind": "port", "mode": label,
            "sample": f"{best['messages']} NewChirp messages ({sample}-message prefix of the last hop, repeated) "
                      f"through the C restatement in {'faithful' if label.startswith('faithful') else 'fast'} mode "
                      f"on {best['threads']} thread(s), the faster of the two modes", "modes": res,
            "usable_cores": cores}


if __name__ == "__main__":
    main()
