#!/usr/bin/env python3
"""Per-kernel times of the library exchange path at world 1 (gd_route_multi_device), its batches NOT
overlapped (keys_ready off), so each kernel's events measure it alone: the partition's own cost beside
the probe and the bucketing it precedes.  BASELINE cfg 2's shape (16M messages over 1M grains).

    python tools/exchange_kernels.py [steps]"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o                                         # noqa: E402
from orleans_amd import graindispatch as g                 # noqa: E402
from orleans_amd.sharded import DeviceEngine, LibraryRouter  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29573")
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    G, N = 1 << 20, 1 << 24
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    for kind, v in (("probe_keys", 3), ("probe_n1", 3), ("bucket", 1)):
        e.tune_set(kind, v)
    reg = o.grain_keys(tc, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg, np.arange(G), own)
    keys = torch.from_numpy(o.grain_keys(tc, np.random.default_rng(1).integers(0, G, N)).view(np.int64)).to(dev)
    eng = DeviceEngine(e, dev)
    lr = LibraryRouter(eng)
    lr.no_keys = True
    with torch.cuda.stream(eng.stream):
        for _ in range(3):
            lr.route_bucket(keys, G, keys_ready=False)
        torch.cuda.synchronize()
        e.set_kernel_timing(1)
        e.kernel_times_reset()
        for _ in range(steps):
            lr.route_bucket(keys, G, keys_ready=False)
        torch.cuda.synchronize()
        kt = e.kernel_times()
        e.set_kernel_timing(0)
    tot = 0.0
    for name, (launches, ms) in sorted(kt.items(), key=lambda x: -x[1][1]):
        print(f"{name:24s} {ms / steps:8.4f} ms a step  ({launches // steps} launches)")
        tot += ms / steps
    print(f"{'sum':24s} {tot:8.4f} ms a step")
    lr.close()
    e.close()


if __name__ == "__main__":
    main()
