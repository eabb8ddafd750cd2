#!/usr/bin/env python3
"""BASELINE cfg 1's shape (1M calls over 10k grains, one silo) through gd_route_bucket_device, the same
loop as bench.py's ping_shape, for a kernel trace (rocprofv3 --kernel-trace -- python3 tools/ping_steps.py)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o                                         # noqa: E402
from orleans_amd import graindispatch as g                 # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda:0")
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    G, N = 10_000, 1 << 20
    e = g.GrainDispatch(device=0, table_capacity=1 << 15, my_silo=0)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in o.bench_silos(1)])
    reg = o.grain_keys(tc, np.arange(G))
    e.register(reg, np.arange(G, dtype=np.uint32), np.zeros(G, np.uint32))
    keys = torch.from_numpy(o.grain_keys(tc, np.random.default_rng(1).integers(0, G, N)).view(np.int64)).to(dev)
    out = [torch.empty(N, dtype=torch.int32, device=dev) for _ in range(2)] + [torch.empty(N, dtype=torch.uint8, device=dev)]
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    off = torch.empty(G + 2, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    e.set_stream(s.cuda_stream)

    def one():
        e.route_bucket_device(keys.data_ptr(), N, G, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                              perm.data_ptr(), off.data_ptr())
    for _ in range(10):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / steps * 1e6:.1f} us a step; bucket variant {e.tune_get('bucket', N, 0)}")
    e.close()


if __name__ == "__main__":
    main()
