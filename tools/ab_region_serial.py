"""Serialized (no pipelining) world-1 gd_route_multi_device at cfg 2's shape: per-kernel times
with the probe running alone on the GPU, GD_REGION_PROBE from the environment.
  GD_REGION_PROBE=1 python tools/ab_region_serial.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from orleans_amd import graindispatch as g  # noqa: E402
import oracle as o  # noqa: E402

G, N = 1 << 20, 1 << 24
tc = o.grain_type_code(o.PING_GRAIN_CLASS)
silos = o.bench_silos(8)
e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0, kernel_timing=False)
e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
reg = o.grain_keys(tc, np.arange(G))
e.register(reg, np.arange(G), np.zeros(G, np.uint32))
keys = torch.from_numpy(o.grain_keys(tc, np.random.default_rng(1).integers(0, G, size=N)).view(np.int64)).cuda()
e.comm_init(g.GrainDispatch.comm_unique_id(), 1, 0)
s = torch.cuda.Stream()
e.set_stream(s.cuda_stream)
torch.cuda.synchronize()
for i in range(25):
    if i == 5:
        e.set_kernel_timing(True)
        t0 = time.perf_counter()
    with torch.cuda.stream(s):
        e.route_multi_device(keys.data_ptr(), N, G, keys_ready=True, no_keys=True)
    e.synchronize()
dt = (time.perf_counter() - t0) / 20
kt = e.kernel_times()
print("GD_REGION_PROBE=%s serial ms/call %.4f" % (os.environ.get("GD_REGION_PROBE", "default"), dt * 1e3),
      {k: round(v[1] / 20, 4) for k, v in kt.items()})
e.comm_destroy()
e.close()
