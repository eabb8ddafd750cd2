"""W = 2 in-process exchange (gd_comm_init_local, one GPU) at cfg 2's per-rank shape, serialized
calls: per-kernel times with GD_IDX16 from the environment (2-B vs 4-B origin indices).  The
transport is device-to-device copies, so this prices the kernels, not xGMI.
  GD_IDX16=1 python tools/ab_idx16_local.py"""
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from orleans_amd import graindispatch as g  # noqa: E402
import oracle as o  # noqa: E402

W, G, N = 2, 1 << 20, 1 << 23
tc = o.grain_type_code(o.PING_GRAIN_CLASS)
silos = o.bench_silos(8)
spec = o.ring_spec(silos, "D")
reg = o.grain_keys(tc, np.arange(G * W))
own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
es, keys, streams = [], [], []
for r in range(W):
    e = g.GrainDispatch(device=0, table_capacity=4 * G, my_silo=r, kernel_timing=False)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    mine = own % W == r
    e.register(reg[mine], np.arange(int(mine.sum())), own[mine])
    es.append(e)
    keys.append(torch.from_numpy(o.grain_keys(tc, np.random.default_rng(r).integers(0, G * W, size=N))
                                 .view(np.int64)).cuda())
    streams.append(torch.cuda.Stream())
    e.set_stream(streams[-1].cuda_stream)
g.GrainDispatch.comm_init_local(es)
n_act = [int((own % W == r).sum()) for r in range(W)]
torch.cuda.synchronize()


def rank(r, i):
    with torch.cuda.stream(streams[r]):
        es[r].route_multi_device(keys[r].data_ptr(), N, n_act[r], keys_ready=True, no_keys=True)
    es[r].synchronize()


for i in range(25):
    if i == 5:
        for e in es:
            e.set_kernel_timing(True)
        t0 = time.perf_counter()
    ts = [threading.Thread(target=rank, args=(r, i)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
dt = (time.perf_counter() - t0) / 20
kt = es[0].kernel_times()
print("GD_IDX16=%s W=%d serial ms/call %.4f" % (os.environ.get("GD_IDX16", "default"), W, dt * 1e3),
      {k: round(v[1] / 20, 4) for k, v in kt.items()})
for e in es:
    e.comm_destroy()
    e.close()
