"""A/B the k_route variants (messages per thread, non-temporal streams) in ONE
process, interleaved rounds (cdna_hip_programming.md rule 24), on the cfg2
workload.  Also checks every variant gives identical results."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g  # noqa: E402

VARIANTS = [(1, 0), (2, 0), (4, 0), (1, 1), (2, 1), (4, 1)]


def main():
    G, N = 1 << 20, 1 << 24
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    silos = [(f"10.0.0.{i + 1}", 11111, 1) for i in range(8)]
    tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
    tcd = (3 << 56) + (tc & 0x00FFFFFFFFFFFFFF)
    keys_h = np.zeros((G, 3), dtype=np.uint64)
    keys_h[:, 1] = np.arange(G, dtype=np.uint64)
    keys_h[:, 2] = np.uint64(tcd)
    ks = np.random.default_rng(0x5EED0001).integers(0, G, size=N)
    msgs = torch.from_numpy(keys_h[ks].view(np.int64)).to(dev)
    stream = torch.cuda.Stream(dev)
    handles = {}
    for m, nt in VARIANTS:
        os.environ["GD_ROUTE_M"], os.environ["GD_ROUTE_NT"] = str(m), str(nt)
        e = g.GrainDispatch(device=0, table_capacity=2 * G)
        pts, own = e.ring_set_silos("D", silos)
        owner = e.ring_owner(keys_h)
        e.register(keys_h, np.arange(G, dtype=np.uint32), owner)
        e.set_stream(stream.cuda_stream)
        handles[(m, nt)] = e
    outs = {k: (torch.empty(N, dtype=torch.int32, device=dev), torch.empty(N, dtype=torch.int32, device=dev),
                torch.empty(N, dtype=torch.uint8, device=dev)) for k in handles}
    times = {k: [] for k in handles}
    reps = 10
    with torch.cuda.stream(stream):
        for r in range(rounds + 1):
            for k, e in handles.items():
                s, a, st = outs[k]
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record(stream)
                for _ in range(reps):
                    e.route_device(msgs.data_ptr(), N, s.data_ptr(), a.data_ptr(), st.data_ptr())
                ev1.record(stream)
                ev1.synchronize()
                if r > 0:
                    times[k].append(ev0.elapsed_time(ev1) / reps)
    ref = outs[VARIANTS[0]]
    for k in handles:
        ok = all(torch.equal(x, y) for x, y in zip(outs[k], ref))
        t = np.array(times[k])
        gbs = N * 65 / (np.median(t) * 1e-3) / 1e9
        print(f"route M={k[0]} nt={k[1]}: median {np.median(t):.4f} ms min {t.min():.4f} ms "
              f"-> {N / np.median(t) / 1e6:.2f} G msg/s, {gbs:.0f} GB/s alg, identical={ok}", flush=True)


if __name__ == "__main__":
    main()
