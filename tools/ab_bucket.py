"""A/B bucketing variants (env knobs read at gd_create) in ONE process, interleaved
rounds, per-kernel times from the library's HIP events.  Checks all variants agree.

usage: python tools/ab_bucket.py ROUNDS VAR=a,b [VAR=...]
"""
import itertools
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g  # noqa: E402


def zipf_acts(n, a_max, s, rng):
    ranks = np.arange(1, a_max + 1, dtype=np.float64)
    p = ranks ** -s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return np.searchsorted(cdf, rng.random(n)).astype(np.uint32)


def main():
    rounds = int(sys.argv[1])
    knobs = [a.split("=") for a in sys.argv[2:]]
    names = [k for k, _ in knobs]
    combos = list(itertools.product(*[v.split(",") for _, v in knobs]))
    N, A = int(os.environ.get("AB_N", 1 << 24)), int(os.environ.get("AB_A", 1 << 20))
    rng = np.random.default_rng(1)
    dev = torch.device("cuda:0")
    workloads = {"uniform": rng.integers(0, A, size=N).astype(np.uint32),
                 "zipf1.1": zipf_acts(N, A, 1.1, rng)}
    stream = torch.cuda.Stream(dev)
    handles = {}
    for c in combos:
        for k, v in zip(names, c):
            os.environ[k] = v
        e = g.GrainDispatch(device=0, table_capacity=1024, kernel_timing=True)
        e.set_stream(stream.cuda_stream)
        handles[c] = e
    for wname, acts_h in workloads.items():
        acts = torch.from_numpy(acts_h.view(np.int32)).to(dev)
        perm = {c: torch.empty(N, dtype=torch.int32, device=dev) for c in combos}
        off = {c: torch.empty(A + 2, dtype=torch.int32, device=dev) for c in combos}
        tot = {c: [] for c in combos}
        per = {c: {} for c in combos}
        with torch.cuda.stream(stream):
            for r in range(rounds + 1):
                for c, e in handles.items():
                    e.kernel_times_reset()
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record(stream)
                    e.bucket_device(acts.data_ptr(), N, A, perm[c].data_ptr(), off[c].data_ptr())
                    ev1.record(stream)
                    ev1.synchronize()
                    kt = e.kernel_times()
                    if r > 0:
                        tot[c].append(ev0.elapsed_time(ev1))
                        for k, (l, ms) in kt.items():
                            per[c].setdefault(k, []).append(ms)
        ref = combos[0]
        for c in combos:
            same = torch.equal(perm[c], perm[ref]) and torch.equal(off[c], off[ref])
            ks = " ".join(f"{k}={np.median(v):.4f}" for k, v in per[c].items() if np.median(v) > 0.003)
            print(f"[{wname}] {dict(zip(names, c))}: total median {np.median(tot[c]):.4f} ms  identical={same}  {ks}",
                  flush=True)


if __name__ == "__main__":
    main()
