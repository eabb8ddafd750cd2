#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 kernel trace (CSV): for the last steady steps of a bench
run, each library kernel's duration and the idle gap before it (end of the previous kernel on the GPU
to this one's start).  tools/trace_gaps.py KERNEL_TRACE.csv [first_kernel_of_step=k_route_m] [steps=3]"""
import csv
import sys


def short(n):
    n = n.replace("void ", "").replace("gd::", "")
    return n[: n.index("(")] if "(" in n else n


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_route_m"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith(first)]
sel = starts[-(steps + 1):]
for a, b in zip(sel[:-1], sel[1:]):
    prev_end = None
    tot_k = tot_g = 0
    print(f"--- step at dispatch {rows[a]['Dispatch_Id']}")
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        tot_k += (e - s) / 1e3
        tot_g += gap
        print(f"  {short(r['Kernel_Name'])[:60]:60s} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f} us")
        prev_end = e
    print(f"  kernels {tot_k:.1f} us, gaps {tot_g:.1f} us")
