#!/usr/bin/env python3
"""Per-kernel table of a bench full record (bench.py --full-out): main config and secondaries.
   tools/kt.py gpurun_out/r05_vN_full.json [more records ...]"""
import json
import sys

for path in sys.argv[1:]:
    d = json.load(open(path))
    print(f"== {path}: {d['value'] / 1e9:.3f} G/s  {d['ms_per_step']} ms/step")
    blocks = [("main", d)] + [(k, v) for k, v in (d.get("secondary") or {}).items() if isinstance(v, dict) and "kernels" in v]
    for name, b in blocks:
        st = (b.get("roofline") or {}).get("bucketing_stage") or {}
        print(f"  [{name}] value {b.get('value', 0) / 1e9:.3f} G/s ms {b.get('ms_per_step')}  stage {st.get('ms_per_step')} ms")
        for n, v in sorted(b["kernels"].items(), key=lambda x: -x[1]["ms_per_step"]):
            print("    %-22s %7.4f ms x%d frac %-7s pmc %-7s tr %s" % (n, v["ms_per_step"], v["launches_per_step"],
                                                                  v.get("frac_hbm"), v.get("frac_pmc"), v.get("traffic_ratio")))
