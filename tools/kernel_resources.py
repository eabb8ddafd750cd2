#!/usr/bin/env python3
"""Per-kernel resources and occupancy from a rocprofv3 kernel_trace.csv, plus the measured mean
resident waves from a pmc_summary.json (SQ_WAVE_CYCLES over the kernel's duration).

    python tools/kernel_resources.py TRACE.csv [PMC_SUMMARY.json] > profiles/rNN_kernel_resources.txt

Theoretical waves per SIMD = min(8, VGPR limit (MI355X_MICROARCH.md register table: allocation
granule 8, 512 per lane), LDS limit (160 KiB per CU), workgroup slots).  Measured: SQ_WAVE_CYCLES /
(duration cycles x 256 CUs x 4 SIMDs), the duration in cycles taken as GRBM_GUI_ACTIVE / 8 (the
counter sums the 8 XCDs) and SQ_WAVE_CYCLES in its 4-cycle unit (CDNA SQ cycle counters); an
estimate, labelled as such.
"""
import csv
import json
import sys
from collections import defaultdict


def vgpr_waves(v):
    alloc = -(-max(v, 1) // 8) * 8
    return min(8, 512 // alloc)


def main():
    rows = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        rows[r["Kernel_Name"]].append(r)
    pmc = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else {}
    print(f"{'kernel':60s} {'calls':>5s} {'avg_us':>8s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'LDS_B':>7s} "
          f"{'WG':>5s} {'waves/SIMD(theory)':>18s} {'waves/SIMD(meas)':>16s}")
    for name, rs in sorted(rows.items(), key=lambda kv: -sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
                                                               for x in kv[1])):
        if "gd::" not in name:
            continue
        r = rs[0]
        dur = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in rs) / len(rs) / 1e3
        v = int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"])
        lds = int(r["LDS_Block_Size"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        wpg = -(-wg // 64)
        by_v = vgpr_waves(v)
        by_lds = (160 * 1024 // lds) * wpg / 4 if lds else 8
        theory = min(by_v, by_lds, 32 // 4)
        short = name.replace("void ", "")
        short = short[: short.index("(")] if "(" in short else short
        meas = ""
        p = pmc.get(short)
        if p and p.get("SQ_WAVE_CYCLES") and p.get("GRBM_GUI_ACTIVE"):
            meas = f"{4 * p['SQ_WAVE_CYCLES'] / (p['GRBM_GUI_ACTIVE'] / 8 * 256 * 4):.2f}"
        print(f"{short[:60]:60s} {len(rs):5d} {dur:8.1f} {r['VGPR_Count']:>5s} {r['Accum_VGPR_Count']:>5s} "
              f"{r['SGPR_Count']:>5s} {lds:7d} {wg:5d} {theory:18.2f} {meas:>16s}")


if __name__ == "__main__":
    main()
