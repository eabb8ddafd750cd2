#!/usr/bin/env python3
"""HBM traffic and LDS conflict ratio per launch of every library kernel of one bench workload, from a
pmc_summary.json (tools/pmc_summary.py) and the same command's rocprofv3 kernel_stats.csv, corrected as
MI355X_MICROARCH.md §HBM prescribes; written to profiles/pmc_<workload>_<kernel>.json, where bench.py's
roofline reads its `traffic` (load_pmc).

    python tools/pmc_traffic.py PMC_SUMMARY.json SOURCE_TAG WORKLOAD N_MESSAGES KERNEL_STATS.csv

<kernel> is the library's launch name (the names of bench.py's `kernels`), not the template function:
k_b2_hist / k_radix_hist16 are launched as k_radix_hist, k_b2_scatter as k_radix_scatter,
k_msd_local_list<512, ...> as k_msd_local_mid and <1024, ...> as k_msd_local, k_route_m as k_route.
Instantiations of one launch name are averaged weighted by their calls; instantiations with under a
quarter of the busiest one's calls (variants the tuner timed and dropped) are left out.

Counters: TCC_EA0_RDREQ[_32B]_sum x 64 B (32 B), TCC_EA0_WRREQ[_64B]_sum x 64 B (else 32 B), collected in
separate passes.  gfx950 tallies a wide coalesced streaming read at half its bytes, so streamed reads
are doubled; k_route's random 32-B slot probes each move one 64-B request and are counted as issued,
so only its 24-B/message key stream is added back at half; k_fan_route (CSR and directory gathers) is
reported as issued (a lower bound).  Writes are counted as issued.  LDS: SQ_LDS_BANK_CONFLICT (extra
cycles) / SQ_LDS_IDX_ACTIVE (all LDS-array cycles).
"""
import csv
import json
import os
import sys

RENAME = {"k_b2_hist": "k_radix_hist", "k_radix_hist16": "k_radix_hist", "k_radix_hist_multi": "k_radix_hist",
          "k_b2_scatter": "k_radix_scatter",
          "k_route_m": "k_route", "k_route_region": "k_route", "k_shard_gather": "k_shard_scatter",
          "k_fill_u32": "k_fill", "k_fan_degree_tiles": "k_fan_degree"}
GATHER = ("k_route", "k_fan_route")


def launch_name(inst: str) -> str:
    """gd::k_msd_local_list<512, 16> -> k_msd_local_mid; gd::k_b2_scatter<...> -> k_radix_scatter;
    gd::k_route<MODE, false> (the ring owner alone, gd_ring_owner_device) -> k_ring_owner, not the probe."""
    s = inst.replace("void ", "").replace("gd::", "")
    base = s.split("<")[0]
    if base == "k_msd_local_list":
        return "k_msd_local_mid" if s.split("<")[1].startswith("512") else "k_msd_local"
    if base == "k_route" and "<" in s and s.split("<")[1].split(">")[0].replace(" ", "").endswith(",false"):
        return "k_ring_owner"
    return RENAME.get(base, base)


def short(name: str) -> str:
    name = name.replace("void ", "").replace("gd::", "")
    return name[: name.index("(")] if "(" in name else name


def main():
    summ = json.load(open(sys.argv[1]))
    src, workload, n = sys.argv[2], sys.argv[3], int(sys.argv[4])
    calls = {}
    for r in csv.DictReader(open(sys.argv[5])):
        nm = short(r["Name"])
        calls[nm] = calls.get(nm, 0) + int(r["Calls"])
    fam = {}
    for name, row in summ.items():
        sn = short(name)
        if "rd_bytes_ea" not in row or "wr_bytes_ea" not in row:
            continue
        fam.setdefault(launch_name(sn), []).append((sn, row, calls.get(sn, 0)))
    out = {}
    for key, members in fam.items():
        top = max(c for _, _, c in members)
        members = [m for m in members if m[2] * 4 >= top and m[2] > 0] or members
        wsum = sum(max(c, 1) for _, _, c in members)
        avg = lambda f: sum(f(r) * max(c, 1) for _, r, c in members) / wsum  # noqa: E731
        rd_raw, wr = avg(lambda r: r["rd_bytes_ea"]), avg(lambda r: r["wr_bytes_ea"])
        if key == "k_route":
            rd = rd_raw + 24 * n / 2
            how = "random slot probes as issued (64-B requests) + the 24-B/message key stream added back at half"
        elif key in GATHER:
            rd = rd_raw
            how = "reads as issued (gathers; a lower bound)"
        else:
            rd = 2 * rd_raw
            how = "streamed reads doubled (gfx950 tallies a wide coalesced read at half its bytes)"
        lds = None
        if all("SQ_LDS_IDX_ACTIVE" in r and "SQ_LDS_BANK_CONFLICT" in r for _, r, _ in members):
            act = avg(lambda r: r["SQ_LDS_IDX_ACTIVE"])
            lds = round(avg(lambda r: r["SQ_LDS_BANK_CONFLICT"]) / act, 4) if act else None
        out[key] = {"kernel": key, "workload": workload, "instantiations": [m for m, _, _ in members],
                    "calls": [c for _, _, c in members],
                    "hbm_bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                    "raw_read_bytes_per_launch": rd_raw, "lds_conflict_ratio": lds, "source": src,
                    "method": "EA request counts x request size, separate --pmc passes; " + how +
                              "; instantiations averaged weighted by calls"}
    os.makedirs("profiles", exist_ok=True)
    for key, v in sorted(out.items()):
        with open(f"profiles/pmc_{workload}_{key}.json", "w") as f:
            json.dump(v, f, indent=1)
        print(f"{key:24s} {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  lds_conflicts {v['lds_conflict_ratio']}")


if __name__ == "__main__":
    main()
