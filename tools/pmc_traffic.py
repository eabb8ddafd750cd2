#!/usr/bin/env python3
"""HBM traffic per launch of the bench's dominant kernels from a pmc_summary.json (tools/pmc_summary.py),
corrected as MI355X_MICROARCH.md §HBM prescribes, written to profiles/pmc_<kernel>.json for bench.py's
roofline `traffic` field.

    python tools/pmc_traffic.py PMC_SUMMARY.json SOURCE_TAG N_MESSAGES [KERNEL_STATS.csv]

Counters: TCC_EA0_RDREQ[_32B]_sum x 64 B (32 B), TCC_EA0_WRREQ[_64B]_sum x 64 B (else 32 B), collected in
separate passes.  gfx950: a wide coalesced streaming read is tallied at half its bytes, so streamed
reads are doubled; k_route's random 32-B slot probes each move one 64-B request and are counted as
issued, so only its 24-B/message key stream is added back at half.  Writes are counted as issued.
"""
import json
import sys


def main():
    summ = json.load(open(sys.argv[1]))
    tag, n = sys.argv[2], int(sys.argv[3])
    calls = {}
    if len(sys.argv) > 4:                      # rocprof kernel_stats.csv: calls per instantiation
        import csv
        for r in csv.DictReader(open(sys.argv[4])):
            nm = r["Name"].split("(")[0].replace("void ", "").replace("gd::", "")
            calls[nm] = calls.get(nm, 0) + int(r["Calls"])
    # the bucketing form the library kept (its first launches time both): the two-level form
    # (k_b2_hist / k_b2_scatter / k_msd_local, gd_msd.h) or the LSD passes (k_radix_*)
    msd_calls = sum(v for k, v in calls.items() if k.startswith("k_msd_local"))
    lsd_calls = max([v for k, v in calls.items() if k.startswith("k_radix_scatter<") and ", true," in k] or [0])
    msd = msd_calls > lsd_calls if calls else any(k.startswith("gd::k_msd_local") for k in summ)
    lsd_fams = ("k_radix_scatter", "k_radix_hist", "k_radix_hist_multi", "k_radix_hist16")
    msd_fams = {"k_b2_scatter": "k_radix_scatter", "k_b2_hist": "k_radix_hist", "k_msd_local": "k_msd_local"}
    fam = {}
    for name, row in summ.items():
        base = name.split("<")[0].replace("gd::", "")
        if "rd_bytes_ea" not in row or "wr_bytes_ea" not in row:
            continue
        if base in ("k_route_m", "k_route_hist"):
            key = "k_route" if base == "k_route_m" else base
        elif not msd and base in lsd_fams:
            key = "k_radix_hist" if base.startswith("k_radix_hist") else base
        elif msd and base in msd_fams:
            key = msd_fams[base]
        else:
            continue
        # the route's probe variants (index group reads / directory / index slot reads) are each timed on
        # a few launches before the library keeps one: with the kernel-trace stats (4th argument) count
        # the steady-state one only, the instantiation with the most calls
        if key == "k_route" and calls:
            mine = calls.get(name.replace("void ", "").replace("gd::", ""), 0)
            if mine < max(v for k, v in calls.items() if k.startswith("k_route_m<")):
                continue
        # launches per cfg 2 step (3 LSD passes): the first pass's scatter (FIRST = true) and
        # histogram (32-bit keys) once, the later passes' instantiations twice; the two-level form
        # launches each of its kernels once
        w = 1.0
        if not msd and key == "k_radix_scatter" and ", false," in name:
            w = 2.0
        if not msd and base == "k_radix_hist16":
            w = 2.0
        fam.setdefault(key, []).append((name, row, w))
    out = {}
    for key, members in fam.items():
        wsum = sum(w for _, _, w in members)
        rd_raw = sum(r["rd_bytes_ea"] * w for _, r, w in members) / wsum
        wr = sum(r["wr_bytes_ea"] * w for _, r, w in members) / wsum
        if key == "k_route" or key == "k_route_hist":
            rd = rd_raw + 24 * n / 2
            how = "random slot probes as issued (64-B requests) + the 24-B/message key stream added back at half"
        else:
            rd = 2 * rd_raw
            how = "streamed reads doubled (gfx950 tallies a wide coalesced read at half its bytes)"
        out[key] = {"kernel": key, "instantiations": [m for m, _, _ in members],
                    "hbm_bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                    "raw_read_bytes_per_launch": rd_raw, "source": tag,
                    "method": "EA request counts x request size, separate --pmc passes; " + how +
                              "; averaged over the instantiations weighted by their launches per cfg 2 step "
                              "(LSD: first radix pass once, later passes twice; two-level form: once each)",
                    "bucketing_form": "msd" if msd else "lsd"}
    for key, v in out.items():
        with open(f"profiles/pmc_{key}.json", "w") as f:
            json.dump(v, f, indent=1)
        print(key, round(v["hbm_bytes_per_launch"] / 1e6, 1), "MB/launch")


if __name__ == "__main__":
    main()
