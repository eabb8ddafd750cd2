#!/usr/bin/env python3
"""HBM traffic per launch of the bench's dominant kernels from a pmc_summary.json (tools/pmc_summary.py),
corrected as MI355X_MICROARCH.md §HBM prescribes, written to profiles/pmc_<kernel>.json for bench.py's
roofline `traffic` field.

    python tools/pmc_traffic.py PMC_SUMMARY.json SOURCE_TAG N_MESSAGES

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
    fam = {}
    for name, row in summ.items():
        base = name.split("<")[0].replace("gd::", "")
        if "rd_bytes_ea" not in row or "wr_bytes_ea" not in row:
            continue
        fam.setdefault(base, []).append((name, row))
    out = {}
    for base, members in fam.items():
        if base not in ("k_route_m", "k_radix_scatter", "k_radix_hist", "k_radix_hist_multi", "k_route_hist"):
            continue
        rd_raw = sum(r["rd_bytes_ea"] for _, r in members) / len(members)
        wr = sum(r["wr_bytes_ea"] for _, r in members) / len(members)
        if base in ("k_route_m", "k_route_hist"):
            rd = rd_raw + 24 * n / 2
            how = "random slot probes as issued (64-B requests) + the 24-B/message key stream added back at half"
        else:
            rd = 2 * rd_raw
            how = "streamed reads doubled (gfx950 tallies a wide coalesced read at half its bytes)"
        key = "k_route" if base == "k_route_m" else ("k_radix_hist" if base.startswith("k_radix_hist") else base)
        out[key] = {"kernel": key, "instantiations": [m for m, _ in members],
                    "hbm_bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                    "raw_read_bytes_per_launch": rd_raw, "source": tag,
                    "method": "EA request counts x request size, separate --pmc passes; " + how +
                              "; averaged over the instantiations (one per radix pass kind)"}
    for key, v in out.items():
        with open(f"profiles/pmc_{key}.json", "w") as f:
            json.dump(v, f, indent=1)
        print(key, round(v["hbm_bytes_per_launch"] / 1e6, 1), "MB/launch")


if __name__ == "__main__":
    main()
