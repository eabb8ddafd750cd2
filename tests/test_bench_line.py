"""bench.py's printed line must reach the driver whole: at most LINE_CAP bytes (the driver keeps only
the tail of stdout; round 4's 21.5-KB line with every kernel table inline went unparsed), and it keeps
the contract's fields -- metric, value, ms_per_step, steps, warmup, config, dtype, a roofline with
bound / kernel / achieved / peak / frac / traffic, cpu_baseline with value / cores / kind / sample --
plus the compact secondary summaries.  Checked on the committed full records of rounds 3 to 5 and on
the printed lines of the N = 2 / 8 one-GPU rehearsals."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


RECORDS = ["profiles/r05_v8_bench_full.json", "profiles/r04_v8_bench.json", "profiles/r03_v8_bench.json",
           "profiles/r04_v7_bench.json"]


@pytest.mark.parametrize("path", RECORDS)
def test_line_under_cap_with_contract_fields(bench, path):
    with open(os.path.join(ROOT, path)) as f:
        full = json.load(f)
    line = bench.compact_line(full, "gpurun_out/bench_full.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_CAP, len(text)
    assert "\n" not in text
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    rf = line["roofline"]
    for k in ("bound", "kernel", "achieved", "peak", "unit", "frac"):
        assert k in rf, k
    assert rf["frac"] == full["roofline"]["frac"]
    assert "bucketing_stage" in rf and "weakest_bucketing_kernel" in rf
    cpu = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cpu, k
    for name in ("cfg3", "cfg4"):
        if name in full.get("secondary", {}):
            s = line["secondary"][name]
            assert s["value"] == full["secondary"][name]["value"]
            if full["secondary"][name].get("roofline"):
                assert "frac" in s["roofline"]


def test_line_cap_holds_for_oversized_records(bench):
    """A record with long strings and many kernels still prints under the cap (secondary tables go
    first)."""
    with open(os.path.join(ROOT, RECORDS[0])) as f:
        full = json.load(f)
    full["exchange"] = "x" * 5000
    full["config"]["silos"] = "y" * 5000
    for name in ("cfg3", "cfg4"):
        sec = full["secondary"][name]
        sec["workload"] = "z" * 3000
        for i in range(40):
            sec["kernels"][f"k_extra_{i}"] = dict(sec["kernels"][next(iter(sec["kernels"]))])
    text = json.dumps(bench.compact_line(full, "gpurun_out/bench_full.json"))
    assert len(text) <= bench.LINE_CAP, len(text)


@pytest.mark.parametrize("rnd", ["r05", "r06"])
@pytest.mark.parametrize("world", [2, 8])
def test_rehearsal_lines_parse_under_cap(bench, world, rnd):
    """The lines `bench.py --gpus N --rehearse-one-gpu` printed through torchrun (rounds 5 and 6): the
    last stdout line is one JSON object under the cap, for N GPUs.  Round 6's also carry VERDICT r05
    item 5's fields: the largest owner share for both silo sets, the line on the other set, the
    communicator's rank count and the exchange's name and per-rank time (null off the library exchange)."""
    with open(os.path.join(ROOT, f"profiles/{rnd}_rehearsal_w{world}_line.json")) as f:
        text = f.read().strip().splitlines()[-1]
    assert len(text) <= bench.LINE_CAP
    line = json.loads(text)
    assert line["n_gpus"] == world and line["rehearsal_one_gpu"] is True
    assert line["value"] > 0 and "roofline" in line and "config" in line
    if rnd == "r06":
        shares = line["config"]["owner_share_max_by_silo_set"]
        assert set(shares) == {"literal", "balanced"} and all(0 < v <= 1 for v in shares.values())
        assert abs(line["config"]["owner_share_max"] - shares["balanced"]) < 0.01
        other = line["secondary"]["cfg2_other_silo_set"]
        assert other["silos"] == "literal" and other["value"] > 0
        assert "n_ranks" in line["comm"] and line["exchange"]
        assert "exchange_ms_per_rank" in line


def test_pmc_kernel_families():
    """tools/pmc_traffic.py groups template instantiations by the name bench.py's kernel tables use:
    the MSD scatter / histogram under the radix names, the list range sorts by their size, the probe
    forms under k_route -- and the ring-owner kernel (k_route<MODE, false>, gd_ring_owner_device) apart
    from them (round 5: averaged in, it had taken cfg 3's k_route bytes from 3.53 down to 2.87 GB)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic as pt
    assert pt.launch_name("gd::k_b2_scatter<512, 16, 1056, 1, false>") == "k_radix_scatter"
    assert pt.launch_name("gd::k_b2_hist<512, 16, 4, 1056>") == "k_radix_hist"
    assert pt.launch_name("gd::k_msd_local_list<512, 16, false>") == "k_msd_local_mid"
    assert pt.launch_name("gd::k_msd_local_list<1024, 24, false>") == "k_msd_local"
    assert pt.launch_name("gd::k_route_m<0, 2, false, 0, false, 4, true>") == "k_route"
    assert pt.launch_name("gd::k_route<0, false>") == "k_ring_owner"
    assert pt.launch_name("gd::k_route<2, true>") == "k_route"
    assert pt.launch_name("gd::k_fan_degree_tiles<16>") == "k_fan_degree"
