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


@pytest.mark.parametrize("world", [2, 8])
def test_rehearsal_lines_parse_under_cap(bench, world):
    """The lines `bench.py --gpus N --rehearse-one-gpu` printed through torchrun (round 5): the last
    stdout line is one JSON object under the cap, for N GPUs."""
    with open(os.path.join(ROOT, f"profiles/r05_rehearsal_w{world}_line.json")) as f:
        text = f.read().strip().splitlines()[-1]
    assert len(text) <= bench.LINE_CAP
    line = json.loads(text)
    assert line["n_gpus"] == world and line["rehearsal_one_gpu"] is True
    assert line["value"] > 0 and "roofline" in line and "config" in line
