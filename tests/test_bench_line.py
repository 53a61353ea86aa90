"""bench.py's output contract (CPU): the driver parses the LAST stdout line and keeps only an ~8 KB tail of
stdout, so the final line must be a compact JSON headline that carries the metric, roofline and cpu_baseline
(round 4's single 21 KB line did not parse). Built here from a recorded full bench result."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

RECORD = os.path.join(ROOT, "profiles", "r04", "r04a5_bench.json")


def _record():
    if not os.path.exists(RECORD):
        pytest.skip("recorded bench result not present")
    return json.load(open(RECORD))


def test_headline_under_cap_and_round_trips():
    import bench
    line = _record()
    text = bench.headline_record(dict(line, full_record="gpurun_out/bench_full.json"))
    assert "\n" not in text
    assert len(text.encode()) < bench.HEADLINE_MAX_BYTES
    rec = json.loads(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline"):
        assert k in rec, k
    assert rec["value"] == pytest.approx(line["value"], rel=1e-4)
    for k in ("kernel_ms", "ops_per_unit", "units_per_launch", "frac", "traffic", "peak", "achieved"):
        assert k in rec["roofline"], k
    assert rec["roofline"]["frac"] == pytest.approx(rec["roofline"]["achieved"] / rec["roofline"]["peak"], rel=1e-3)
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in rec["cpu_baseline"], k
    legs = rec["secondary_summary"]
    assert len(legs) == len(line["secondary"])
    assert all("value" in s for s in legs)


def test_headline_drops_optional_parts_past_the_cap():
    import bench
    line = _record()
    # a pathological record: many large legs; the mandatory fields still fit and parse
    line = dict(line, secondary=line["secondary"] * 40)
    text = bench.headline_record(line)
    assert len(text.encode()) < bench.HEADLINE_MAX_BYTES
    rec = json.loads(text)
    assert "roofline" in rec and "cpu_baseline" in rec and "secondary_summary" not in rec


def test_write_final_last_line(tmp_path):
    import bench
    line = _record()
    r, w = os.pipe()
    bench.write_final(w, line, str(tmp_path / "full.json"))
    os.close(w)
    out = os.read(r, 1 << 20).decode()
    os.close(r)
    assert out.endswith("\n") and out.count("\n") == 1
    rec = json.loads(out.strip())
    assert rec["full_record"].endswith("full.json")
    full = json.load(open(tmp_path / "full.json"))
    assert full["secondary"] == line["secondary"]
