"""bench.py's output contract (CPU): the headline JSON is the LAST stdout line, at most 8 KB, with the
contract's keys; the per-tier censuses, PMC blocks and tail notes go to the BENCH_DETAIL line on stderr
(the round-4 line had grown to 20.8 KB and the driver could not parse it)."""
import contextlib
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

R04D = os.path.join(ROOT, "tests", "golden", "bench_r04d_line.json")


def _emit(out):
    so, se = io.StringIO(), io.StringIO()
    with contextlib.redirect_stdout(so), contextlib.redirect_stderr(se):
        bench.emit(out)
    return so.getvalue(), se.getvalue()


def _check_head(line):
    assert len(line.encode()) <= bench.LINE_MAX_BYTES
    h = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "roofline", "cpu_baseline", "steps", "warmup",
              "higher_is_better", "scaling", "dtype", "config"):
        assert k in h, k
    assert isinstance(h["roofline"], dict) and "frac" in h["roofline"] and "bound" in h["roofline"]
    return h


def test_recorded_r04d_line_fits_and_parses():
    with open(R04D) as f:
        out = json.load(f)
    assert len(json.dumps(out)) > 20000              # the line the driver could not parse
    so, se = _emit(dict(out))
    lines = so.strip().splitlines()
    assert len(lines) == 1                           # stdout: the headline only
    h = _check_head(lines[-1])
    assert h["value"] == out["value"] and h["cpu_baseline"]["value"] == out["cpu_baseline"]["value"]
    # every secondary line kept, in brief
    for k in ("md_only_c3", "sharded", "sharded_1m", "pump_models", "mcmd", "jobs_per_gpu", "end_to_end"):
        assert k in h["lines"], k
    assert h["lines"]["sharded_1m"]["roofline"]["bound"] == "fp64"
    assert h["lines"]["md_only_c3"]["cpu_baseline"] == bench._sig(out["md_only_c3"]["cpu_baseline"]["value"])
    assert '"tiers"' not in so and '"force_tail":' not in so and '"pmc"' not in so
    # the detail line keeps everything
    det = [l for l in se.splitlines() if l.startswith("BENCH_DETAIL ")]
    assert len(det) == 1
    full = json.loads(det[0][len("BENCH_DETAIL "):])
    assert full["sharded_1m"]["roofline"]["tiers"] == out["sharded_1m"]["roofline"]["tiers"]


def test_oversized_secondary_lines_are_dropped_not_the_headline():
    with open(R04D) as f:
        out = json.load(f)
    for i in range(40):                              # a pathological number of secondary lines
        out[f"extra_{i}"] = {"value": 1.0, "unit": "x" * 300, "N": i}
    so, _ = _emit(out)
    h = _check_head(so.strip().splitlines()[-1])
    assert h["lines_in_detail_only"]


def test_watchdog_path_prints_a_parseable_line():
    with open(R04D) as f:
        out = json.load(f)
    out["secondary_errors"] = {"sharded_1m": "did not finish within 420 s (watchdog) " + "x" * 5000}
    so, _ = _emit(out)
    h = _check_head(so.strip().splitlines()[-1])
    assert len(h["secondary_errors"]["sharded_1m"]) <= 200


def test_md_only_config_list():
    assert bench.md_only_configs("c3,c4") == ["c3", "c4"]
    assert bench.md_only_configs("none") == []
    import pytest
    with pytest.raises(SystemExit):
        bench.md_only_configs("c5")                  # QT on: not an MD-only line


def test_synthetic_world8_line_fits():
    """a W = 8 line — every large line sharded over 8 ranks with its force-call
    breakdown, load imbalance and Epotential timing, plus the large end-to-end lines — stays within the
    8 KB budget with no secondary line dropped"""
    with open(R04D) as f:
        out = json.load(f)
    out["n_gpus"] = out["comm_size"] = 8
    bd = {k: 12.3456789 for k in ("allgather", "sort_boxes", "plan", "block_kernel", "slot_reduce", "tail_pass",
                                  "reduce_scatter", "forces_total", "stages_sum")}
    bd["stages_sum_vs_force_call"] = 0.99876543
    for k in ("md_only_c3", "md_only_c4", "sharded", "sharded_1m"):
        line = dict(out.get(k) or out["sharded_1m"])
        line["n_gpus"] = 8
        line["force_breakdown_ms"] = dict(bd)
        line["epotential"] = {"wall_ms": 123.456789, "block_kernel_ms": 101.23456, "vs_force_call": 0.987654321}
        roof = dict(line.get("roofline") or {})
        roof.update(bound="fp64+fp32", frac=0.412345678, fp64_frac=0.31234567, f32_frac=0.1012345678,
                    load_imbalance=1.0123456789)
        line["roofline"] = roof
        out[k] = line
    for k in ("end_to_end_c5", "end_to_end_1m"):
        out[k] = dict(out["end_to_end"], N=1000258, epot_ms=190.123456)
    so, _ = _emit(out)
    h = _check_head(so.strip().splitlines()[-1])
    assert "lines_in_detail_only" not in h, h.get("lines_in_detail_only")
    for k in ("md_only_c3", "md_only_c4", "sharded", "sharded_1m", "end_to_end_c5", "end_to_end_1m"):
        assert k in h["lines"], k
    assert h["lines"]["sharded_1m"]["force_breakdown_ms"]["reduce_scatter"] == 12.346
    assert h["lines"]["sharded_1m"]["roofline"]["f32_frac"] == 0.10123
    print(f"W = 8 headline line: {len(so.strip().splitlines()[-1])} bytes")
