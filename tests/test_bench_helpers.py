"""bench.py's measurement helpers on CPU: the committed profile (roofline.json "profile") yields the
traffic, VALU and chain-check / tally figures the bench line carries; the CPU-baseline scaling;
and tools/bench_summary.py reads a line whose secondary legs failed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_committed_profile_figures():
    assert os.path.isdir(bench.PMC_PROFILE), bench.PMC_PROFILE
    t = bench.pmc_traffic()
    assert t["bytes"] > 0 and t["per_kernel"]["k_rec_main"]["write_bytes"] > 0
    # per 640k-vote launch: the recovery kernels move a few GB, not MB and not tens of GB
    assert 1e9 < t["bytes"] < 3e10
    # reads from the L2's request counters by size (the committed profile has the pass): every request of
    # the recovery kernels is a 128-B one, twice what FETCH_SIZE tallies (profiles/r05/FETCH_CALIBRATION.md)
    for k, v in t["per_kernel"].items():
        assert v["read_basis"] == "request counters (pmc_req)", k
        assert 1.9 < v["read_bytes"] / v["fetch_raw_bytes"] < 2.1, k
    v = bench.valu_figures()
    assert 0.2 < v["valu_lane_op_frac"] < 0.6
    assert 2e5 < v["valu_instr_per_vote"]["k_rec_main"] < 4e5
    for trace, fetch, write in (("trace_serial", "pmc_fetch", "pmc_write"), ("c3_trace", "c3_fetch", "c3_write")):
        c = bench.chain_counters(trace, fetch, write)
        assert c is not None and c["GBps"] > 100 and 0 < c["frac_of_hbm_achievable"] < 1.2
        assert set(bench.CHAIN_KERNELS) <= set(c["per_kernel"])


def test_whole_host_estimate():
    e = bench.whole_host_estimate(8000.0, 7000.0)
    assert e["physical_cores"] >= 1
    assert e["value"] == 7000.0 * e["physical_cores"]  # the slower per-thread rate


def test_bench_summary_reads_failed_legs(tmp_path):
    line = {"metric": "m", "value": 1e8, "ms_per_step": 6.4, "n_gpus": 1,
            "roofline": {"kernel_ms_avg": 6.3, "frac": 0.87},
            "wire": {"value": 9.6e7}, "end_to_end": {"error": "RuntimeError: boom"},
            "cpu_baseline": {"error": "OSError: x"}}
    p = tmp_path / "b.json"
    p.write_text("noise\n" + json.dumps(line) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_summary.py"), str(p)],
                         capture_output=True, text=True, check=True).stdout
    assert "100.0 M votes/s" in out and "wire 96.0 M" in out
    assert "end_to_end error: RuntimeError: boom" in out and "cpu error: OSError: x" in out


def _full_record():
    """A full bench record of round 5 (every leg, phases, NUMA facts, histograms) plus this round's
    config4_shard leg and scaling basis."""
    d = json.load(open(os.path.join(ROOT, "profiles", "r05", "bench_r5h.json")))
    d["config4_shard"] = {"metric": "m", "value": 1.07e8, "unit": "votes/s", "ms_per_step": 117.0}
    d["scaling_basis"] = {"n1_headline": "config 2", "n_gt_1": "config 4 shards", "n1_same_workload": "x"}
    return d


def test_compact_line_fits_and_carries_every_leg(tmp_path):
    """the stdout line is at most 4 KB, carries a flat `legs` object with every leg
    (wire_from_host included) and the roofline / CPU-baseline essentials; the full record goes to the
    side file."""
    d = _full_record()
    assert len(json.dumps(d)) > 12_000  # what the driver's tail cut in round 5
    path = bench.write_detail(d, str(tmp_path / "detail.json"))
    line = bench.compact_line(d, path)
    text = json.dumps(line)
    assert len(text) <= 4096, len(text)
    assert set(line["legs"]) == set(bench.LEG_NAMES), line["legs"]
    assert line["legs"]["wire_from_host"] == d["wire"]["from_host_buffers"]["value"]
    assert line["legs"]["end_to_end"] == d["end_to_end"]["value"]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "config"):
        assert line[k] == d[k], k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert line["roofline"][k] == d["roofline"][k], k
    for k in ("value", "unit", "cores", "kind"):
        assert line["cpu_baseline"][k] == d["cpu_baseline"][k], k
    assert line["scaling_basis"]["n_gt_1"] == "config 4 shards"
    assert json.load(open(path)) == d


def test_compact_line_reports_failed_legs():
    d = _full_record()
    d["stream"] = {"error": "RuntimeError: " + "x" * 1000}
    line = bench.compact_line(d, None)
    assert "stream" not in line["legs"] and line["leg_errors"]["stream"].startswith("RuntimeError")
    assert len(json.dumps(line)) <= 4096
