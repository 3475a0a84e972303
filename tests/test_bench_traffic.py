"""bench.py's roofline.traffic lookup (CPU): the stored PMC bytes are reported
only for the build and the row count they were measured on."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402


def _same_build(src):
    return src.get("csrc_sha256") == src["this_build_csrc_sha256"]


def test_traffic_matches_this_build_and_size():
    b, src = bench.pmc_traffic_entry("filter_agg", 1_000_000_000)
    if not _same_build(src):  # sources edited since the last PMC passes: null, and said why
        assert b is None and "digest" in src["why_null"], src
        return
    assert b is not None and 8.0e9 <= b < 8.01e9, src  # C2: 8 B/row read once


def test_row_keyed_entry_for_c5():
    b, src = bench.pmc_traffic_entry("filter_agg", 1_250_000_000)
    assert src["entry"] == "filter_agg@1250000000"
    if not _same_build(src):
        assert b is None and "digest" in src["why_null"], src
        return
    assert b is not None and 1.0e10 <= b < 1.001e10, src


def test_other_sizes_and_builds_report_why():
    b, src = bench.pmc_traffic_entry("filter_agg", 500_000_000)
    assert b is None and ("rows" if _same_build(src) else "digest") in src["why_null"], src
    b, src = bench.pmc_traffic_entry("no_such_kernel", 1_000_000_000)
    assert b is None and "no entry" in src["why_null"], src


def test_digest_mismatch_nulls_traffic(monkeypatch):
    monkeypatch.setattr(bench, "csrc_digest", lambda: "0" * 64)
    b, src = bench.pmc_traffic_entry("group_direct", 1_000_000_000)
    assert b is None and "digest" in src["why_null"], src


def test_multi_pass_traffic_is_the_sum_of_its_passes():
    """c3h / c3s name three kernels each: their traffic is the sum of the
    passes' stored bytes (about 41 and 58 GB per query at 1e9 rows), or null
    as soon as one pass is missing or stale."""
    for cfg, lo, hi in (("c3h", 4.0e10, 4.3e10), ("c3s", 5.6e10, 6.0e10), ("c3n", 1.27e10, 1.29e10)):
        w = bench.workload(cfg, 0, 1_000_000_000)
        b, src = bench.pmc_traffic_keys(w["pmc_keys"], 1_000_000_000)
        entries = src.get("entries", [src])
        assert len(entries) == len(w["pmc_keys"])
        if not all(_same_build(e) for e in entries):
            assert b is None
            continue
        assert b is not None and lo <= b <= hi, (cfg, b)
    b, src = bench.pmc_traffic_keys(["pg_hist", "no_such_pass"], 1_000_000_000)
    assert b is None and any("no entry" in e.get("why_null", "") for e in src["entries"])


def test_new_workloads_account_their_bytes():
    """The round-6 configs name the query's own bytes per row (the roofline's
    algorithmic bytes), a multi-kernel scope and their PMC passes."""
    for cfg, bpr in (("c3n", 12.25), ("c3h", 16), ("c3s", 16)):
        w = bench.workload(cfg, 0, 1_000_000_000, 100_000)
        assert w["bytes_per_row"] == bpr and w["pmc_keys"], (cfg, w)
        assert "GROUP BY k" in w["sql"] and "CREATE TABLE" in w["setup"]
    assert bench.workload("c3s", 0, 10, 7)["setup"].count(str(bench.C3S_MULT)) == 1
