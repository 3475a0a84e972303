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
