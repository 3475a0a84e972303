"""The oracle (test infrastructure) checked against the reference's golden
vectors and closed forms before it is trusted as the GPU checker."""
import struct

import numpy as np
import pytest

from oracle import fmt, mb, wire


def test_splitmix64_known_values(oracle):
    # splitmix64 reference outputs (Vigna's generator; state increment 0x9E3779B97F4A7C15)
    assert oracle.splitmix64(0) == 0xE220A8397B1DCDAF
    assert oracle.splitmix64(1) == 0x910A2DEC89025CC1


def test_synth_matches_python(oracle):
    def sm(z):
        z = (z + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return z ^ (z >> 31)
    x = oracle.synth_i64(1000, 42, 5, 50, 1)
    assert list(x) == [sm(42 + 5 + i) % 50 + 1 for i in range(1000)]


def test_filter_agg_vs_numpy(oracle):
    rng = np.random.default_rng(1)
    x = rng.integers(-2**62, 2**62, size=100_003, dtype=np.int64)
    c, s, mn, mx = oracle.filter_agg_i64(x, -2**40, 2**61, threads=4)
    sel = x[(x >= -2**40) & (x <= 2**61)]
    assert c == len(sel)
    assert s == sum(int(v) for v in sel)  # exact int128 vs Python int
    assert mn == sel.min() and mx == sel.max()


def test_synth_filter_count_equals_materialized(oracle):
    x = oracle.synth_i64(1_000_000, 42, 0, 50, 1)
    assert oracle.synth_filter_count(42, 0, 1_000_000, 50, 1, 25, 2**63 - 1, 4)[0] == \
        oracle.filter_agg_i64(x, 25, 2**63 - 1, 2)[0]


def test_range_mod_closed_form(oracle):
    # C1: SELECT i FROM range(1e6) WHERE i%2=0 -> 500 000 rows, sum 249 999 500 000
    out = oracle.range_mod_select(1_000_000, 2, 0, 1)
    assert len(out) == 500_000 and int(out.sum()) == 249_999_500_000
    # fixture "range with modulo" (duckdb_fixture_cases.mbt:159-165): evens of range(4)
    assert list(oracle.range_mod_select(4, 2, 0, 1)) == [0, 2]
    # fixture "range with expression": range*2 of range(3)
    assert list(oracle.range_mod_select(3, 1, 0, 2)) == [0, 2, 4]


def test_groupby_vs_python(oracle):
    k = oracle.synth_i32(50_000, 7, 0, 32, 0)
    v = oracle.synth_i64(50_000, 9, 0, 2**40, -2**39)
    counts, sums = oracle.groupby_sum(k, v, 0, 32, threads=3)
    ref_c = [0] * 32
    ref_s = [0] * 32
    for a, b in zip(k.tolist(), v.tolist()):
        ref_c[a] += 1
        ref_s[a] += b
    assert counts == ref_c and sums == ref_s


def test_fmt_against_fixtures(fixtures):
    by = {c["name"]: c for c in fixtures}
    assert fmt.integer(9223372036854775807) == by["bigint extremes"]["rows"][0][0]
    assert fmt.integer(-9223372036854775808) == by["bigint extremes"]["rows"][0][1]
    assert fmt.decimal(123456, 3) == by["decimal positive"]["rows"][0][0]
    assert fmt.decimal(-99999999, 2) == by["decimal negative"]["rows"][0][0]
    assert fmt.double(16 / 3) == by["multiple aggregates"]["rows"][0][3]
    assert [fmt.double(float("nan")), fmt.double(float("inf")), fmt.double(float("-inf"))] == \
        by["float special values"]["rows"][0]
    assert fmt.boolean(True) == "true" and fmt.boolean(False) == "false"


def test_wire_formats_layout():
    b = wire.int64([100])
    assert b == struct.pack("<iq", 1, 100)
    b = wire.int32([1, None, 3], nullable=True)
    assert b == struct.pack("<iiii", 3, 1, 0, 3) + bytes([1, 0, 1])
    b = wire.string(["hello", None], nullable=True)
    assert b == struct.pack("<ii", 2, 7) + b"hello\0\0" + bytes([1, 0])
    assert wire.schema(["a", "b"], [4, 11]) == b'[{"name":"a","nullable":true,"type_id":"int32"},' \
                                               b'{"name":"b","nullable":true,"type_id":"double"}]'
    assert wire.int32([2**33 + 5]) == struct.pack("<ii", 1, 5)  # (int32) truncation, duckdb_native.c:2384-2385


def test_parse_int_boundaries():
    # prop_parse_int_max_boundary / min_boundary (duckdb_pbt_test.mbt:1765-1814)
    assert mb.parse_int(str(2**31 - 1)) == 2**31 - 1
    assert mb.parse_int(str(2**31 - 1) + "0") == 2**31 - 1
    assert mb.parse_int(str(-2**31)) == -2**31
    assert mb.parse_int("9223372036854775807") == 2**31 - 1  # typed bigint saturation (duckdb_test.mbt:1251-1287)


def test_synth_groupby_matches_materialised(oracle):
    # the generator-fused C3 oracle (bench parity at 1e9 rows) equals the
    # array-based one on the same rows, including a shifted shard start
    for start, n in [(0, 100_003), (5_000_000_000, 77_777)]:
        k = oracle.synth_i32(n, 7, start, 32, 0)
        v = oracle.synth_i64(n, 9, start, 2**40, -2**39)
        assert oracle.synth_groupby(7, 9, start, n, 32, 2**40, -2**39, 3) == oracle.groupby_sum(k, v, 0, 32, 2)


def test_select_i64_matches_numpy(oracle):
    # the order-preserving selection oracle (bench --config sel parity and CPU
    # baseline): equal to numpy's boolean mask over ragged sizes and thread
    # counts, including empty, all-pass and single-row chunks
    import numpy as np
    for n in (0, 1, 7, 1_000, 100_003):
        x = oracle.synth_i64(n, 42, 3, 50, 1)
        for threads in (1, 3, 8, 64):
            for lo, hi in ((25, 2**63 - 1), (100, 200), (-5, 200), (10, 10)):
                got = oracle.select_i64(x, lo, hi, threads)
                assert np.array_equal(got, x[(x >= lo) & (x <= hi)]), (n, threads, lo, hi)
