"""Hot-path parity: scan -> filter -> project -> aggregate on
the MI355X against the CPU oracle, bit-exact for integer work.

Sizes: exact comparisons at sizes the oracle finishes in seconds; full
BASELINE sizes (1e9 rows) through size-independent properties (closed forms,
sum of disjoint predicates, monotonicity)."""
import numpy as np
import pytest

from conftest import one, q

pytestmark = pytest.mark.gpu

SYNTH_C2 = "CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({a}, {b}) tbl(i)"
SYNTH_C3 = ("CREATE TABLE g AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
            "mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")


# ---- C1: SELECT i FROM range(1e6) WHERE i%2=0 ------------------------------
def test_c1_range_filter_stream(conn, oracle):
    exp = oracle.range_mod_select(1_000_000, 2, 0, 1)
    s = conn.query_stream("SELECT i FROM range(1000000) tbl(i) WHERE i%2=0").value
    got = []
    while True:
        r = s.next().value
        if r is None:
            break
        got.extend(int(row[0]) for row in r.rows)
    s.close()
    assert len(got) == 500_000 and got == exp.tolist()
    assert sum(got) == 249_999_500_000


def test_c1_arrow_and_count(conn, mbx):
    a = conn.query_arrow("SELECT i FROM range(1000000) tbl(i) WHERE i%2=0").value
    v = a.raw_int64(0)
    assert len(v) == 500_000 and v[:3] == [0, 2, 4] and v[-1] == 999_998
    assert one(conn, "SELECT COUNT(*), SUM(i) FROM range(1000000) tbl(i) WHERE i%2=0") == ["500000", "249999500000"]


# ---- C2: scan + filter COUNT over INT64 -------------------------------------
@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 1023, 4097, 1_000_003, 10_000_000])
def test_c2_count_parity(conn, oracle, n):
    q(conn, SYNTH_C2.format(a=0, b=n))
    for k in (24, 0, 50, -5, 49):
        c, s = oracle.synth_filter_count(42, 0, n, 50, 1, k + 1, 2**63 - 1, 8)
        got = one(conn, f"SELECT COUNT(*), SUM(x) FROM t WHERE x > {k}")
        assert int(got[0]) == c
        assert (got[1] == "" and c == 0) or int(got[1]) == s


def test_c2_all_aggregates_and_predicates(conn, oracle):
    n = 2_000_001
    q(conn, SYNTH_C2.format(a=100, b=100 + n))
    x = oracle.synth_i64(n, 42, 100, 50, 1)
    for where, lo, hi in [("x > 24", 25, 50), ("x >= 10 AND x < 20", 10, 19), ("x = 7", 7, 7),
                          ("x BETWEEN 3 AND 5", 3, 5), ("24 < x", 25, 50), ("x <= 1", 1, 1), ("x > 50", 51, 50)]:
        c, s, mn, mx = oracle.filter_agg_i64(x, lo, hi, 8)
        got = one(conn, f"SELECT COUNT(*), SUM(x), MIN(x), MAX(x), AVG(x) FROM t WHERE {where}")
        assert int(got[0]) == c, where
        if c:
            assert [int(got[1]), int(got[2]), int(got[3])] == [s, mn, mx], where
            assert abs(float(got[4]) - s / c) <= 1e-12 * abs(s / c), where
        else:
            assert got[1:] == ["", "", "", ""]


def test_c2_decimal_variant(conn, oracle):
    # DECIMAL(15,2) l_quantity-style: raw = 100*x, `x > 24` <=> raw > 2400
    n = 1_000_000
    q(conn, f"CREATE TABLE d AS SELECT CAST(mbx_synth(42, i, 50) + 1 AS DECIMAL(15,2)) AS q FROM range({n}) tbl(i)")
    c, s = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 8)
    got = one(conn, "SELECT COUNT(*), SUM(q) FROM d WHERE q > 24")
    assert int(got[0]) == c and got[1] == f"{s}.00"
    assert q(conn, "SELECT SUM(q) FROM d WHERE q > 24").column_types == ["Decimal"]


def test_c2_full_size_properties(conn, oracle):
    # 1e9 rows (BASELINE size): exact COUNT vs the oracle's streaming generator,
    # and the partition property COUNT(x>24) + COUNT(x<=24) = N
    n = 1_000_000_000
    q(conn, SYNTH_C2.format(a=0, b=n))
    c_gt = int(one(conn, "SELECT COUNT(*) FROM t WHERE x > 24")[0])
    c_le = int(one(conn, "SELECT COUNT(*) FROM t WHERE x <= 24")[0])
    assert c_gt + c_le == n
    oc, osum = oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 16)
    assert c_gt == oc
    got = one(conn, "SELECT SUM(x) FROM t WHERE x > 24")
    assert int(got[0]) == osum
    q(conn, "DROP TABLE t")


# ---- C3: GROUP BY 32-key INT32 + SUM(INT64) -------------------------------------
@pytest.mark.parametrize("n", [1, 1000, 3_000_001])
def test_c3_groupby_parity(conn, oracle, n):
    q(conn, SYNTH_C3.format(n=n))
    k = oracle.synth_i32(n, 7, 0, 32, 0)
    v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
    counts, sums = oracle.groupby_sum(k, v, 0, 32, 8)
    res = q(conn, "SELECT k, SUM(v), COUNT(*), MIN(v), MAX(v), AVG(v) FROM g GROUP BY k ORDER BY k")
    assert res.column_types == ["Integer", "HugeInt", "BigInt", "BigInt", "BigInt", "Double"]
    exp = [(i, sums[i], counts[i]) for i in range(32) if counts[i]]
    assert [(int(r[0]), int(r[1]), int(r[2])) for r in res.rows] == exp
    for r in res.rows:
        kk = int(r[0])
        sel = v[k == kk]
        assert int(r[3]) == sel.min() and int(r[4]) == sel.max()
        assert abs(float(r[5]) - sums[kk] / counts[kk]) <= 1e-9 * max(1.0, abs(sums[kk] / counts[kk]))


def test_c3_full_size_properties(conn, oracle):
    """C3 at BASELINE size (1e9 rows): every group's COUNT and exact int128 SUM
    against the oracle's streaming generator over all rows (orc_synth_groupby,
    no host arrays), plus the checksum of checksums."""
    n = 1_000_000_000
    q(conn, SYNTH_C3.format(n=n))
    res = q(conn, "SELECT k, SUM(v), COUNT(*) FROM g GROUP BY k ORDER BY k")
    assert len(res.rows) == 32
    oc, osum = oracle.synth_groupby(7, 9, 0, n, 32, 1 << 40, -(1 << 39), 16)
    assert [(int(r[0]), int(r[1]), int(r[2])) for r in res.rows] == [(k, osum[k], oc[k]) for k in range(32)]
    total_c = sum(int(r[2]) for r in res.rows)
    total_s = sum(int(r[1]) for r in res.rows)
    assert total_c == n
    # checksum of checksums: the per-group sums add up to the global sum
    assert total_s == int(one(conn, "SELECT SUM(v) FROM g")[0])
    q(conn, "DROP TABLE g")


# ---- C5 (single-GPU shard): global SUM/COUNT over a shifted shard ---------------
def test_c5_shard_sum_count(conn, oracle):
    start, n = 7_000_000_000, 5_000_000
    q(conn, SYNTH_C2.format(a=start, b=start + n))
    c, s = oracle.synth_filter_count(42, start, n, 50, 1, 25, 2**63 - 1, 8)
    assert one(conn, "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24") == [str(c), str(s)]


# ---- generic path vs numpy on random data ----------------------------------------
def _load_random(conn, mbx, rng, n, nulls=True):
    q(conn, "CREATE TABLE r (a INTEGER, b BIGINT, c DOUBLE, k SMALLINT)")
    a = rng.integers(-1000, 1000, n).astype(np.int32)
    b = rng.integers(-2**40, 2**40, n).astype(np.int64)
    c = rng.standard_normal(n)
    k = rng.integers(-5, 6, n).astype(np.int16)
    va = (rng.random(n) > 0.1).astype(np.uint8) if nulls else None
    ap = conn.create_appender("main", "r").value
    assert isinstance(ap.append_column(0, a, va), mbx.Ok)
    assert isinstance(ap.append_column(1, b), mbx.Ok)
    assert isinstance(ap.append_column(2, c), mbx.Ok)
    assert isinstance(ap.append_column(3, k), mbx.Ok)
    assert isinstance(ap.commit(n), mbx.Ok)
    ap.close()
    return a, b, c, k, (va.astype(bool) if nulls else np.ones(n, bool))


def test_generic_filter_project(conn, mbx):
    rng = np.random.default_rng(7)
    n = 300_001
    a, b, c, k, va = _load_random(conn, mbx, rng, n)
    a64 = a.astype(np.int64)
    sel = va & (a64 * 3 + 1 > 100) & (b % 7 != 0)
    res = conn.query_raw("SELECT a * 3 + 1, b // 7, b % 7, CASE WHEN a > 500 THEN 1 ELSE 0 END FROM r "
                         "WHERE a * 3 + 1 > 100 AND b % 7 <> 0")
    assert res.row_count() == int(sel.sum())
    idx = np.nonzero(sel)[0]
    for j in list(range(5)) + [len(idx) // 2, len(idx) - 1]:
        i = idx[j]
        assert res.value(0, j) == str(a64[i] * 3 + 1)
        assert res.value(1, j) == str(int(b[i] / 7))  # integer division truncates toward zero
        assert res.value(2, j) == str(int(np.fmod(b[i], 7)))
        assert res.value(3, j) == ("1" if a[i] > 500 else "0")
    res.close()


def test_generic_aggregates_with_nulls(conn, mbx):
    rng = np.random.default_rng(11)
    n = 500_000
    a, b, c, k, va = _load_random(conn, mbx, rng, n)
    got = one(conn, "SELECT COUNT(*), COUNT(a), SUM(a), MIN(a), MAX(a), SUM(b), SUM(c), MIN(c), MAX(c) FROM r")
    av = a[va].astype(np.int64)
    assert got[:6] == [str(n), str(len(av)), str(int(av.sum())), str(av.min()), str(av.max()), str(int(b.sum()))]
    assert abs(float(got[6]) - float(np.sum(c))) <= 1e-9 * np.sum(np.abs(c))
    assert float(got[7]) == c.min() and float(got[8]) == c.max()
    # GROUP BY a SMALLINT key (generic direct-index path) with NULL-free keys
    res = q(conn, "SELECT k, COUNT(*), SUM(b), COUNT(a) FROM r GROUP BY k ORDER BY k")
    for row in res.rows:
        kk = int(row[0])
        m = k == kk
        assert int(row[1]) == int(m.sum()) and int(row[2]) == int(b[m].sum()) and int(row[3]) == int((m & va).sum())
    # GROUP BY a nullable key: one NULL group
    res = q(conn, "SELECT a % 3 AS g, COUNT(*) FROM r GROUP BY a % 3 ORDER BY g NULLS FIRST")
    assert res.nulls[0][0] and int(res.rows[0][1]) == int((~va).sum())
    assert sum(int(r[1]) for r in res.rows) == n


def test_order_by_limit_offset(conn, mbx):
    rng = np.random.default_rng(3)
    n = 10_000
    a, b, c, k, va = _load_random(conn, mbx, rng, n, nulls=False)
    res = conn.query_raw("SELECT b FROM r ORDER BY b DESC LIMIT 5 OFFSET 2")
    exp = np.sort(b)[::-1][2:7]
    assert [int(res.value(0, i)) for i in range(5)] == exp.tolist()
    res.close()
    res = q(conn, "SELECT k, a FROM r ORDER BY k, a LIMIT 50")
    pairs = sorted(zip(k.tolist(), a.tolist()))[:50]
    assert [(int(x), int(y)) for x, y in res.rows] == pairs


def test_empty_and_edge_tables(conn, mbx):
    q(conn, "CREATE TABLE e (x BIGINT)")
    assert one(conn, "SELECT COUNT(*), SUM(x), MIN(x) FROM e WHERE x > 1") == ["0", "", ""]
    assert q(conn, "SELECT x FROM e").rows == []
    assert q(conn, "SELECT x, COUNT(*) FROM e GROUP BY x").rows == []
    q(conn, "INSERT INTO e VALUES (9223372036854775807), (-9223372036854775808), (NULL)")
    assert one(conn, "SELECT COUNT(*), COUNT(x), SUM(x), MIN(x), MAX(x) FROM e") == \
        ["3", "2", "-1", "-9223372036854775808", "9223372036854775807"]
    r = conn.query("SELECT x + 1 FROM e")
    assert isinstance(r, mbx.Err) and "Overflow" in r.error.message


def test_ctas_and_types_roundtrip(conn):
    q(conn, "CREATE TABLE s AS SELECT i AS a, CAST(i AS INTEGER) AS b, CAST(i AS SMALLINT) AS c, "
            "CAST(i AS DOUBLE) / 4 AS d, i % 2 = 0 AS e, CAST(i AS DECIMAL(20,3)) AS f FROM range(-5, 5) tbl(i)")
    res = q(conn, "SELECT * FROM s ORDER BY a")
    assert res.column_types == ["BigInt", "Integer", "SmallInt", "Double", "Boolean", "Decimal"]
    assert res.rows[0] == ["-5", "-5", "-5", "-1.25", "false", "-5.000"]
    assert res.rows[9] == ["4", "4", "4", "1.0", "true", "4.000"]


# ---- every fused filter-aggregate launch shape gives the same bits ----------
FA_VARIANTS = ["", "u8_nt_ch_g4", "u4_nt_gs_g16", "u2_pl_gs_g4_v4", "u8_nt_ch_g4_v4", "d4_g1", "d8_g1", "d16_g2"]


@pytest.mark.parametrize("variant", FA_VARIANTS)
def test_filter_agg_variants_parity(conn, oracle, monkeypatch, variant):
    monkeypatch.setenv("MBX_FA_VARIANT", variant)
    for n in (0, 1, 127, 128, 129, 255, 257, 4099, 1_000_003):
        x = oracle.synth_i64(n, 42, 0, 50, 1)
        v = oracle.synth_i64(n, 9, 0, 1000, -500)
        q(conn, "DROP TABLE IF EXISTS fv")
        q(conn, f"CREATE TABLE fv AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(42, i, 50) + 1 AS INTEGER) AS y, "
                f"mbx_synth(9, i, 1000) - 500 AS v, CAST(mbx_synth(9, i, 1000) - 500 AS INTEGER) AS w "
                f"FROM range({n}) tbl(i)")
        m = x > 24
        exp_cnt = int(m.sum())
        for sql, vals in [("SELECT COUNT(*) FROM fv WHERE x > 24", None),
                          ("SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM fv WHERE x > 24", x),
                          ("SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM fv WHERE x > 24", v),
                          ("SELECT COUNT(*) FROM fv WHERE y > 24", None),
                          ("SELECT COUNT(*), SUM(y), MIN(y), MAX(y) FROM fv WHERE y > 24", x),
                          ("SELECT COUNT(*), SUM(w), MIN(w), MAX(w) FROM fv WHERE y > 24", v),
                          ("SELECT COUNT(*), SUM(v) FROM fv WHERE y > 24", v)]:
            got = one(conn, sql)
            assert int(got[0]) == exp_cnt, (variant, n, sql)
            if vals is not None and exp_cnt:
                sel = vals[m]
                want = [int(sel.sum(dtype=np.int64)), int(sel.min()), int(sel.max())][:len(got) - 1]
                assert [int(g) for g in got[1:]] == want, (variant, n, sql)


# ---- every fused GROUP BY launch shape gives the same bits ------------------
# (+atomic: the table flush through global atomics instead of the per-workgroup
# records that group_partials_compact reduces)
GD_VARIANTS = ["", "seg", "d2_g1", "d3_g2", "d4_g2", "d6_g1", "d8_g1", "+atomic", "d3_g2+atomic"]


@pytest.mark.parametrize("variant", GD_VARIANTS)
def test_group_direct_variants_parity(conn, oracle, monkeypatch, variant):
    base, *opts = variant.split("+")
    monkeypatch.setenv("MBX_GD_VARIANT", base)
    if "atomic" in opts:
        monkeypatch.setenv("MBX_GD_ATOMIC_FLUSH", "1")
    for n in (1, 255, 256, 257, 1023, 70_001, 1_000_003):
        k = oracle.synth_i64(n, 7, 0, 40, -20)           # keys -20..19
        v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
        u = oracle.synth_i64(n, 11, 0, 1000, -500)
        q(conn, "DROP TABLE IF EXISTS gv")
        q(conn, f"CREATE TABLE gv AS SELECT mbx_synth(7, i, 40) - 20 AS k, CAST(mbx_synth(7, i, 40) - 20 AS INTEGER) AS k4, "
                f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(11, i, 1000) - 500 AS u, "
                f"CAST(mbx_synth(11, i, 1000) - 500 AS INTEGER) AS u4, CAST(mbx_synth(9, i, 1000000) AS INTEGER) AS w4 "
                f"FROM range({n}) tbl(i)")
        w = oracle.synth_i64(n, 9, 0, 1_000_000, 0)
        keys = sorted(set(k.tolist()))
        for kc in ("k", "k4"):
            exp_c = [int((k == kk).sum()) for kk in keys]
            got = q(conn, f"SELECT {kc}, COUNT(*) FROM gv GROUP BY {kc} ORDER BY {kc}").rows
            assert [(int(r[0]), int(r[1])) for r in got] == list(zip(keys, exp_c)), (variant, n, kc)
            for sql, cols in [(f"SELECT {kc}, SUM(v), COUNT(*) FROM gv GROUP BY {kc} ORDER BY {kc}", [v]),
                              (f"SELECT {kc}, SUM(u), SUM(v), COUNT(*) FROM gv GROUP BY {kc} ORDER BY {kc}", [u, v]),
                              (f"SELECT {kc}, SUM(u4), MIN(u4), MAX(u4), SUM(w4) FROM gv GROUP BY {kc} ORDER BY {kc}", None),
                              (f"SELECT {kc}, MIN(v), MAX(v), SUM(v) FROM gv GROUP BY {kc} ORDER BY {kc}", None)]:
                got = q(conn, sql).rows
                for r, kk in zip(got, keys):
                    m = k == kk
                    assert int(r[0]) == kk
                    if "SUM(u4), MIN(u4)" in sql:
                        want = [int(u[m].sum()), int(u[m].min()), int(u[m].max()), int(w[m].sum())]
                    elif "MIN(v), MAX(v)" in sql:
                        want = [int(v[m].min()), int(v[m].max()), int(v[m].astype(object).sum())]
                    else:
                        want = [int(c[m].astype(object).sum()) for c in cols] + [int(m.sum())]
                    assert [int(x) for x in r[1:]] == want, (variant, n, sql, kk)


# ---- hash GROUP BY: several keys, VARCHAR / wide-range / NULL keys ---------------
def _expect_groups(keys, vals):
    acc = {}
    for kt, v in zip(keys, vals):
        c, s, mn, mx = acc.get(kt, (0, 0, None, None))
        acc[kt] = (c + 1, s + v, v if mn is None else min(mn, v), v if mx is None else max(mx, v))
    return acc


def _sort_key(kt):
    return tuple((k is None, k if k is not None else 0) for k in kt)


@pytest.mark.parametrize("n", [1, 1000, 200_003])
def test_hash_groupby_multi_key(conn, oracle, n):
    a = oracle.synth_i64(n, 3, 0, 97, 0)
    b = oracle.synth_i64(n, 5, 0, 13, -6)
    v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
    q(conn, "DROP TABLE IF EXISTS hg")
    q(conn, f"CREATE TABLE hg AS SELECT mbx_synth(3, i, 97) AS a, CAST(mbx_synth(5, i, 13) - 6 AS INTEGER) AS b, "
            f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    exp = _expect_groups(list(zip(a.tolist(), b.tolist())), v.tolist())
    res = q(conn, "SELECT a, b, COUNT(*), SUM(v), MIN(v), MAX(v) FROM hg GROUP BY a, b ORDER BY a, b")
    assert res.column_types == ["BigInt", "Integer", "BigInt", "HugeInt", "BigInt", "BigInt"]
    want = [[str(k[0]), str(k[1])] + [str(x) for x in exp[k]] for k in sorted(exp)]
    assert res.rows == want


def test_hash_groupby_wide_range_and_null_keys(conn, oracle):
    n = 100_000
    # wide-range BIGINT keys (range >> rows): hash path; every 7th key NULL
    q(conn, f"CREATE TABLE wk AS SELECT CASE WHEN i % 7 = 0 THEN NULL ELSE (i % 1000) * 1000000007 END AS k, "
            f"i AS v FROM range({n}) tbl(i)")
    keys = [None if i % 7 == 0 else (i % 1000) * 1000000007 for i in range(n)]
    exp = _expect_groups([(k,) for k in keys], list(range(n)))
    res = q(conn, "SELECT k, COUNT(*), SUM(v) FROM wk GROUP BY k ORDER BY k")
    want = [[("" if k[0] is None else str(k[0])), str(exp[k][0]), str(exp[k][1])] for k in sorted(exp, key=_sort_key)]
    assert [[r[0], r[1], r[2]] for r in res.rows] == want
    assert res.nulls[-1][0] is True  # NULL group last


def test_hash_groupby_varchar_keys(conn):
    n = 50_000
    q(conn, f"CREATE TABLE sk AS SELECT CASE WHEN i % 3 = 0 THEN 'alpha' WHEN i % 3 = 1 THEN 'beta' ELSE NULL END AS s, "
            f"i % 5 AS t, i AS v FROM range({n}) tbl(i)")
    exp = {}
    for i in range(n):
        s = "alpha" if i % 3 == 0 else "beta" if i % 3 == 1 else None
        kt = (s, i % 5)
        c, sm = exp.get(kt, (0, 0))
        exp[kt] = (c + 1, sm + i)
    res = q(conn, "SELECT s, t, COUNT(*), SUM(v) FROM sk GROUP BY s, t ORDER BY s, t")
    want = [[("" if k[0] is None else k[0]), str(k[1]), str(c), str(sm)]
            for k, (c, sm) in sorted(exp.items(), key=lambda kv: _sort_key(kv[0]))]
    assert res.rows == want
    # HAVING over the hash path
    res = q(conn, "SELECT s, COUNT(*) AS c FROM sk GROUP BY s HAVING COUNT(*) > 16666 ORDER BY s")
    assert res.rows == [["alpha", "16667"], ["beta", "16667"]]


def test_hash_groupby_double_keys(conn):
    q(conn, "CREATE TABLE dk AS SELECT CAST(i % 4 AS DOUBLE) / 2 AS d, i AS v FROM range(1000) tbl(i)")
    res = q(conn, "SELECT d, COUNT(*), SUM(v) FROM dk GROUP BY d ORDER BY d")
    assert res.rows == [["0.0", "250", str(sum(range(0, 1000, 4)))], ["0.5", "250", str(sum(range(1, 1000, 4)))],
                        ["1.0", "250", str(sum(range(2, 1000, 4)))], ["1.5", "250", str(sum(range(3, 1000, 4)))]]


def test_order_by_extremes_and_varchar(conn):
    # adjacent extremes must stay distinct (the NULL pass is separate from the value key)
    q(conn, "CREATE TABLE ox (x BIGINT, s VARCHAR)")
    vals = [(-9223372036854775807, "prefix_longer_than_8_b"), (None, None), (-9223372036854775808, "prefix_longer_than_8_a"),
            (9223372036854775807, "b"), (9223372036854775806, ""), (0, "prefix_longer"), (None, "a")]
    for x, s in vals:
        q(conn, "INSERT INTO ox VALUES ({}, {})".format("NULL" if x is None else x, "NULL" if s is None else f"'{s}'"))
    res = q(conn, "SELECT x FROM ox ORDER BY x")
    assert [r[0] for r in res.rows] == ["-9223372036854775808", "-9223372036854775807", "0", "9223372036854775806",
                                        "9223372036854775807", "", ""]
    res = q(conn, "SELECT x FROM ox ORDER BY x DESC NULLS FIRST")
    assert [r[0] for r in res.rows][2:] == ["9223372036854775807", "9223372036854775806", "0", "-9223372036854775807",
                                            "-9223372036854775808"]
    res = q(conn, "SELECT s FROM ox ORDER BY s")
    got = [(None if n[0] else r[0]) for r, n in zip(res.rows, res.nulls)]
    assert got == ["", "a", "b", "prefix_longer", "prefix_longer_than_8_a", "prefix_longer_than_8_b", None]
    res = q(conn, "SELECT s, x FROM ox ORDER BY s DESC, x")
    got = [(None if n[0] else r[0]) for r, n in zip(res.rows, res.nulls)]
    assert got == ["prefix_longer_than_8_b", "prefix_longer_than_8_a", "prefix_longer", "b", "a", "", None]


# ---- filter -> GROUP BY fused (range predicate inside the LDS group kernel) -------
@pytest.mark.parametrize("variant", ["", "d3_g2", "d4_g1", "jit"])
def test_filter_groupby_fused_parity(conn, oracle, monkeypatch, variant):
    # group_direct_lds with fused predicates, at its default shape and others
    # (MBX_JIT=0); "jit": with run-time compilation on, which a range-filtered
    # GROUP BY no longer prefers (the LDS kernel is faster at 1e9 rows), so the
    # same kernel runs with the compiler live
    if variant == "jit":
        monkeypatch.setenv("MBX_JIT", "sync")
    else:
        monkeypatch.setenv("MBX_JIT", "0")
        monkeypatch.setenv("MBX_GD_VARIANT", variant)
    for n in (255, 257, 100_003, 1_000_000):
        k = oracle.synth_i64(n, 7, 0, 32, 0)
        v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
        x = oracle.synth_i64(n, 42, 0, 50, 1)
        q(conn, "DROP TABLE IF EXISTS fg")
        q(conn, f"CREATE TABLE fg AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
                f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x, "
                f"CAST(mbx_synth(42, i, 50) + 1 AS INTEGER) AS x4 FROM range({n}) tbl(i)")
        cases = [("x > 24", x > 24), ("x4 BETWEEN 10 AND 20", (x >= 10) & (x <= 20)), ("k < 16", k < 16),
                 ("v >= 0", v >= 0), ("x = 7", x == 7), ("x > 50", x > 50),
                 ("x > 24 AND k < 16", (x > 24) & (k < 16)),
                 ("x4 BETWEEN 10 AND 20 AND v >= 0 AND x < 45", (x >= 10) & (x <= 20) & (v >= 0)),
                 ("x4 > 5 AND x < 40 AND k BETWEEN 3 AND 29", (x > 5) & (x < 40) & (k >= 3) & (k <= 29))]
        for where, m in cases:
            res = q(conn, f"SELECT k, SUM(v), COUNT(*), MIN(v), MAX(v) FROM fg WHERE {where} GROUP BY k ORDER BY k")
            want = []
            for kk in range(32):
                sel = m & (k == kk)
                c = int(sel.sum())
                if c:
                    vs = v[sel]
                    want.append([str(kk), str(int(vs.astype(object).sum())), str(c), str(int(vs.min())), str(int(vs.max()))])
            assert res.rows == want, (variant, n, where)


# ---- streams read device-resident results back in batches ------------------------
def test_stream_device_batches(conn):
    n = 150_001  # > 2 device->host batches of 65 536 rows, ragged last chunk
    q(conn, f"CREATE TABLE st AS SELECT i AS a, CASE WHEN i % 5 = 0 THEN NULL ELSE i * 3 END AS b, "
            f"CASE WHEN i % 2 = 0 THEN 'even' ELSE 'odd' END AS s FROM range({n}) tbl(i)")
    s = conn.query_stream("SELECT a, b, s FROM st WHERE a % 3 <> 1").value
    assert s.columns() == ["a", "b", "s"]
    rows, nulls, chunks = [], [], 0
    while True:
        r = s.next().value
        if r is None:
            break
        chunks += 1
        assert len(r.rows) <= 2048
        rows.extend(r.rows)
        nulls.extend(r.nulls)
    s.close()
    want = [i for i in range(n) if i % 3 != 1]
    assert len(rows) == len(want) and chunks == (len(want) + 2047) // 2048
    for (a, b, st), nl, i in zip(rows, nulls, want):
        assert int(a) == i
        assert nl[1] == (i % 5 == 0)
        if i % 5:
            assert int(b) == 3 * i
        assert st == ("even" if i % 2 == 0 else "odd")
    # the connection keeps working between and after partial reads
    s2 = conn.query_stream("SELECT a FROM st").value
    first = s2.next().value
    assert one(conn, "SELECT COUNT(*) FROM st")[0] == str(n)
    second = s2.next().value
    assert int(first.rows[0][0]) == 0 and int(second.rows[0][0]) == 2048
    s2.close()


def test_groupby_direct_wide_slot_table(conn):
    # 100 000-slot direct-index table (> one workgroup's compaction): device-wide slot scan
    n = 300_007
    q(conn, f"CREATE TABLE ws AS SELECT i % 100000 AS k, i AS v FROM range({n}) tbl(i)")
    res = q(conn, "SELECT k, COUNT(*), SUM(v) FROM ws WHERE v % 7 <> 3 GROUP BY k ORDER BY k")
    exp = {}
    for i in range(n):
        if i % 7 != 3:
            c, s = exp.get(i % 100000, (0, 0))
            exp[i % 100000] = (c + 1, s + i)
    assert res.rows == [[str(k), str(c), str(s)] for k, (c, s) in sorted(exp.items())]


def test_groupby_direct_sparse_keys_count_on_device(mbx, oracle, monkeypatch):
    """The direct GROUP BY of the statement's own result leaves its group count on
    the device and ToHost trims the slot rows to it in the same copy; sparse keys
    (3 of 16 slots present) make the count smaller than the slot table.  HAVING,
    ORDER BY, LIMIT, a projection, a stream and the Arrow path read the count
    first; each must give the same groups."""
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    try:
        for flush in ("", "1"):
            monkeypatch.setenv("MBX_GD_ATOMIC_FLUSH", flush)
            for n in (3, 1000, 1_000_003):
                q(c, "DROP TABLE IF EXISTS sk")
                # keys -3, 7, 12 (range 16), values i - 500
                q(c, f"CREATE TABLE sk AS SELECT CASE WHEN i % 3 = 0 THEN -3 WHEN i % 3 = 1 THEN 7 ELSE 12 END AS k, "
                     f"i - 500 AS v, CAST(i - 500 AS DECIMAL(15,2)) AS d FROM range({n}) tbl(i)")
                exp = {}
                for kk, r in ((-3, 0), (7, 1), (12, 2)):
                    vals = [i - 500 for i in range(r, n, 3)]
                    if vals:
                        exp[kk] = (sum(vals), len(vals), min(vals), max(vals))
                got = q(c, "SELECT k, SUM(v), COUNT(*), MIN(v), MAX(v) FROM sk GROUP BY k").rows
                assert "group_direct" in [x["name"] for x in c.last_profile()["kernels"]], n
                assert sorted((int(r[0]), int(r[1]), int(r[2]), int(r[3]), int(r[4])) for r in got) == \
                    sorted((kk,) + t for kk, t in exp.items()), (flush, n)
                assert [r[0] for r in got] == [str(kk) for kk in sorted(exp)]  # key order
                keys = sorted(exp)
                r = q(c, "SELECT k, COUNT(*) FROM sk GROUP BY k HAVING COUNT(*) > 0 ORDER BY k DESC").rows
                assert [int(x[0]) for x in r] == keys[::-1]
                r = q(c, "SELECT k, COUNT(*) FROM sk GROUP BY k LIMIT 2").rows
                assert [int(x[0]) for x in r] == keys[:2]
                r = q(c, "SELECT k + 1, COUNT(*) FROM sk GROUP BY k").rows
                assert sorted(int(x[0]) for x in r) == [kk + 1 for kk in keys]
                st = c.query_stream("SELECT k, COUNT(*) FROM sk GROUP BY k").value
                rows = []
                while True:
                    ch = st.next().value
                    if ch is None or not ch.rows:
                        break
                    rows += ch.rows
                st.close()
                assert [int(x[0]) for x in rows] == keys
                a = c.query_arrow("SELECT k, COUNT(*) FROM sk GROUP BY k").value
                assert a.row_count() == len(keys)
                a.close()
                # no group at all (a fused predicate no row passes): the count 0 trims every slot
                r = q(c, "SELECT k, COUNT(*), SUM(v) FROM sk WHERE v > 1000000000000 GROUP BY k")
                assert r.rows == [] and len(r.columns) == 3
                # DECIMAL sums (16-byte results) through the same trimmed copy
                r = q(c, "SELECT k, SUM(d) FROM sk GROUP BY k").rows
                assert [(int(x[0]), x[1]) for x in r] == [(kk, f"{exp[kk][0]}.00") for kk in keys]
    finally:
        c.close()


# ---- multi-column conjunctions fused into one LDS-DMA pass ----------------------
def test_filter_multi_parity(mbx, oracle):
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    try:
        for n in (1, 255, 256, 257, 70_001, 1_000_003):
            x = oracle.synth_i64(n, 42, 0, 50, 1)
            k = oracle.synth_i64(n, 7, 0, 32, 0)
            v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
            q(c, "DROP TABLE IF EXISTS fm")
            q(c, f"CREATE TABLE fm AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
                 f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, "
                 f"(mbx_synth(9, i, 1099511627776) - 549755813888) * 4194304 AS w FROM range({n}) tbl(i)")
            w = v.astype(object) * 4194304  # |w| < 2^61: the int64 SUM would overflow -> int128 mode
            cases = [("x > 24 AND k < 16", (x > 24) & (k < 16), "v"),
                     ("x BETWEEN 5 AND 30 AND k >= 3 AND v > 0", (x >= 5) & (x <= 30) & (k >= 3) & (v > 0), "v"),
                     ("k = 7 AND x < 40", (k == 7) & (x < 40), "x"),
                     ("k < 16", k < 16, "v"),            # one predicate column of another width
                     ("x > 24 AND k < 16", (x > 24) & (k < 16), None)]
            for where, m, col in cases:
                if col is None:
                    got = one(c, f"SELECT COUNT(*) FROM fm WHERE {where}")
                    assert int(got[0]) == int(m.sum()), (n, where)
                else:
                    got = one(c, f"SELECT COUNT(*), SUM({col}), MIN({col}), MAX({col}) FROM fm WHERE {where}")
                    sel = (v if col == "v" else x)[m]
                    assert int(got[0]) == int(m.sum()), (n, where)
                    if m.sum():
                        assert [int(g) for g in got[1:]] == [int(sel.astype(object).sum()), int(sel.min()), int(sel.max())]
                    else:
                        assert got[1:] == ["", "", ""]
                if n >= 256:
                    names = [kk["name"] for kk in c.last_profile()["kernels"]]
                    assert "filter_multi" in names, (where, names)
            # SUM without MIN/MAX: int64 accumulation (narrow) and int128 (w), agg column not first
            for col, vals in (("v", v.astype(object)), ("w", w), ("x", x.astype(object))):
                for where, m in (("x > 24 AND k < 16", (x > 24) & (k < 16)), ("k >= 3 AND x <= 30", (k >= 3) & (x <= 30))):
                    got = one(c, f"SELECT COUNT(*), SUM({col}) FROM fm WHERE {where}")
                    assert int(got[0]) == int(m.sum()), (n, col, where)
                    assert got[1] == (str(sum(vals[m])) if m.sum() else ""), (n, col, where)
                    if n >= 256:
                        assert "filter_multi" in [kk["name"] for kk in c.last_profile()["kernels"]]
    finally:
        c.close()


# ---- fused run-time compiled GROUP BY (jit::VmGroupAggregate) ---------------------
def _jit_conn(mbx, monkeypatch):
    monkeypatch.setenv("MBX_JIT", "sync")
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    return mbx.connect_with_config(cfg).value


def _kernels(c):
    return [kk["name"] for kk in c.last_profile()["kernels"]]


def _groups_expect(keys, cols, mask):
    """keys: list of per-row key tuples; cols: {name: list of per-row values
    (None = NULL)}; returns {key: {name: (count, sum, min, max)}} over rows
    where mask; plus COUNT(*) under name '*'."""
    acc = {}
    for i, kt in enumerate(keys):
        if not mask[i]:
            continue
        d = acc.setdefault(kt, {"*": [0, 0, None, None]})
        d["*"][0] += 1
        for name, vals in cols.items():
            v = vals[i]
            st = d.setdefault(name, [0, 0, None, None])
            if v is None:
                continue
            st[0] += 1
            st[1] += v
            st[2] = v if st[2] is None else min(st[2], v)
            st[3] = v if st[3] is None else max(st[3], v)
    return acc


def _cell(x):
    return "" if x is None else str(x)


@pytest.mark.parametrize("n", [1, 257, 100_003, 1_000_003])
def test_jit_groupby_expressions_parity(mbx, oracle, monkeypatch, n):
    c = _jit_conn(mbx, monkeypatch)
    try:
        k = oracle.synth_i64(n, 7, 0, 32, 0).tolist()
        k2 = oracle.synth_i64(n, 8, 0, 4, 0).tolist()
        v = oracle.synth_i64(n, 9, 0, 2**40, -2**39).tolist()
        x = oracle.synth_i64(n, 42, 0, 50, 1).tolist()
        q(c, "DROP TABLE IF EXISTS jg")
        q(c, f"CREATE TABLE jg AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
             f"CAST(mbx_synth(8, i, 4) AS INTEGER) AS k2, mbx_synth(9, i, 1099511627776) - 549755813888 AS v, "
             f"mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
        keys1 = [(a,) for a in k]
        keys2 = list(zip(k, k2))
        allrows = [True] * n
        # c3_project: an expression argument over one key
        exp = _groups_expect(keys1, {"v2": [2 * a for a in v]}, allrows)
        res = q(c, "SELECT k, SUM(v * 2), COUNT(*) FROM jg GROUP BY k ORDER BY k")
        assert res.rows == [[str(kk[0]), str(exp[kk]["v2"][1]), str(exp[kk]["*"][0])] for kk in sorted(exp)]
        if n >= 256:
            assert "jit_group" in _kernels(c)
        # two keys, a WHERE over an expression, several statistics
        tmod3 = [(abs(a) % 3) * (1 if a >= 0 else -1) for a in v]  # SQL % truncates
        m = [(x[i] + k2[i] > 24) and (tmod3[i] != 1) for i in range(n)]
        cols = {"vx": [v[i] + x[i] for i in range(n)], "vm": [v[i] - x[i] for i in range(n)],
                "v3": [3 * v[i] for i in range(n)], "v": v}
        exp = _groups_expect(keys2, cols, m)
        res = q(c, "SELECT k, k2, COUNT(*), SUM(v + x), MIN(v - x), MAX(v * 3), COUNT(v) FROM jg "
                   "WHERE x + k2 > 24 AND v % 3 <> 1 GROUP BY k, k2 ORDER BY k, k2")
        want = [[str(kk[0]), str(kk[1]), str(exp[kk]["*"][0]), str(exp[kk]["vx"][1]), str(exp[kk]["vm"][2]),
                 str(exp[kk]["v3"][3]), str(exp[kk]["v"][0])] for kk in sorted(exp)]
        assert res.rows == want
        if n >= 256:
            assert "jit_group" in _kernels(c)
        # the same query without ORDER BY comes out in key order too
        res2 = q(c, "SELECT k, k2, COUNT(*), SUM(v + x), MIN(v - x), MAX(v * 3), COUNT(v) FROM jg "
                    "WHERE x + k2 > 24 AND v % 3 <> 1 GROUP BY k, k2")
        assert res2.rows == want
    finally:
        c.close()


def test_jit_groupby_null_keys_and_args(mbx, monkeypatch):
    c = _jit_conn(mbx, monkeypatch)
    try:
        n = 300_007
        q(c, f"CREATE TABLE jn AS SELECT CASE WHEN i % 7 = 0 THEN NULL ELSE i % 5 END AS a, "
             f"CASE WHEN i % 11 = 0 THEN NULL ELSE CAST(i % 3 AS INTEGER) END AS b, "
             f"CASE WHEN i % 3 = 0 THEN NULL ELSE i * 7 - 1000000 END AS v FROM range({n}) tbl(i)")
        keys = [(None if i % 7 == 0 else i % 5, None if i % 11 == 0 else i % 3) for i in range(n)]
        vals = [None if i % 3 == 0 else i * 7 - 1000000 for i in range(n)]
        exp = _groups_expect(keys, {"v": vals}, [True] * n)
        res = q(c, "SELECT a, b, COUNT(*), COUNT(v), SUM(v + 1), MIN(v), MAX(v), AVG(v) FROM jn GROUP BY a, b "
                   "ORDER BY a, b")
        want = []
        for kk in sorted(exp, key=_sort_key):
            st = exp[kk]["v"]
            want.append([_cell(kk[0]), _cell(kk[1]), str(exp[kk]["*"][0]), str(st[0]),
                         _cell(st[1] + st[0] if st[0] else None), _cell(st[2]), _cell(st[3])])
        assert [r[:7] for r in res.rows] == want
        for r, kk in zip(res.rows, sorted(exp, key=_sort_key)):
            st = exp[kk]["v"]
            if st[0]:
                assert abs(float(r[7]) - st[1] / st[0]) <= 1e-9 * max(1.0, abs(st[1] / st[0]))
            else:
                assert r[7] == ""
        assert "jit_group" in _kernels(c)
        # a NULL group is emitted last with NULL key cells
        assert res.nulls[-1][0] is True and res.nulls[-1][1] is True
    finally:
        c.close()


def test_jit_groupby_int64_wrap_is_exact(mbx, monkeypatch):
    # values near 2^62 in few groups: the per-block int64 LDS sums wrap many
    # times; the wrap counter keeps SUM exact (HUGEINT)
    c = _jit_conn(mbx, monkeypatch)
    try:
        n = 2_000_003
        big = 4611686018427387000
        q(c, f"CREATE TABLE jw AS SELECT CAST(i % 3 AS INTEGER) AS k, "
             f"CASE WHEN i % 5 = 0 THEN -{big} - i ELSE {big} + i END AS v FROM range({n}) tbl(i)")
        exp = {}
        for kk in range(3):
            idx = range(kk, n, 3)
            s = sum((-big - i) if i % 5 == 0 else (big + i) for i in idx)
            exp[kk] = (len(idx), s)
        res = q(c, "SELECT k, COUNT(*), SUM(v + 1) FROM jw GROUP BY k ORDER BY k")
        assert res.rows == [[str(kk), str(exp[kk][0]), str(exp[kk][1] + exp[kk][0])] for kk in range(3)]
        assert "jit_group" in _kernels(c)
        # an overflowing expression raises the interpreter's error
        r = c.query("SELECT k, SUM(v * 4) FROM jw GROUP BY k")
        assert isinstance(r, mbx.Err) and "Overflow in multiplication" in r.error.message
    finally:
        c.close()


# ---- beyond 2^31 rows: 64-bit row indexing through every hot-path kernel ------
BIG_N = 2**31 + 4097


def test_c2_c5_beyond_int32_rows(mbx, oracle):
    import os as _os
    th = min(16, len(_os.sched_getaffinity(0)))
    c = mbx.connect().value
    q(c, f"CREATE TABLE big AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({BIG_N}) tbl(i)")
    cnt, s = oracle.synth_filter_count(42, 0, BIG_N, 50, 1, 25, 2**63 - 1, th)
    assert one(c, "SELECT COUNT(*) FROM big WHERE x > 24") == [str(cnt)]
    assert one(c, "SELECT COUNT(*), SUM(x) FROM big WHERE x > 24") == [str(cnt), str(s)]
    assert one(c, "SELECT COUNT(*) FROM big") == [str(BIG_N)]
    # compaction with output positions past 2^31, checked by aggregates and the tail rows
    q(c, "CREATE TABLE bigsel AS SELECT x FROM big WHERE x > 24")
    assert one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM bigsel") == [str(cnt), str(s), "25", "50"]
    tail = oracle.synth_i64(4097, 42, BIG_N - 4097, 50, 1)
    exp_tail = tail[tail > 24][-5:].tolist()
    got = q(c, f"SELECT x FROM bigsel LIMIT 5 OFFSET {cnt - 5}").rows
    assert [int(r[0]) for r in got] == exp_tail
    c.close()


def test_select_rounds_output_positions_beyond_int32(mbx, oracle):
    """The one-pass compaction (select_rounds) with OUTPUT positions past 2^31:
    every one of 2^31 + 4097 rows passes, so the run bases, per-round prefix and
    storer addresses all cross the int32 range; checked by COUNT/SUM/MIN/MAX of
    the result, its head and tail rows, and the kernel that ran."""
    import os as _os
    th = min(16, len(_os.sched_getaffinity(0)))
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    q(c, f"CREATE TABLE big2 AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({BIG_N}) tbl(i)")
    cnt, s = oracle.synth_filter_count(42, 0, BIG_N, 50, 1, 1, 2**63 - 1, th)
    assert cnt == BIG_N
    a = c.query_arrow("SELECT x FROM big2 WHERE x >= 1").value  # device-resident result
    names = [k["name"] for k in c.last_profile()["kernels"]]
    assert "select_rounds" in names, names
    # the reference's arrow row count is an int32 (duckdb_native.c:2277): the low 32 bits
    assert a.row_count() == BIG_N - 2**32
    a.close()
    q(c, "CREATE TABLE bigall AS SELECT x FROM big2 WHERE x >= 1")
    assert one(c, "SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM bigall") == [str(BIG_N), str(s), "1", "50"]
    head = oracle.synth_i64(5, 42, 0, 50, 1).tolist()
    tail = oracle.synth_i64(5, 42, BIG_N - 5, 50, 1).tolist()
    assert [int(r[0]) for r in q(c, "SELECT x FROM bigall LIMIT 5").rows] == head
    assert [int(r[0]) for r in q(c, f"SELECT x FROM bigall LIMIT 5 OFFSET {BIG_N - 5}").rows] == tail
    mid = 2**31 - 2  # the rows either side of output position 2^31
    assert ([int(r[0]) for r in q(c, f"SELECT x FROM bigall LIMIT 4 OFFSET {mid}").rows] ==
            oracle.synth_i64(4, 42, mid, 50, 1).tolist())
    c.close()


def test_c3_beyond_int32_rows(mbx, oracle):
    import os as _os
    th = min(16, len(_os.sched_getaffinity(0)))
    c = mbx.connect().value
    q(c, SYNTH_C3.replace("TABLE g", "TABLE gbig").format(n=BIG_N))
    oc, osum = oracle.synth_groupby(7, 9, 0, BIG_N, 32, 1 << 40, -(1 << 39), th)
    got = q(c, "SELECT k, SUM(v), COUNT(*) FROM gbig GROUP BY k ORDER BY k").rows
    assert [(int(r[0]), int(r[1]), int(r[2])) for r in got] == [(k, osum[k], oc[k]) for k in range(32)]
    c.close()


def test_hbm_calibrate_reports_every_shape(mbx):
    """duckdb_mbx_hbm_calibrate_ex: the box's measured ceilings bench.py reports
    beside the 8 TB/s spec; every shape runs and lands in a sane
    range, and the 3-value entry agrees on the first three slots' meaning."""
    import ctypes
    c = mbx.connect().value
    cal = c.hbm_calibrate(1 << 28, 2)
    for k in ("copy_gbs", "read_nt_gbs", "read_gbs", "ring_read_gbs", "copy_nt4_gbs", "ring_copy_gbs",
              "ring_copy_half_gbs"):
        assert 100.0 < cal[k] < 9000.0, (k, cal)
    out3 = (ctypes.c_double * 3)()
    assert mbx.lib.duckdb_mbx_hbm_calibrate(c._h, 1 << 28, 1, out3) == 1 and all(100.0 < x < 9000.0 for x in out3)
    out2 = (ctypes.c_double * 2)()
    assert mbx.lib.duckdb_mbx_hbm_calibrate_ex(c._h, 1 << 28, 1, out2, 2) == 2
    c.close()


@pytest.mark.parametrize("n", [1, 257, 100_003, 1_000_003])
def test_group_direct_nullable_value(mbx, oracle, monkeypatch, n):
    """F2's group_direct_lds with a NULL-able value column (VV: validity words
    in the ring, COUNT(*) apart from the value's count): COUNT(*), COUNT(vn),
    SUM, MIN, MAX, AVG per key, a key whose values are all NULL (SUM / MIN /
    MAX / AVG NULL, COUNT(vn) 0), with and without a fused WHERE, exact vs
    numpy and equal to the generic path (MBX_GD_NULLS=0)."""
    import numpy as np
    cfg = mbx.Config.create()
    cfg.set("mbx_profile", "true")
    c = mbx.connect_with_config(cfg).value
    q(c, f"CREATE TABLE gn AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, mbx_synth(42, i, 50) + 1 AS x, "
         f"CASE WHEN mbx_synth(19, i, 7) = 0 OR mbx_synth(7, i, 32) = 5 THEN NULL "
         f"ELSE mbx_synth(9, i, 1099511627776) - 549755813888 END AS vn FROM range({n}) tbl(i)")
    k = oracle.synth_i64(n, 7, 0, 32, 0)
    x = oracle.synth_i64(n, 42, 0, 50, 1)
    v = oracle.synth_i64(n, 9, 0, 2**40, -2**39)
    valid = (oracle.synth_i64(n, 19, 0, 7, 0) != 0) & (k != 5)
    for where, m in (("", np.ones(n, bool)), (" WHERE x > 24", x > 24), (" WHERE x > 24 AND k < 20", (x > 24) & (k < 20))):
        sql = f"SELECT k, COUNT(*), COUNT(vn), SUM(vn), MIN(vn), MAX(vn), AVG(vn) FROM gn{where} GROUP BY k ORDER BY k"
        res = q(c, sql)
        if n >= 256:
            assert "group_direct" in _kernels(c), (sql, _kernels(c))
        want = []
        for kk in sorted(set(k[m].tolist())):
            sel = m & (k == kk)
            vs = v[sel & valid]
            want.append([str(kk), str(int(sel.sum())), str(len(vs)), str(int(vs.astype(object).sum())) if len(vs) else "",
                         str(int(vs.min())) if len(vs) else "", str(int(vs.max())) if len(vs) else ""])
        assert [r[:6] for r in res.rows] == want, (n, sql)
        for r in res.rows:  # AVG: DOUBLE of the exact sum / count
            if r[2] == "0":
                assert r[6] == ""
            else:
                assert abs(float(r[6]) - int(r[3]) / int(r[2])) <= 1e-9 * max(1.0, abs(int(r[3]) / int(r[2])))
        monkeypatch.setenv("MBX_GD_NULLS", "0")
        res2 = q(c, sql)
        monkeypatch.delenv("MBX_GD_NULLS")
        if n >= 256:
            assert "group_direct" not in _kernels(c)
        assert [r[:6] for r in res2.rows] == [r[:6] for r in res.rows], (n, sql)
    c.close()
