"""The reference's native integration tests (src/duckdb_test.mbt), re-expressed
over the host mirror; every statement that reads rows runs on the MI355X."""
import pytest

from conftest import q, one

pytestmark = pytest.mark.gpu


def test_native_stream_large_range(conn, mbx):
    # duckdb_test.mbt:100-113
    s = conn.query_stream("SELECT i FROM RANGE(1000000) tbl(i)").value
    assert s.columns() == ["i"]
    total, chunks = 0, 0
    while True:
        n = s.next_count()
        if n is None:
            break
        assert 0 < n <= 2048
        total += n
        chunks += 1
    assert total == 1000000 and chunks == 489
    s.close()


def test_stream_values_and_end(conn, mbx):
    s = conn.query_stream("SELECT i, i * 2 AS d FROM range(5000) tbl(i) WHERE i % 3 = 0").value
    seen = []
    while True:
        r = s.next()
        assert isinstance(r, mbx.Ok)
        if r.value is None:
            break
        for row in r.value.rows:
            seen.append((int(row[0]), int(row[1])))
    assert seen == [(i, 2 * i) for i in range(0, 5000, 3)]
    s.close()


def test_stream_rejects_decimal(conn, mbx):
    # duckdb_native.c:271-303 whitelist: DECIMAL is not streamable
    r = conn.query_stream("SELECT CAST(i AS DECIMAL(10,2)) FROM range(3) tbl(i)")
    assert isinstance(r, mbx.Err) and r.error.message == "streaming query has unsupported column type"


def _prep(conn, sql, bind):
    st = conn.prepare(sql).value
    bind(st)
    r = st.execute()
    st.close()
    return r


def test_prepare_simple_and_binds(conn, mbx):
    assert _prep(conn, "SELECT 1 AS x", lambda s: None).value.rows == [["1"]]           # :166-187
    assert _prep(conn, "SELECT ? * 2 AS x", lambda s: s.bind_int(1, 21)).value.rows == [["42"]]  # :190-207
    assert _prep(conn, "SELECT ? * 2 AS x", lambda s: s.bind_bigint(1, 1000000000)).value.rows == [["2000000000"]]
    v = _prep(conn, "SELECT ? * 2.0 AS x", lambda s: s.bind_double(1, 2.5)).value.rows[0][0]
    assert v in ("5", "5.0")                                                               # :230-247
    assert _prep(conn, "SELECT ? AS x", lambda s: s.bind_varchar(1, "hello")).value.rows == [["hello"]]
    assert _prep(conn, "SELECT ? AS x", lambda s: s.bind_bool(1, True)).value.rows == [["true"]]
    r = _prep(conn, "SELECT ? AS x", lambda s: s.bind_null(1)).value
    assert r.nulls == [[True]]


def test_prepare_multiple_params_and_rows(conn, mbx):
    r = _prep(conn, "SELECT ? + ? AS s, ? AS t", lambda s: (s.bind_int(1, 10), s.bind_int(2, 32), s.bind_varchar(3, "x")))
    assert r.value.rows == [["42", "x"]]
    r = _prep(conn, "SELECT i FROM range(?) tbl(i) WHERE i > ?", lambda s: (s.bind_int(1, 10), s.bind_int(2, 6)))
    assert r.value.rows == [["7"], ["8"], ["9"]]


def test_prepared_predicate_rebinding(conn, mbx, oracle):
    # 1e9 rows, 5 constants, each answer against the CPU oracle; after the first
    # execute the bound plan is reused with only the constant overwritten
    n = 1_000_000_000
    q(conn, f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
    st = conn.prepare("SELECT COUNT(*), SUM(x) FROM t WHERE x > ?").value
    for k in (0, 24, 37, 49, 50):
        st.bind_bigint(1, k)
        got = st.execute().value.rows[0]
        c, s = oracle.synth_filter_count(42, 0, n, 50, 1, k + 1, 2**63 - 1, 16)
        assert got == [str(c), str(s) if c else ""], k
    assert st.plan_stats() == {"binds": 1, "reuses": 4}
    # a parameter of another type binds again; a catalog change invalidates the plan
    st.bind_int(1, 24)
    assert st.execute().value.rows[0][0] == str(oracle.synth_filter_count(42, 0, n, 50, 1, 25, 2**63 - 1, 16)[0])
    q(conn, "CREATE TABLE other (a INTEGER)")
    st.bind_int(1, 25)
    st.execute()
    assert st.plan_stats() == {"binds": 3, "reuses": 4}
    st.close()
    q(conn, "DROP TABLE t")


def test_prepared_plan_cache_falls_back_to_binding(conn, mbx):
    # parameters folded away or outside expressions (LIMIT, range arguments)
    # leave nothing to patch: every execute binds, and the answers follow the values
    st = conn.prepare("SELECT i FROM range(?) tbl(i) WHERE i > ? + 1 LIMIT ?").value
    for n, lo, lim in ((10, 3, 2), (20, 15, 10), (5, 0, 1)):
        st.bind_bigint(1, n)
        st.bind_bigint(2, lo)
        st.bind_bigint(3, lim)
        assert st.execute().value.rows == [[str(i)] for i in range(lo + 2, n)][:lim]
    assert st.plan_stats()["reuses"] == 0
    st.close()
    st = conn.prepare("SELECT ? AS v, i FROM range(3) tbl(i) WHERE i >= ?").value
    for v in ("a", "bb", "ccc"):
        st.bind_varchar(1, v)
        st.bind_bigint(2, 1)
        assert st.execute().value.rows == [[v, "1"], [v, "2"]]
    assert st.plan_stats() == {"binds": 1, "reuses": 2}
    st.close()


def _appender(conn, mbx, setup, fn, verify):
    q(conn, setup)
    ap = conn.create_appender("main", "test_table").value
    r = fn(ap)
    assert isinstance(r, mbx.Ok), r.error.message
    ap.close()  # close implies flush (duckdb_test.mbt:430-447)
    return q(conn, verify)


def test_appender_basic_int(conn, mbx):
    def f(a):
        a.begin_row(); a.append_int(1); a.append_int(100); return a.end_row()
    res = _appender(conn, mbx, "CREATE TABLE test_table (id INTEGER, value INTEGER)", f,
                    "SELECT * FROM test_table ORDER BY id")                                   # :478-523
    assert res.rows == [["1", "100"]]


def test_appender_types(conn, mbx):
    def f(a):
        a.begin_row(); a.append_int(1); a.append_varchar("hello"); a.append_double(3.5); a.append_bool(True)
        return a.end_row()
    res = _appender(conn, mbx, "CREATE TABLE test_table (id INTEGER, name VARCHAR, d DOUBLE, b BOOLEAN)", f,
                    "SELECT * FROM test_table ORDER BY id")
    assert res.rows == [["1", "hello", "3.5", "true"]]


def test_appender_null_and_multiple_rows(conn, mbx):
    def f(a):
        a.begin_row(); a.append_int(2); a.append_int(20); a.end_row()
        a.begin_row(); a.append_int(1); a.append_null(); return a.end_row()
    res = _appender(conn, mbx, "CREATE TABLE test_table (id INTEGER, value INTEGER)", f,
                    "SELECT * FROM test_table ORDER BY id")                                    # :643-760
    assert res.rows == [["1", ""], ["2", "20"]] and res.nulls == [[False, True], [False, False]]
    assert res.cell(0, 1) is None


def test_appender_bigint(conn, mbx):
    def f(a):
        a.begin_row(); a.append_int(1); a.append_bigint(1000000000); return a.end_row()
    res = _appender(conn, mbx, "CREATE TABLE test_table (id INTEGER, value BIGINT)", f,
                    "SELECT * FROM test_table ORDER BY id")                                    # :763-799
    assert res.rows == [["1", "1000000000"]]


def test_appender_errors(conn, mbx):
    q(conn, "CREATE TABLE test_table (id INTEGER, value INTEGER)")
    a = conn.create_appender("main", "test_table").value
    a.begin_row()
    a.append_int(1)
    r = a.end_row()
    assert isinstance(r, mbx.Err) and "EndRow" in r.error.message
    a.append_int(2)
    r = a.append_int(3)
    assert isinstance(r, mbx.Err) and r.error.message == "Too many appends for chunk!"
    a.close()
    assert isinstance(conn.create_appender("main", "no_such_table"), mbx.Err)


def test_appender_decimal_date(conn, mbx):
    def f(a):
        a.begin_row(); a.append_decimal(15, 2, 12345); a.append_date(19877); a.append_timestamp(0); return a.end_row()
    res = _appender(conn, mbx, "CREATE TABLE test_table (d DECIMAL(15,2), dt DATE, ts TIMESTAMP)", f,
                    "SELECT * FROM test_table")
    assert res.rows == [["123.45", "2024-06-03", "1970-01-01 00:00:00"]]


def test_typed_result_columnar_access(conn, mbx):
    # duckdb_test.mbt:1198-1248
    res = q(conn, "SELECT * FROM (VALUES (1, 'a'), (2, 'b'), (3, NULL)) AS t(id, name)")
    typed = res.to_typed()
    assert typed.get_int_column(0) == [1, 2, 3]
    assert typed.get_string_column(1) == ["a", "b", None]


def test_typed_result_bigint_extremes(conn, mbx):
    # duckdb_test.mbt:1251-1287: Int is 32-bit; typed ints saturate
    typed = q(conn, "SELECT 9223372036854775807 AS max_val, -9223372036854775808 AS min_val").to_typed()
    i = typed.get_int(0, 0)
    assert i == 2**31 - 1 and ((i + 1 + 2**31) % 2**32) - 2**31 < 0
    j = typed.get_int(0, 1)
    assert j == -2**31 and ((j - 1 + 2**31) % 2**32) - 2**31 > 0


def test_typed_get_value(conn, mbx):
    typed = q(conn, "SELECT 42 AS num, 'text' AS str, NULL AS nul").to_typed()
    assert typed.get_value(0, 0) == mbx.Value("Int", 42)
    assert typed.get_value(0, 1) == mbx.Value("String", "text")
    assert typed.get_value(0, 2) == mbx.Value("Null")


def test_typed_hugeint_and_decimal_stay_strings(conn, mbx):
    # duckdb_parsing.mbt:124-141: HUGEINT/DECIMAL -> Value::String
    q(conn, "CREATE TABLE t AS SELECT i AS x, CAST(i AS DECIMAL(15,2)) AS d FROM range(10) tbl(i)")
    res = q(conn, "SELECT SUM(x), SUM(d) FROM t")
    assert res.column_types == ["HugeInt", "Decimal"] and res.rows == [["45", "45.00"]]
    typed = res.to_typed()
    assert typed.get_value(0, 0) == mbx.Value("String", "45")


def test_separate_connections_do_not_share_tables(conn, mbx):
    q(conn, "CREATE TABLE only_here (x INTEGER)")
    other = mbx.connect().value
    assert isinstance(other.query("SELECT * FROM only_here"), mbx.Err)
    other.close()


def test_insert_values_and_select(conn):
    q(conn, "CREATE TABLE t (a INTEGER, b VARCHAR, c DOUBLE)")
    assert q(conn, "INSERT INTO t VALUES (1, 'x', 1.5), (2, NULL, NULL), (3, 'z', -2.0)").rows == [["3"]]
    res = q(conn, "SELECT a, b, c FROM t WHERE a >= 2 ORDER BY a DESC")
    assert res.rows == [["3", "z", "-2.0"], ["2", "", ""]]
    assert res.nulls == [[False, False, False], [False, True, True]]
    assert q(conn, "INSERT INTO t SELECT a + 10, b, c FROM t").rows == [["3"]]
    assert one(conn, "SELECT COUNT(*), SUM(a), COUNT(b), MIN(c), MAX(c) FROM t") == ["6", "42", "4", "-2.0", "1.5"]


@pytest.mark.gpu
def test_bulk_text_pull_matches_per_cell_on_device(conn):
    # multi-row device results with NULLs, VARCHAR, DECIMAL, HUGEINT and DOUBLE
    conn.query("DROP TABLE IF EXISTS bt")
    r = conn.query("CREATE TABLE bt AS SELECT i AS a, CASE WHEN i % 3 = 0 THEN NULL WHEN i % 3 = 1 THEN 'one' "
                   "ELSE 'twó' END AS b, CAST(i AS DECIMAL(15,2)) AS c, i * 0.5 AS d, "
                   "CAST(i AS HUGEINT) * 1000000000000 AS h FROM range(3000) tbl(i)")
    assert hasattr(r, "value"), r
    for sql in ["SELECT * FROM bt", "SELECT a % 7 AS k, SUM(a), COUNT(b), SUM(c) FROM bt GROUP BY a % 7 ORDER BY k",
                "SELECT b, h FROM bt WHERE a > 2990 ORDER BY a"]:
        a = conn.query(sql).value
        b = conn.query_percell(sql).value
        assert a.rows == b.rows and a.nulls == b.nulls and a.columns == b.columns, sql
        assert len(a.rows) > 0
