"""Front end on the CPU: parser, binder (DuckDB typing rules) and constant
folding, checked against the reference's golden fixtures
(src/duckdb_fixture_cases.mbt) for every fixture whose SQL reads no table
rows.  Fixtures that scan rows (VALUES / range) need the GPU and are covered by
tests/test_gpu_fixtures.py; here we check they plan onto the device."""
import pytest

from conftest import q

SCANNING = {"multi row values", "simple aggregate", "range function", "range with expression", "range with modulo",
            "multiple aggregates", "sum aggregate", "comparison boolean", "null in values", "case expression"}


def test_fixture_partition(fixtures):
    names = {c["name"] for c in fixtures}
    assert SCANNING <= names and len(fixtures) == 35


@pytest.mark.parametrize("idx", range(35))
def test_constant_fixture(hostconn, fixtures, idx, mbx):
    case = fixtures[idx]
    if case["name"] in SCANNING:
        plan = hostconn.explain(case["sql"])
        assert plan.rstrip().endswith("[device]"), plan
        r = hostconn.query(case["sql"])
        assert isinstance(r, mbx.Err) and "GPU" in r.error.message  # no CPU fallback
        return
    res = q(hostconn, case["sql"])
    assert res.columns == case["columns"], case["name"]
    assert res.rows == case["rows"], case["name"]
    assert res.nulls == case["nulls"], case["name"]


def test_types_of_literals(hostconn):
    res = q(hostconn, "select 42 as i, 3000000000 as b, 170141183460469231731687303715884105727 as h, "
                      "3.5 as d, 1e3 as f, 'x' as s, true as t, NULL as n")
    assert res.column_types == ["Integer", "BigInt", "HugeInt", "Decimal", "Double", "Varchar", "Boolean", "Integer"]
    assert res.rows[0][:6] == ["42", "3000000000", "170141183460469231731687303715884105727", "3.5", "1000.0", "x"]


def test_bigint_min_literal_is_bigint(hostconn):
    # typed test "typed result bigint extremes" (duckdb_test.mbt:1251-1287) needs an integer column type
    res = q(hostconn, "SELECT 9223372036854775807 AS max_val, -9223372036854775808 AS min_val")
    assert res.column_types == ["BigInt", "BigInt"]


def test_arithmetic_typing_and_errors(hostconn, mbx):
    assert q(hostconn, "select 7/2, 7//2, 7%2, -7%2, 1/0, 5%0").rows == [["3.5", "3", "1", "-1", "", ""]]
    r = hostconn.query("select 2147483647 + 1")
    assert isinstance(r, mbx.Err) and r.error.message.startswith("Out of Range Error: Overflow in addition of INT32")
    assert q(hostconn, "select 2147483647::BIGINT + 1").rows == [["2147483648"]]
    r = hostconn.query("select 9223372036854775807 * 2")
    assert isinstance(r, mbx.Err) and "Overflow" in r.error.message


def test_decimal_arithmetic(hostconn):
    res = q(hostconn, "select 1.25 + 2.5, 1.25 * 2.5, 10.00::DECIMAL(15,2) > 24, CAST(24 AS DECIMAL(15,2))")
    assert res.rows == [["3.75", "3.125", "false", "24.00"]]
    assert res.column_types == ["Decimal", "Decimal", "Boolean", "Decimal"]


def test_double_rendering(hostconn):
    rows = q(hostconn, "select 1e20::DOUBLE, 0.1::DOUBLE, 100.0::DOUBLE, 1e-5::DOUBLE, 123456789012345678::DOUBLE, "
                       "(1/3)::DOUBLE, -0.0::DOUBLE").rows[0]
    assert rows == ["1e+20", "0.1", "100.0", "1e-05", "1.2345678901234568e+17", "0.3333333333333333", "-0.0"]


def test_union_all_constants(hostconn):
    res = q(hostconn, "SELECT 1::INTEGER UNION ALL SELECT NULL::INTEGER UNION ALL SELECT 3::INTEGER")
    assert res.rows == [["1"], [""], ["3"]] and res.nulls == [[False], [True], [False]]
    res = q(hostconn, "SELECT 1 UNION ALL SELECT 2 UNION ALL SELECT 3")
    assert res.column_types == ["Integer"]


def test_case_coalesce_in_list(hostconn):
    rows = q(hostconn, "select case when 1 > 2 then 'a' else 'b' end, coalesce(NULL, 2, 3), 3 in (1, 2, 3), "
                       "4 not in (1, 2), 5 between 1 and 10, NULL is null").rows[0]
    assert rows == ["b", "2", "true", "true", "true", "true"]


def test_parse_errors(hostconn, mbx):
    for sql in ["selec 1", "select from", "select 1 +", "select (1", "select 'abc"]:
        r = hostconn.query(sql)
        assert isinstance(r, mbx.Err) and "Error" in r.error.message, sql


def test_binder_errors(hostconn, mbx):
    r = hostconn.query("select * from nonexistent_table")
    assert isinstance(r, mbx.Err) and r.error.message.startswith("Catalog Error: Table with name nonexistent_table")
    r = hostconn.query("select nosuchfunc(1)")
    assert isinstance(r, mbx.Err) and "Catalog Error" in r.error.message


def test_ddl_without_rows_runs_on_host(hostconn):
    q(hostconn, "CREATE TABLE t (id INTEGER, v BIGINT, d DECIMAL(15,2), s VARCHAR)")
    plan = hostconn.explain("SELECT COUNT(*), SUM(v) FROM t WHERE v > 24")
    assert "AGGREGATE" in plan and plan.rstrip().endswith("[device]")
    q(hostconn, "DROP TABLE t")
    q(hostconn, "DROP TABLE IF EXISTS t")


def test_hot_path_plans(hostconn):
    q(hostconn, "CREATE TABLE lineitem (l_quantity DECIMAL(15,2), x BIGINT, k INTEGER)")
    # DECIMAL(15,2) > 24  ->  raw > 2400 on the unscaled int64 (SURVEY.md §8(d) C2 variant)
    plan = hostconn.explain("SELECT COUNT(*) FROM lineitem WHERE l_quantity > 24")
    assert "(#0 > 24.00)" in plan, plan
    plan = hostconn.explain("SELECT i FROM range(1000000) tbl(i) WHERE i%2=0")
    assert "RANGE(0, 1000000, 1)" in plan and "((#0 % 2) = 0)" in plan


def test_prepared_parameter_binding(hostconn, mbx):
    st = hostconn.prepare("SELECT ? * 2 AS x").value
    assert isinstance(st.bind_int(1, 21), mbx.Ok)
    assert st.execute().value.rows == [["42"]]
    assert isinstance(st.bind_bigint(1, 1000000000), mbx.Ok)
    assert st.execute().value.rows == [["2000000000"]]  # duckdb_test.mbt:210-227
    bad = st.bind_int(2, 1)
    assert isinstance(bad, mbx.Err) and "parameter" in bad.error.message
    st.clear_bindings()
    r = st.execute()
    assert isinstance(r, mbx.Err)
    st.close()


def test_bulk_text_pull_matches_per_cell(hostconn):
    # query() pulls every cell in one C call (duckdb_mbx_result_text);
    # query_percell() is the reference's literal per-cell loop
    # (duckdb_native.mbt:477-497).  Same strings, same NULL flags.
    for sql in ["SELECT 1 AS a, NULL AS b, 'héllo' AS c, 2.5 AS d, -9223372036854775808 AS e, '' AS f",
                "SELECT NULL, NULL AS n2, 1e300 AS big, CAST(NULL AS VARCHAR) AS v",
                "SELECT 42 WHERE 1 = 0",
                "CREATE TABLE bulk_t (a INTEGER)"]:
        a = hostconn.query(sql).value
        b = hostconn.query_percell(sql.replace("bulk_t", "bulk_t2")).value
        assert a.rows == b.rows and a.nulls == b.nulls, sql
        assert a.columns == b.columns and a.column_types == b.column_types


def _dec_text(raw, scale):
    # DuckDB's DECIMAL spelling: [-]int.frac with frac zero-padded to the scale
    if scale == 0:
        return str(raw)
    a = abs(raw)
    return ("-" if raw < 0 else "") + f"{a // 10 ** scale}.{a % 10 ** scale:0{scale}d}"


def test_integer_cell_text_random(hostconn):
    """The per-cell and bulk text paths format integer, HUGEINT and DECIMAL
    cells with a 64-bit two-digit formatter (HostColumn::FormatInto); check it
    against Python's exact text over random magnitudes and the extremes."""
    import random
    rng = random.Random(5)
    ints = [0, 1, -1, 9, 10, 99, 100, -100, 2 ** 63 - 1, -2 ** 63, 10 ** 18, -10 ** 18]
    ints += [rng.randrange(-2 ** 63, 2 ** 63) >> rng.randrange(0, 63) for _ in range(60)]
    huge = [2 ** 127 - 1, -2 ** 127 + 1, 10 ** 19 - 1, 10 ** 19, -10 ** 19, 10 ** 38 - 1, 2 ** 64, -(2 ** 64) - 1]
    huge += [rng.randrange(-2 ** 127, 2 ** 127) >> rng.randrange(0, 127) for _ in range(60)]
    cols = [f"({v})::BIGINT" for v in ints] + [f"({v})::HUGEINT" for v in huge]
    want = [str(v) for v in ints] + [str(v) for v in huge]
    decs = []
    for _ in range(60):
        w = rng.choice([4, 9, 15, 18, 30, 38])
        sc = rng.randrange(0, w + 1)
        raw = rng.randrange(-10 ** w + 1, 10 ** w) // 10 ** rng.randrange(0, w)
        decs.append((raw, w, sc))
    decs += [(5, 15, 2), (-5, 15, 2), (-50, 15, 2), (0, 15, 2), (10 ** 38 - 1, 38, 38), (-(10 ** 18) + 1, 18, 18)]
    for raw, w, sc in decs:
        cols.append(f"CAST('{_dec_text(raw, sc)}' AS DECIMAL({w},{sc}))")
        want.append(_dec_text(raw, sc))
    cols += ["true", "false", "42::TINYINT", "(-7)::SMALLINT", "255::UTINYINT", "18446744073709551615::UBIGINT"]
    want += ["true", "false", "42", "-7", "255", "18446744073709551615"]
    sql = "SELECT " + ", ".join(cols)
    assert q(hostconn, sql).rows == [want]
    assert hostconn.query_percell(sql).value.rows == [want]
