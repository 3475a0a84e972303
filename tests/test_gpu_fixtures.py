"""All 35 golden fixtures (src/duckdb_fixture_cases.mbt, compared exactly like
expect_query_result in src/duckdb_fixture_helpers.mbt:137-142: columns, row
strings and null masks) through the device path — mirrors the reference test
"native fixtures" (src/duckdb_test.mbt:87-97)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("idx", range(35))
def test_native_fixture(conn, fixtures, idx, mbx):
    case = fixtures[idx]
    r = conn.query(case["sql"])
    assert isinstance(r, mbx.Ok), f"fixture '{case['name']}' failed: {r.error.message}"
    res = r.value
    assert res.columns == case["columns"], case["name"]
    assert res.rows == case["rows"], case["name"]
    assert res.nulls == case["nulls"], case["name"]
